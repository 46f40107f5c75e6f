"""Diagnostic: physics launch time vs the number of contact lanes per wave.
Contact and free states are taken from a steady-state pointmaze-large rollout
(step 300); each batch of 65,536 envs has k contact lanes in every wave of 64
(the rest free), so only the per-wave composition changes."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, ogbench_amd
dev = torch.device('cuda', 0)
n = 65536
env = ogbench_amd.make('pointmaze-large-v0', num_envs=n, device=dev, auto_reset=True)
env.reset(seed=0, options=dict(task_id=(torch.arange(n, device=dev, dtype=torch.int32) % 5) + 1))
g = torch.Generator(device=dev); g.manual_seed(1)
acts = torch.rand(64, n, 2, device=dev, generator=g) * 2 - 1
for i in range(300):
    env.step(acts[i % 64])
q = env.get_xy().clone(); a = acts[0]
cf = env.physics(q, a)[1].bool()
qc, ac, qf, af = q[cf], a[cf], q[~cf], a[~cf]


def t(qq, aa, reps=20):
    for _ in range(3):
        env.physics(qq, aa)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); s.record()
    for _ in range(reps):
        env.physics(qq, aa)
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


W = n // 64
ORDER = [int(x) for x in os.environ.get('KS', '0,1,2,4,8,13,24,48,64').split(',')]
for k in ORDER:
    ic = torch.arange(W * k, device=dev) % qc.shape[0]
    jf = torch.arange(W * (64 - k), device=dev) % qf.shape[0]
    qq = torch.cat([qc[ic].view(W, k, 2), qf[jf].view(W, 64 - k, 2)], 1).reshape(n, 2).contiguous()
    aa = torch.cat([ac[ic].view(W, k, 2), af[jf].view(W, 64 - k, 2)], 1).reshape(n, 2).contiguous()
    # same contact lanes placed at the end of each wave instead of the start
    qq2 = torch.cat([qf[jf].view(W, 64 - k, 2), qc[ic].view(W, k, 2)], 1).reshape(n, 2).contiguous()
    aa2 = torch.cat([af[jf].view(W, 64 - k, 2), ac[ic].view(W, k, 2)], 1).reshape(n, 2).contiguous()
    # contact lanes spread over the wave (lane j*64//k)
    pos = torch.zeros(64, dtype=torch.bool, device=dev)
    if k:
        pos[(torch.arange(k, device=dev) * 64) // k] = True
    qq3 = torch.empty(W, 64, 2, dtype=q.dtype, device=dev); aa3 = torch.empty(W, 64, 2, dtype=a.dtype, device=dev)
    qq3[:, pos] = qc[ic].view(W, k, 2); qq3[:, ~pos] = qf[jf].view(W, 64 - k, 2)
    aa3[:, pos] = ac[ic].view(W, k, 2); aa3[:, ~pos] = af[jf].view(W, 64 - k, 2)
    # k contact lanes per wave drawn from the LAST contact states instead of the first
    ic4 = qc.shape[0] - 1 - (torch.arange(W * k, device=dev) % qc.shape[0])
    qq4 = torch.cat([qc[ic4].view(W, k, 2), qf[jf].view(W, 64 - k, 2)], 1).reshape(n, 2).contiguous()
    aa4 = torch.cat([ac[ic4].view(W, k, 2), af[jf].view(W, 64 - k, 2)], 1).reshape(n, 2).contiguous()
    print(f'k={k:2d} contact lanes/wave: {t(qq, aa):6.1f} us (first lanes)  {t(qq2, aa2):6.1f} us (last lanes)  '
          f'{t(qq3.view(n, 2), aa3.view(n, 2)):6.1f} us (spread)  {t(qq4, aa4):6.1f} us (other states)', flush=True)
