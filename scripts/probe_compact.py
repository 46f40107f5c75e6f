"""Perf probe: would compacting contact envs help?  Times the physics kernel on
the bench's stationary state distribution: all envs, only the envs in contact,
only the free ones.  Not part of the bench contract."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch, ogbench_amd

dev = torch.device('cuda', 0)
n = 65536
env = ogbench_amd.make('pointmaze-large-v0', num_envs=n, device=dev, auto_reset=True)
env.reset(seed=0, options=dict(task_id=(torch.arange(n, device=dev, dtype=torch.int32) % 5) + 1))
g = torch.Generator(device=dev); g.manual_seed(1)
for i in range(600):
    env.step(torch.rand(n, 2, device=dev, generator=g) * 2 - 1)
q = env.get_xy()
a = torch.rand(n, 2, device=dev, generator=g) * 2 - 1


def t_us(qq, aa, reps=50):
    env.physics(qq, aa)
    torch.cuda.synchronize()
    torch.cuda._sleep(int(reps * 60e-6 * 2.4e9))
    ev = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(); env.physics(qq, aa); e.record(); ev.append((s, e))
    torch.cuda.synchronize()
    return float(np.median([s.elapsed_time(e) for s, e in ev])) * 1e3


out, cf = env.physics(q, a)
c = cf.bool()
print(f'contact fraction {c.float().mean().item():.3f}')
print(f'all     {t_us(q, a):8.1f} us  n={n}')
qc, ac = q[c].contiguous(), a[c].contiguous()
qf, af = q[~c].contiguous(), a[~c].contiguous()
print(f'contact {t_us(qc, ac):8.1f} us  n={qc.shape[0]}')
print(f'free    {t_us(qf, af):8.1f} us  n={qf.shape[0]}')
# contact envs sorted by cell (coherent waves)
ij = env.xy_to_ij(qc)
key = ij[:, 0].long() * 64 + ij[:, 1].long()
o = torch.argsort(key)
print(f'contact sorted-by-cell {t_us(qc[o].contiguous(), ac[o].contiguous()):8.1f} us')
for epw in (32, 16):
    env._L.ogbx_maze_set_envs_per_wave(env._h, epw)
    print(f'contact epw{epw} {t_us(qc, ac):8.1f} us')
env._L.ogbx_maze_set_envs_per_wave(env._h, 64)
