"""Diagnostic: is the slow phase after a synchronized reset in the physics?
Times the physics-only launch (env.physics) on the states of step 10 and
step 300 after reset; with OGBX_LIB=<stamps build> also the per-wave cycle
split (collide / solve / update / total) of point_step on those states."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch, ogbench_amd
from ogbench_amd import _lib
dev = torch.device('cuda', 0)
n = 65536
env = ogbench_amd.make('pointmaze-large-v0', num_envs=n, device=dev, auto_reset=True)
L = _lib.lib()
stamps = hasattr(L, 'ogbx_diag_phys_stamps')
env.reset(seed=0, options=dict(task_id=(torch.arange(n, device=dev, dtype=torch.int32) % 5) + 1))
g = torch.Generator(device=dev); g.manual_seed(1)
acts = torch.rand(64, n, 2, device=dev, generator=g) * 2 - 1


def t(q, a, reps=20):
    for _ in range(3):
        env.physics(q, a)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); s.record()
    for _ in range(reps):
        env.physics(q, a)
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


for i in range(301):
    env.step(acts[i % 64])
    if i in (10, 30, 300):
        torch.cuda.synchronize()
        q = env.get_xy().clone(); a = acts[(i + 1) % 64]
        cf = env.physics(q, a)[1].bool()
        line = f'step {i}: physics all {t(q, a):6.1f} us, contact {t(q[cf].contiguous(), a[cf].contiguous()):6.1f} us, free {t(q[~cf].contiguous(), a[~cf].contiguous()):6.1f} us ({int(cf.sum())} contact)'
        # sorted by env-index: contact lanes per wave
        per_wave = cf.view(-1, 64).sum(1).float()
        line += f' | contact lanes/wave mean {per_wave.mean():.1f} max {int(per_wave.max())}, waves with any {int((per_wave > 0).sum())}'
        if stamps:
            buf = (ctypes.c_ulonglong * (4096 * 4))()
            L.ogbx_diag_phys_stamps(buf)
            env.physics(q, a); torch.cuda.synchronize()
            L.ogbx_diag_phys_stamps(buf)
            st = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 4)[: n // 64].astype(np.float64)
            tot = st[:, 3]; w = int(np.argmax(tot))
            line += (f' | wave cycles mean {tot.mean():.0f} p50/p99/max {np.percentile(tot, [50, 99, 100]).astype(int)}'
                     f' slowest c/s/u {st[w, 0]:.0f}/{st[w, 1]:.0f}/{st[w, 2]:.0f}')
        print(line, flush=True)
