"""Diagnostic: physics-kernel time on the bench's stationary states, all envs
vs the contact envs only (compacted) vs the free envs only, with HIP events
around launches queued behind a spin kernel (device-paced: env.physics()
allocates its outputs, so a host-paced loop measures the host).  If the
compacted launch (~1/12 of the envs and waves) takes as long as the full one,
the kernel is bound by one wave's contact chain, not by the number of
waves.  (Rounds 3-4 ran this host-paced: their "free only" 9.1 us was the
Python call, not the kernel.)"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch, ogbench_amd

dev = torch.device('cuda', 0)
n = 65536
env = ogbench_amd.make('pointmaze-large-v0', num_envs=n, device=dev, auto_reset=True)
env.reset(seed=0, options=dict(task_id=(torch.arange(n, device=dev, dtype=torch.int32) % 5) + 1))
g = torch.Generator(device=dev); g.manual_seed(1)
for i in range(300):
    env.step(torch.rand(n, 2, device=dev, generator=g) * 2 - 1)
q = env.get_xy()
a = torch.rand(n, 2, device=dev, generator=g) * 2 - 1
out, cf = env.physics(q, a)
c = cf.bool()
qc, ac = q[c].contiguous(), a[c].contiguous()
qf, af = q[~c].contiguous(), a[~c].contiguous()


def t(qq, aa, reps=200):
    for _ in range(5):
        env.physics(qq, aa)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    torch.cuda._sleep(int(reps * 60e-6 * 2.4e9))
    s.record()
    for _ in range(reps):
        env.physics(qq, aa)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


print(f'contact envs {qc.shape[0]} of {n} ({qc.shape[0] / n:.3f})')
print(f'physics all envs      : {t(q, a):7.1f} us')
print(f'physics contact only  : {t(qc, ac):7.1f} us')
print(f'physics free only     : {t(qf, af):7.1f} us')
