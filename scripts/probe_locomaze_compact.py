"""Diagnostic: physics-kernel time on the bench's stationary states, all envs
vs the contact envs only (compacted), with HIP events.  If the compacted launch
(~1/5 of the envs, ~1/5 of the waves) takes as long as the full one, the
kernel is bound by one wave's contact chain, not by the number of waves."""
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


def t(qq, aa, reps=50):
    for _ in range(5):
        env.physics(qq, aa)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
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
