"""PMC probe of the point physics kernel on the bench's stationary states:
one launch over all envs and one over the contact envs only (run under
rocprofv3 --pmc).  Not part of the bench contract."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, ogbench_amd

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
for _ in range(3):
    env.physics(q, a)
for _ in range(3):
    env.physics(qc, ac)
torch.cuda.synchronize()
print('contact envs', qc.shape[0])
