"""Probe: powderworld-medium cell-update throughput at 32x32 (NT = 256, 29 KB
LDS, several worlds per CU) vs 64x64 (NT = 1024, 116 KB LDS, one world per
CU) at the same total cell count; random valid actions, auto-reset."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, ogbench_amd
dev = torch.device('cuda', 0)
for size, n in ((64, 4096), (32, 16384)):
    env = ogbench_amd.make('powderworld-medium-v0', num_envs=n, device=dev, world_size=size, auto_reset=True)
    env.reset(seed=0, options=dict(task_id=(torch.arange(n, dtype=torch.int32, device=dev) % 5) + 1))
    ne, xy = 5, env._xy_action_size
    hi = torch.tensor([ne if i % 3 == 0 else xy for i in range(96)], device=dev).view(96, 1)
    acts = (torch.rand(96, n, device=dev) * hi).to(torch.int32)
    for i in range(60):
        env.step(acts[i % 96])
    torch.cuda.synchronize()
    steps = 450
    t0 = time.perf_counter()
    for i in range(steps):
        env.step(acts[i % 96])
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    print(f'size {size} n {n}: {dt*1e3:.3f} ms/step, {n*size*size/dt/1e9:.2f} G cell-steps/s', flush=True)
    env.close()
