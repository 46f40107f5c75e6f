"""Diagnostic: maze_step_kernel time per step over a 2,000-step timed region
(one event pair around the region, as bench.py) for envs-per-wave 64/32/16 at
the strong-scaling shares N = 8,192 / 16,384 / 32,768 (warmed-up states)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, ogbench_amd
dev = torch.device('cuda', 0)
for n in (8192, 16384, 32768):
    env = ogbench_amd.make('pointmaze-large-v0', num_envs=n, device=dev, auto_reset=True)
    env.reset(seed=0, options=dict(task_id=(torch.arange(n, device=dev, dtype=torch.int32) % 5) + 1))
    g = torch.Generator(device=dev); g.manual_seed(1)
    acts = torch.rand(64, n, 2, device=dev, generator=g) * 2 - 1
    for i in range(300):
        env.step(acts[i % 64])
    for epw in (64, 32, 16, 64):
        env._L.ogbx_maze_set_envs_per_wave(env._h, epw)
        for i in range(50):
            env.step(acts[i % 64])
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(); s.record()
        for i in range(2000):
            env.step(acts[i % 64])
        e.record(); torch.cuda.synchronize()
        print(f'N={n:6d} epw={epw:2d}: {s.elapsed_time(e) / 2000 * 1e3:6.2f} us/step', flush=True)
    env.close()
