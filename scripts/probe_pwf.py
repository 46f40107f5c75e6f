"""Time the full powderworld forward (pwf_forward_kernel, Philox rand fields)
on realistic medium/hard 64x64 worlds: N envs driven by random actions for a
while, then `steps` forwards of all worlds timed with HIP events."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ogbench_amd  # noqa: E402

dev = torch.device('cuda', 0)
lib = os.environ.get('OGBX_LIB', 'default').split('/')[-1]
for level in ('medium', 'hard'):
    n, size = 4096, 64
    ne = 5 if level == 'medium' else 8
    env = ogbench_amd.make(f'powderworld-{level}-v0', num_envs=n, device=dev, world_size=size)
    cache = os.path.join('gpurun_out', f'pwf_worlds_{level}.pt')  # same worlds for every build variant
    if os.path.exists(cache):
        w = torch.load(cache, weights_only=True).to(dev)
    else:
        env.reset(seed=1, options=dict(task_id=(torch.arange(n, device=dev) % 5 + 1)))
        rng = np.random.RandomState(0)
        xy = env._xy_action_size
        K = 150
        acts = np.stack([rng.randint(0, ne if t % 3 == 0 else xy, size=n) for t in range(K)])
        env.rollout(acts)
        w = env.world_full().contiguous()
        os.makedirs('gpurun_out', exist_ok=True)
        torch.save(w.cpu(), cache)
    env.forward_full(w, 1)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    steps = 6
    a.record()
    env.forward_full(w, steps)
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / steps
    vel = (w[:, 3:5].abs() > 0).float().mean().item()
    print(f'{lib:28s} {level:6s} forward of {n} worlds {size}x{size}: {ms:.3f} ms  '
          f'({n * size * size / ms / 1e6:.2f} Gcell/s; vel!=0 frac {vel:.3f})', flush=True)
    env.close()
