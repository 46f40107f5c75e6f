"""Diagnostic: fraction of powderworld medium/hard envs whose world holds any
non-zero velocity, over a bench-like rollout (4096 envs, 64x64, random
actions, auto-reset)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, ogbench_amd
dev = torch.device('cuda', 0)
n = 4096
for level in ('medium', 'hard'):
    env = ogbench_amd.make(f'powderworld-{level}-v0', num_envs=n, device=dev, world_size=64, auto_reset=True)
    env.reset(seed=0, options=dict(task_id=(torch.arange(n, dtype=torch.int32, device=dev) % 5) + 1))
    gen = torch.Generator(device=dev); gen.manual_seed(5)
    xy = env._xy_action_size
    fr = []
    for i in range(600):
        hi = 5 if i % 3 == 0 else xy
        env.step((torch.rand(n, device=dev, generator=gen) * hi).to(torch.int32))
        if i % 60 == 59:
            m, v, g = env._full_views()
            anyv = (v.view(n, -1) != 0).any(1).float().mean().item()
            fr.append(round(anyv, 3))
    print(level, 'fraction of envs with any velocity, every 60 steps:', fr, flush=True)
    env.close()
