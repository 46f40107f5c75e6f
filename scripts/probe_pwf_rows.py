"""Diagnostic: how sparse are powderworld-medium/hard worlds per row?  Over a
bench-like rollout (4096 envs, 64x64, random actions, auto-reset), the mean
fraction of rows (and of 3-row neighbourhoods) that hold each rule's trigger
elements -- the headroom of per-row rule skipping."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch, ogbench_amd
dev = torch.device('cuda', 0)
n = 4096
SETS = {'sand|dust': [2, 12], 'fluid trig': [3, 4, 7, 10, 11, 16, 18], 'fire|lava': [7, 10], 'plant': [8],
        'ice': [6], 'non-empty non-wall': None}
for level in sys.argv[1:] or ['medium']:
    env = ogbench_amd.make(f'powderworld-{level}-v0', num_envs=n, device=dev, world_size=64, auto_reset=True)
    env.reset(seed=0, options=dict(task_id=(torch.arange(n, dtype=torch.int32, device=dev) % 5) + 1))
    gen = torch.Generator(device=dev); gen.manual_seed(5)
    xy = env._xy_action_size
    ne = {'medium': 5, 'hard': 8}[level]
    acc = {k: [] for k in SETS}
    for i in range(450):
        hi = ne if i % 3 == 0 else xy
        env.step((torch.rand(n, device=dev, generator=gen) * hi).to(torch.int32))
        if i % 75 == 74:
            ids = env.world_ids().long()  # [n, 64, 64]
            for k, s in SETS.items():
                m = (ids > 1) if s is None else torch.isin(ids, torch.tensor(s, device=dev))
                row = m.any(2).float()  # [n, 64]
                nb3 = torch.maximum(torch.maximum(row, torch.roll(row, 1, 1)), torch.roll(row, -1, 1))
                acc[k].append((round(row.mean().item(), 3), round(nb3.mean().item(), 3)))
    print(level, 'fraction of rows (row, 3-row neighbourhood) holding the set, every 75 steps:', flush=True)
    for k, v in acc.items():
        print(f'  {k:20s}', v, flush=True)
    env.close()
