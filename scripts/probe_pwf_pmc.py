"""PMC probe of the full powderworld forward (run under rocprofv3 --pmc): builds
realistic medium 64x64 worlds with a short random rollout, then launches
pwf_forward_kernel three times on them.  Not part of the bench contract."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ogbench_amd  # noqa: E402

dev = torch.device('cuda', 0)
n, size, ne = 4096, 64, 5
env = ogbench_amd.make('powderworld-medium-v0', num_envs=n, device=dev, world_size=size)
env.reset(seed=1, options=dict(task_id=(torch.arange(n, device=dev) % 5 + 1)))
rng = np.random.RandomState(0)
acts = np.stack([rng.randint(0, ne if t % 3 == 0 else env._xy_action_size, size=n) for t in range(150)])
env.rollout(acts)
w = env.world_full().contiguous()
for _ in range(3):
    env.forward_full(w, 1)
torch.cuda.synchronize()
print('done')
