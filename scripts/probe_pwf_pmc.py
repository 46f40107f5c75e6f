"""PMC probe of the full powderworld forward (run under rocprofv3 --pmc): loads
the medium 64x64 worlds cached by scripts/probe_pwf.py (gpurun_out/
pwf_worlds_medium.pt) and launches pwf_forward_kernel three times on them.
Not part of the bench contract."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ogbench_amd  # noqa: E402

dev = torch.device('cuda', 0)
w = torch.load(os.path.join('gpurun_out', 'pwf_worlds_medium.pt'), weights_only=True).to(dev)
env = ogbench_amd.make('powderworld-medium-v0', num_envs=1, device=dev, world_size=64)
for _ in range(3):
    env.forward_full(w, 1)
torch.cuda.synchronize()
print('done')
