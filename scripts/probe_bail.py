"""Diagnostic: how often the lean contact loop bails to the full loop
(point_contact.h point_step_as; counter 14 = waves that redo the step).
Inputs: the near-wall random states of tests/test_locomaze_gpu.py and the
bench's warmed-up pointmaze-large states.
Run with OGBX_LIB=_abx/libogbx_stats.so (scripts/build_maze_variant.sh stats -DOGBX_PHYS_STATS)."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch, ogbench_amd
from ogbench_amd import _lib
from oracle import locomaze as orc
dev = torch.device('cuda', 0)
L = _lib.lib()
buf = (ctypes.c_ulonglong * 32)()
L.ogbx_diag_phys_stats(buf)
for maze in ('medium', 'large', 'giant', 'arena'):
    rng = np.random.RandomState(sum(map(ord, maze)))
    mp, _ = orc.tables(maze)
    cells = np.argwhere(mp == 0)
    n = 20000
    c = cells[rng.randint(len(cells), size=n)]
    q = np.stack([c[:, 1] * 4.0 - 4 + rng.uniform(-1.9, 1.9, n), c[:, 0] * 4.0 - 4 + rng.uniform(-1.9, 1.9, n)], 1)
    a = rng.uniform(-1, 1, (n, 2)).astype(np.float32)
    env = ogbench_amd.MazeEnv('point', maze, num_envs=1, device=dev)
    env.physics(torch.tensor(q), torch.tensor(a))
    torch.cuda.synchronize()
    L.ogbx_diag_phys_stats(buf)
    s = list(buf)
    print(f'{maze:7s} near-wall: contact wave-steps {s[9] // 20} bail waves {s[14]} slow wave-stages {s[12]}', flush=True)
n = 65536
env = ogbench_amd.MazeEnv('point', 'large', num_envs=n, device=dev, auto_reset=True)
env.reset(seed=0, options=dict(task_id=torch.arange(n, device=dev) % 5 + 1))
acts = torch.rand(64, n, 2, device=dev) * 2 - 1
L.ogbx_diag_phys_stats(buf)
for i in range(300):
    env.step(acts[i % 64])
torch.cuda.synchronize()
L.ogbx_diag_phys_stats(buf)
s = list(buf)
print(f'bench 300 steps: contact wave-stages {s[9]} bail waves {s[14]} slow wave-stages {s[12]} '
      f'iterating wave-stages {s[13]} band wave-stages {s[10]}', flush=True)
print(f'  lean loop: lane mismatches {s[0]} (1 edge {s[1]}, 2 edges {s[2]}, more {s[3]}), '
      f'iterations {s[4]}, single-trip fixes {s[5]}', flush=True)
print(f'  lanes iterating {s[0]}: new contact {s[1]}, friction edge {s[2]}, normal edge {s[3]}; '
      f'trips {s[4]}, settled in one trip {s[5]}; by RK stage 0/1/2: {s[6]} {s[7]} {s[8]}', flush=True)
print(f'  flipping-edge |residual| max: <1e-12 {s[16]}, <1e-9 {s[17]}, <1e-6 {s[18]}, <1e-3 {s[19]}, larger {s[20]}',
      flush=True)
print(f'  first stage of the step {s[21]} (with >= 2 contacts {s[22]}), stage 4 {s[23]}', flush=True)
print(f'  by stage e = 1, 2, 3: {s[24]} {s[25]} {s[26]}; e = 5, 6, 7: {s[27]} {s[28]} {s[29]}; e >= 8: {s[30]}', flush=True)
print(f'  (local loop) flipped edges per iterating lane: one {s[1]}, two {s[2]}, more {s[3]}', flush=True)
