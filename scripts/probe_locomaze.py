"""Perf probe: physics-kernel time vs contact fraction (separates launch cost
from contact compute).  Not part of the bench contract."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch, ogbench_amd

dev = torch.device('cuda', 0)
env = ogbench_amd.MazeEnv('point', 'large', num_envs=1, device=dev)
mp = env.maze_map
cells = np.argwhere(mp == 0)
rng = np.random.RandomState(0)
n = 65536
def mk(spread):
    c = cells[rng.randint(len(cells), size=n)]
    q = np.stack([c[:, 1] * 4.0 - 4 + rng.uniform(-spread, spread, n), c[:, 0] * 4.0 - 4 + rng.uniform(-spread, spread, n)], 1)
    a = rng.uniform(-1, 1, (n, 2)).astype(np.float32)
    return torch.tensor(q, device=dev), torch.tensor(a, device=dev)
for spread in [0.5, 1.1, 1.3, 1.5, 1.9]:
    q, a = mk(spread)
    out, c = env.physics(q, a)
    torch.cuda.synchronize()
    evs = []
    for _ in range(50):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(); env.physics(q, a); e.record(); evs.append((s, e))
    torch.cuda.synchronize()
    ms = np.median([s.elapsed_time(e) for s, e in evs])
    print(f'spread {spread}: contact frac {c.float().mean().item():.3f}  physics kernel {ms*1e3:.1f} us', flush=True)
