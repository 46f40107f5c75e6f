"""Perf probe: physics/step kernel time vs envs-per-wave."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch, ogbench_amd
from ogbench_amd import _lib
dev = torch.device('cuda', 0)
env = ogbench_amd.MazeEnv('point', 'large', num_envs=65536, device=dev, auto_reset=True)
cells = np.argwhere(env.maze_map == 0)
rng = np.random.RandomState(0)
n = 65536
def timeit(fn, reps=30):
    evs = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(); fn(); e.record(); evs.append((s, e))
    torch.cuda.synchronize()
    return np.median([s.elapsed_time(e) for s, e in evs]) * 1e3
c = cells[rng.randint(len(cells), size=n)]
q = np.stack([c[:, 1] * 4.0 - 4 + rng.uniform(-1.5, 1.5, n), c[:, 0] * 4.0 - 4 + rng.uniform(-1.5, 1.5, n)], 1)
a = torch.tensor(rng.uniform(-1, 1, (n, 2)).astype(np.float32), device=dev)
q = torch.tensor(q, device=dev)
env.reset(seed=0, options=dict(task_id=torch.arange(n, device=dev) % 5 + 1))
acts = torch.rand(64, n, 2, device=dev) * 2 - 1
for _ in range(200):
    env.step(acts[_ % 64])
ref = None
for epw in [64, 32, 16, 8]:
    _lib.check(env._L.ogbx_maze_set_envs_per_wave(env._h, epw))
    out, cf = env.physics(q, a)
    if ref is None: ref = out.clone()
    same = bool(torch.equal(out, ref))
    tp = timeit(lambda: env.physics(q, a))
    ts = timeit(lambda: env.step(acts[0]))
    print(f'epw {epw}: physics {tp:.1f} us  step {ts:.1f} us  identical={same}', flush=True)
