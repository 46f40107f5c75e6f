"""Perf probe: physics-kernel time vs contact fraction (separates launch cost
from contact compute).  Not part of the bench contract.  OGBX_LIB selects a
diagnostic build (any libogbx.so variant under _abx/)."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch, ogbench_amd
from ogbench_amd import _lib

dev = torch.device('cuda', 0)
env = ogbench_amd.MazeEnv('point', 'large', num_envs=1, device=dev)
L = _lib.lib()
stats = getattr(L, 'ogbx_diag_phys_stats', None)
cells = np.argwhere(env.maze_map == 0)
rng = np.random.RandomState(0)
n = 65536
tag = os.path.basename(os.environ.get('OGBX_LIB', 'libogbx.so'))
for spread in [0.5, 1.3, 1.9]:
    c = cells[rng.randint(len(cells), size=n)]
    q = np.stack([c[:, 1] * 4.0 - 4 + rng.uniform(-spread, spread, n), c[:, 0] * 4.0 - 4 + rng.uniform(-spread, spread, n)], 1)
    a = rng.uniform(-1, 1, (n, 2)).astype(np.float32)
    q, a = torch.tensor(q, device=dev), torch.tensor(a, device=dev)
    out, cf = env.physics(q, a)
    torch.cuda.synchronize()
    if stats:
        buf = (ctypes.c_ulonglong * 32)()
        stats(buf)
    evs = []
    for _ in range(30):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(); env.physics(q, a); e.record(); evs.append((s, e))
    torch.cuda.synchronize()
    ms = np.median([s.elapsed_time(e) for s, e in evs])
    line = f'{tag} spread {spread}: contact {cf.float().mean().item():.3f} kernel {ms*1e3:.1f} us'
    if stats:
        buf = (ctypes.c_ulonglong * 32)()
        env.physics(q, a); torch.cuda.synchronize(); stats(buf)
        line += f' | stages n0..3={list(buf)[:4]} newton_its={buf[4]} fallbacks={buf[5]} slowpaths={buf[6]}'
    print(line, flush=True)
