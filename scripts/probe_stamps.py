"""Diagnostic: per-wave cycle split of point_step (collide / solve / update),
from build/variants/libogbx_stamps.so (OGBX_LIB)."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch, ogbench_amd
from ogbench_amd import _lib
dev = torch.device('cuda', 0)
env = ogbench_amd.MazeEnv('point', 'large', num_envs=1, device=dev)
L = _lib.lib()
cells = np.argwhere(env.maze_map == 0)
rng = np.random.RandomState(0)
n = 65536
for spread in [1.3, 1.9]:
    c = cells[rng.randint(len(cells), size=n)]
    q = np.stack([c[:, 1] * 4.0 - 4 + rng.uniform(-spread, spread, n), c[:, 0] * 4.0 - 4 + rng.uniform(-spread, spread, n)], 1)
    a = rng.uniform(-1, 1, (n, 2)).astype(np.float32)
    q, a = torch.tensor(q, device=dev), torch.tensor(a, device=dev)
    env.physics(q, a); torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * (4096 * 4))()
    L.ogbx_diag_phys_stamps(buf)
    env.physics(q, a); torch.cuda.synchronize()
    L.ogbx_diag_phys_stamps(buf)
    st = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 4)[: n // 64].astype(np.float64)
    tot = st[:, 3]
    w = np.argmax(tot)
    print(f'spread {spread}: waves total cycles mean {tot.mean():.0f} max {tot.max():.0f} | slowest wave split collide/solve/update = {st[w,0]:.0f}/{st[w,1]:.0f}/{st[w,2]:.0f} | mean split {st[:,0].mean():.0f}/{st[:,1].mean():.0f}/{st[:,2].mean():.0f}', flush=True)
    print('  percentiles of total:', np.percentile(tot, [50, 90, 99, 100]).astype(int))
