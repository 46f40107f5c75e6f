"""Diagnostic: per-wave (max over lanes) cycle split of point_step
(collide / solve / update) on realistic states: a warmed-up pointmaze-large
rollout.  Run with OGBX_LIB=<a -DOGBX_PHYS_STAMPS build>."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch, ogbench_amd
from ogbench_amd import _lib
dev = torch.device('cuda', 0)
n = 65536
env = ogbench_amd.MazeEnv('point', 'large', num_envs=n, device=dev, auto_reset=True)
L = _lib.lib()
env.reset(seed=0, options=dict(task_id=torch.arange(n, device=dev) % 5 + 1))
acts = torch.rand(64, n, 2, device=dev) * 2 - 1
for i in range(300):
    env.step(acts[i % 64])
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * (4096 * 4))()
L.ogbx_diag_phys_stamps(buf)
for rep in range(3):
    env.step(acts[rep]); torch.cuda.synchronize()
    L.ogbx_diag_phys_stamps(buf)
    st = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 4)[: n // 64].astype(np.float64)
    tot = st[:, 3]
    w = np.argmax(tot)
    print(f'step {rep}: wave total cycles mean {tot.mean():.0f} p50/p90/p99/max {np.percentile(tot,[50,90,99,100]).astype(int)} '
          f'| slowest wave collide/solve/update {st[w,0]:.0f}/{st[w,1]:.0f}/{st[w,2]:.0f} | mean {st[:,0].mean():.0f}/{st[:,1].mean():.0f}/{st[:,2].mean():.0f}', flush=True)
