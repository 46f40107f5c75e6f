"""Diagnostic: per-wave duration distribution of one maze_step_kernel launch in
the bench setting (pointmaze-large, N envs, after `warm` auto-reset steps).
Run with OGBX_LIB=_abx/libogbx_<v>.so built with -DOGBX_WAVE_STAMPS
(scripts/build_maze_variant.sh <v> -DOGBX_WAVE_STAMPS [...])."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch, ogbench_amd
from ogbench_amd import _lib
dev = torch.device('cuda', 0)
L = _lib.lib()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
env = ogbench_amd.MazeEnv('point', 'large', num_envs=n, device=dev, auto_reset=True)
env.reset(seed=0, options=dict(task_id=torch.arange(n, device=dev) % 5 + 1))
gen = torch.Generator(device=dev).manual_seed(1)
acts = torch.rand(64, n, 2, device=dev, generator=gen) * 2 - 1
buf = (ctypes.c_ulonglong * (4096 * 4))()
durs, cycs, spans, paths = [], [], [], []
for i in range(400):
    if i >= 100 and i % 10 == 0:
        torch.cuda.synchronize()
        L.ogbx_diag_wave_stamps(buf)  # clears the path counters
    env.step(acts[i % 64])
    if i >= 100 and i % 10 == 0:
        torch.cuda.synchronize()
        L.ogbx_diag_wave_stamps(buf)
        a = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 4)[: (n + 63) // 64].astype(np.int64)
        t0, t1 = a[:, 0], a[:, 1]
        durs.append((t1 - t0) / 100.0)  # us (100 MHz)
        cycs.append(a[:, 2])
        p = a[:, 3].astype(np.uint64)
        paths.append(np.stack([p & 0xFFFFF, (p >> 20) & 0xFFFFF, p >> 40], 1).astype(np.int64))
        spans.append(((t1.max() - t0.min()) / 100.0, (t0.max() - t0.min()) / 100.0))
d = np.concatenate(durs); c = np.concatenate(cycs); sp = np.array(spans)
print(f'N={n}: wave us mean {d.mean():.2f} p50 {np.median(d):.2f} p90 {np.percentile(d, 90):.2f} '
      f'p99 {np.percentile(d, 99):.2f} max {d.max():.2f}; cycles mean {c.mean():.0f} max {c.max()} '
      f'-> {c.mean() / d.mean() / 1e3:.2f} GHz; launch span (first start..last end) {sp[:, 0].mean():.2f} us, '
      f'start spread {sp[:, 1].mean():.2f} us; per-launch max wave {np.mean([x.max() for x in durs]):.2f} us', flush=True)
P = np.concatenate(paths)
order = np.argsort(d)
for name, sel in (('fastest 50%', order[: len(d) // 2]), ('p90-p99', order[int(.9 * len(d)):int(.99 * len(d))]),
                  ('top 1%', order[int(.99 * len(d)):])):
    print(f'  {name:12s}: wave us {d[sel].mean():.2f}; per wave cold entries {P[sel, 0].mean():.1f}, '
          f'iteration trips {P[sel, 1].mean():.1f}, band stages {P[sel, 2].mean():.1f}', flush=True)
