"""Diagnostic: physics path counters on realistic states (a warmed-up
pointmaze-large rollout).  Run with OGBX_LIB=_abx/libogbx_stats.so.
Counters: [0..3] lane-stages with n contacts, 4 Newton iterations (lanes),
5 Armijo fallbacks, 6 contact steps (lanes), 8 wave-stages in Newton mode,
9 wave-stages on the contact path, 10 wave-stages with a transition-band gain,
11 wave-stages with a diagonal candidate, 12 wave-stages with a slow collide,
13 wave Newton iterations."""
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
buf = (ctypes.c_ulonglong * 32)()
L.ogbx_diag_phys_stats(buf)
for rep in range(3):
    env.step(acts[rep]); torch.cuda.synchronize()
    L.ogbx_diag_phys_stats(buf)
    s = list(buf)
    print(f'step {rep}: lane-stages n0..3 {s[:4]} newton_its {s[4]} fallbacks {s[5]} contact_steps {s[6]} | '
          f'wave-stages contact {s[9]} newton {s[8]} band {s[10]} diag {s[11]} slow {s[12]} wave_newton_its {s[13]}', flush=True)
