"""Diagnostic: maze_step cost right after a synchronized reset vs steady state.
Per-step kernel time (HIP events) in buckets of steps after reset; with
OGBX_LIB=<stats build> also the physics path counters per bucket (see
probe_stats.py for the counter meanings)."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, ogbench_amd
from ogbench_amd import _lib
dev = torch.device('cuda', 0)
n = 65536
env = ogbench_amd.make('pointmaze-large-v0', num_envs=n, device=dev, auto_reset=True)
L = _lib.lib()
stats = hasattr(L, 'ogbx_diag_phys_stats')
buf = (ctypes.c_ulonglong * 32)()
env.reset(seed=0, options=dict(task_id=(torch.arange(n, device=dev, dtype=torch.int32) % 5) + 1))
g = torch.Generator(device=dev); g.manual_seed(1)
acts = torch.rand(64, n, 2, device=dev, generator=g) * 2 - 1
ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(400)]
if stats:
    torch.cuda.synchronize(); L.ogbx_diag_phys_stats(buf)
for b0 in range(0, 400, 25):
    for i in range(b0, b0 + 25):
        ev[i][0].record(); env.step(acts[i % 64]); ev[i][1].record()
    torch.cuda.synchronize()
    t = sum(ev[i][0].elapsed_time(ev[i][1]) for i in range(b0, b0 + 25)) / 25 * 1e3
    cont = float(env.physics(env.get_xy(), acts[0])[1].float().mean())
    line = f'steps {b0:3d}-{b0 + 24:3d}: {t:6.1f} us/step  contact frac {cont:.3f}'
    if stats:
        L.ogbx_diag_phys_stats(buf); s = list(buf)
        line += (f' | lane-stages n0..3 {s[:4]} newton_its {s[4]} fallbacks {s[5]} contact_steps {s[6]}'
                 f' wave: contact {s[9]} newton {s[8]} band {s[10]} diag {s[11]} slow {s[12]} newton_its {s[13]}')
    print(line, flush=True)
