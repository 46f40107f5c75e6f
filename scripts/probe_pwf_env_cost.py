"""Diagnostic: spread of the per-env forward cost in the powder-medium/hard
bench setting (rule-stamp build: SRC=powder scripts/build_maze_variant.sh
pwfrs -DOGBX_PWF_RULE_STAMPS, then OGBX_LIB=_abx/libogbx_pwfrs.so python
scripts/probe_pwf_env_cost.py [medium|hard]).  Per env: stamped cycles per
forward over windows of 30 steps (10 forwards) along an episode; prints the
mean, percentiles and max over envs -- how much a longest-first schedule of
the 4,096 workgroups could take off a forward launch's tail."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch, ogbench_amd
from ogbench_amd import _lib
dev = torch.device('cuda', 0)
L = _lib.lib()
n = 4096
level = sys.argv[1] if len(sys.argv) > 1 else 'medium'
env = ogbench_amd.make(f'powderworld-{level}-v0', num_envs=n, device=dev, world_size=64, auto_reset=True)
env.reset(seed=0, options=dict(task_id=(torch.arange(n, dtype=torch.int32, device=dev) % 5) + 1))
gen = torch.Generator(device=dev); gen.manual_seed(5)
ring = 96
xy = env._xy_action_size
hi = torch.tensor([5 if i % 3 == 0 else xy for i in range(ring)], device=dev).view(ring, 1)
acts = (torch.rand(ring, n, device=dev, generator=gen) * hi).to(torch.int32)
buf = (ctypes.c_ulonglong * (4096 * 16))()
def snap():
    torch.cuda.synchronize()
    L.ogbx_diag_pwf_rules(buf)
    return np.frombuffer(buf, dtype=np.uint64).reshape(4096, 16).astype(np.int64).copy()
step = 0
for w0 in (60, 150, 300, 450):
    while step < w0:
        env.step(acts[step % ring]); step += 1
    a = snap()
    for _ in range(30):
        env.step(acts[step % ring]); step += 1
    d = snap() - a
    fw = np.maximum(d[:, 15], 1)
    c = d[:, :10].sum(1) / fw
    q = np.percentile(c, [50, 90, 99])
    print(f'{level} steps {w0}-{w0 + 30}: cycles per forward mean {c.mean():.0f}, p50 {q[0]:.0f}, p90 {q[1]:.0f}, '
          f'p99 {q[2]:.0f}, max {c.max():.0f} (max/mean {c.max() / c.mean():.2f})', flush=True)
