"""Diagnostic: phase times of pwf_step_kernel per env (workgroup) in the
powder-medium bench setting: state load, step body (forward + paint + success),
observation + state store; and the launch span.  Run with
OGBX_LIB=_ab/libogbx_pwfst.so (scripts/build_pwf_variant.sh pwfst ... no:
SRC=powder scripts/build_maze_variant.sh pwfst -DOGBX_PWF_STAMPS)."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch, ogbench_amd
from ogbench_amd import _lib
dev = torch.device('cuda', 0)
L = _lib.lib()
n = 4096
env = ogbench_amd.make('powderworld-medium-v0', num_envs=n, device=dev, world_size=64, auto_reset=True)
env.reset(seed=0, options=dict(task_id=(torch.arange(n, dtype=torch.int32, device=dev) % 5) + 1))
gen = torch.Generator(device=dev); gen.manual_seed(5)
ring = 96
xy = env._xy_action_size
hi = torch.tensor([5 if i % 3 == 0 else xy for i in range(ring)], device=dev).view(ring, 1)
acts = (torch.rand(ring, n, device=dev, generator=gen) * hi).to(torch.int32)
buf = (ctypes.c_ulonglong * (4096 * 4))()
rows = []
for i in range(240):
    env.step(acts[i % ring])
    if i >= 120 and i % 3 == 2:
        torch.cuda.synchronize()
        L.ogbx_diag_pwf_stamps(buf)
        a = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 4).astype(np.int64)
        rows.append(a.copy())
A = np.stack(rows)  # [launches, env, 4]
load = (A[..., 1] - A[..., 0]) / 100.0
body = (A[..., 2] - A[..., 1]) / 100.0
tail = (A[..., 3] - A[..., 2]) / 100.0
tot = (A[..., 3] - A[..., 0]) / 100.0
span = (A[..., 3].max(1) - A[..., 0].min(1)) / 100.0
print(f'forward launches {len(rows)}: span {span.mean():.1f} us; per env: load {load.mean():.2f} us, '
      f'body {body.mean():.2f} us (p90 {np.percentile(body, 90):.2f}), observe+store {tail.mean():.2f} us, '
      f'total {tot.mean():.2f} us; envs per CU in sequence ~{span.mean() / tot.mean() / 1:.1f} '
      f'(256 CUs, {n} envs = {n / 256:.0f} per CU)', flush=True)
