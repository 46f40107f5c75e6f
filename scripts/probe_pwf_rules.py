"""Diagnostic: shader-clock cycles per rule of the powder forward (per env and
forward, averaged) in the powder-medium bench setting, from the rule-stamp
build: SRC=powder scripts/build_maze_variant.sh pwfrs -DOGBX_PWF_RULE_STAMPS,
then OGBX_LIB=_abx/libogbx_pwfrs.so python scripts/probe_pwf_rules.py [medium|hard]."""
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
names = ['presence+rands', 'stone', 'gravity', 'sand', 'fluid', 'ice', 'water', 'fire', 'plant', 'velocity']


def report(tag, d):
    fw = d[:, 15].sum()
    tot = d[:, :10].sum()
    print(f'{level} {tag}: {fw} forwards; cycles per forward (mean over envs): {tot / fw:.0f}')
    for k, nm in enumerate(names):
        print(f'  {nm:15s} {d[:, k].sum() / fw:8.0f} cyc  {100 * d[:, k].sum() / tot:5.1f} %')
    for k, nm in zip(range(10, 14), ['vel: bins', 'vel: rounds', 'vel: commit', 'vel: blur']):
        print(f'    {nm:13s} {d[:, k].sum() / fw:8.0f} cyc')


for i in range(120):
    env.step(acts[i % ring])
a = snap()
for i in range(120, 420):
    env.step(acts[i % ring])
b = snap()
report('steady state, 300 steps', b - a)
# the synchronized auto-reset: every env truncates at step 500 (a render-only
# step), whose launch then replays the task's goal sequence, one forward per
# goal action, and the reset's own forward
for i in range(420, 499):
    env.step(acts[i % ring])
a = snap()
env.step(acts[499 % ring])
b = snap()
report('synchronized reset step', b - a)
