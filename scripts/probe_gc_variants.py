"""Diagnostic: GC / HGC sample(1024, out=) time per call (2,000 back-to-back
calls in one event span) on the bench's humanoid buffer, with the periodic
closed form on and off (ogbx_gc_buffer.period), for the library in OGBX_LIB."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from ogbench_amd.datasets import Dataset, GCDataset, HGCDataset
dev = torch.device('cuda', 0)
n_traj, L = 500, 2000
R = n_traj * L
g = torch.Generator(device=dev).manual_seed(3)
term = torch.zeros(R, device=dev)
term[L - 1 :: L] = 1
data = dict(observations=torch.randn(R, 69, device=dev, generator=g),
            actions=torch.rand(R, 21, device=dev, generator=g) * 2 - 1,
            terminals=torch.clamp(term + torch.cat([term[1:], torch.ones(1, device=dev)]), max=1.0),
            valids=1.0 - term)
cfg = dict(discount=0.995, value_p_curgoal=0.2, value_p_trajgoal=0.5, value_p_randomgoal=0.3,
           value_geom_sample=True, actor_p_curgoal=0.0, actor_p_trajgoal=1.0, actor_p_randomgoal=0.0,
           actor_geom_sample=False, gc_negative=True, p_aug=0.0, frame_stack=None, subgoal_steps=100)
lib = os.path.basename(os.environ.get('OGBX_LIB', 'libogbx.so'))
for cls in (GCDataset, HGCDataset):
    for period in (True, False, True):
        d = cls(Dataset(data, device=dev), cfg, seed=0)
        if not period:
            d._buf.period = d._buf.period_picks = d._buf.period_end = 0
        out = d.sample(1024)
        for _ in range(200):
            d.sample(1024, out=out)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(); s.record()
        for _ in range(2000):
            d.sample(1024, out=out)
        e.record(); torch.cuda.synchronize()
        print(f'{lib:24s} {cls.__name__:10s} period={"on " if period else "off"}: '
              f'{s.elapsed_time(e) / 2000 * 1e3:6.2f} us/call', flush=True)
