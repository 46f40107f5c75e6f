"""Diagnostic: what bounds one HGCDataset.sample(1024) look-ahead launch on
the bench's humanoid buffer.  hgc_ahead_kernel through the raw C-ABI
(ogbx_hgc_sample_ahead), 2,000 launches queued behind a spin kernel, per
launch:  steady (record in, next record out), gather only (record in, no
next chain), chain only (no record: this call's chain, then gather; no next),
and the miss path (this call's chain, gather, next chain)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from ogbench_amd import _lib
from ogbench_amd.datasets import Dataset, GcColumn, HGCDataset, HgcOutputs, _HGC_SCALARS

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
h = HGCDataset(Dataset(data, device=dev), cfg, seed=0)
B = 1024
out, cols = h._hcolumns(B)
arr = (GcColumn * len(cols))(*cols)
ptr = lambda k: out[k].data_ptr() if k in out else None  # noqa: E731
outs = HgcOutputs(None, None, None, None, *[ptr(k) for k in _HGC_SCALARS[4:]])
bufs = [torch.zeros(B * 20, dtype=torch.int64, device=dev) for _ in range(2)]
L_ = h._Lh
stream = _lib.stream_of(dev)


def launch(i, mode):
    src = bufs[i & 1] if mode in ('steady', 'gather') else None
    dst = bufs[1 - (i & 1)] if mode in ('steady', 'miss') else None
    _lib.check(L_.ogbx_hgc_sample_ahead(h._buf, h._cfg, h._hcfg, ctypes.cast(arr, ctypes.c_void_p), len(arr), B, 1,
                                        0, i, _lib.ptr(src), _lib.ptr(dst), outs, stream))


for mode in ('miss', 'steady', 'gather', 'chain', 'steady'):
    n = 2000
    for i in range(100):
        launch(i, 'miss')
    torch.cuda.synchronize()
    torch.cuda._sleep(int(n * 60e-6 * 2.4e9))
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(n):
        launch(i, mode)
    e.record()
    torch.cuda.synchronize()
    print(f'hgc_ahead_kernel {mode:7s}: {s.elapsed_time(e) / n * 1e3:6.2f} us/launch', flush=True)
