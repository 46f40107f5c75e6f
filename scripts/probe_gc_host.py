"""Host cost of the pieces of one steady GCDataset.sample(1024, out=prev)
(verdict r05 item 6): the whole call, the row-record staleness check, the
stream lookup and the bare C-ABI call, each with the device held by a spin
kernel so that nothing waits on the GPU; beside them the back-to-back device
time of one launch.

  python scripts/probe_gc_host.py
"""

import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    from ogbench_amd.datasets import Dataset, GCDataset, HGCDataset

    n_traj, L = 500, 2000
    R = n_traj * L
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    term = torch.zeros(R, device=dev)
    term[L - 1 :: L] = 1
    data = dict(observations=torch.randn(R, 69, device=dev, generator=g),
                actions=torch.rand(R, 21, device=dev, generator=g) * 2 - 1,
                terminals=torch.clamp(term + torch.cat([term[1:], torch.ones(1, device=dev)]), max=1.0),
                valids=1.0 - term)
    cfg = dict(discount=0.995, value_p_curgoal=0.2, value_p_trajgoal=0.5, value_p_randomgoal=0.3,
               value_geom_sample=True, actor_p_curgoal=0.0, actor_p_trajgoal=1.0, actor_p_randomgoal=0.0,
               actor_geom_sample=False, gc_negative=True, p_aug=0.0, frame_stack=None)
    res = {}
    for name, cls, c in (('gc', GCDataset, cfg), ('hgc', HGCDataset, dict(cfg, subgoal_steps=100))):
        ds = cls(Dataset(data, device=dev), c, seed=0)
        batch = ds.sample(1024)
        for _ in range(20):
            ds.sample(1024, out=batch)

        def per_call(fn, calls=400):
            torch.cuda.synchronize(dev)
            torch.cuda._sleep(int(calls * 40e-6 * 2.4e9))
            t0 = time.perf_counter()
            for i in range(calls):
                fn(i)
            dt = time.perf_counter() - t0
            torch.cuda.synchronize(dev)
            return dt / calls * 1e6

        hit = ds._out_cache[id(batch)]
        plan, slot = ds._plan, hit[2]
        raw = ds._raw_stream
        res[name] = dict(
            sample_out=per_call(lambda i: ds.sample(1024, out=batch)),
            refresh_record=per_call(lambda i: ds._refresh_record()),
            raw_stream=per_call(lambda i: raw(0)),
            cabi_plan_sample=per_call(lambda i: ds._plan_sample(plan, slot, 10**6 + i, raw(0))),
            noop_python_call=per_call(lambda i: None),
            kernel_ms_back_to_back=bench._per_launch_ms(lambda i: ds.sample(1024, out=batch), 1000, dev, 60.0),
        )
    print(json.dumps(res), flush=True)


if __name__ == '__main__':
    main()
