"""Where does the device sit idle inside bench.py's 20-step timed region?
(verdict r05 item 3.)

Replays bench_pointmaze's setup (65,536 envs, action ring, warmup) and then
R windows of exactly bench._timed's shape (synchronize, event a, K env.step
calls, event b, synchronize), stamping the host clock (CLOCK_MONOTONIC and
CLOCK_BOOTTIME, ns) before the first call and after every call.  Run it under
`rocprofv3 --kernel-trace` to get each maze_step_kernel's device start/end;
scripts/window_summary.py lines the two up.  Also prints the host cost of the
pieces of one env.step (device held by a spin kernel, so nothing waits on the
GPU).

  python scripts/probe_window.py --out gpurun_out/window_host.json
"""

import argparse
import ctypes
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def now():
    return time.clock_gettime_ns(time.CLOCK_MONOTONIC)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--num-envs', type=int, default=65536)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=5)
    ap.add_argument('--windows', type=int, default=12)
    ap.add_argument('--out', default=os.path.join(ROOT, 'gpurun_out', 'window_host.json'))
    a = ap.parse_args()
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    n = a.num_envs
    env, actions = bench._maze_job(n, 0, n, 128, dev)
    ring = actions.shape[0]

    def step(i):
        env.step(actions[i % ring])

    for i in range(a.warmup):
        step(i)
    wins = []
    for w in range(a.windows):
        torch.cuda.synchronize(dev)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record(torch.cuda.current_stream(dev))
        host = [now()]
        boot0 = time.clock_gettime_ns(time.CLOCK_BOOTTIME)
        for i in range(a.steps):
            step(i)
            host.append(now())
        ev1.record(torch.cuda.current_stream(dev))
        torch.cuda.synchronize(dev)
        host.append(now())
        wins.append(dict(host_ns=host, boottime_minus_monotonic_ns=boot0 - host[0], span_ms=ev0.elapsed_time(ev1)))
        time.sleep(0.02)  # separates the windows in the kernel trace

    # host cost of the pieces of one env.step, the device held by a spin kernel
    def per_call(fn, calls=400):
        torch.cuda.synchronize(dev)
        torch.cuda._sleep(int(calls * 40e-6 * 2.4e9))
        t0 = time.perf_counter()
        for i in range(calls):
            fn(i)
        dt = time.perf_counter() - t0
        torch.cuda.synchronize(dev)
        return dt / calls * 1e6

    from ogbench_amd import _lib

    L = env._L
    act = actions[0]
    out = env._step_out
    pieces = dict(
        env_step=per_call(step),
        action_check=per_call(lambda i: env._action(actions[i % ring])),
        ring_index=per_call(lambda i: actions[i % ring]),
        stream_of=per_call(lambda i: _lib.stream_of(env.device)),
        raw_stream=per_call(lambda i: torch._C._cuda_getCurrentRawStream(0)),
        ctypes_step_prebound=per_call(lambda i: L.ogbx_maze_step(env._h, act.data_ptr(), 0, 1, *out, 1,
                                                                 ctypes.c_void_p(torch._C._cuda_getCurrentRawStream(0)))),
    )
    # the back-to-back device time of one launch (bench._per_launch_ms)
    b2b = bench._per_launch_ms(step, 1000, dev, host_us=60.0)
    rec = dict(num_envs=n, steps=a.steps, windows=wins, host_us=pieces, kernel_ms_back_to_back=b2b)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, 'w') as f:
        json.dump(rec, f)
    spans = [w['span_ms'] / a.steps for w in wins]
    print(json.dumps(dict(span_ms_per_step=spans, b2b_ms=b2b, host_us=pieces)), flush=True)
    env.close()


if __name__ == '__main__':
    main()
