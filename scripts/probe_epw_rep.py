"""Envs-per-wave layouts at the strong-scaling shares (round 6): the default
64 envs per wave against 32 / 16 / 8 envs per wave whose spare lanes step
copies (OGBX_EPW_REPLICATE) -- results are bit-identical across layouts, only
which envs share a wave changes.  Per layout, the back-to-back device time of
one launch (1,000 launches behind a spin kernel, bench._per_launch_ms), on the
bench's states (reset with task i%5+1, warmed 300 steps), layouts interleaved.

  python scripts/probe_epw_rep.py [N ...]
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

REP = 0x100


def main():
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    ns = [int(a) for a in sys.argv[1:]] or [8192, 16384, 32768, 65536]
    layouts = [64, 32 | REP, 16 | REP, 8 | REP, 32, 64]
    out = {}
    for n in ns:
        env, acts = bench._maze_job(n, 0, n, 128, dev)
        for i in range(300):
            env.step(acts[i % 128])
        res = {}
        for rnd in range(2):
            for epw in layouts:
                env._L.ogbx_maze_set_envs_per_wave(env._h, epw)
                ms = bench._per_launch_ms(lambda i: env.step(acts[i % 128]), 1000, dev, host_us=60.0)
                key = f'{epw & 0xFF}{"r" if epw & REP else ""}'
                res.setdefault(key, []).append(round(ms * 1e3, 3))
                print(f'N={n:6d} epw={key:>4}: {ms * 1e3:6.2f} us/launch', flush=True)
        env._L.ogbx_maze_set_envs_per_wave(env._h, 64)
        out[n] = res
        env.close()
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
