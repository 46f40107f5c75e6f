"""Which envs differ between envs-per-wave layouts (diagnostic for the
layout-independence test): near-wall states as in
tests/test_locomaze_gpu.py::test_results_do_not_depend_on_envs_per_wave, one
physics step (ogbx_point_physics) per layout, compared with the 64-envs layout."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))
import ogbench_amd  # noqa: E402
from oracle import locomaze as orc  # noqa: E402


def main():
    dev = torch.device('cuda', 0)
    rng = np.random.RandomState(17)
    mp, _ = orc.tables('large')
    free_cells = np.argwhere(mp == 0)
    n, K = 3000, 12
    c = free_cells[rng.randint(len(free_cells), size=n)]
    q = np.stack([c[:, 1] * 4.0 - 4 + rng.uniform(-1.9, 1.9, n), c[:, 0] * 4.0 - 4 + rng.uniform(-1.9, 1.9, n)], 1)
    acts = torch.tensor(rng.uniform(-1, 1, (K, n, 2)).astype(np.float32)).to(dev)
    res = {}
    for epw in (64, 32, 16, 8, 32 | 0x100, 16 | 0x100, 8 | 0x100):
        env = ogbench_amd.make('pointmaze-large-v0', num_envs=n, device=dev, max_episode_steps=9, auto_reset=True)
        env._L.ogbx_maze_set_envs_per_wave(env._h, epw)
        env.reset(seed=5)
        sd = env.state_dict()
        sd['qpos'] = torch.tensor(q, dtype=torch.float64)
        env.load_state_dict(sd)
        obs = []
        for t in range(K):
            ob = env.step(acts[t])[0]
            obs.append(ob.cpu().numpy().copy())
        res[epw] = np.stack(obs)
        env.close()
    for epw, r in res.items():
        d = np.abs(r - res[64]).max(axis=2)  # [K, n]
        bad = np.argwhere(d > 0)
        first = bad[:5].tolist()
        print(f'epw {epw:#x}: {len(bad)} (step, env) rows differ, max {d.max():.3g}, first {first}', flush=True)


if __name__ == '__main__':
    main()
