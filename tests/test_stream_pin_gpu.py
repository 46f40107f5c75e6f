"""GPU: pinned outputs of every Philox consumer at OGBX_STREAM_VERSION.

Parity tests inject the reference's draws, and the shard tests compare the
kernels with themselves, so neither notices when a layout change alters which
Philox words feed which draw -- and with it every seeded run (the
powderworld medium/hard rand fields changed in round 3 unannounced).  This
test hashes seeded runs of each consumer and compares them with digests
recorded at the current stream version; a change that moves the streams must
bump OGBX_STREAM_VERSION (include/ogbx.h) and re-record the digests on purpose
(run with OGBX_WRITE_PINS=<file> to write them).

Consumers: pointmaze reset noise + task draws + auto-reset (maze_reset /
maze_step), the on-device expert's noise, powderworld-easy invalid-action
replacements, powderworld-medium rand fields and goal replays, GCDataset and
HGCDataset sample draws.
"""

import hashlib
import json
import os

import numpy as np
import pytest
import torch

import ogbench_amd
from ogbench_amd import _lib
from ogbench_amd.datasets import Dataset, GCDataset, HGCDataset

pytestmark = pytest.mark.gpu

STREAM_VERSION = 2
PINNED = {
    'pointmaze': '86126b859d3c30f41d8249ec',
    'powder_easy': '408325547e866809b750a981',
    'powder_medium': 'd1d796b7afa8af8c9738fe06',
    'gc_sample': 'bf2b89ee32edf7c0e11c4556',
    'hgc_sample': '6edbb3d30cfcf326a6cda844',
}


def _digest(*tensors):
    h = hashlib.sha256()
    for t in tensors:
        h.update(np.ascontiguousarray(t.detach().cpu().numpy()).tobytes())
    return h.hexdigest()[:24]


def _runs(gpu):
    out = {}
    # pointmaze: reset noise / task draws, auto-reset draws and expert noise,
    # kept free of contact arithmetic (whose rounding is not a stream
    # property): max_episode_steps = 1 makes every step an auto-reset, whose
    # returned obs is the fresh reset; the expert runs on given (start, goal)
    env = ogbench_amd.make('pointmaze-large-v0', num_envs=1000, device=gpu, auto_reset=True,
                           max_episode_steps=1)
    obs, info = env.reset(seed=123)
    rows = [obs.clone(), info['goal'].clone()]
    g = torch.Generator().manual_seed(1)
    for _ in range(6):
        o, r, te, tr, inf = env.step(torch.rand(1000, 2, generator=g).to(gpu) * 2 - 1)
        rows += [o.clone(), env.cur_goal_xy, tr.clone()]
    start = torch.rand(1000, 2, generator=g, dtype=torch.float64).to(gpu) * 30
    goal = torch.rand(1000, 2, generator=g, dtype=torch.float64).to(gpu) * 30
    for _ in range(3):
        rows.append(env.expert_action(noise=0.2, start_xy=start, goal_xy=goal, seed=5).clone())
    out['pointmaze'] = _digest(*rows)
    env.close()
    for name, kw in (('powder_easy', dict(world_size=32)), ('powder_medium', dict(world_size=32))):
        env_id = 'powderworld-easy-v0' if name == 'powder_easy' else 'powderworld-medium-v0'
        env = ogbench_amd.make(env_id, num_envs=16, device=gpu, auto_reset=True, max_episode_steps=9, **kw)
        obs, _ = env.reset(seed=77)
        g = torch.Generator().manual_seed(3)
        rows = [obs.clone()]
        for _ in range(24):
            o, r, te, tr, inf = env.step(torch.randint(-2, 40, (16,), generator=g, dtype=torch.int32).to(gpu))
            rows += [o.clone(), r.clone(), te.clone(), tr.clone()]
        out[name] = _digest(*rows)
        env.close()
    rng = np.random.RandomState(0)
    R, L = 4000, 40
    term = np.zeros(R, np.float32)
    term[L - 1::L] = 1
    shifted = np.concatenate([term[1:], np.ones(1, np.float32)])
    data = dict(observations=rng.normal(size=(R, 5)).astype(np.float32),
                actions=rng.normal(size=(R, 3)).astype(np.float32),
                terminals=np.minimum(term + shifted, 1.0), valids=1.0 - term)
    cfg = dict(discount=0.99, value_p_curgoal=0.2, value_p_trajgoal=0.5, value_p_randomgoal=0.3,
               value_geom_sample=True, actor_p_curgoal=0.0, actor_p_trajgoal=1.0, actor_p_randomgoal=0.0,
               actor_geom_sample=False, gc_negative=True, p_aug=None, frame_stack=None)
    gc = GCDataset(Dataset(data, device=gpu), cfg, seed=17)
    b = gc.sample(512, num_batches=2)
    out['gc_sample'] = _digest(*b.values())
    hgc = HGCDataset(Dataset(data, device=gpu), dict(cfg, subgoal_steps=10, low_discount=0.95), seed=19)
    b = hgc.sample(512)
    out['hgc_sample'] = _digest(*b.values())
    return out


def test_stream_version_matches_library():
    assert _lib.lib().ogbx_stream_version() == STREAM_VERSION


def test_philox_streams_pinned(gpu):
    got = _runs(gpu)
    path = os.environ.get('OGBX_WRITE_PINS')
    if path:
        with open(path, 'w') as f:
            json.dump(got, f, indent=1)
    assert PINNED, 'no digests recorded yet: run with OGBX_WRITE_PINS=<file> and paste them into PINNED'
    assert got == PINNED, (f'seeded outputs changed at stream version {STREAM_VERSION}: bump OGBX_STREAM_VERSION '
                           f'and re-record PINNED if this was on purpose\n{got}')
