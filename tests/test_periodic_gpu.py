"""GPU parity of the closed-form (periodic) sampler path of gc_sample_kernel /
hgc_sample_kernel (gcsample.hip periodic_row: a pick's row and trajectory end
computed, not loaded) -- the path BASELINE configs[3] runs.

  * the reference's own GCDataset / HGCDataset outputs on an equal-length
    buffer (tests/golden/gc_periodic_golden.npz), picks forced to the period
    boundaries, replayed with injected draws: bit-exact for every key;
  * HGC at configs[3]'s full size (1M rows, B = 1024 x 64, Philox) against
    the oracle fed the kernel's recorded draws: bit-exact for every key;
  * the DEFAULT HGC path -- the look-ahead kernel (hgc_ahead_kernel: call c
    gathers the selectors call c-1's launch stored), which is what
    HGCDataset.sample(1024) and the hgcsample bench run -- on configs[3]'s
    layout at configs[3]'s own HIQL config (impls/hyperparameters.sh:272:
    subgoal_steps=100, discount=0.995), over a stream of fresh and out=
    calls: every key of every call bit-identical to direct sampling, whose
    recorded draws replayed through the oracle give the same indices, masks,
    rewards and rows; the same for the opt-in GC look-ahead; and calls
    alternating between two streams.
Reference: impls/utils/datasets.py:65-70, 213-327, 478-491, 496-643.
"""

import numpy as np
import pytest
import torch

from ogbench_amd.datasets import Dataset, GCDataset, HGCDataset
from oracle import gcdataset_np as orc
from test_gc_gpu import humanoid_layout
from test_oracle_gc import CONFIGS
from test_oracle_hgc import HGC_CONFIGS
from test_oracle_periodic import L, periodic_case, pgold  # noqa: F401

pytestmark = pytest.mark.gpu


def _cmp(out, exp, keys):
    for k in keys:
        got = out[k].cpu().numpy()
        assert got.dtype == exp[k].dtype, (k, got.dtype, exp[k].dtype)
        assert np.array_equal(got, exp[k]), k


@pytest.mark.parametrize('cname', list(CONFIGS))
def test_gc_periodic_injected_matches_reference(gpu, pgold, cname):  # noqa: F811
    data, draws, exp, keys = periodic_case(pgold, f'gc_{cname}')
    gc = GCDataset(Dataset(data, device=gpu), dict(CONFIGS[cname], p_aug=None, frame_stack=None), seed=1)
    assert gc.period == (L, L - 1, L - 2)  # the closed form is what runs
    out = gc.sample(len(draws['pick']), draws=draws)
    assert set(exp) <= set(out)
    _cmp(out, exp, keys)


@pytest.mark.parametrize('cname', list(HGC_CONFIGS))
def test_hgc_periodic_injected_matches_reference(gpu, pgold, cname):  # noqa: F811
    data, draws, exp, keys = periodic_case(pgold, f'hgc_{cname}')
    hgc = HGCDataset(Dataset(data, device=gpu), dict(HGC_CONFIGS[cname]), seed=1)
    assert hgc.period == (L, L - 1, L - 2)
    out = hgc.sample(len(draws['pick']), draws=draws)
    assert list(out) == keys
    _cmp(out, exp, keys)


@pytest.mark.parametrize('cname', ['hiql', 'hlow'])
def test_hgc_humanoid_scale_matches_oracle(gpu, cname):
    """configs[3] with the HIQL sampler: 1M rows, 500 x 2,000, B = 1024 x 64."""
    Lh = 2000
    data = humanoid_layout(L=Lh)
    cfg = dict(HGC_CONFIGS[cname], subgoal_steps=100, discount=0.995)  # hyperparameters.sh:272
    hgc = HGCDataset(Dataset(data, device=gpu), cfg, seed=11)
    assert hgc.period == (Lh, Lh - 1, Lh - 2)
    out = hgc.sample(1024, num_batches=64, record_draws=True)
    draws = {k: v.cpu().numpy() for k, v in out['_draws'].items()}
    ref, ids = orc.hgc_sample(data, cfg, draws)
    assert np.array_equal(out['_idxs'].cpu().numpy(), ids['idxs'])
    assert np.array_equal(out['_high_value_goal_idxs'].cpu().numpy(), ids['hvg'])
    assert np.array_equal(out['_high_actor_goal_idxs'].cpu().numpy(), ids['hag'])
    if ids['lvg'] is not None:
        assert np.array_equal(out['_low_value_goal_idxs'].cpu().numpy(), ids['lvg'])
    keys = [k for k in ref]
    _cmp(out, ref, keys)


_HIQL_C3 = dict(HGC_CONFIGS['hiql'], subgoal_steps=100, discount=0.995)  # impls/hyperparameters.sh:272
_GCIQL_C3 = dict(CONFIGS['gciql'], discount=0.995, p_aug=None, frame_stack=None)  # hyperparameters.sh:266


@pytest.fixture(scope='module')
def humanoid():
    return humanoid_layout(L=2000)


def _oracle_call(kind, data, cfg, y):
    """The oracle's batch for the draws direct sampling recorded in `y`."""
    draws = {k: v.cpu().numpy() for k, v in y['_draws'].items()}
    if kind == 'hgc':
        ref, ids = orc.hgc_sample(data, cfg, draws)
        assert np.array_equal(y['_idxs'].cpu().numpy(), ids['idxs'])
        assert np.array_equal(y['_high_value_goal_idxs'].cpu().numpy(), ids['hvg'])
        assert np.array_equal(y['_high_actor_goal_idxs'].cpu().numpy(), ids['hag'])
        return ref
    ref, idxs, vg, ag = orc.sample(data, cfg, draws)
    assert np.array_equal(y['_idxs'].cpu().numpy(), idxs)
    assert np.array_equal(y['_value_goal_idxs'].cpu().numpy(), vg)
    assert np.array_equal(y['_actor_goal_idxs'].cpu().numpy(), ag)
    return ref


@pytest.mark.parametrize('kind', ['hgc', 'gc'])
def test_lookahead_default_path_configs3_matches_oracle(gpu, humanoid, kind):
    """configs[3] (1M rows, 500 x 2,000, B = 1,024) through the look-ahead
    kernel as HGCDataset runs it by default (GC: opt-in), at HIQL's /
    GCIQL's humanoidmaze config.  Each call is checked three ways: bit-equal
    to the direct kernel's batch of the same (seed, call), and -- through the
    draws the direct kernel recorded -- bit-exact against the oracle for every
    key; the look-ahead must actually have served calls from stored
    selectors (ahead_hits)."""
    data = humanoid
    if kind == 'hgc':
        cls, cfg = HGCDataset, _HIQL_C3
    else:
        cls, cfg = GCDataset, dict(_GCIQL_C3, lookahead=True)
    ds = Dataset(data, device=gpu)
    a = cls(ds, cfg, seed=17)
    b = cls(ds, dict(cfg, lookahead=False), seed=17)
    assert a._lookahead and a.period == (2000, 1999, 1998)
    plan = ['fresh', 'fresh', 'out', 'out', 'out', 'fresh', 'out', 'out']
    prev = None
    for i, mode in enumerate(plan):
        x = a.sample(1024, out=prev) if mode == 'out' else a.sample(1024)
        if mode == 'out':
            assert x is prev
        y = b.sample(1024, record_draws=True)
        ref = _oracle_call(kind, data, cfg, y)
        for k in ref:
            assert torch.equal(x[k], y[k]), (i, k)
            got = x[k].cpu().numpy()
            assert got.dtype == ref[k].dtype, (i, k)
            assert np.array_equal(got, ref[k]), (i, k)
        prev = x
    # every call after the first gathered the selectors its predecessor stored
    assert a.ahead_hits == len(plan) - 1


def test_lookahead_two_streams(gpu, humanoid):
    """Look-ahead calls enqueued on two streams without synchronising between
    them (a shared buffer pair let a launch on one stream
    overwrite the selectors an in-flight launch on the other was reading):
    each stream has its own pair, so every batch equals direct sampling's."""
    ds = Dataset(humanoid, device=gpu)
    a = HGCDataset(ds, _HIQL_C3, seed=23)
    b = HGCDataset(ds, dict(_HIQL_C3, lookahead=False), seed=23)
    s1, s2 = torch.cuda.Stream(gpu), torch.cuda.Stream(gpu)
    pattern = [s1, s1, s2, s2, s2, s1, s1, s2, s1, s2, s2, s1]
    got = []
    for st in pattern:
        with torch.cuda.stream(st):
            got.append(a.sample(1024))
    torch.cuda.synchronize(gpu)
    assert a.ahead_hits == 5  # s1 s1 | s2 s2 s2 | s1 s1 | s2 | s1 | s2 s2 | s1
    for i, x in enumerate(got):
        y = b.sample(1024)
        for k in y:
            assert torch.equal(x[k], y[k]), (i, k)
