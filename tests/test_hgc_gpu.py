"""GPU parity of the hierarchical sampler (hgc_sample_kernel via
ogbx_hgc_sample) against the reference HGCDataset.sample outputs with
injected draws, and against the oracle replaying the kernel's own Philox
draws.  Bit-exact for every key (indices, gathered rows, float64 rewards)."""

import numpy as np
import pytest
import torch

from ogbench_amd.datasets import Dataset, HGCDataset
from oracle import gcdataset_np as orc
from test_oracle_hgc import HGC_CONFIGS, gold, hgc_case  # noqa: F401

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('cname', list(HGC_CONFIGS))
@pytest.mark.parametrize('oracle_rep', [False, True])
def test_hgc_injected_draws_match_reference(gpu, gold, cname, oracle_rep):  # noqa: F811
    data, draws, exp, keys = hgc_case(gold, cname, oracle_rep)
    hgc = HGCDataset(Dataset(data, device=gpu), dict(HGC_CONFIGS[cname]), seed=3)
    out = hgc.sample(len(draws['pick']), draws=draws)
    assert list(out) == keys
    for k in keys:
        got = out[k].cpu().numpy()
        assert got.dtype == exp[k].dtype, (k, got.dtype, exp[k].dtype)
        assert np.array_equal(got, exp[k]), k


@pytest.mark.parametrize('cname', list(HGC_CONFIGS))
def test_hgc_philox_draws_replay_in_oracle(gpu, gold, cname):  # noqa: F811
    data, _, _, keys = hgc_case(gold, cname, True)
    cfg = dict(HGC_CONFIGS[cname])
    hgc = HGCDataset(Dataset(data, device=gpu), cfg, seed=99)
    out = hgc.sample(1000, num_batches=4, record_draws=True)
    draws = {k: v.cpu().numpy() for k, v in out['_draws'].items()}
    ref, ids = orc.hgc_sample(data, cfg, draws)
    assert np.array_equal(out['_idxs'].cpu().numpy(), ids['idxs'])
    assert np.array_equal(out['_high_value_goal_idxs'].cpu().numpy(), ids['hvg'])
    assert np.array_equal(out['_high_actor_goal_idxs'].cpu().numpy(), ids['hag'])
    for k in keys:
        assert np.array_equal(out[k].cpu().numpy(), ref[k]), k
    # goal statistics sanity: value goals are the current state at ~p_curgoal
    p = cfg['value_p_curgoal']
    frac = float((ids['hvg'] == ids['idxs']).mean())
    assert abs(frac - p) < 0.05 or (p == 1.0 and frac == 1.0)


def test_hgc_out_reuse(gpu, gold):  # noqa: F811
    data, _, _, keys = hgc_case(gold, 'hlow', False)
    h1 = HGCDataset(Dataset(data, device=gpu), dict(HGC_CONFIGS['hlow']), seed=5)
    h2 = HGCDataset(Dataset(data, device=gpu), dict(HGC_CONFIGS['hlow']), seed=5)
    h1.sample(128)
    b1 = h1.sample(128)
    a2 = h2.sample(128)
    b2 = h2.sample(128, out=a2)
    assert b2 is a2
    for k in keys:
        assert torch.equal(b1[k], b2[k]), k


@pytest.mark.parametrize('cname', list(HGC_CONFIGS))
def test_hgc_lookahead_matches_direct_sampling(gpu, gold, cname):  # noqa: F811
    """hgc_ahead_kernel (selectors of call c stored by the launch of call c-1)
    returns the batches of direct sampling bit for bit, over out= refills,
    size changes and an interleaved recorded call."""
    data, _, _, keys = hgc_case(gold, cname, True)
    a = HGCDataset(Dataset(data, device=gpu), dict(HGC_CONFIGS[cname]), seed=8)
    b = HGCDataset(Dataset(data, device=gpu), dict(HGC_CONFIGS[cname], lookahead=False), seed=8)
    prev_a = prev_b = None
    for i, (B, mode) in enumerate([(1024, 'fresh'), (1024, 'out'), (1024, 'out'), (300, 'fresh'), (300, 'record'),
                                   (300, 'fresh'), (300, 'fresh'), (2048, 'fresh'), (1024, 'fresh')]):
        if mode == 'record':
            x, y = a.sample(B, record_draws=True), b.sample(B, record_draws=True)
        elif mode == 'out':
            x, y = a.sample(B, out=prev_a), b.sample(B, out=prev_b)
        else:
            x, y = a.sample(B), b.sample(B)
        for k in keys:
            assert torch.equal(x[k], y[k]), (i, k)
        if mode != 'record':
            prev_a, prev_b = x, y


def test_hgc_lookahead_reads_the_callers_tables(gpu, gold):  # noqa: F811
    """The look-ahead chain looks masks and rewards up in the config's tables
    (held in registers for K < 128), so tables other than the canonical
    1 - (s < K) give the same batches as direct sampling."""
    data, _, _, keys = hgc_case(gold, 'hiql', True)
    a = HGCDataset(Dataset(data, device=gpu), dict(HGC_CONFIGS['hiql']), seed=4)
    b = HGCDataset(Dataset(data, device=gpu), dict(HGC_CONFIGS['hiql'], lookahead=False), seed=4)
    for h in (a, b):  # in place: the config keeps the table pointers
        for masks, rewards in (h._hv_tab, h._lv_tab):
            masks.copy_(torch.linspace(0.25, 0.75, masks.numel(), dtype=torch.float64, device=gpu))
            rewards.mul_(3.0).add_(0.5)
    assert a._lookahead and not b._lookahead
    for i in range(4):
        x, y = a.sample(512), b.sample(512)
        for k in keys:
            assert torch.equal(x[k], y[k]), (i, k)
    assert a.ahead_hits >= 2


def test_hgc_lookahead_long_subgoals_read_tables_in_memory(gpu, gold):  # noqa: F811
    """subgoal_steps >= 128: the chain's table lookups fall back to memory
    reads; still bit-identical to direct sampling and to the oracle."""
    data, _, _, keys = hgc_case(gold, 'hiql', True)
    cfg = dict(HGC_CONFIGS['hiql'], subgoal_steps=150)
    a = HGCDataset(Dataset(data, device=gpu), cfg, seed=6)
    b = HGCDataset(Dataset(data, device=gpu), dict(cfg, lookahead=False), seed=6)
    assert a.value_subgoal_steps >= 128
    for i in range(3):
        x, y = a.sample(700), b.sample(700)
        for k in keys:
            assert torch.equal(x[k], y[k]), (i, k)
    assert a.ahead_hits >= 1
    out = b.sample(400, record_draws=True)
    draws = {k: v.cpu().numpy() for k, v in out['_draws'].items()}
    ref, _ = orc.hgc_sample(data, cfg, draws)
    for k in keys:
        assert np.array_equal(out[k].cpu().numpy(), ref[k]), k


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason='needs two GPUs')
def test_sampler_on_a_non_current_device(gold):  # noqa: F811
    """A dataset on cuda:1 with cuda:0 current: the plan allocates its
    look-ahead buffers on the dataset's device and samples match cuda:0's."""
    data, _, _, keys = hgc_case(gold, 'hiql', True)
    torch.cuda.set_device(0)
    a = HGCDataset(Dataset(data, device='cuda:1'), dict(HGC_CONFIGS['hiql']), seed=2)
    b = HGCDataset(Dataset(data, device='cuda:0'), dict(HGC_CONFIGS['hiql']), seed=2)
    for i in range(3):
        x, y = a.sample(256), b.sample(256)
        for k in keys:
            assert torch.equal(x[k].cpu(), y[k].cpu()), (i, k)
