"""CPU: pin the offline-sampler oracle (oracle/gcdataset_np.py) on the
equal-length-trajectory layout that libogbx samples through its closed form
(ogbx_gc_buffer.period).  tests/golden/gc_periodic_golden.npz holds the
reference's own GCDataset / HGCDataset outputs (impls/utils/datasets.py:65-70,
213-327, 478-491, 496-643) on 30 trajectories of 50 rows, with the sample,
value-goal and actor-goal picks forced to the period boundaries in their first
entries (made by tests/golden/make_golden_gc.py:main_periodic)."""

import os

import numpy as np
import pytest

from oracle import gcdataset_np as orc
from test_oracle_gc import CONFIGS
from test_oracle_hgc import HGC_CONFIGS

GOLD = os.path.join(os.path.dirname(__file__), 'golden', 'gc_periodic_golden.npz')
N_TRAJ, L = 30, 50


@pytest.fixture(scope='module')
def pgold():
    return dict(np.load(GOLD))


def periodic_case(gold, tag):
    raw = {k[4:]: v for k, v in gold.items() if k.startswith('raw_')}
    data = orc.load_dataset(raw, compact_dataset=True)
    p = f'{tag}_draw_'
    draws = {k[len(p):]: v for k, v in gold.items() if k.startswith(p)}
    p = f'{tag}_out_'
    exp = {k[len(p):]: v for k, v in gold.items() if k.startswith(p)}
    keys = [str(k) for k in gold[f'{tag}_keys']] if f'{tag}_keys' in gold else list(exp)
    return data, draws, exp, keys


def test_fixture_is_periodic_with_boundary_picks(pgold):
    data, draws, _, _ = periodic_case(pgold, 'gc_gciql')
    valid = np.nonzero(data['valids'] > 0)[0]
    npick = len(valid)
    assert npick == N_TRAJ * (L - 1)
    q = np.arange(npick) // (L - 1)
    assert np.array_equal(valid, q * L + np.arange(npick) % (L - 1))
    assert np.array_equal(orc.traj_end(data['terminals'])[valid], q * L + L - 2)
    forced = pgold['forced_picks']
    for k in ('pick', 'v_pick', 'a_pick'):
        assert np.array_equal(draws[k][: len(forced)], forced), k
    assert {0, npick - 1, L - 2, L - 1} <= set(forced.tolist())


@pytest.mark.parametrize('cname', list(CONFIGS))
def test_gc_periodic_matches_reference(pgold, cname):
    data, draws, exp, _ = periodic_case(pgold, f'gc_{cname}')
    out, *_ = orc.sample(data, CONFIGS[cname], draws)
    assert set(out) == set(exp)
    for k in exp:
        assert out[k].dtype == exp[k].dtype, k
        assert np.array_equal(out[k], exp[k]), k


@pytest.mark.parametrize('cname', list(HGC_CONFIGS))
def test_hgc_periodic_matches_reference(pgold, cname):
    data, draws, exp, keys = periodic_case(pgold, f'hgc_{cname}')
    out, _ = orc.hgc_sample(data, HGC_CONFIGS[cname], draws)
    assert list(out) == keys
    for k in keys:
        assert out[k].dtype == exp[k].dtype, k
        assert np.array_equal(out[k], exp[k]), k
