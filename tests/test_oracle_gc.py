"""CPU: pin the offline-sampler oracle (oracle/gcdataset_np.py) against the
reference's own GCDataset outputs with recorded draws (tests/golden/gc_golden.npz)."""

import os

import numpy as np
import pytest

from oracle import gcdataset_np as orc

GOLD = os.path.join(os.path.dirname(__file__), 'golden', 'gc_golden.npz')
CONFIGS = {
    'gciql': dict(discount=0.99, value_p_curgoal=0.2, value_p_trajgoal=0.5, value_p_randomgoal=0.3,
                  value_geom_sample=True, actor_p_curgoal=0.0, actor_p_trajgoal=1.0, actor_p_randomgoal=0.0,
                  actor_geom_sample=False, gc_negative=True),
    'crl': dict(discount=0.995, value_p_curgoal=0.0, value_p_trajgoal=1.0, value_p_randomgoal=0.0,
                value_geom_sample=True, actor_p_curgoal=0.0, actor_p_trajgoal=0.5, actor_p_randomgoal=0.5,
                actor_geom_sample=False, gc_negative=False),
    'curone': dict(discount=0.9, value_p_curgoal=1.0, value_p_trajgoal=0.0, value_p_randomgoal=0.0,
                   value_geom_sample=False, actor_p_curgoal=0.3, actor_p_trajgoal=0.3, actor_p_randomgoal=0.4,
                   actor_geom_sample=True, gc_negative=True),
}


@pytest.fixture(scope='module')
def gold():
    return dict(np.load(GOLD))


def raw(gold):
    return {k[4:]: v for k, v in gold.items() if k.startswith('raw_')}


@pytest.mark.parametrize('compact', [True, False])
def test_load_dataset(gold, compact):
    tag = 'compact' if compact else 'regular'
    got = orc.load_dataset(raw(gold), compact_dataset=compact, add_info=True)
    exp = {k[len(f'load_{tag}_'):]: v for k, v in gold.items() if k.startswith(f'load_{tag}_')}
    assert set(got) == set(exp)
    for k in exp:
        assert got[k].dtype == exp[k].dtype, k
        assert np.array_equal(got[k], exp[k]), k


def _draws(gold, tag):
    p = f'gc_{tag}_draw_'
    return {k[len(p):]: v for k, v in gold.items() if k.startswith(p)}


@pytest.mark.parametrize('cname', list(CONFIGS))
@pytest.mark.parametrize('oracle_rep', [False, True])
def test_gc_sample_matches_reference(gold, cname, oracle_rep):
    tag = f'{cname}_{"oracle" if oracle_rep else "obs"}'
    data = orc.load_dataset(raw(gold), compact_dataset=True)
    if oracle_rep:
        data['oracle_reps'] = raw(gold)['qpos'][: len(data['observations'])].astype(np.float32)
    out, *_ = orc.sample(data, CONFIGS[cname], _draws(gold, tag))
    p = f'gc_{tag}_out_'
    exp = {k[len(p):]: v for k, v in gold.items() if k.startswith(p)}
    assert set(out) == set(exp)
    for k in exp:
        assert out[k].dtype == exp[k].dtype, k
        assert np.array_equal(out[k], exp[k]), k


def test_gc_explicit_idxs_regular_dataset(gold):
    data = orc.load_dataset(raw(gold), compact_dataset=False)
    out, *_ = orc.sample(data, CONFIGS['crl'], _draws(gold, 'regidx'), idxs=gold['gc_regidx_idxs'])
    p = 'gc_regidx_out_'
    for k in [k[len(p):] for k in gold if k.startswith(p)]:
        assert np.array_equal(out[k], gold[p + k]), k


def test_legacy_geometric_inversion(gold):
    """np.random.geometric (legacy RandomState, p < 1/3) == ceil(log(1-u)/log(1-p))."""
    u, g = gold['geom_u'], gold['geom_g']
    p = 1 - 0.99
    assert np.array_equal(np.ceil(np.log(1 - u) / np.log(1 - p)).astype(np.int64), g)
