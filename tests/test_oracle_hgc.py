"""CPU: pin the HGCDataset restatement (oracle/gcdataset_np.py:hgc_sample)
against the reference's own HGCDataset.sample outputs with recorded draws
(tests/golden/hgc_golden.npz, made by tests/golden/make_golden_gc.py)."""

import os

import numpy as np
import pytest

from oracle import gcdataset_np as orc

GOLD = os.path.join(os.path.dirname(__file__), 'golden', 'hgc_golden.npz')
HGC_CONFIGS = {
    'hiql': dict(discount=0.99, value_p_curgoal=0.2, value_p_trajgoal=0.5, value_p_randomgoal=0.3,
                 value_geom_sample=True, actor_p_curgoal=0.0, actor_p_trajgoal=1.0, actor_p_randomgoal=0.0,
                 actor_geom_sample=False, gc_negative=True, p_aug=0.0, frame_stack=None, subgoal_steps=10),
    'hlow': dict(discount=0.97, value_p_curgoal=0.3, value_p_trajgoal=0.4, value_p_randomgoal=0.3,
                 value_geom_sample=False, actor_p_curgoal=0.2, actor_p_trajgoal=0.5, actor_p_randomgoal=0.3,
                 actor_geom_sample=True, gc_negative=False, p_aug=None, frame_stack=None, subgoal_steps=6,
                 value_subgoal_steps=7, actor_subgoal_steps=4, low_subgoal_steps=3, low_discount=0.95),
    'hcur': dict(discount=0.9, value_p_curgoal=1.0, value_p_trajgoal=0.0, value_p_randomgoal=0.0,
                 value_geom_sample=True, actor_p_curgoal=0.0, actor_p_trajgoal=0.5, actor_p_randomgoal=0.5,
                 actor_geom_sample=False, gc_negative=True, p_aug=None, frame_stack=None, subgoal_steps=5,
                 high_subgoal_steps=12, low_discount=0.9),
}


@pytest.fixture(scope='module')
def gold():
    return dict(np.load(GOLD))


def hgc_case(gold, cname, oracle_rep):
    raw = {k[4:]: v for k, v in gold.items() if k.startswith('raw_')}
    data = orc.load_dataset(raw, compact_dataset=True)
    if oracle_rep:
        data['oracle_reps'] = raw['qpos'][: len(data['observations'])].astype(np.float32)
    tag = f'{cname}_{"oracle" if oracle_rep else "obs"}'
    p = f'hgc_{tag}_draw_'
    draws = {k[len(p):]: v for k, v in gold.items() if k.startswith(p)}
    p = f'hgc_{tag}_out_'
    exp = {k[len(p):]: v for k, v in gold.items() if k.startswith(p)}
    keys = [str(k) for k in gold[f'hgc_{tag}_keys']]
    return data, draws, exp, keys


@pytest.mark.parametrize('cname', list(HGC_CONFIGS))
@pytest.mark.parametrize('oracle_rep', [False, True])
def test_hgc_oracle_matches_reference(gold, cname, oracle_rep):
    data, draws, exp, keys = hgc_case(gold, cname, oracle_rep)
    out, _ = orc.hgc_sample(data, HGC_CONFIGS[cname], draws)
    assert list(out) == keys
    for k in keys:
        assert out[k].dtype == exp[k].dtype, k
        assert np.array_equal(out[k], exp[k]), k
