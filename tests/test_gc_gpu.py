"""GPU parity of the fused index-gather + hindsight-relabel kernel
(gc_sample_kernel via ogbx_gc_sample) against the reference outputs with
injected draws, and against the oracle replaying the kernel's own Philox draws.
All integer / gathered outputs are compared bit-exactly."""

import functools
import os

import numpy as np
import pytest
import torch

from ogbench_amd import _lib

from ogbench_amd.datasets import Dataset, GCDataset, nonzero_positive
from oracle import gcdataset_np as orc

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), 'golden', 'gc_golden.npz')
from test_oracle_gc import CONFIGS  # noqa: E402


@pytest.fixture(scope='module')
def gold():
    return dict(np.load(GOLD))


def _raw(gold):
    return {k[4:]: v for k, v in gold.items() if k.startswith('raw_')}


def _cmp(out, exp):
    for k, v in exp.items():
        got = out[k].cpu().numpy()
        assert got.dtype == v.dtype, (k, got.dtype, v.dtype)
        assert np.array_equal(got, v), k


@pytest.mark.parametrize('cname', list(CONFIGS))
@pytest.mark.parametrize('oracle_rep', [False, True])
def test_injected_draws_match_reference(gpu, gold, cname, oracle_rep):
    tag = f'{cname}_{"oracle" if oracle_rep else "obs"}'
    data = orc.load_dataset(_raw(gold), compact_dataset=True)
    if oracle_rep:
        data['oracle_reps'] = _raw(gold)['qpos'][: len(data['observations'])].astype(np.float32)
    ds = Dataset(data, device=gpu)
    gc = GCDataset(ds, dict(CONFIGS[cname], p_aug=None, frame_stack=None), seed=1)
    p = f'gc_{tag}_draw_'
    draws = {k[len(p):]: v for k, v in gold.items() if k.startswith(p)}
    out = gc.sample(len(draws['pick']), draws=draws)
    p = f'gc_{tag}_out_'
    exp = {k[len(p):]: v for k, v in gold.items() if k.startswith(p)}
    assert set(exp) <= set(out)
    _cmp(out, exp)


def test_explicit_idxs_regular_dataset(gpu, gold):
    data = orc.load_dataset(_raw(gold), compact_dataset=False)
    gc = GCDataset(Dataset(data, device=gpu), dict(CONFIGS['crl'], p_aug=None, frame_stack=None))
    p = 'gc_regidx_draw_'
    draws = {k[len(p):]: v for k, v in gold.items() if k.startswith(p)}
    out = gc.sample(64, idxs=gold['gc_regidx_idxs'], draws=draws)
    p = 'gc_regidx_out_'
    _cmp(out, {k[len(p):]: v for k, v in gold.items() if k.startswith(p)})


@pytest.mark.parametrize('cname', list(CONFIGS))
def test_philox_draws_replay_in_oracle(gpu, gold, cname):
    """Philox mode: the oracle, fed the draws the kernel reports, must produce
    the identical batch (8 batches of 1000 in one launch)."""
    data = orc.load_dataset(_raw(gold), compact_dataset=True)
    data['oracle_reps'] = _raw(gold)['qpos'][: len(data['observations'])].astype(np.float32)
    gc = GCDataset(Dataset(data, device=gpu), dict(CONFIGS[cname], p_aug=None, frame_stack=None), seed=42)
    out = gc.sample(1000, num_batches=8, record_draws=True)
    draws = {k: v.cpu().numpy() for k, v in out['_draws'].items()}
    ref, idxs, vg, ag = orc.sample(data, CONFIGS[cname], draws)
    assert np.array_equal(out['_idxs'].cpu().numpy(), idxs)
    for k, v in ref.items():
        assert np.array_equal(out[k].cpu().numpy(), v), k
    # draws are in range and idxs are valid transitions
    valid = np.nonzero(data['valids'] > 0)[0]
    assert np.isin(idxs, valid).all()
    assert (draws['v_pick'] >= 0).all() and (draws['v_pick'] < len(valid)).all()


def test_goal_statistics(gpu):
    """Distribution check of Philox-mode relabelling on a long synthetic buffer."""
    rng = np.random.RandomState(0)
    n_traj, L = 200, 500
    term = np.zeros(n_traj * L, np.float32)
    term[L - 1 :: L] = 1
    raw = dict(observations=rng.normal(size=(n_traj * L, 4)).astype(np.float32),
               actions=rng.normal(size=(n_traj * L, 2)).astype(np.float32), terminals=term)
    data = orc.load_dataset(raw, compact_dataset=True)
    cfg = dict(CONFIGS['gciql'], p_aug=None, frame_stack=None)
    gc = GCDataset(Dataset(data, device=gpu), cfg, seed=3)
    out = gc.sample(1 << 18, record_draws=True)
    idx = out['_idxs'].cpu().numpy()
    vg = out['_value_goal_idxs'].cpu().numpy()
    ag = out['_actor_goal_idxs'].cpu().numpy()
    cur = (vg == idx).mean()
    assert abs(cur - 0.2) < 0.01  # value_p_curgoal (+ rare traj/random coincidences)
    same_traj = (vg // L == idx // L) & (vg > idx)
    assert abs(same_traj.mean() - 0.5) < 0.02
    # actor goals: always future states of the same trajectory (uniform)
    assert ((ag // L) == (idx // L)).all() and (ag >= idx).all()
    # geometric offsets have mean 1/(1-discount) = 100 (before clipping)
    geo = out['_draws']['v_geom'].cpu().numpy()
    assert abs(geo.mean() - 100.0) < 2.0
    assert (geo >= 1).all()
    masks = out['masks'].cpu().numpy()
    assert np.array_equal(masks, 1.0 - (idx == vg))


def test_nonzero_and_traj_end(gpu):
    rng = np.random.RandomState(1)
    x = (rng.rand(1_000_003) < 0.01).astype(np.float32) * rng.rand(1_000_003).astype(np.float32)
    x[-1] = 1.0
    got = nonzero_positive(torch.tensor(x, device=gpu)).cpu().numpy()
    assert np.array_equal(got, np.nonzero(x > 0)[0])
    data = dict(observations=np.zeros((len(x), 1), np.float32), terminals=x)
    gc = GCDataset(Dataset(data, device=gpu), dict(CONFIGS['crl'], p_aug=None, frame_stack=None))
    assert np.array_equal(gc.traj_end.cpu().numpy(), orc.traj_end(x))


def test_plain_dataset_sample_and_random_idxs(gpu, gold):
    data = orc.load_dataset(_raw(gold), compact_dataset=True)
    ds = Dataset(data, device=gpu)
    idx = ds.get_random_idxs(5000).cpu().numpy()
    assert np.isin(idx, np.nonzero(data['valids'] > 0)[0]).all()
    sub = ds.get_subset(torch.tensor(idx[:100]))
    assert np.array_equal(sub['observations'].cpu().numpy(), data['observations'][idx[:100]])
    nxt = np.minimum(idx[:100] + 1, len(data['observations']) - 1)
    assert np.array_equal(sub['next_observations'].cpu().numpy(), data['observations'][nxt])


@functools.lru_cache(maxsize=1)
def humanoid_layout(n_traj=500, L=2000, seed=3):
    """configs[3]'s buffer shape (1M rows, obs 69, act 21; equal trajectories,
    the last row of each invalid) in the compact layout, as host arrays
    (shared between tests: treat as read-only)."""
    rng = np.random.default_rng(seed)
    R = n_traj * L
    term = np.zeros(R, np.float32)
    term[L - 1::L] = 1
    raw = dict(observations=rng.standard_normal((R, 69), dtype=np.float32),
               actions=rng.standard_normal((R, 21), dtype=np.float32), terminals=term)
    return orc.load_dataset(raw, compact_dataset=True)


def test_humanoid_scale_properties(gpu):
    """BASELINE configs[3] (1M rows, obs 69, act 21, B = 1024) through the
    closed-form (periodic) path: a fused 64-batch Philox launch, every key --
    rows, goal indices, masks, rewards -- bit-exact against the oracle fed the
    draws the kernel reports, plus size-independent properties."""
    L = 2000
    data = humanoid_layout(L=L)
    R = len(data['observations'])
    ds = Dataset(data, device=gpu)
    cfg = dict(CONFIGS['gciql'], discount=0.995, p_aug=None, frame_stack=None)
    gc = GCDataset(ds, cfg, seed=9)
    assert gc.period == (L, L - 1, L - 2)
    out = gc.sample(1024, num_batches=64, record_draws=True)
    draws = {k: v.cpu().numpy() for k, v in out['_draws'].items()}
    ref, idxs, vg, ag = orc.sample(data, cfg, draws)
    assert np.array_equal(out['_idxs'].cpu().numpy(), idxs)
    assert np.array_equal(out['_value_goal_idxs'].cpu().numpy(), vg)
    assert np.array_equal(out['_actor_goal_idxs'].cpu().numpy(), ag)
    assert set(ref) <= set(out)
    for k, v in ref.items():
        got = out[k].cpu().numpy()
        assert got.dtype == v.dtype, k
        assert np.array_equal(got, v), k
    valids = data['valids']
    assert (valids[idxs] == 1).all()
    assert ((ag // L) == (idxs // L)).all()
    assert abs(float((vg == idxs).mean()) - 0.2) < 0.01
    assert R == 1_000_000


def test_humanoid_scale_boundary_picks(gpu):
    """The injected-draw kernel on the same 1M-row closed-form buffer, with the
    sample / goal picks at every period boundary q*1999 - 1, q*1999 (and 0,
    npick - 1), against the oracle."""
    L = 2000
    data = humanoid_layout(L=L)
    ds = Dataset(data, device=gpu)
    cfg = dict(CONFIGS['crl'], p_aug=None, frame_stack=None)
    gc = GCDataset(ds, cfg, seed=2)
    assert gc.period == (L, L - 1, L - 2)
    npick = 500 * (L - 1)
    q = np.arange(1, 500)
    forced = np.concatenate([[0, npick - 1], q * (L - 1) - 1, q * (L - 1)])
    rec = gc.sample(1024, record_draws=True)['_draws']
    draws = {k: v.cpu().numpy() for k, v in rec.items()}
    n = len(forced)
    draws['pick'][:n] = forced
    draws['v_pick'][:n] = forced[::-1]
    draws['a_pick'][:n] = np.roll(forced, 7)
    draws['v_geom'][:n] = np.arange(n) % 5 + 1  # goals at and just past the trajectory end
    out = gc.sample(1024, draws=draws, record_draws=True)
    ref, idxs, vg, ag = orc.sample(data, cfg, draws)
    assert np.array_equal(out['_idxs'].cpu().numpy(), idxs)
    assert np.array_equal(out['_value_goal_idxs'].cpu().numpy(), vg)
    assert np.array_equal(out['_actor_goal_idxs'].cpu().numpy(), ag)
    for k, v in ref.items():
        assert np.array_equal(out[k].cpu().numpy(), v), k


def test_out_reuse_matches_fresh_calls(gpu, gold):
    """sample(B, out=prev) refills prev in place with exactly the batch a fresh
    call would return (same seed, same call index)."""
    data = orc.load_dataset(_raw(gold), compact_dataset=True)
    cfg = dict(CONFIGS['gciql'] if 'gciql' in CONFIGS else next(iter(CONFIGS.values())), p_aug=None, frame_stack=None)
    g1 = GCDataset(Dataset(data, device=gpu), cfg, seed=7)
    g2 = GCDataset(Dataset(data, device=gpu), cfg, seed=7)
    a1 = {k: v.clone() for k, v in g1.sample(256).items()}
    b1 = g1.sample(256)
    a2 = g2.sample(256)
    for k in a1:
        assert torch.equal(a1[k], a2[k]), k
    ptrs = {k: v.data_ptr() for k, v in a2.items()}
    b2 = g2.sample(256, out=a2)
    assert b2 is a2 and all(v.data_ptr() == ptrs[k] for k, v in b2.items())
    for k in b1:
        assert torch.equal(b1[k], b2[k]), k


def test_periodic_closed_form_matches_tables(gpu):
    """The OGBench layout (equal trajectories, last row invalid) is sampled
    through the closed form (ogbx_gc_buffer.period, no index loads); the same
    dataset with the closed form switched off (tables) gives identical
    batches, for GC and HGC."""
    from ogbench_amd.datasets import HGCDataset

    n_traj, L = 40, 250
    R = n_traj * L
    g = torch.Generator(device=gpu).manual_seed(5)
    term = torch.zeros(R, device=gpu)
    term[L - 1 :: L] = 1
    data = dict(observations=torch.randn(R, 69, device=gpu, generator=g),
                actions=torch.randn(R, 21, device=gpu, generator=g),
                terminals=torch.clamp(term + torch.cat([term[1:], torch.ones(1, device=gpu)]), max=1.0),
                valids=1.0 - term)
    from test_oracle_hgc import HGC_CONFIGS

    cases = [(GCDataset, dict(c, p_aug=None, frame_stack=None)) for c in CONFIGS.values()]
    cases += [(HGCDataset, dict(c, p_aug=None)) for c in HGC_CONFIGS.values()]
    for cls, cfg in cases:
        a = cls(Dataset(data, device=gpu), cfg, seed=4)
        b = cls(Dataset(data, device=gpu), cfg, seed=4)
        assert a.period == (L, L - 1, L - 2)
        b._buf.period = b._buf.period_picks = b._buf.period_end = 0
        for B, nb in ((1024, 1), (96, 3), (4096, 16)):
            x, y = a.sample(B, num_batches=nb), b.sample(B, num_batches=nb)
            for k in x:
                assert torch.equal(x[k], y[k]), (cls.__name__, B, k)


def test_row_record_stride_and_in_place_updates(gpu, gold):
    """The sampler's packed copy of the small columns: its row
    stride is the power of two at or above the packed bytes, it is skipped for
    the plain sampler and under row_record=False, and a column modified in
    place (or replaced) after the sampler was built is re-packed before the
    next sample -- batches always show the dataset's current values."""
    data = orc.load_dataset(_raw(gold), compact_dataset=True)  # actions 3 f32 + terminals + valids = 20 B
    ds = Dataset(data, device=gpu)
    cfg = dict(CONFIGS['gciql'], p_aug=None, frame_stack=None)
    gc = GCDataset(ds, cfg, seed=3)
    assert gc._rec_stride == 32 and gc._record.shape == (ds.size, 32)
    assert ds._sampler()._record is None
    off = GCDataset(ds, dict(cfg, row_record=False), seed=3)
    assert off._record is None
    a = gc.sample(512, record_draws=True)
    b = off.sample(512, record_draws=True)
    for k in a:
        if not k.startswith('_'):
            assert torch.equal(a[k], b[k]), k
    prev = gc.sample(512)
    ds['actions'].mul_(-2.0)  # in place: version counter moves
    out = gc.sample(512, record_draws=True)
    assert torch.equal(out['actions'], ds['actions'][out['_idxs']])
    ds['terminals'].add_(0.0)
    ds['actions'].add_(1.0)
    refill = gc.sample(512, out=prev)
    assert refill is prev
    rows = ds['actions']
    hit = (refill['actions'][:, None, :] == rows[None, :, :]).all(-1).any(-1)
    assert bool(hit.all())  # every refilled row is a current dataset row
    chk = gc.sample(512, record_draws=True)
    assert torch.equal(chk['actions'], ds['actions'][chk['_idxs']])


def test_lookahead_matches_direct_sampling(gpu, gold):
    """The look-ahead kernel (ogbx_gc_sample_ahead: call c gathers from the
    selectors call c-1 stored, and stores call c+1's) returns the batches of
    direct sampling bit for bit, across out= refills, batch-size changes,
    interleaved recorded / injected calls (which consume a call index and
    invalidate the stored selectors), num_batches > 1, and calls above the
    look-ahead's 1,024-sample limit."""
    data = orc.load_dataset(_raw(gold), compact_dataset=True)
    for cname in ('gciql', 'crl'):
        cfg = dict(CONFIGS[cname], p_aug=None, frame_stack=None)
        a = GCDataset(Dataset(data, device=gpu), dict(cfg, lookahead=True), seed=21)
        b = GCDataset(Dataset(data, device=gpu), dict(cfg, lookahead=False), seed=21)
        prev_a = prev_b = None
        plan = [(1024, 1, 'fresh'), (1024, 1, 'out'), (1024, 1, 'out'), (256, 2, 'fresh'), (256, 2, 'fresh'),
                (1024, 1, 'record'), (1024, 1, 'fresh'), (1024, 1, 'fresh'), (1000, 2, 'fresh'), (1024, 1, 'fresh'),
                (64, 1, 'fresh'), (64, 1, 'out')]
        for i, (B, nb, mode) in enumerate(plan):
            if mode == 'record':
                x, y = a.sample(B, record_draws=True), b.sample(B, record_draws=True)
            elif mode == 'out' and prev_a is not None and prev_a['masks'].numel() == B * nb:
                x, y = a.sample(B, num_batches=nb, out=prev_a), b.sample(B, num_batches=nb, out=prev_b)
            else:
                x, y = a.sample(B, num_batches=nb), b.sample(B, num_batches=nb)
            for k in y:
                if not k.startswith('_'):
                    assert torch.equal(x[k], y[k]), (cname, i, k)
            if mode != 'record':
                prev_a, prev_b = x, y
        assert a.ahead_hits > 0  # calls were served from stored selectors
    # Dataset.sample (plain sampler) and get_random_idxs
    d1, d2 = Dataset(data, device=gpu), Dataset(data, device=gpu)
    d1._sampler()._lookahead, d2._sampler()._lookahead = True, False
    d1._sampler()._seed = d2._sampler()._seed = 5
    for _ in range(3):
        x, y = d1.sample(512), d2.sample(512)
        for k in y:
            assert torch.equal(x[k], y[k]), k


def test_raw_ahead_abi_matches_direct(gpu, gold):
    """ogbx_gc_sample_ahead driven directly through the C-ABI as INTEGRATION.md
    section 5 shows a non-Python host doing it (two caller-owned buffers that
    alternate, ahead_in = NULL on the first call and after a call-index gap):
    every batch bit-identical to ogbx_gc_sample with the same seed and call."""
    import ctypes

    from ogbench_amd import datasets as D

    data = orc.load_dataset(_raw(gold), compact_dataset=True)
    cfg = dict(CONFIGS['gciql'], p_aug=None, frame_stack=None, lookahead=False)
    gc = GCDataset(Dataset(data, device=gpu), cfg, seed=31)
    L = gc._L
    B = 512
    words = 8  # OGBX_GC_AHEAD_WORDS
    bufs = [torch.empty(B * words, dtype=torch.int64, device=gpu) for _ in range(2)]
    stream = _lib.stream_of(gpu)

    def batch():
        out, cols = gc._columns(B, None)
        arr = (D.GcColumn * len(cols))(*cols)
        m = torch.empty(B, dtype=torch.float64, device=gpu)
        r = torch.empty(B, dtype=torch.float64, device=gpu)
        return out, arr, m, r

    prev = None
    for call in [0, 1, 2, 3, 7, 8, 9]:
        xa, arr_a, ma, ra = batch()
        xb, arr_b, mb, rb = batch()
        src = prev[1] if prev is not None and prev[0] == call else None
        dst = bufs[call & 1]
        _lib.check(L.ogbx_gc_sample_ahead(gc._buf, gc._cfg, ctypes.cast(arr_a, ctypes.c_void_p), len(arr_a), B, 1,
                                          31, call, _lib.ptr(src), _lib.ptr(dst), None, None, None, _lib.ptr(ma),
                                          _lib.ptr(ra), stream))
        _lib.check(L.ogbx_gc_sample(gc._buf, gc._cfg, ctypes.cast(arr_b, ctypes.c_void_p), len(arr_b), B, 1, None,
                                    31, call, None, None, None, _lib.ptr(mb), _lib.ptr(rb), None, stream))
        prev = (call + 1, dst)
        assert torch.equal(ma, mb) and torch.equal(ra, rb), call
        for k in xa:
            assert torch.equal(xa[k], xb[k]), (call, k)
