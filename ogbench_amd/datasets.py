"""HBM-resident offline datasets and the goal-conditioned sampler.

Batched, device-side counterparts of impls/utils/datasets.py (hliuson/ogbench):

  Dataset    ~ Dataset (datasets.py:36-83): a dict of device tensors with
               ``size``, ``valid_idxs``, ``get_random_idxs``, ``sample``,
               ``get_subset``;
  GCDataset  ~ GCDataset (datasets.py:149-366): ``sample(batch_size, idxs=None,
               evaluation=False)`` returns the same keys as the reference
               (every dataset key, ``next_observations``, ``value_goals``,
               ``actor_goals``, ``masks``, ``rewards``).

Every sample is ONE launch of ``gc_sample_kernel`` (libogbx): index draw,
trajectory-end lookup, hindsight goal relabel and the row gathers of every
column are fused.  Random numbers come from a counter-based Philox stream
(key = seed, counter = (sample, call)); the reference's NumPy draws can be
injected bit-exactly through ``draws=`` for parity tests.
"""

from __future__ import annotations

import ctypes
import operator
import weakref

import numpy as np

from . import _lib


def _torch():
    import torch

    return torch


_VERSION = operator.attrgetter('_version')


class GcColumn(ctypes.Structure):
    _fields_ = [
        ('src', ctypes.c_void_p),
        ('dst', ctypes.c_void_p),
        ('row_bytes', ctypes.c_int64),
        ('select', ctypes.c_int32),
        ('src_stride', ctypes.c_int32),
    ]


def periodic_layout(num_rows, valid, ends):
    """(period, picks per period, trajectory-end offset) when the buffer is a
    run of equal trajectories -- the OGBench layout: every episode the same
    length, its last row invalid -- else (0, 0, 0).  ``valid``: valid_idxs or
    None (every row pickable); ``ends``: the trajectory end of every pick.
    The kernels then compute a pick's row and trajectory end instead of
    loading them (``ogbx_gc_buffer.period``).  Accepted only if the closed
    form equals ``valid`` and ``ends`` for every pick (checked where the
    tensors live), so the samples are identical either way."""
    torch = _torch()
    R = int(num_rows)
    if valid is not None:
        V = valid.numel()
        ntraj = R - V  # one invalid row per trajectory
        if ntraj <= 0 or R % ntraj or V % ntraj:
            return (0, 0, 0)
        P, pp = R // ntraj, V // ntraj
    else:
        if ends.numel() != R:
            return (0, 0, 0)
        P = int(ends[0]) + 1
        if R % P:
            return (0, 0, 0)
        pp = P
    E = int(ends[0])
    if not 0 <= E < P:
        return (0, 0, 0)
    k = torch.arange(ends.numel(), dtype=torch.int64, device=ends.device)
    q = torch.div(k, pp, rounding_mode='floor')
    if valid is not None and not torch.equal(q * P + (k - q * pp), valid):
        return (0, 0, 0)
    if not torch.equal(q * P + E, ends):
        return (0, 0, 0)
    return (P, pp, E)


class GcBuffer(ctypes.Structure):
    _fields_ = [
        ('num_rows', ctypes.c_int64),
        ('valid_idxs', ctypes.c_void_p),
        ('num_valid', ctypes.c_int64),
        ('traj_end', ctypes.c_void_p),
        ('valid_traj_end', ctypes.c_void_p),
        ('valid_pairs', ctypes.c_void_p),
        ('period', ctypes.c_int64),
        ('period_picks', ctypes.c_int64),
        ('period_end', ctypes.c_int64),
    ]


class GcConfig(ctypes.Structure):
    _fields_ = [
        ('value_p_curgoal', ctypes.c_double),
        ('value_traj_thresh', ctypes.c_double),
        ('value_discount', ctypes.c_double),
        ('actor_p_curgoal', ctypes.c_double),
        ('actor_traj_thresh', ctypes.c_double),
        ('actor_discount', ctypes.c_double),
        ('value_geom_sample', ctypes.c_int32),
        ('actor_geom_sample', ctypes.c_int32),
        ('value_cur_is_one', ctypes.c_int32),
        ('actor_cur_is_one', ctypes.c_int32),
        ('gc_negative', ctypes.c_int32),
        ('pad_', ctypes.c_int32),
    ]


_DRAW_INT = ('pick', 'v_pick', 'v_geom', 'a_pick', 'a_geom')
_DRAW_FLOAT = ('v_dist', 'v_u_traj', 'v_u_cur', 'a_dist', 'a_u_traj', 'a_u_cur')
_DRAW_ORDER = ('pick', 'v_pick', 'v_geom', 'v_dist', 'v_u_traj', 'v_u_cur',
               'a_pick', 'a_geom', 'a_dist', 'a_u_traj', 'a_u_cur')


class GcDraws(ctypes.Structure):
    _fields_ = [('idxs', ctypes.c_void_p)] + [(k, ctypes.c_void_p) for k in _DRAW_ORDER]


class GcDrawRecord(ctypes.Structure):
    _fields_ = [(k, ctypes.c_void_p) for k in _DRAW_ORDER]


def _bind():
    L = _lib.lib()
    if not getattr(L, '_gc_bound', False):
        P = ctypes.POINTER
        L.ogbx_gc_sample.restype = ctypes.c_int32
        L.ogbx_gc_sample.argtypes = [
            P(GcBuffer), P(GcConfig), ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_int64,
            P(GcDraws), ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
            ctypes.c_void_p, ctypes.c_void_p, P(GcDrawRecord), ctypes.c_void_p,
        ]
        L.ogbx_gc_sample_ahead.restype = ctypes.c_int32
        L.ogbx_gc_sample_ahead.argtypes = [
            P(GcBuffer), P(GcConfig), ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_int64,
            ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
        ]
        L.ogbx_gc_plan_create.restype = ctypes.c_int32
        L.ogbx_gc_plan_create.argtypes = [P(GcBuffer), P(GcConfig), ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int32,
                                          P(ctypes.c_void_p)]
        L.ogbx_gc_plan_set_batch.restype = ctypes.c_int32
        L.ogbx_gc_plan_set_batch.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32,
                                             ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                             ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.ogbx_gc_plan_sample.restype = ctypes.c_int32
        L.ogbx_gc_plan_sample.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_uint64, ctypes.c_void_p]
        L.ogbx_gc_plan_hits.restype = ctypes.c_int64
        L.ogbx_gc_plan_hits.argtypes = [ctypes.c_void_p]
        L.ogbx_gc_plan_destroy.restype = ctypes.c_int32
        L.ogbx_gc_plan_destroy.argtypes = [ctypes.c_void_p]
        L.ogbx_gc_traj_end.restype = ctypes.c_int32
        L.ogbx_gc_traj_end.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p,
                                       ctypes.c_void_p]
        L.ogbx_nonzero_f32.restype = ctypes.c_int32
        L.ogbx_nonzero_f32.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_void_p]
        L._gc_bound = True
    return L


def nonzero_positive(x):
    """nonzero(x > 0) of a float32 device vector, via the libogbx compaction."""
    torch = _torch()
    x = x.reshape(-1)
    if x.dtype != torch.float32:
        x = x.to(torch.float32)
    x = x.contiguous()
    L = _bind()
    out = torch.empty(x.numel(), dtype=torch.int64, device=x.device)
    cnt = torch.zeros(1, dtype=torch.int64, device=x.device)
    _lib.check(L.ogbx_nonzero_f32(_lib.ptr(x), x.numel(), _lib.ptr(out), _lib.ptr(cnt),
                                  _lib.stream_of(x.device)))
    return out[: int(cnt.item())]


def _to_device(v, device):
    torch = _torch()
    if isinstance(v, torch.Tensor):
        t = v.to(device)
    else:
        t = torch.as_tensor(np.ascontiguousarray(v), device=device)
    return t.contiguous()


class Dataset(dict):
    """Dataset of device tensors (reference: datasets.py:36-83).

    Keys are kept in insertion order; arrays are moved to ``device`` once
    (HBM-resident).  ``valid_idxs`` is computed on the device when 'valids'
    exists (datasets.py:59-60).
    """

    @classmethod
    def create(cls, freeze=True, device=None, **fields):
        assert 'observations' in fields
        return cls(fields, device=device)

    def __init__(self, data=(), device=None, **kw):
        torch = _torch()
        data = dict(data, **kw)
        if device is None:
            first = next(iter(data.values()))
            device = first.device if isinstance(first, torch.Tensor) and first.is_cuda else 'cuda'
        self.device = torch.device(device)
        if self.device.index is None:
            self.device = torch.device('cuda', torch.cuda.current_device())
        super().__init__({k: _to_device(v, self.device) for k, v in data.items()})
        self.size = max(len(v) for v in self.values())
        if 'valids' in self:
            self.valid_idxs = nonzero_positive(self['valids'])
        self._seed = None
        self._calls = 0

    # column replacements bump _gen, so that a sampler's per-call staleness
    # check is one int compare plus the packed columns' version counters
    _gen = 0

    def __setitem__(self, key, value):
        self._gen += 1
        super().__setitem__(key, value)

    def __delitem__(self, key):
        self._gen += 1
        super().__delitem__(key)

    def update(self, *a, **kw):
        self._gen += 1
        super().update(*a, **kw)

    def pop(self, *a):
        self._gen += 1
        return super().pop(*a)

    def popitem(self):
        self._gen += 1
        return super().popitem()

    def clear(self):
        self._gen += 1
        super().clear()

    def setdefault(self, key, default=None):
        self._gen += 1
        return super().setdefault(key, default)

    def __ior__(self, other):
        self._gen += 1
        return super().__ior__(other)

    def copy(self, add_or_replace=None):
        d = dict(self)
        if add_or_replace:
            d.update(add_or_replace)
        return Dataset(d, device=self.device)

    # the sampling entry points go through GCDataset's kernel with both goal
    # relabels disabled (p_curgoal = 1 short-circuit, datasets.py:318-319)
    def _sampler(self):
        if getattr(self, '_plain_sampler', None) is None:
            self._plain_sampler = GCDataset(self, _PLAIN_CONFIG, _plain=True)
        return self._plain_sampler

    def get_random_idxs(self, num_idxs):
        """datasets.py:65-70 (Philox draws on the device)."""
        return self._sampler().sample(num_idxs, _keys=())['_idxs']

    def sample(self, batch_size, idxs=None):
        out = self._sampler().sample(batch_size, idxs=idxs)
        for k in ('value_goals', 'actor_goals', 'masks', 'rewards', '_idxs'):
            out.pop(k, None)
        return out

    def get_subset(self, idxs):
        return self.sample(len(idxs), idxs=idxs)


_PLAIN_CONFIG = dict(
    discount=0.99, value_p_curgoal=1.0, value_p_trajgoal=0.0, value_p_randomgoal=0.0, value_geom_sample=False,
    actor_p_curgoal=1.0, actor_p_trajgoal=0.0, actor_p_randomgoal=0.0, actor_geom_sample=False,
    gc_negative=False, p_aug=None, frame_stack=None,
)


class GCDataset:
    """Goal-conditioned sampler (reference: datasets.py:149-366).

    config keys read (as the reference): discount, value_/actor_ p_curgoal,
    p_trajgoal, p_randomgoal, geom_sample, gc_negative, p_aug, frame_stack;
    and two of this sampler's own: row_record (default True; False skips the
    interleaved copy of the small columns, ``_row_record``) and lookahead
    (default True: each plain call of <= 1,024 samples also computes the next
    call's selectors, so the next call only gathers; ``ogbx_gc_plan_*``).
    """

    def __init__(self, dataset, config, preprocess_frame_stack=True, seed=None, _plain=False):
        torch = _torch()
        if not isinstance(dataset, Dataset):
            dataset = Dataset(dataset)
        self.dataset = dataset
        self.config = config
        self.preprocess_frame_stack = preprocess_frame_stack
        self.size = dataset.size
        self.device = dataset.device
        if config.get('frame_stack') is not None:
            raise NotImplementedError('frame stacking (visual datasets) is out of scope')
        if config.get('agent_name') in ('trl', 'latent_trl', 'discrete_latent_trl'):
            raise NotImplementedError('the TRL sampling branches are out of scope')
        L = _bind()
        self._L = L
        stream = _lib.stream_of(self.device)
        if 'terminals' in dataset:
            self.terminal_locs = nonzero_positive(dataset['terminals'])
        else:
            self.terminal_locs = torch.tensor([self.size - 1], dtype=torch.int64, device=self.device)
        if not _plain:
            assert self.terminal_locs.numel() > 0 and int(self.terminal_locs[-1]) == self.size - 1
            assert np.isclose(
                config['value_p_curgoal'] + config['value_p_trajgoal'] + config['value_p_randomgoal'], 1.0)
            assert np.isclose(
                config['actor_p_curgoal'] + config['actor_p_trajgoal'] + config['actor_p_randomgoal'], 1.0)
        self.initial_locs = torch.cat([torch.zeros(1, dtype=torch.int64, device=self.device),
                                       self.terminal_locs[:-1] + 1])
        self.traj_end = torch.empty(self.size, dtype=torch.int64, device=self.device)
        if self.terminal_locs.numel() > 0:
            _lib.check(L.ogbx_gc_traj_end(_lib.ptr(self.terminal_locs), self.terminal_locs.numel(), self.size,
                                          _lib.ptr(self.traj_end), stream))
        else:
            self.traj_end.fill_(self.size - 1)
        valid = getattr(dataset, 'valid_idxs', None)
        # trajectory end of every valid row: the drawn index and its end load in parallel
        self.valid_traj_end = self.traj_end[valid].contiguous() if valid is not None else None
        # (index, trajectory end) of every valid row interleaved: one 16-B load per pick
        self.valid_pairs = torch.stack([valid, self.valid_traj_end], 1).contiguous() if valid is not None else None
        self.period = periodic_layout(self.size, valid, self.valid_traj_end if valid is not None else self.traj_end)
        self._buf = GcBuffer(self.size, valid.data_ptr() if valid is not None else None,
                             valid.numel() if valid is not None else 0, self.traj_end.data_ptr(),
                             self.valid_traj_end.data_ptr() if valid is not None else None,
                             self.valid_pairs.data_ptr() if valid is not None else None, *self.period)
        self._valid = valid
        self._plain = _plain
        self._record, self._rec_off, self._rec_stride, self._rec_src = self._row_record(dataset)
        self._rec_index()

        def thresh(p_traj, p_cur):
            return p_traj / (1.0 - p_cur) if p_cur != 1.0 else 0.0  # datasets.py:321

        c = config
        self._cfg = GcConfig(
            float(c['value_p_curgoal']), thresh(c['value_p_trajgoal'], c['value_p_curgoal']), float(c['discount']),
            float(c['actor_p_curgoal']), thresh(c['actor_p_trajgoal'], c['actor_p_curgoal']), float(c['discount']),
            int(bool(c['value_geom_sample'])), int(bool(c['actor_geom_sample'])),
            int(c['value_p_curgoal'] == 1.0), int(c['actor_p_curgoal'] == 1.0), int(bool(c['gc_negative'])), 0,
        )
        self._seed = int(seed) if seed is not None else None
        self._calls = 0
        self._out_cache = {}
        # plain (Philox, no idxs / draws / recording) calls go through a sampler
        # plan (ogbx_gc_plan_*): the prepared output batches and the look-ahead
        # state live in libogbx, so a steady call is one lookup and one launch
        self._lookahead = bool(config.get('lookahead', self._LOOKAHEAD_DEFAULT))
        self._p_aug = config.get('p_aug')
        # the reference draws np.random.rand() < p_aug per call (datasets.py:278);
        # with p_aug 0 the test can never pass and the draw would only advance
        # numpy's global stream (which this sampler's Philox draws do not
        # follow), so the steady call skips it
        self._p_aug_live = self._p_aug is not None and float(self._p_aug) > 0.0
        self._dev_idx = self.device.index
        self._plan_sample = L.ogbx_gc_plan_sample
        self._raw_stream = torch._C._cuda_getCurrentRawStream  # hipStream_t of the current stream, as an int
        self._plan = None
        self._plan_seed = None
        self._plan_final = None
        self._slot = 0

    # ---------------------------------------------------------------- helpers
    _RECORD_MAX = 128  # one L2 line

    def _row_record(self, ds):
        """The sampler's own interleaved copy of the dataset's small columns
        (every key but the goal sources whose row is 4-byte granular, packed in
        key order while they fit one 128-B line per row, e.g. actions 84 +
        terminals 4 + valids 4 of the humanoid layout): a sample's rows of them
        then come from one line of HBM instead of one line per column.  The row
        stride is the power of two (16..128 B) at or above the packed bytes, so
        a row never straddles a line and the copy costs no more than it must
        (pointmaze: actions 8 + terminals 4 + valids 4 = 16 B per row).  The
        dataset's own tensors (and the returned batch) keep the reference
        shapes.  Not built for the plain Dataset.sample sampler, with fewer
        than two packable columns, or with config['row_record'] = False.

        The reference freezes its dataset (Dataset.create sets the arrays
        read-only, impls/utils/datasets.py:45-56); torch tensors cannot be made
        read-only, so sample() checks the packed columns' version counters
        and identities and refreshes the copy if one was modified
        (``_refresh_record``)."""
        torch = _torch()
        if self._plain or not self.config.get('row_record', True):
            return None, {}, 0, ()
        goal_srcs = {'observations', 'oracle_reps'}
        off, picks = 0, []
        for k, v in ds.items():
            if k in goal_srcs:
                continue
            rb = (v[0].numel() if v.dim() > 1 else 1) * v.element_size()
            if rb % 4 or off + rb > self._RECORD_MAX:
                continue
            picks.append((k, off, rb))
            off += rb
        if len(picks) < 2:
            return None, {}, 0, ()
        stride = 16
        while stride < off:
            stride *= 2
        rec = torch.zeros(self.size, stride, dtype=torch.uint8, device=self.device)
        src = tuple((k, ds[k], o, rb) for k, o, rb in picks)
        self._fill_record(rec, src)
        return rec, {k: o for k, o, _ in picks}, stride, tuple((k, t, o, rb, t._version) for k, t, o, rb in src)

    def _fill_record(self, rec, src):
        torch = _torch()
        for k, t, o, rb in src:
            rec[:, o:o + rb] = t.reshape(self.size, -1).contiguous().view(torch.uint8)

    def _refresh_record(self):
        """Re-pack the row record if a packed column was modified in place or
        replaced since it was built (same layout, same record buffer: the
        cached column descriptors stay valid, except on replacement)."""
        ds = self.dataset
        # fast check (every sample() call): the packed columns are the same
        # tensor objects with the same version counters
        gen = getattr(ds, '_gen', None)
        if (gen is not None and gen == self._rec_gen) or \
                all(map(operator.is_, map(ds.get, self._rec_keys), self._rec_tensors)):
            if tuple(map(_VERSION, self._rec_tensors)) == self._rec_versions:
                self._rec_gen = gen  # verified: the next calls compare the generation only
                return
        stale = False
        for k, t, _, _, ver in self._rec_src:
            cur = ds.get(k)
            if cur is not t:
                if cur is None or cur.shape != t.shape or cur.dtype != t.dtype:
                    raise ValueError(f'dataset column {k!r} changed shape or dtype after the sampler was built')
                self._out_cache.clear()  # the batch descriptors hold the old column pointers
                stale = True
            elif t._version != ver:
                stale = True
        if stale:
            src = tuple((k, ds[k], o, rb) for k, _, o, rb, _ in self._rec_src)
            self._fill_record(self._record, src)
            self._rec_src = tuple((k, t, o, rb, t._version) for k, t, o, rb in src)
            self._rec_index()

    def _rec_index(self):
        self._rec_keys = tuple(e[0] for e in self._rec_src)
        self._rec_tensors = tuple(e[1] for e in self._rec_src)
        self._rec_versions = tuple(e[4] for e in self._rec_src)
        self._rec_gen = None  # set by the next clean check (Dataset._gen of a verified state)

    def _column(self, src_key, dst, select):
        """Descriptor of one gathered column (from the row record when the key
        lives there)."""
        src = self.dataset[src_key]
        row_bytes = src[0].numel() * src.element_size() if src.dim() > 1 else src.element_size()
        o = self._rec_off.get(src_key)
        if o is not None:
            return GcColumn(self._record.data_ptr() + o, dst.data_ptr(), row_bytes, select, self._rec_stride)
        return GcColumn(src.data_ptr(), dst.data_ptr(), row_bytes, select, 0)

    def _p_aug_draw(self, out, evaluation):
        # p_aug draw (datasets.py:278-279): image crops apply only to 4-D arrays
        p_aug = self.config.get('p_aug')
        if p_aug is not None and not evaluation:
            if np.random.rand() < p_aug and any(v.dim() == 4 for v in out.values()):
                raise NotImplementedError('image augmentation (visual datasets) is out of scope')

    def _next_seed(self):
        if self._seed is None:
            self._seed = int(np.random.randint(0, 2**63 - 1))
        call = self._calls
        self._calls += 1
        return self._seed, call

    def _columns(self, total, keys):
        """Column descriptors and the output dict (reference key order)."""
        torch = _torch()
        ds = self.dataset
        out, cols = {}, []

        def add(src_key, dst_key, select):
            src = ds[src_key]
            dst = torch.empty((total,) + tuple(src.shape[1:]), dtype=src.dtype, device=self.device)
            out[dst_key] = dst
            cols.append(self._column(src_key, dst, select))

        for k in (ds.keys() if keys is None else keys):
            add(k, k, 0)
        if keys is None and 'next_observations' not in ds:
            add('observations', 'next_observations', 1)  # datasets.py:81-82
        if not self._plain and keys is None:
            goal_src = 'oracle_reps' if 'oracle_reps' in ds else 'observations'  # datasets.py:348-357
            add(goal_src, 'value_goals', 2)
            add(goal_src, 'actor_goals', 3)
        return out, cols

    # GC: with the look-ahead actually hitting (round 5), 4.7 vs 5.8 us per
    # B = 1,024 launch back to back (profiles/r05_gcsample_*), so on by
    # default for both samplers
    _LOOKAHEAD_DEFAULT = True

    def _hcfg_ptr(self):
        return None  # GCDataset; HGCDataset passes its ogbx_hgc_config

    def _plan_for(self, seed):
        """The sampler plan of this (dataset, config, seed), created on the
        first plain call (the seed is drawn then if none was given)."""
        if self._plan is None or self._plan_seed != seed:
            self._drop_plan()
            L = self._L
            h = ctypes.c_void_p()
            # the plan also takes its device from the buffer (hipPointerGetAttributes)
            with _torch().cuda.device(self.device):
                _lib.check(L.ogbx_gc_plan_create(self._buf, self._cfg, self._hcfg_ptr(), seed, int(self._lookahead),
                                                 ctypes.byref(h)), 'gc_plan_create')
            self._plan, self._plan_seed = h.value, seed
            self._plan_final = weakref.finalize(self, L.ogbx_gc_plan_destroy, h.value)
            self._out_cache.clear()  # their slots belong to the old plan
        return self._plan

    def _drop_plan(self):
        if self._plan_final is not None:
            self._plan_final()
        self._plan, self._plan_final = None, None

    @property
    def ahead_hits(self):
        """Calls served from selectors the previous launch stored (diagnostic)."""
        return int(self._L.ogbx_gc_plan_hits(self._plan)) if self._plan is not None else 0

    def _next_slot(self):
        slot = self._slot
        self._slot = (slot + 1) % 8  # OGBX_GC_PLAN_SLOTS; the out cache holds at most the last two
        return slot

    def sample(self, batch_size, idxs=None, evaluation=False, draws=None, record_draws=False,
               num_batches=1, _keys=None, out=None):
        """GCDataset.sample (datasets.py:213-294), one fused launch.

        draws: optional dict of injected reference draws (see ``_DRAW_ORDER``;
        device or host arrays of length num_batches*batch_size).
        record_draws: also return the draws the kernel used (``out['_draws']``).
        num_batches > 1: sample that many independent batches in the same launch
        (outputs have a leading num_batches*batch_size dimension).
        out: a batch dict returned by an earlier call with the same batch_size /
        num_batches (and no idxs/draws/record_draws): its tensors are refilled
        in place (stream ordered, so consumers enqueued earlier read the old
        batch) and it is returned.  Skips all per-call allocation.
        """
        plain_call = idxs is None and not draws and not record_draws and _keys is None
        if self._rec_src:
            # staleness of the packed row record: a Dataset's generation (no
            # column replaced since the last verified check) and the packed
            # columns' version counters; anything else takes the full check
            gen = getattr(self.dataset, '_gen', None)
            if (gen is None or gen != self._rec_gen
                    or tuple(map(_VERSION, self._rec_tensors)) != self._rec_versions):
                self._refresh_record()
        if out is not None and plain_call:
            # the steady refill: one dict lookup, one ctypes call (host time
            # per call is what bounds sample(1024)'s rate, bench 'extra')
            hit = self._out_cache.get(id(out))
            if (hit is not None and hit[0] is out and hit[1] == (batch_size, num_batches)
                    and self._plan_seed == self._seed):
                call = self._calls
                self._calls = call + 1
                st = self._plan_sample(self._plan, hit[2], call, self._raw_stream(self._dev_idx))
                if st:
                    _lib.check(st, 'gc_sample')
                if self._p_aug_live and not evaluation:
                    self._p_aug_draw(out, evaluation)
                return out
        torch = _torch()
        total = int(batch_size) * int(num_batches)
        out, cols = self._columns(total, _keys)
        col_arr = (GcColumn * max(1, len(cols)))(*cols)
        masks = torch.empty(total, dtype=torch.float64, device=self.device)
        rewards = torch.empty(total, dtype=torch.float64, device=self.device)
        # index outputs only when asked for (plain sampling or draw recording)
        idx_out = torch.empty(total, dtype=torch.int64, device=self.device) if (self._plain or record_draws) else None
        vg = torch.empty(total, dtype=torch.int64, device=self.device) if record_draws else None
        ag = torch.empty(total, dtype=torch.int64, device=self.device) if record_draws else None
        keep = []
        dr = GcDraws()
        if idxs is not None:
            t = _to_device(idxs, self.device).to(torch.int64).reshape(-1)
            assert t.numel() == total
            keep.append(t)
            dr.idxs = t.data_ptr()
        if draws:
            for k, v in draws.items():
                if k == 'idxs':
                    continue
                dt = torch.int64 if k in _DRAW_INT else torch.float64
                t = _to_device(v, self.device).to(dt).reshape(-1)
                assert t.numel() == total, k
                keep.append(t)
                setattr(dr, k, t.data_ptr())
        rec = None
        rec_t = None
        if record_draws:
            rec_t = {k: torch.empty(total, dtype=torch.int64 if k in _DRAW_INT else torch.float64,
                                    device=self.device) for k in _DRAW_ORDER}
            rec = GcDrawRecord(*[rec_t[k].data_ptr() for k in _DRAW_ORDER])
        seed, call = self._next_seed()
        slot = None
        if plain_call:
            plan = self._plan_for(seed)
            slot = self._next_slot()
            _lib.check(self._L.ogbx_gc_plan_set_batch(plan, slot, ctypes.cast(col_arr, ctypes.c_void_p), len(cols),
                                                      int(batch_size), int(num_batches), _lib.ptr(idx_out),
                                                      _lib.ptr(vg), _lib.ptr(ag), _lib.ptr(masks),
                                                      _lib.ptr(rewards), None), 'gc_plan_set_batch')
            st = self._L.ogbx_gc_plan_sample(plan, slot, call, _lib.stream_of(self.device))
        else:
            st = self._L.ogbx_gc_sample(
                self._buf, self._cfg, ctypes.cast(col_arr, ctypes.c_void_p), len(cols), int(batch_size),
                int(num_batches), dr, seed, call, _lib.ptr(idx_out), _lib.ptr(vg), _lib.ptr(ag), _lib.ptr(masks),
                _lib.ptr(rewards), rec, _lib.stream_of(self.device))
        _lib.check(st, 'gc_sample')
        if self._plain:
            out['_idxs'] = idx_out
        else:
            out['masks'] = masks
            out['rewards'] = rewards
        if plain_call:
            # remember the batch's plan slot so that sample(..., out=this) skips
            # setup (the output tensors stay alive in `out`)
            if len(self._out_cache) >= 2:
                self._out_cache.clear()
            self._out_cache[id(out)] = (out, (batch_size, num_batches), slot, masks, rewards, idx_out)
        if self._plain:
            return out
        self._p_aug_draw(out, evaluation)
        if record_draws:
            out['_draws'] = rec_t
            out['_idxs'] = idx_out
            out['_value_goal_idxs'] = vg
            out['_actor_goal_idxs'] = ag
        return out


# ----------------------------------------------------------------------------- HGCDataset

_HDRAW_LOW = ('l_pick', 'l_geom', 'l_u_traj', 'l_u_cur')
_HDRAW_INT = _DRAW_INT + ('l_pick', 'l_geom')


class HgcConfig(ctypes.Structure):
    _fields_ = [
        ('value_subgoal_steps', ctypes.c_int64),
        ('low_subgoal_steps', ctypes.c_int64),
        ('actor_subgoal_steps', ctypes.c_int64),
        ('has_low_value_goals', ctypes.c_int32),
        ('pad_', ctypes.c_int32),
        ('low_discount', ctypes.c_double),
        ('hv_mask_table', ctypes.c_void_p),
        ('hv_reward_table', ctypes.c_void_p),
        ('lv_mask_table', ctypes.c_void_p),
        ('lv_reward_table', ctypes.c_void_p),
    ]


class HgcDraws(ctypes.Structure):
    _fields_ = [('gc', GcDraws)] + [(k, ctypes.c_void_p) for k in _HDRAW_LOW]


class HgcDrawRecord(ctypes.Structure):
    _fields_ = [('gc', GcDrawRecord)] + [(k, ctypes.c_void_p) for k in _HDRAW_LOW]


_HGC_SCALARS = ('idxs', 'high_value_goal_idxs', 'high_actor_goal_idxs', 'low_value_goal_idxs',
                'high_value_offsets', 'high_value_subgoal_steps', 'high_value_masks', 'high_value_rewards',
                'low_value_subgoal_steps', 'low_value_masks', 'low_value_rewards', 'masks', 'rewards')


class HgcOutputs(ctypes.Structure):
    _fields_ = [(k, ctypes.c_void_p) for k in _HGC_SCALARS]


def _bind_hgc():
    L = _bind()
    if not getattr(L, '_hgc_bound', False):
        P = ctypes.POINTER
        L.ogbx_hgc_sample_ahead.restype = ctypes.c_int32
        L.ogbx_hgc_sample_ahead.argtypes = [
            P(GcBuffer), P(GcConfig), P(HgcConfig), ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64,
            ctypes.c_int64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, P(HgcOutputs),
            ctypes.c_void_p,
        ]
        L.ogbx_hgc_sample.restype = ctypes.c_int32
        L.ogbx_hgc_sample.argtypes = [
            P(GcBuffer), P(GcConfig), P(HgcConfig), ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64,
            ctypes.c_int64, P(HgcDraws), ctypes.c_uint64, ctypes.c_uint64, P(HgcOutputs), P(HgcDrawRecord),
            ctypes.c_void_p,
        ]
        L._hgc_bound = True
    return L


def _subgoal_tables(discount, K, gc_negative, device):
    """masks / rewards of HGCDataset.sample as functions of the clipped subgoal
    step count s in [0, K] (datasets.py:533-541, 550-556), computed with the
    reference's own float64 NumPy expressions so the device lookup is bit-exact."""
    torch = _torch()
    s = np.arange(K + 1, dtype=np.int64)
    succ = (s < K).astype(float)
    masks = 1.0 - succ
    rewards = -(1 - discount ** s) / (1 - discount) if gc_negative else (discount ** s) * succ
    return (torch.as_tensor(np.ascontiguousarray(masks), device=device),
            torch.as_tensor(np.ascontiguousarray(rewards, dtype=np.float64), device=device))


class HGCDataset(GCDataset):
    """Hierarchical goal-conditioned sampler (reference: datasets.py:467-643).

    Extra config keys (as the reference): subgoal_steps, optional
    high_subgoal_steps, value_subgoal_steps, actor_subgoal_steps,
    low_subgoal_steps, low_discount.  One fused launch of hgc_sample_kernel
    per sample() returns the reference's 27 (28 with low_discount) keys.
    """

    def _hcfg_ptr(self):
        return ctypes.byref(self._hcfg)

    def __init__(self, dataset, config, preprocess_frame_stack=True, seed=None):
        super().__init__(dataset, config, preprocess_frame_stack=preprocess_frame_stack, seed=seed)
        c = config
        high = c.get('high_subgoal_steps', c['subgoal_steps'])
        self.value_subgoal_steps = int(high if c.get('value_subgoal_steps') is None else c['value_subgoal_steps'])
        self.actor_subgoal_steps = int(high if c.get('actor_subgoal_steps') is None else c['actor_subgoal_steps'])
        self.low_subgoal_steps = int(c.get('low_subgoal_steps', c['subgoal_steps']))
        self._has_low = c.get('low_discount') is not None
        dev = self.device
        self._hv_tab = _subgoal_tables(c['discount'], self.value_subgoal_steps, c['gc_negative'], dev)
        self._lv_tab = _subgoal_tables(c['discount'], self.low_subgoal_steps, c['gc_negative'], dev)
        self._hcfg = HgcConfig(
            self.value_subgoal_steps, self.low_subgoal_steps, self.actor_subgoal_steps, int(self._has_low), 0,
            float(c['low_discount']) if self._has_low else 0.0,
            self._hv_tab[0].data_ptr(), self._hv_tab[1].data_ptr(),
            self._lv_tab[0].data_ptr(), self._lv_tab[1].data_ptr(),
        )
        self._Lh = _bind_hgc()

    def _hcolumns(self, total):
        """Output tensors in the reference's key order, and column descriptors."""
        torch = _torch()
        ds = self.dataset
        out, cols = {}, []
        goal_src = 'oracle_reps' if 'oracle_reps' in ds else 'observations'

        def col(src_key, select):
            src = ds[src_key]
            dst = torch.empty((total,) + tuple(src.shape[1:]), dtype=src.dtype, device=self.device)
            cols.append(self._column(src_key, dst, select))
            return dst

        def scalar(dtype):
            return torch.empty(total, dtype=dtype, device=self.device)

        for k in ds.keys():
            out[k] = col(k, 0)
        if 'next_observations' not in ds:
            out['next_observations'] = col('observations', 1)
        i64, f64 = torch.int64, torch.float64
        out['high_value_reps'] = out['observations']
        out['high_value_goals'] = col(goal_src, 2)
        out['high_value_actions'] = col(goal_src, 4)
        out['high_value_next_observations'] = col('observations', 4)
        for k, dt in (('high_value_offsets', i64), ('high_value_subgoal_steps', i64), ('high_value_masks', f64),
                      ('high_value_rewards', f64)):
            out[k] = scalar(dt)
        out['low_value_next_observations'] = col('observations', 5)
        for k, dt in (('low_value_subgoal_steps', i64), ('low_value_masks', f64), ('low_value_rewards', f64)):
            out[k] = scalar(dt)
        if self._has_low:
            out['low_value_goals'] = col(goal_src, 6)
        out['value_goals'] = out['high_value_goals']
        out['masks'] = scalar(f64)
        out['rewards'] = scalar(f64)
        out['high_actor_goals'] = col(goal_src, 3)
        out['high_actor_actions'] = col(goal_src, 7)
        out['high_actor_next_observations'] = col('observations', 7)
        out['high_actor_targets'] = out['high_actor_actions']
        out['low_actor_goals'] = col(goal_src, 8)
        out['low_actor_goal_observations'] = col('observations', 8)
        out['low_actor_next_observations'] = col('observations', 9)
        return out, cols

    def sample(self, batch_size, idxs=None, evaluation=False, draws=None, record_draws=False, num_batches=1,
               out=None):
        """HGCDataset.sample (datasets.py:496-643), one fused launch.  Arguments
        as GCDataset.sample; draws may also carry the low-level l_* draws."""
        torch = _torch()
        total = int(batch_size) * int(num_batches)
        plain_call = idxs is None and not draws and not record_draws
        if self._rec_src:
            # staleness of the packed row record: a Dataset's generation (no
            # column replaced since the last verified check) and the packed
            # columns' version counters; anything else takes the full check
            gen = getattr(self.dataset, '_gen', None)
            if (gen is None or gen != self._rec_gen
                    or tuple(map(_VERSION, self._rec_tensors)) != self._rec_versions):
                self._refresh_record()
        hit = self._out_cache.get(id(out)) if (out is not None and plain_call) else None
        if (hit is not None and hit[0] is out and hit[1] == (batch_size, num_batches)
                and self._plan_seed == self._seed):
            call = self._calls
            self._calls = call + 1
            st = self._plan_sample(self._plan, hit[2], call, self._raw_stream(self._dev_idx))
            if st:
                _lib.check(st, 'hgc_sample')
            if self._p_aug_live and not evaluation:
                self._p_aug_draw(out, evaluation)
            return out
        else:
            out, cols = self._hcolumns(total)
            col_keep = (GcColumn * max(1, len(cols)))(*cols)
            col_arr = ctypes.cast(col_keep, ctypes.c_void_p)
            ncols = len(cols)
            ptr = lambda k: out[k].data_ptr() if k in out else None  # noqa: E731
            outs = HgcOutputs(None, None, None, None, *[ptr(k) for k in _HGC_SCALARS[4:]])
            keep = []
            dr = HgcDraws()
            if idxs is not None:
                t = _to_device(idxs, self.device).to(torch.int64).reshape(-1)
                assert t.numel() == total
                keep.append(t)
                dr.gc.idxs = t.data_ptr()
            for k, v in (draws or {}).items():
                if k == 'idxs':
                    continue
                t = _to_device(v, self.device).to(torch.int64 if k in _HDRAW_INT else torch.float64).reshape(-1)
                assert t.numel() == total, k
                keep.append(t)
                setattr(dr.gc if hasattr(dr.gc, k) else dr, k, t.data_ptr())
            rec = None
            if record_draws:
                rec_t = {k: torch.empty(total, dtype=torch.int64 if k in _HDRAW_INT else torch.float64,
                                        device=self.device) for k in _DRAW_ORDER + _HDRAW_LOW}
                rec = HgcDrawRecord(GcDrawRecord(*[rec_t[k].data_ptr() for k in _DRAW_ORDER]),
                                    *[rec_t[k].data_ptr() for k in _HDRAW_LOW])
                idx_t = {k: torch.empty(total, dtype=torch.int64, device=self.device) for k in _HGC_SCALARS[:4]}
                for k, t in idx_t.items():
                    setattr(outs, k, t.data_ptr())
        seed, call = self._next_seed()
        stream = _lib.stream_of(self.device)
        B, nb = int(batch_size), int(num_batches)
        if plain_call:
            plan = self._plan_for(seed)
            slot = self._next_slot()
            _lib.check(self._Lh.ogbx_gc_plan_set_batch(plan, slot, col_arr, ncols, B, nb, None, None, None, None,
                                                       None, ctypes.byref(outs)), 'gc_plan_set_batch')
            if len(self._out_cache) >= 2:
                self._out_cache.clear()
            self._out_cache[id(out)] = (out, (batch_size, num_batches), slot, outs, col_keep)
            st = self._Lh.ogbx_gc_plan_sample(plan, slot, call, stream)
        else:
            st = self._Lh.ogbx_hgc_sample(self._buf, self._cfg, self._hcfg, col_arr, ncols, B, nb, dr, seed, call,
                                          outs, rec, stream)
        _lib.check(st, 'hgc_sample')
        self._p_aug_draw(out, evaluation)
        if record_draws:
            out['_draws'] = rec_t
            for k, t in idx_t.items():
                out['_' + k] = t
            if not self._has_low:
                for k in _HDRAW_LOW:
                    out['_draws'].pop(k)
        del keep
        return out
