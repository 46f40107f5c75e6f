"""ctypes binding of libogbx.so (the C-ABI declared in include/ogbx.h).

The library is built in-tree (``ogbench_amd/libogbx.so``) by
``__graft_entry__.build()`` / ``make -C ogbench_amd/csrc``.  There is no CPU
fallback: if the library is missing or no gfx950 device is visible, every
entry point that needs the GPU raises ``RuntimeError``.
"""

from __future__ import annotations

import ctypes
import os
import re
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('OGBX_LIB', os.path.join(_HERE, 'libogbx.so'))
HEADER_PATH = os.path.join(os.path.dirname(_HERE), 'include', 'ogbx.h')

OGBX_OK = 0
OGBX_EINVAL = -1
OGBX_EDEVICE = -2
OGBX_ENOMEM = -3
OGBX_ESTATE = -4

c_void_p = ctypes.c_void_p
c_int32 = ctypes.c_int32
c_int64 = ctypes.c_int64
c_uint64 = ctypes.c_uint64
c_double = ctypes.c_double
c_char_p = ctypes.c_char_p
P = ctypes.POINTER


class MazeOpts(ctypes.Structure):
    _fields_ = [
        ('loco_type', c_int32),
        ('success_timing', c_int32),
        ('terminate_at_goal', c_int32),
        ('add_noise_to_goal', c_int32),
        ('reward_task_id', c_int32),
        ('max_episode_steps', c_int32),
        ('env_base', c_int64),
    ]


class PowderOpts(ctypes.Structure):
    _fields_ = [
        ('world_size', c_int32),
        ('grid_size', c_int32),
        ('brush_size', c_int32),
        ('num_elems', c_int32),
        ('max_episode_steps', c_int32),
        ('pad', c_int32),
        ('env_base', c_int64),
    ]


# name -> (restype, argtypes)
_SIGNATURES = {
    'ogbx_last_error': (c_char_p, []),
    'ogbx_abi_version': (c_int32, []),
    'ogbx_stream_version': (c_int32, []),
    'ogbx_build_arch': (c_char_p, []),
    # locomaze
    'ogbx_maze_create': (c_int32, [c_char_p, c_int64, c_int32, P(MazeOpts), P(c_void_p)]),
    'ogbx_maze_destroy': (c_int32, [c_void_p]),
    'ogbx_maze_num_envs': (c_int64, [c_void_p]),
    'ogbx_maze_set_envs_per_wave': (c_int32, [c_void_p, c_int32]),
    'ogbx_maze_describe': (c_int32, [c_void_p, P(c_int32), P(c_int32), P(c_int32), P(c_double), P(c_double)]),
    'ogbx_maze_tables': (c_int32, [c_void_p, c_void_p, c_void_p]),
    'ogbx_maze_static_tables': (c_int32, [c_char_p, P(c_int32), P(c_int32), P(c_int32), c_void_p, c_void_p]),
    'ogbx_maze_reset': (
        c_int32,
        [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_uint64, c_void_p],
    ),
    'ogbx_maze_step': (
        c_int32,
        [c_void_p, c_void_p, c_int32, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
         c_int32, c_void_p],
    ),
    'ogbx_maze_bind_step': (c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int32]),
    'ogbx_maze_step_bound': (c_int32, [c_void_p, c_void_p, c_int32, c_void_p]),
    'ogbx_antmaze_step_bound': (c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    'ogbx_antmaze_state': (c_int32, [c_void_p, P(c_void_p), P(c_void_p)]),
    'ogbx_antmaze_reset': (
        c_int32,
        [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
         c_uint64, c_void_p],
    ),
    'ogbx_antmaze_step': (
        c_int32,
        [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int32,
         c_void_p, c_void_p],
    ),
    'ogbx_maze_rollout_until_done': (
        c_int32,
        [c_void_p, c_void_p, c_int32, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    ),
    'ogbx_maze_state': (c_int32, [c_void_p, P(c_void_p), P(c_void_p), P(c_void_p), P(c_void_p), P(c_void_p)]),
    'ogbx_maze_set_seed': (c_int32, [c_void_p, c_uint64]),
    'ogbx_point_physics': (c_int32, [c_void_p, c_void_p, c_void_p, c_int32, c_int64, c_void_p, c_void_p, c_void_p]),
    'ogbx_maze_xy_to_ij': (c_int32, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p]),
    'ogbx_maze_ij_to_xy': (c_int32, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p]),
    'ogbx_maze_oracle_subgoal': (c_int32, [c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p]),
    'ogbx_maze_expert_action': (
        c_int32, [c_void_p, c_void_p, c_void_p, c_int64, c_double, c_void_p, c_uint64, c_uint64, c_void_p, c_void_p]
    ),
    'ogbx_maze_set_goal': (c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_uint64, c_uint64, c_void_p]),
    # powderworld
    'ogbx_powder_create': (c_int32, [P(PowderOpts), c_int64, c_int32, P(c_void_p)]),
    'ogbx_powder_destroy': (c_int32, [c_void_p]),
    'ogbx_powder_describe': (c_int32, [c_void_p, P(c_int32), P(c_int32), P(c_int32), P(c_int32), P(c_int32)]),
    'ogbx_powder_goal_worlds': (c_int32, [c_void_p, c_void_p]),
    'ogbx_powder_reset': (
        c_int32,
        [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_void_p, c_void_p, c_uint64, c_void_p],
    ),
    'ogbx_powder_step': (
        c_int32,
        [c_void_p, c_void_p, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
         c_int32, c_void_p],
    ),
    'ogbx_powder_state': (c_int32, [c_void_p, P(c_void_p), P(c_void_p), P(c_void_p), P(c_void_p)]),
    'ogbx_powder_set_seed': (c_int32, [c_void_p, c_uint64]),
    'ogbx_powder_full_state': (c_int32, [c_void_p, P(c_void_p), P(c_void_p), P(c_void_p)]),
    'ogbx_powder_state_view': (c_int32, [c_void_p, P(c_void_p), P(c_void_p), P(c_void_p), P(c_void_p)]),
    'ogbx_powder_state_written': (c_int32, [c_void_p]),
    'ogbx_powder_set_phase': (c_int32, [c_void_p, c_int64]),
    'ogbx_powder_forward': (c_int32, [c_void_p, c_void_p, c_int64, c_int32, c_void_p, c_void_p]),
    'ogbx_powder_forward_full': (
        c_int32, [c_void_p, c_void_p, c_int64, c_int32, c_void_p, c_void_p, c_void_p, c_void_p]
    ),
    'ogbx_powder_task_table': (c_int32, [c_int32, c_int32, c_void_p, c_int32, P(c_int32), P(c_int32)]),
    # evaluation
    'ogbx_eval_accumulate': (
        c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int32, c_void_p, c_void_p]
    ),
    'ogbx_comm_unique_id': (c_int32, [c_void_p]),
    'ogbx_comm_create': (c_int32, [c_void_p, c_int32, c_int32, c_int32, P(c_void_p)]),
    'ogbx_comm_destroy': (c_int32, [c_void_p]),
    'ogbx_eval_allgather': (c_int32, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p]),
}

_lock = threading.Lock()
_lib = None


class OgbxError(RuntimeError):
    """Failure reported by libogbx (status code + thread-local message)."""

    def __init__(self, status, message):
        super().__init__(f'libogbx status {status}: {message}')
        self.status = status
        self.message = message


def lib():
    """Load libogbx.so (once) and declare every signature.  Raises if missing."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f'libogbx.so not found at {LIB_PATH}; build it with '
                f'`python -c "import __graft_entry__ as g; g.build()"` or `make -C ogbench_amd/csrc`. '
                f'There is no CPU fallback.'
            )
        handle = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        # Every entry point include/ogbx.h declares must be exported, whichever
        # library is loaded (the in-tree build or an OGBX_LIB override): a stale
        # or partial library fails here, not at the first call of a missing symbol.
        missing = [n for n in declared_symbols() if not hasattr(handle, n)]
        missing += [n for n in _SIGNATURES if not hasattr(handle, n)]
        if missing:
            raise RuntimeError(f'{LIB_PATH} lacks entry points declared in {HEADER_PATH}: '
                               f'{", ".join(sorted(set(missing)))}; rebuild it (make -C ogbench_amd/csrc)')
        for name, (res, args) in _SIGNATURES.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        # struct layouts follow the header's ABI version: a library built
        # from another version would misread them
        want = header_abi_version()
        if handle.ogbx_abi_version() != want:
            raise RuntimeError(f'{LIB_PATH} has ABI version {handle.ogbx_abi_version()}, {HEADER_PATH} '
                               f'declares {want}; rebuild it (make -C ogbench_amd/csrc)')
        _lib = handle
        return _lib


def header_abi_version(header_path=HEADER_PATH):
    """OGBX_ABI_VERSION as include/ogbx.h defines it."""
    return int(re.search(r'#define\s+OGBX_ABI_VERSION\s+(\d+)', open(header_path).read()).group(1))


def declared_symbols(header_path=HEADER_PATH):
    """Every function name declared in include/ogbx.h."""
    text = open(header_path).read()
    text = re.sub(r'/\*.*?\*/', '', text, flags=re.S)
    names = re.findall(r'\b(ogbx_[a-z0-9_]+)\s*\(', text)
    return sorted(set(names))


def last_error():
    return lib().ogbx_last_error().decode(errors='replace')


def check(status, what=''):
    """Raise the reference-compatible exception for a non-OK status."""
    if status == OGBX_OK:
        return
    msg = last_error()
    if what:
        msg = f'{what}: {msg}'
    if status == OGBX_EINVAL:
        raise ValueError(msg)
    raise OgbxError(status, msg)


def ptr(t):
    """Device pointer of a torch tensor (or None -> NULL)."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())


_dev_index = {}


def stream_of(device):
    """hipStream_t of torch's current stream on `device`, as a void*.

    Reads the raw stream handle (no torch.cuda.Stream object per call: that
    costs microseconds, the same order as a latency-bound sampler launch)."""
    import torch

    idx = _dev_index.get(device)
    if idx is None:
        d = torch.device('cuda', device) if isinstance(device, int) else torch.device(device)
        if d.index is None:  # 'cuda': the current device, which may change
            return ctypes.c_void_p(torch._C._cuda_getCurrentRawStream(torch.cuda.current_device()))
        idx = _dev_index[device] = d.index
    return ctypes.c_void_p(torch._C._cuda_getCurrentRawStream(idx))
