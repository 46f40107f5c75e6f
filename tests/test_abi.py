"""CPU checks of the C-ABI boundary: libogbx.so loads, exports every symbol of
include/ogbx.h, and its device-free tables match the reference fixtures."""

import ctypes

import numpy as np

from ogbench_amd import _lib


def test_library_loads_and_reports_abi():
    L = _lib.lib()
    assert L.ogbx_abi_version() == 5
    assert L.ogbx_build_arch() == b'gfx950'


def test_every_declared_symbol_is_exported():
    L = _lib.lib()
    declared = _lib.declared_symbols()
    assert len(declared) >= 15
    missing = [s for s in declared if not hasattr(L, s)]
    assert missing == []
    # every symbol the Python layer binds is declared in the header
    assert set(_lib._SIGNATURES) <= set(declared)


# Every entry point of include/ogbx.h at OGBX_ABI_VERSION 5, enumerated: a
# symbol added to (or dropped from) the header must be added here on purpose,
# documented in INTEGRATION.md and, if it changes the ABI, bump the version.
ABI5_SYMBOLS = {
    'ogbx_last_error', 'ogbx_abi_version', 'ogbx_stream_version', 'ogbx_build_arch',
    # locomaze (point) + antmaze wrapper
    'ogbx_maze_create', 'ogbx_maze_destroy', 'ogbx_maze_num_envs', 'ogbx_maze_set_envs_per_wave',
    'ogbx_maze_describe', 'ogbx_maze_tables', 'ogbx_maze_static_tables', 'ogbx_maze_reset', 'ogbx_maze_step', 'ogbx_maze_bind_step', 'ogbx_maze_step_bound',
    'ogbx_maze_rollout_until_done', 'ogbx_maze_state', 'ogbx_maze_set_seed', 'ogbx_point_physics',
    'ogbx_maze_xy_to_ij', 'ogbx_maze_ij_to_xy', 'ogbx_maze_oracle_subgoal', 'ogbx_maze_expert_action',
    'ogbx_maze_set_goal', 'ogbx_antmaze_state', 'ogbx_antmaze_reset', 'ogbx_antmaze_step', 'ogbx_antmaze_step_bound',
    # powderworld
    'ogbx_powder_create', 'ogbx_powder_destroy', 'ogbx_powder_describe', 'ogbx_powder_goal_worlds',
    'ogbx_powder_reset', 'ogbx_powder_step', 'ogbx_powder_state', 'ogbx_powder_state_view',
    'ogbx_powder_state_written', 'ogbx_powder_set_phase', 'ogbx_powder_set_seed', 'ogbx_powder_full_state', 'ogbx_powder_forward',
    'ogbx_powder_forward_full', 'ogbx_powder_task_table',
    # offline replay
    'ogbx_gc_sample', 'ogbx_gc_sample_ahead', 'ogbx_hgc_sample', 'ogbx_hgc_sample_ahead', 'ogbx_gc_traj_end',
    'ogbx_nonzero_f32', 'ogbx_compact_terminals', 'ogbx_gather_rows', 'ogbx_relabel_maze',
    'ogbx_gc_plan_create', 'ogbx_gc_plan_set_batch', 'ogbx_gc_plan_sample', 'ogbx_gc_plan_hits',
    'ogbx_gc_plan_destroy',
    # evaluation + collective
    'ogbx_eval_accumulate', 'ogbx_comm_unique_id', 'ogbx_comm_create', 'ogbx_comm_destroy', 'ogbx_eval_allgather',
}


def test_header_declares_exactly_the_abi5_symbols():
    assert set(_lib.declared_symbols()) == ABI5_SYMBOLS
    L = _lib.lib()
    assert [s for s in sorted(ABI5_SYMBOLS) if not hasattr(L, s)] == []


def test_integration_documents_every_symbol():
    """INTEGRATION.md names every entry point of the header (verdict r04 #8)."""
    import os

    doc = open(os.path.join(os.path.dirname(os.path.dirname(__file__)), 'INTEGRATION.md')).read()
    assert [s for s in sorted(ABI5_SYMBOLS) if s not in doc] == []


def test_static_tables_match_reference(golden_locomaze):
    from ogbench_amd.locomaze import static_tables

    for name in ['arena', 'medium', 'large', 'giant', 'teleport']:
        mp, tk = static_tables(name)
        assert np.array_equal(mp, golden_locomaze[f'map_{name}'])
        assert np.array_equal(tk, golden_locomaze[f'tasks_{name}'])


def test_unknown_maze_type_is_value_error():
    import pytest

    from ogbench_amd.locomaze import static_tables

    with pytest.raises(ValueError, match='Unknown maze type'):
        static_tables('spiral')


def test_create_without_gpu_fails_loudly():
    """No CPU fallback: creating a handle without a gfx950 device must fail."""
    import torch

    if torch.cuda.is_available():
        return
    L = _lib.lib()
    h = ctypes.c_void_p()
    opts = _lib.MazeOpts(0, 0, 1, 1, -1, 1000)
    st = L.ogbx_maze_create(b'large', 16, 0, opts, h)
    assert st == _lib.OGBX_EDEVICE
    assert 'CPU fallback' in _lib.last_error() or 'device' in _lib.last_error()


def test_powder_task_tables_match_reference():
    """The C++ task tables (every element set) vs the reference's set_tasks."""
    import os

    gold = np.load(os.path.join(os.path.dirname(__file__), 'golden', 'powder_full_golden.npz'))
    L = _lib.lib()
    for ne in (2, 5, 8):
        for t in range(1, 6):
            buf = np.zeros((256, 3), np.int32)
            n, tol = ctypes.c_int32(), ctypes.c_int32()
            assert L.ogbx_powder_task_table(ne, t, buf.ctypes.data_as(ctypes.c_void_p), 256, n, tol) == 0
            assert np.array_equal(buf[:n.value], gold[f'tasks{ne}_{t}_seq']), (ne, t)
            assert tol.value == int(gold[f'tasks{ne}_{t}_tol'])
    assert L.ogbx_powder_task_table(5, 6, None, 0, None, None) != 0
