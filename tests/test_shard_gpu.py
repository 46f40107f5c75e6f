"""GPU: sharded runs reproduce the single-GPU run bit for bit.

Two fresh rank processes (started by conftest.pytest_sessionstart before any
GPU call of this process; gloo process group; both on cuda:0) each step their
contiguous half of the job's envs with handles created at ``env_base`` =
rank * N/2 and one shared seed.  This process runs the same job as ONE batch
of N envs.  Every per-env output (reset obs/goal, obs, reward, terminated,
truncated, success, final qpos) must be identical, and the all-gathered eval
counters must equal the single-run counters.  pointmaze-large: 4096 envs x
300 steps, expert actions with Philox noise, TimeLimit 250 with auto-reset;
powderworld-easy: 128 envs x 30 steps with invalid actions (Philox
replacements) and auto-reset; antmaze-large wrapper (configs[4]): 1024 envs x
60 steps on caller post-physics states, TimeLimit 25, auto-reset alternating
caller reset states and Philox bodies, gathered eval counters.
"""

import os
import signal
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import shard_worker as sw  # noqa: E402

pytestmark = pytest.mark.gpu


def _wait(job, timeout=240):
    assert job, 'the sharded job was not started (run with -m gpu)'
    for p in job['procs']:
        try:
            rc = p.wait(timeout=timeout)
        except Exception:
            for q in job['procs']:
                try:
                    os.killpg(q.pid, signal.SIGKILL)
                except OSError:
                    pass
            raise
        if rc != 0:
            logs = ''.join(open(os.path.join(job['out'], f'rank{r}.log')).read()[-3000:]
                           for r in range(len(job['procs'])))
            raise AssertionError(f'rank process exited with {rc}:\n{logs}')
    return [dict(np.load(os.path.join(job['out'], f'rank{r}.npz'))) for r in range(len(job['procs']))]


@pytest.fixture(scope='module')
def ranks(shard_job):
    return _wait(shard_job)


def test_maze_shards_equal_single_gpu_run(gpu, ranks):
    ref, counters = sw.run_maze(0, sw.MAZE_TOTAL, gpu)
    keys = ('obs0', 'goal0', 'obs', 'reward', 'terminated', 'truncated', 'success', 'qpos')
    for r, got in enumerate(ranks):
        b, n = int(got['base']), int(got['n'])
        for k in keys:
            exp = ref[k][b:b + n] if k in ('obs0', 'goal0', 'qpos') else ref[k][:, b:b + n]
            assert np.array_equal(got['maze_' + k], exp), f'rank {r}: {k} differs from the single run'
    assert sum(int(g['n']) for g in ranks) == sw.MAZE_TOTAL
    # the all-gathered counters equal the single run's, and are non-trivial
    for got in ranks:
        assert np.array_equal(got['maze_gathered_total'], ref['counters'])
        assert np.array_equal(got['maze_gathered_per_rank'].sum(0), ref['counters'])
    assert ref['counters'][:, 0].sum() > 0 and ref['truncated'].sum() > 0


def test_powder_shards_equal_single_gpu_run(gpu, ranks):
    ref = sw.run_powder(0, sw.POWDER_TOTAL, gpu)
    for r, got in enumerate(ranks):
        b, n = int(got['pbase']), int(got['pn'])
        assert np.array_equal(got['powder_obs0'], ref['obs0'][b:b + n])
        for k in ('obs', 'reward', 'terminated', 'truncated', 'success'):
            assert np.array_equal(got['powder_' + k], ref[k][:, b:b + n]), f'rank {r}: powder {k}'
    assert ref['truncated'].sum() > 0


def test_ant_shards_equal_single_gpu_run(gpu, ranks):
    ref, counters = sw.run_ant(0, sw.ANT_TOTAL, gpu)
    per_env = ('obs0', 'goal0', 'body', 'goal_xy')
    for r, got in enumerate(ranks):
        b, n = int(got['abase']), int(got['an'])
        for k in per_env + ('obs', 'final_obs', 'reward', 'terminated', 'truncated', 'success'):
            exp = ref[k][b:b + n] if k in per_env else ref[k][:, b:b + n]
            assert np.array_equal(got['ant_' + k], exp), f'rank {r}: ant {k} differs from the single run'
    assert sum(int(g['an']) for g in ranks) == sw.ANT_TOTAL
    for got in ranks:
        assert np.array_equal(got['ant_gathered_total'], ref['counters'])
        assert np.array_equal(got['ant_gathered_per_rank'].sum(0), ref['counters'])
    # goal ends and TimeLimit ends both happen, so both reset paths ran
    assert ref['terminated'].sum() > 100 and ref['truncated'].sum() > 100
    assert ref['counters'][:, 0].sum() > 0
