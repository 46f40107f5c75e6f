"""GPU: bench.py keeps the driver's output contract (one JSON line with the
metric, value, roofline and cpu_baseline fields) and its per-launch time never
exceeds the timed region's per-step time.  Short runs of the default workload
and of the antmaze wrapper workload, each in a child process."""

import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args, timeout=240):
    out = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), *args], cwd=ROOT, capture_output=True,
                         text=True, timeout=timeout)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, out.stdout[-2000:]
    return json.loads(lines[0])


def _contract(r):
    for k in ('metric', 'value', 'unit', 'n_gpus', 'steps', 'warmup', 'ms_per_step', 'higher_is_better', 'scaling',
              'vs_baseline', 'dtype', 'data', 'config', 'roofline'):
        assert k in r, k
    assert r['value'] > 0 and r['n_gpus'] == 1 and r['higher_is_better'] is True
    rf = r['roofline']
    for k in ('bound', 'achieved', 'peak', 'unit', 'frac', 'traffic', 'kernel_ms'):
        assert k in rf, k
    assert abs(rf['frac'] - rf['achieved'] / rf['peak']) < 1e-12
    # per-launch device time (one event span over back-to-back launches)
    # within the timed region's per-step time (5 % slack for run-to-run noise)
    assert rf['kernel_ms'] <= r['ms_per_step'] * 1.05, (rf['kernel_ms'], r['ms_per_step'])


def test_default_bench_line():
    r = _run('--steps', '1000', '--warmup', '50', '--cpu-seconds', '2')
    _contract(r)
    assert r['metric'].startswith('env steps/sec at N=65536 parallel envs, pointmaze-large')
    assert r['config']['total_envs'] == 65536 and r['scaling'] == 'strong' and r['dtype'] == 'f64'
    assert r['extra']['eval_allgather']['overall_success'] > 0.5
    cb = r['cpu_baseline']
    assert cb['value'] > 0 and cb['cores'] >= 1 and cb['kind'] in ('port', 'reference') and cb['sample']


def test_two_rank_line_without_a_launcher():
    # `bench.py --gpus 2` with no torchrun: bench.py starts both ranks itself
    # (gloo, both on this box's GPU) and rank 0's line covers the 2-rank job
    env = {k: v for k, v in os.environ.items() if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK')}
    out = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), '--gpus', '2', '--dist-backend', 'gloo',
                          '--steps', '20', '--warmup', '5'], cwd=ROOT, env=env, capture_output=True, text=True,
                         timeout=400)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, out.stdout[-2000:]
    r = json.loads(lines[0])
    assert r['n_gpus'] == 2 and r['ranks_seen'] == 2
    assert r['extra']['eval_allgather']['ranks'] == 2
    assert r['config']['num_envs_per_gpu'] == 32768 and r['config']['total_envs'] == 65536
    assert r['metric'] == 'env steps/sec at N=65536 parallel envs, pointmaze-large, 1/2/4/8 MI355X'
    assert 'cpu_baseline' not in r  # rank 0 at N = 1 only


def test_antmaze_bench_line():
    r = _run('--workload', 'antmaze', '--steps', '1000', '--warmup', '50', '--no-cpu-baseline')
    _contract(r)
    assert r['config']['num_envs_per_gpu'] == 16384 and r['roofline']['kernel'] == 'ant_step_kernel'
