import os
import socket
import subprocess
import sys
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, 'tests', 'golden')
SHARD_WORLD = 2
_shard_job = {}


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs a real MI355X (gfx950) and libogbx.so')


def _gpu_session(config):
    expr = (config.getoption('markexpr') or '').replace(' ', '')
    return 'gpu' in expr and 'notgpu' not in expr


def pytest_sessionstart(session):
    """GPU sessions: start the 2-rank sharded rollout (tests/shard_worker.py)
    here, before this process makes any GPU call -- the ranks are fresh
    processes (gloo process group, both on cuda:0); tests/test_shard_gpu.py
    waits for them and compares their outputs with the single-process run."""
    if not _gpu_session(session.config):
        return
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    out = tempfile.mkdtemp(prefix='ogbx_shard_')
    procs = []
    for r in range(SHARD_WORLD):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(SHARD_WORLD), LOCAL_RANK=str(r),
                   MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
        log = open(os.path.join(out, f'rank{r}.log'), 'w')
        procs.append(subprocess.Popen([sys.executable, '-u', os.path.join(ROOT, 'tests', 'shard_worker.py'), out],
                                      env=env, stdout=log, stderr=subprocess.STDOUT, start_new_session=True))
    _shard_job.update(out=out, procs=procs)


def pytest_sessionfinish(session, exitstatus):
    """Never leave a rank process behind (e.g. after -x stopped the session)."""
    import signal

    for p in _shard_job.get('procs', []):
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except OSError:
                pass
            p.wait()


@pytest.fixture(scope='session')
def shard_job():
    return _shard_job


@pytest.fixture(scope='session')
def gpu():
    """The GPU device; GPU tests fail loudly (never skip) without one."""
    import torch

    assert torch.cuda.is_available(), 'gpu-marked test run without a visible GPU'
    from ogbench_amd import _lib

    _lib.lib()
    return torch.device('cuda', 0)


@pytest.fixture(scope='session')
def golden_locomaze():
    import numpy as np

    return dict(np.load(os.path.join(GOLDEN, 'locomaze_golden.npz')))
