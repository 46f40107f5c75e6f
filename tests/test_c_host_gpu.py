"""GPU: a plain-C host (examples/c_host_pointmaze.c: gcc, libogbx.so and the HIP
runtime only -- no Python, no torch) drives pointmaze-large through the C-ABI:
create, reset, 1,100 auto-reset steps, the on-device eval counters, twice with
the same seed.  The program checks its own results (obs inside the maze,
one counted episode per env, bit-identical rerun) and prints OK."""

import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, 'examples', 'c_host_pointmaze')


def test_c_host_drives_the_c_abi():
    assert os.path.exists(EXE), 'examples/c_host_pointmaze not built (run __graft_entry__.build())'
    out = subprocess.run([EXE, '65536', '1100'], capture_output=True, text=True, timeout=180)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.strip().endswith('OK'), out.stdout
    assert 'episodes=65536' in out.stdout
