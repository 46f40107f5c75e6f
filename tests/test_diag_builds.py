"""The diagnostic build toggles still compile (CPU: hipcc cross-compiles gfx950).

The shipped kernels carry exactly five compile-time toggles, all diagnostic
(they add counters or clock stamps and change no result):
  * OGBX_PHYS_STATS  -- contact-path counters (point_physics.h, point_contact.h)
  * OGBX_WAVE_STAMPS -- per-wave wall-clock stamps + path counts (locomaze.hip)
  * OGBX_STAGE_STAMPS -- per-wave cycles of each part of the lean contact stage
  * OGBX_MASK_TRACE  -- per-env start / settled active-edge masks of every lean stage
  * OGBX_PWF_RULE_STAMPS -- per-rule cycle stamps of the full powderworld forward
No test builds them otherwise, so this one does (device code only, -O1 to keep
the CPU suite short; the two source files compile in parallel).
"""
import os
import shutil
import subprocess

import pytest

CSRC = os.path.join(os.path.dirname(__file__), '..', 'ogbench_amd', 'csrc')
HIPCC = '/opt/rocm/bin/hipcc'
FLAGS = ['-O1', '-std=c++17', '--offload-arch=gfx950', '-ffp-contract=off', '-Wall', '-Werror',
         '-Wno-unused-function', '-Wno-unused-variable', '-Wno-bitwise-instead-of-logical',
         '-Wno-unused-command-line-argument', '--cuda-device-only', '-c']


@pytest.mark.skipif(not os.path.exists(HIPCC), reason='hipcc not installed')
def test_diagnostic_toggles_compile(tmp_path):
    jobs = {
        'locomaze': ['-DOGBX_PHYS_STATS', '-DOGBX_WAVE_STAMPS', '-DOGBX_STAGE_STAMPS', '-DOGBX_MASK_TRACE'],
        'powder': ['-DOGBX_PWF_RULE_STAMPS'],
    }
    procs = {}
    for src, defs in jobs.items():
        cmd = [HIPCC] + FLAGS + defs + [os.path.join(CSRC, src + '.hip'), '-o', str(tmp_path / (src + '.o'))]
        procs[src] = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    errors = []
    for src, p in procs.items():
        out, _ = p.communicate(timeout=600)
        if p.returncode != 0:
            errors.append('%s %s:\n%s' % (src, jobs[src], out[-4000:]))
    assert not errors, '\n'.join(errors)


def test_no_ab_toggles_left_in_kernels():
    """Only the diagnostic toggles remain: no compiled-out A/B variant code."""
    allowed = {'OGBX_PHYS_STATS', 'OGBX_WAVE_STAMPS', 'OGBX_STAGE_STAMPS', 'OGBX_MASK_TRACE', 'OGBX_PWF_RULE_STAMPS'}
    found = set()
    for name in os.listdir(CSRC):
        if not name.endswith(('.hip', '.h')):
            continue
        for line in open(os.path.join(CSRC, name)):
            s = line.strip()
            if s.startswith(('#if', '#elif')):
                toks = s.replace('(', ' ').replace(')', ' ').replace('!', ' ').split()
                found.update(t for t in toks[1:] if t.startswith('OGBX_'))
    assert found <= allowed, sorted(found - allowed)
