"""CPU: bench.py's host-side helpers -- the traffic record is used only for a
run of the same workload, per-launch units and world size (else null), and the
sharding of the metric's fixed total N."""

import json
import os
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from ogbench_amd.sharding import shard  # noqa: E402


def test_traffic_record_selected_by_configuration():
    with open(os.path.join(ROOT, 'profiles', 'traffic.json')) as f:
        rec = json.load(f)['maze_step_kernel@pointmaze']
    assert bench._traffic('maze_step_kernel', 'pointmaze', rec['units'], rec.get('world', 1)) == \
        rec['hbm_bytes_per_launch']
    assert bench._traffic('maze_step_kernel', 'pointmaze', rec['units'] // 2, 1) is None  # other N
    assert bench._traffic('maze_step_kernel', 'pointmaze', rec['units'], 2) is None  # other world size
    assert bench._traffic('maze_step_kernel', 'powder', rec['units'], 1) is None  # other workload
    # the committed record is within 1.15x of the 87 B/env-step algorithmic
    # bytes plus the kernel's instruction fetch: the fully unrolled contact
    # loop is 348 KB of code (86 KB at unroll 4, where the record was 1.06x),
    # fetched again every launch (the FETCH_SIZE pass grows by
    # 355 KiB per launch between the two builds)
    code_fetch = 2 * 355 * 1024
    assert rec['hbm_bytes_per_launch'] <= 1.15 * 87 * rec['units'] + code_fetch


def test_rank_layout_checks():
    # no launcher: one GPU runs in-process, N > 1 self-launches
    assert bench._check_world(1, 'gloo', env={}) == 'rank'
    assert bench._check_world(2, 'gloo', env={}) == 'self-launch'
    assert bench._check_world(2, 'gloo', env={'WORLD_SIZE': '2'}) == 'rank'
    # a launcher whose world size differs from --gpus is refused, not noted
    with pytest.raises(SystemExit) as e:
        bench._check_world(8, 'gloo', env={'WORLD_SIZE': '2'})
    assert e.value.code == 2
    # more RCCL ranks than visible GPUs (none here) is refused
    with pytest.raises(SystemExit) as e:
        bench._check_world(torch.cuda.device_count() + 1, 'nccl', env={})
    assert e.value.code == 2


def test_mismatched_world_exits_before_touching_the_gpu():
    env = dict(os.environ, WORLD_SIZE='3', RANK='0', LOCAL_RANK='0')
    out = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), '--gpus', '2', '--dist-backend', 'gloo'],
                         env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode == 2, (out.returncode, out.stderr[-2000:])
    assert 'WORLD_SIZE=3' in out.stderr and not any(ln.startswith('{') for ln in out.stdout.splitlines())


def test_self_launch_returns_the_worst_rank_status(tmp_path, monkeypatch):
    # the launcher itself, on a stand-in script: every rank sees its own
    # RANK / WORLD_SIZE and a shared 127.0.0.1 rendezvous, and the parent
    # returns the worst status
    probe = tmp_path / 'rank.py'
    probe.write_text('import os, sys\n'
                     'print(os.environ["RANK"], os.environ["WORLD_SIZE"], os.environ["MASTER_ADDR"], flush=True)\n'
                     'sys.exit(3 if os.environ["RANK"] == "1" else 0)\n')
    monkeypatch.setattr(bench, '__file__', str(probe))
    rc, rcs = bench._self_launch(3, [])
    assert rcs == [0, 3, 0] and rc == 3


def test_strong_scaling_shards_cover_the_total():
    for world in (1, 2, 4, 8):
        spans = [shard(65536, world, r) for r in range(world)]
        assert spans[0][0] == 0 and sum(n for _, n in spans) == 65536
        for (b0, n0), (b1, _) in zip(spans, spans[1:]):
            assert b0 + n0 == b1
        assert all(n % 64 == 0 for _, n in spans)  # whole waves per rank
