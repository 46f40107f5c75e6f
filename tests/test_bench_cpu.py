"""CPU: bench.py's host-side helpers -- the traffic record is used only for a
run of the same workload, per-launch units and world size (else null), and the
sharding of the metric's fixed total N."""

import json
import os
import sys

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


def test_strong_scaling_shards_cover_the_total():
    for world in (1, 2, 4, 8):
        spans = [shard(65536, world, r) for r in range(world)]
        assert spans[0][0] == 0 and sum(n for _, n in spans) == 65536
        for (b0, n0), (b1, _) in zip(spans, spans[1:]):
            assert b0 + n0 == b1
        assert all(n % 64 == 0 for _, n in spans)  # whole waves per rank
