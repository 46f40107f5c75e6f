"""CPU: record hygiene (verdict r05 item 7).  Every number that DESIGN.md's
summary table (section 0) and README.md's summary quote from a committed
record is recomputed here from the record it names -- the bench lines
(``BENCH_r05.json``, ``profiles/r06_*_bench.json``), the rocprofv3 kernel-trace
summaries (``profiles/r06_*_kernel_stats.csv``) and the PMC traffic records
(``profiles/traffic.json``) -- formatted as the document prints it, and must
appear in that document verbatim.  A number edited in a document without its
record (or a record replaced without the document) fails here."""

import csv
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _json(rel):
    with open(os.path.join(ROOT, rel)) as f:
        return json.load(f)


def _trace_us(rel, kernel):
    """Average duration (us) of the kernel-trace rows whose name contains
    `kernel` (template instances of one kernel pooled, as prof_summary does)."""
    tot = n = 0
    with open(os.path.join(ROOT, rel)) as f:
        for row in csv.DictReader(f):
            if kernel in row['Name']:
                tot += float(row['TotalDurationNs'])
                n += int(row['Calls'])
    assert n, (rel, kernel)
    return tot / n / 1e3


def _traffic(key):
    return _json('profiles/traffic.json')[key]['hbm_bytes_per_launch']


def _bench(wl):
    return _json(f'profiles/r06_{wl}_bench.json')


def _b05():
    return _json('BENCH_r05.json')['parsed']  # the driver's record of its own run


def _runs():
    return _json('profiles/r06_pointmaze_driver_runs.json')['runs']


def _window():
    return _json('profiles/r06_driver_window.json')['runs']


def _pm_trace(n):
    return _trace_us(f'profiles/r06_pointmaze-n{n}_kernel_stats.csv', 'maze_step_kernel')


def _pwf_dense(wl):
    return _trace_us(f'profiles/r06_{wl}_kernel_stats.csv', 'pwf_step_kernel<64, false>')


_PWF_BYTES = 64 * 64 * 16 + 27  # bench.py: algorithmic bytes per env-step, medium/hard
_HGC_BYTES = 2 * (12 * 276 + 84 + 8) + 16 + 72  # bench.py: algorithmic bytes per HGC sample


# (document, the text the document must contain, built from the records)
CLAIMS = [
    # the driver's own last run of the BASELINE metric
    ('README.md', lambda: f"**{_b05()['value'] / 1e9:.2f} G env-steps/s**"),
    ('DESIGN.md', lambda: f"**{_b05()['value'] / 1e9:.2f} G env-steps/s** ({_b05()['value'] / 1e7:.0f}× the 10 M target)"),
    ('DESIGN.md', lambda: f"{_b05()['ms_per_step'] * 1e3:.2f} µs per step "
                          f"({_b05()['roofline']['kernel_ms_back_to_back'] * 1e3:.2f} µs launch back to back)"),
    ('DESIGN.md', lambda: f"| {_b05()['roofline']['frac']:.3f} | {_b05()['cpu_baseline']['value'] / 1e6:.1f} M env-steps/s "
                          f"(C port, {_b05()['cpu_baseline']['cores']} threads) | `BENCH_r05.json` |"),
    # the driver's command on the round-6 build
    ('DESIGN.md', lambda: f"{min(r['value'] for r in _runs()) / 1e9:.2f}–{max(r['value'] for r in _runs()) / 1e9:.2f} "
                          f"G env-steps/s ({min(r['value'] for r in _window()[2:]) / 1e9:.2f}–"
                          f"{max(r['value'] for r in _window()[2:]) / 1e9:.2f} G on another box"),
    ('DESIGN.md', lambda: f"window / back to back {min(r['timed_over_b2b'] for r in _runs()):.2f}–"
                          f"{max(r['timed_over_b2b'] for r in _runs()):.2f}× on this box "
                          f"({min(r['timed_over_b2b'] for r in _window()[2:]):.2f}–"
                          f"{max(r['timed_over_b2b'] for r in _window()[2:]):.2f}× on the other)"),
    ('README.md', lambda: f"{min(r['value'] for r in _runs()) / 1e9:.2f}–{max(r['value'] for r in _runs()) / 1e9:.2f} G"),
    # pointmaze-large, 2,000 timed steps
    ('DESIGN.md', lambda: f"| **{_bench('pointmaze')['value'] / 1e9:.2f} G env-steps/s** | **{_pm_trace(65536):.2f} µs "
                          f"trace avg** | {_bench('pointmaze')['roofline']['frac']:.3f} (latency-bound, §4.1); traffic "
                          f"{_traffic('maze_step_kernel@pointmaze') / 1e6:.2f} MB = "
                          f"{_traffic('maze_step_kernel@pointmaze') / (87 * 65536):.2f}× algorithmic | "
                          f"{_bench('pointmaze')['cpu_baseline']['value'] / 1e6:.1f} M env-steps/s (C port, 16 threads)"),
    ('README.md', lambda: f"{_bench('pointmaze')['value'] / 1e9:.2f} G env-steps/s on the 2,000-step bench"),
    ('README.md', lambda: f"{_pm_trace(65536):.1f} µs per launch"),
    # strong-scaling shares
    ('DESIGN.md', lambda: f"{_pm_trace(32768):.2f} / {_pm_trace(16384):.2f} / {_pm_trace(8192):.2f} µs trace avg"),
    ('README.md', lambda: f"{_pm_trace(8192):.2f} µs at the 8-GPU share"),
    # pointmaze-medium, one env
    ('DESIGN.md', lambda: f"{_bench('pointmaze-medium-n1')['value'] / 1e3:.0f} k env-steps/s (Gymnasium surface"),
    ('DESIGN.md', lambda: f"{_bench('pointmaze-medium-n1')['cpu_baseline']['value'] / 1e3:.0f} k env-steps/s (C port, 1 core)"),
    # antmaze wrapper
    ('DESIGN.md', lambda: f"{_bench('antmaze')['value'] / 1e9:.2f} G env-steps/s (timed loop "
                          f"{_bench('antmaze')['ms_per_step'] * 1e3:.2f} µs per call"),
    ('DESIGN.md', lambda: f"**{_trace_us('profiles/r06_antmaze_kernel_stats.csv', 'ant_step_kernel'):.2f} µs** trace avg, "
                          f"{_bench('antmaze')['roofline']['kernel_ms'] * 1e3:.2f} µs back to back | "
                          f"{_bench('antmaze')['roofline']['frac']:.2f} | "
                          f"{_bench('antmaze')['cpu_baseline']['value'] / 1e6:.0f} M env-steps/s (NumPy port, 1 core)"),
    # powderworld easy / medium / hard
    ('DESIGN.md', lambda: f"| {_bench('powder')['value'] / 1e6:.0f} M env-steps/s (K=48 fused "
                          f"{_bench('powder')['extra']['fused_k48_steps_per_s'] / 1e6:.0f} M) | "
                          f"{_bench('powder')['roofline']['kernel_ms'] * 1e3:.1f} µs | "
                          f"{_bench('powder')['roofline']['frac']:.2f} (fused "
                          f"{_bench('powder')['extra']['fused_k48_achieved_GBs'] / 8000:.2f}) | "
                          f"{_bench('powder')['cpu_baseline']['value'] / 1e3:.1f} k env-steps/s"),
    ('DESIGN.md', lambda: f"{_bench('powder-medium')['value'] / 1e6:.1f} M env-steps/s = "
                          f"{_bench('powder-medium')['ms_per_step']:.4f} ms per step (medium; steady window "
                          f"{_bench('powder-medium')['extra']['steady_state_ms_per_step']:.3f} ms; four synchronized "
                          f"resets of {_bench('powder-medium')['extra']['sync_reset_step_ms']:.1f} ms)"),
    ('DESIGN.md', lambda: f"forward-step launch {_pwf_dense('powder-medium'):.0f} µs trace avg"),
    ('DESIGN.md', lambda: f"**{_bench('powder-medium')['roofline']['frac']:.3f} / "
                          f"{_bench('powder-hard')['roofline']['frac']:.3f}** on the render-cache basis"),
    ('DESIGN.md', lambda: f"PMC {_traffic('pwf_light_step_kernel+pwf_step_kernel@powder-medium') / 1e6:.0f} MB per step = "
                          f"{_traffic('pwf_light_step_kernel+pwf_step_kernel@powder-medium') / (_PWF_BYTES * 4096):.2f}×"),
    ('DESIGN.md', lambda: f"{_bench('powder-medium')['cpu_baseline']['value'] / 1e3:.2f} k env-steps/s (NumPy port, 1 core)"),
    ('DESIGN.md', lambda: f"{_bench('powder-hard')['value'] / 1e6:.1f} M env-steps/s = "
                          f"{_bench('powder-hard')['ms_per_step']:.4f} ms per step (hard; steady "
                          f"{_bench('powder-hard')['extra']['steady_state_ms_per_step']:.3f} ms; resets "
                          f"{_bench('powder-hard')['extra']['sync_reset_step_ms']:.1f} ms)"),
    ('DESIGN.md', lambda: f"forward-step launch {_pwf_dense('powder-hard'):.0f} µs trace avg | "
                          f"{_bench('powder-hard')['roofline']['frac']:.3f} | "
                          f"{_bench('powder-hard')['cpu_baseline']['value'] / 1e3:.2f} k env-steps/s"),
    # offline replay
    ('DESIGN.md', lambda: f"**{_bench('gcsample')['value'] / 1e6:.0f} M samples/s** "
                          f"({_bench('gcsample')['ms_per_step'] * 1e3:.2f} µs per call"),
    ('DESIGN.md', lambda: f"**{_trace_us('profiles/r06_gcsample_kernel_stats.csv', 'gc_ahead_kernel<true'):.2f} µs** "
                          f"trace avg (`gc_ahead_kernel<true, …>`) | {_bench('gcsample')['roofline']['frac']:.3f} "
                          f"(fused {_bench('gcsample')['extra']['fused_256x1024_achieved_GBs'] / 8000:.2f}); traffic "
                          f"{_traffic('gc_ahead_kernel<true>@gcsample') / 1e6:.2f} MB = "
                          f"{_traffic('gc_ahead_kernel<true>@gcsample') / (2424 * 1024):.2f}× | "
                          f"{_bench('gcsample')['cpu_baseline']['value'] / 1e6:.2f} M samples/s"),
    ('DESIGN.md', lambda: f"**{_bench('hgcsample')['value'] / 1e6:.0f} M samples/s** (128×1024 fused "
                          f"{_bench('hgcsample')['extra']['fused_128x1024_samples_per_s'] / 1e6:.0f} M)"),
    ('DESIGN.md', lambda: f"**{_trace_us('profiles/r06_hgcsample_kernel_stats.csv', 'hgc_ahead_kernel<true'):.2f} µs** "
                          f"trace avg (`hgc_ahead_kernel<true, …>`) | {_bench('hgcsample')['roofline']['frac']:.3f} "
                          f"(fused {_bench('hgcsample')['extra']['fused_128x1024_achieved_GBs'] / 8000:.2f}); traffic "
                          f"{_traffic('hgc_ahead_kernel<true>@hgcsample') / 1e6:.2f} MB = "
                          f"{_traffic('hgc_ahead_kernel<true>@hgcsample') / (_HGC_BYTES * 1024):.2f}× (repeated rows hit L2) | "
                          f"{_bench('hgcsample')['cpu_baseline']['value'] / 1e6:.2f} M samples/s"),
]


@pytest.mark.parametrize('i', range(len(CLAIMS)))
def test_document_number_equals_its_record(i):
    doc, fn = CLAIMS[i]
    want = fn()
    with open(os.path.join(ROOT, doc), encoding='utf-8') as f:
        body = ' '.join(f.read().split())  # line breaks of wrapped prose are spaces
    assert want in body, f'{doc} does not say {want!r} (the records formatted as the document prints them)'
