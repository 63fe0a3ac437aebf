"""The bench line's PMC half: bench.py reads traffic and VALU issue from the tracked
roofline_pmc.json, which travels to the GPU box (profiles/ does not), and every number in it
reproduces from the committed rocprofv3 summaries it names (scripts/prof_summary.py)."""
import csv
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _db():
    return json.load(open(os.path.join(ROOT, "roofline_pmc.json")))


def _counter(src, name):
    import glob
    for f in glob.glob(os.path.join(ROOT, src, "pmc_*_zb_step_kernel.csv")):
        for row in csv.DictReader(open(f)):
            if row["counter"] == name:
                return float(row["mean_per_dispatch"])
    raise KeyError(name)


def test_headline_grid_present_and_reproducible():
    # 4096 envs = 1024 workgroups x 64 work-items = 65536
    e = _db()["zb_step_kernel@65536"]
    src = e["source"]
    assert src.startswith("profiles/") and os.path.isdir(os.path.join(ROOT, src))
    traffic = (2 * _counter(src, "FETCH_SIZE") + _counter(src, "WRITE_SIZE")) * 1024
    assert traffic == pytest.approx(e["traffic_bytes"], rel=1e-4)
    assert _counter(src, "SQ_ACTIVE_INST_VALU") / _counter(src, "SQ_WAVE_CYCLES") == pytest.approx(e["issue_frac"], rel=1e-4)
    assert _counter(src, "SQ_INSTS_VALU") / _counter(src, "SQ_WAVES") == pytest.approx(e["valu_insts_per_wave"], rel=1e-4)
    gaps = open(os.path.join(ROOT, src, "kernel_gaps.txt")).read()
    assert f"mean {e['rocprof_mean_us']:.2f}" in gaps


def test_bench_reads_it():
    import bench
    traffic, src = bench.pmc_traffic(4096)
    assert traffic and src.startswith("profiles/")
    iss = bench.pmc_issue(4096)
    assert 0 < iss["frac"] < 1
    v = bench.valu_roofline(4096, 125e-6)
    assert v["unit"].startswith("TFLOP/s") and 0 < v["frac"] < 1 and 0 < v["issue_frac_device"] < 1
    assert bench.pmc_traffic(12345 * 4) == (None, None)  # no pass for that grid: null, never a guess


def test_roofline_file_travels_to_the_gpu_box():
    pats = [l.strip() for l in open(os.path.join(ROOT, ".gpurunignore")) if l.strip()]
    assert not any(p in ("roofline_pmc.json", "./roofline_pmc.json", "*.json") for p in pats), pats
