"""bench.py helpers (CPU): FLOP accounting of SURVEY.md §8(d) and the committed
PMC evidence the default bench line quotes as `roofline.traffic`."""

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_lu_flops_matches_survey():
    # 2N³/3 + 2N² per Newton step; N=32: 23,893; N=64: 182,955; N=6: 216
    assert round(bench.lu_flops(32)) == 23893
    assert round(bench.lu_flops(64)) == 182955
    assert round(bench.lu_flops(6)) == 216


def test_solve_dims():
    assert bench.solve_dim(32, 16, "dense") == 64
    assert bench.solve_dim(32, 16, "reduced") == 48
    assert bench.solve_dim(32, 16, "schur") == 32


def test_pmc_summary_matches_default_config():
    """The default bench line (C3, schur, 65,536 instances) must find its PMC summary;
    other configurations must not borrow it."""
    traffic, src = bench.pmc_traffic(32, 16, 65536, "schur")
    d = json.load(open(os.path.join(ROOT, src)))
    assert traffic == pytest.approx((d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024.0)
    assert traffic > 0
    assert bench.pmc_traffic(32, 16, 4096, "schur") == (None, None)
    assert bench.pmc_traffic(16, 8, 65536, "schur") == (None, None)
    assert bench.pmc_traffic(32, 16, 65536, "dense") == (None, None)


def test_trace_summary_agrees_with_bench_events():
    """profiles/r01: rocprofv3's average fast-pass duration and the bench's HIP-event
    launch time (both passes) of the same command agree within 10 %."""
    tr = json.load(open(os.path.join(ROOT, "profiles", "r01", "trace_c3_schur.json")))
    b = json.load(open(os.path.join(ROOT, "profiles", "r01", "bench_c3_schur.json")))
    assert tr["Grid_Size"] == 64 * b["config"]["batch_per_gpu"]
    assert tr["avg_ms"] == pytest.approx(b["roofline"]["kernel_ms"], rel=0.10)


def test_cli_has_every_baseline_mode():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--help"], capture_output=True,
                         text=True, check=True).stdout
    for flag in ("--gpus", "--steps", "--warmup", "--sens", "--lane-change", "--gather", "--cpu-sample"):
        assert flag in out


@pytest.mark.gpu
def test_gpu_bench_lane_change_line():
    """The C4 bench line on a small batch: one JSON line, statuses equal to the C oracle's."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--lane-change", "2", "--batch", "64",
                        "--steps", "1", "--warmup", "1", "--cpu-sample", "64"], capture_output=True, text=True,
                       timeout=110, check=True)
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["config"]["kkt_dim"] == 140 and d["n_gpus"] == 1
    assert d["value"] > 0 and 0 < d["roofline"]["frac"] < 1
    assert d["cpu_baseline"]["status_match"] is True
