"""bench.py helpers (CPU): FLOP accounting of SURVEY.md §8(d), the workload plan
(strong / weak scaling), the rank launcher, the summary statistics of
benchmark/path.jl and the rule that a bench line quotes rocprofv3 evidence only
when it was taken on exactly its configuration and build."""

import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_lu_flops_matches_survey():
    # 2N³/3 + 2N² per Newton step; N=32: 23,893; N=64: 182,955; N=6: 216
    assert round(bench.lu_flops(32)) == 23893
    assert round(bench.lu_flops(64)) == 182955
    assert round(bench.lu_flops(6)) == 216


def test_solve_dims_and_executed_flops():
    assert bench.solve_dim(32, 16, "dense") == 64
    assert bench.solve_dim(32, 16, "reduced") == 48
    assert bench.solve_dim(32, 16, "schur") == 32
    resid = 2 * (32 * 48 + 16 * 32)
    # Gauss-Jordan of the SPD S: every other row at every step, (n-1)·n·(n+1) = 32,736 at n = 32
    assert bench.executed_flops(32, 16, "schur") == resid + 2 * 32 * 32 * 16 + 4 * 32 * 16 + 31 * 32 * 33
    assert bench.executed_flops(32, 16, "dense") == resid + bench.lu_flops(64)
    # m = 15: residual −2·(32 + 32), rr/δy −4·32, the Schur GEMM's K stays padded to 16
    assert bench.executed_flops(32, 16, "schur") - bench.executed_flops(32, 15, "schur") == 256



def test_roofline_bound_from_pmc():
    """bound = the unit the PMC counters show busiest (≥ 0.3), else latency; without PMC
    evidence of the build, the stated fallback, marked as assumed."""
    assert bench.roofline_bound({}, 5.0, "valu")[0] == "valu"
    assert "assumed" in bench.roofline_bound({}, 5.0, "valu")[1]["source"]
    act = 1e7 * bench.XCDS  # 10 M cycles per XCD
    sim = 1e7 * bench.SIMDS
    valu = {"pmc": {"GRBM_GUI_ACTIVE": act, "SQ_INSTS_VALU": 0.8 * sim / 4, "SQ_VALU_MFMA_BUSY_CYCLES": 0.1 * sim,
                    "FETCH_SIZE": 1e6, "WRITE_SIZE": 0.0, "_source": "x"}}
    assert bench.roofline_bound(valu, 5.0, "hbm")[0] == "valu"
    hbm = {"pmc": dict(valu["pmc"], SQ_INSTS_VALU=0.1 * sim / 4, FETCH_SIZE=5.0 * 8e12 / 1024 * 5e-3)}
    b, e = bench.roofline_bound(hbm, 5.0, "valu")
    assert b == "hbm" and e["utilisation"]["hbm"] == pytest.approx(5.0)
    lat = {"pmc": dict(valu["pmc"], SQ_INSTS_VALU=0.05 * sim / 4)}
    assert bench.roofline_bound(lat, 5.0, "valu")[0] == "latency"


def test_parity_report_counts_instances():
    got = {"x": np.array([[1.0, np.nan], [2.0, 3.0], [4.0, 5.0]]), "status": np.array([0, 1, 0], np.int32)}
    ref = {"x": np.array([[1.0, np.nan], [2.0, 3.5], [4.0, 5.0]]), "status": np.array([0, 1, 1], np.int32)}
    r = bench.parity_report(got, ref, ("x", "status"), 3, "t")
    assert r["mismatches"] == {"x": 1, "status": 1} and not r["pass"] and r["bit_exact_fields"] == []
    r = bench.parity_report(got, got, ("x", "status"), 3, "t")
    assert r["pass"] and r["bit_exact_fields"] == ["x", "status"]


def test_plan_strong_scaling_is_the_baseline_config():
    """BASELINE C3: global 65,536 sharded over the GPUs (8,192 per GPU at N=8); C5: 4,096."""
    a = bench.parse([])
    assert bench.plan(a, 1, 0) == dict(start=0, count=65536, cap=65536, global_batch=65536, scaling="strong")
    shards = [bench.plan(a, 8, r) for r in range(8)]
    assert all(p["count"] == 8192 and p["cap"] == 8192 for p in shards)
    assert [p["start"] for p in shards] == [8192 * r for r in range(8)]
    assert bench.plan(bench.parse(["--sens"]), 8, 7)["count"] == 512
    assert bench.plan(bench.parse(["--lane-change", "2"]), 1, 0)["count"] == 1024
    ragged = [bench.plan(bench.parse(["--global-batch", "10"]), 4, r) for r in range(4)]
    assert [p["count"] for p in ragged] == [3, 3, 2, 2] and all(p["cap"] == 3 for p in ragged)
    weak = bench.plan(bench.parse(["--batch", "1000"]), 4, 3)
    assert weak == dict(start=3000, count=1000, cap=1000, global_batch=4000, scaling="weak")


def test_launcher_refuses_missing_gpus(capsys):
    assert bench.launch_ranks(8, "unused.py", [], have_devices=1) == 2
    assert "only 1 GPU" in capsys.readouterr().err


@pytest.mark.slow
def test_launch_ranks_spawns_world2(tmp_path):
    """The `--gpus N` spawn path with world size 2 on CPU: torch.distributed.run as a
    child, two ranks join a gloo group at 127.0.0.1 and shard the global batch."""
    out = tmp_path / "ranks.json"
    rc = bench.launch_ranks(2, os.path.join(ROOT, "tests", "helpers", "rank_probe.py"), [str(out), "65537"],
                            have_devices=2)
    assert rc == 0
    d = json.load(open(out))
    assert d["world"] == 2
    assert d["shards"] == [[0, 0, 32769, 32769], [1, 32769, 32768, 32769]]


def test_summary_statistics_format():
    """benchmark/path.jl:101-126: success_rate, μ, σ of the runtimes."""
    s = bench.summary_statistics([0.010, 0.012, 0.011], 1000, 0.95)["ip"]
    assert s["success_rate"] == 0.95
    assert s["μ"] == pytest.approx(1.1e-5)
    assert s["σ"] == pytest.approx(np.std([1e-5, 1.2e-5, 1.1e-5], ddof=1))


def test_evidence_only_for_its_config_and_build(tmp_path, monkeypatch):
    from mcp_amd import build as b

    monkeypatch.setattr(bench, "PROFILE_DIR", str(tmp_path))
    monkeypatch.setattr(b, "built_hash", lambda: "abc")
    cfg = {"mode": "c3", "n": 32, "m": 16, "batch_per_gpu": 65536, "linear_solver": "schur", "sparsity": 0.0}
    json.dump({"config": cfg, "lib_hash": "abc", "FETCH_SIZE": 1000.0, "WRITE_SIZE": 24.0},
              open(tmp_path / "pmc_x.json", "w"))
    json.dump({"config": cfg, "lib_hash": "abc", "avg_ms": 6.0, "launch_avg_ms_all_passes": 6.01},
              open(tmp_path / "trace_x.json", "w"))
    ev = bench.evidence("x", cfg)
    assert set(ev) == {"pmc", "trace"}
    assert bench.pmc_traffic(ev)[0] == 1024.0 * 1024
    r = bench.roofline(6.01, 78.6e9 * 6.01 * 0.5, 1e9, 1e9, ev, "k", ("valu", {}), "")
    assert r["frac_trace"] == pytest.approx(0.5) and r["frac"] == pytest.approx(0.5)
    assert bench.evidence("x", dict(cfg, batch_per_gpu=8192)) == {}  # another configuration
    monkeypatch.setattr(b, "built_hash", lambda: "other")
    assert bench.evidence("x", cfg) == {}  # another build of libmcpx.so


def test_roofline_frac_never_exceeds_peak():
    """A dense §8(d) count above the FP64 peak is not a roofline for the kernel:
    `frac` falls back to the structural count (the elimination the kernel performs) and the dense
    figure is flagged; a structural count above the peak too makes `frac` null with an error."""
    import bench

    peak_flops_ms = bench.FP64_PEAK_TFLOPS * 1e12 * 1e-3  # FLOPs in 1 ms at peak
    r = bench.roofline(1.0, 0.5 * peak_flops_ms, 0.2 * peak_flops_ms, 1e9, {}, "k", ("latency", {}), "")
    assert r["frac"] == pytest.approx(0.5) and "dense_count_exceeds_peak" not in r
    r = bench.roofline(1.0, 1.02 * peak_flops_ms, 0.0015 * peak_flops_ms, 1e9, {}, "k", ("latency", {}), "")
    assert r["frac"] == pytest.approx(0.0015) and r["dense_count_exceeds_peak"]
    assert r["frac_dense_kkt"] == pytest.approx(1.02) and r["frac_basis"].startswith("structural")
    r = bench.roofline(1.0, 2.0 * peak_flops_ms, 1.5 * peak_flops_ms, 1e9, {}, "k", ("latency", {}), "")
    assert r["frac"] is None and "frac_error" in r
    r = bench.roofline(1.0, 0.99 * peak_flops_ms, 0.002 * peak_flops_ms, 1e9, {}, "k", ("latency", {}), "",
                       structural=True)  # a generated module's line: the structural basis always
    assert r["frac"] == pytest.approx(0.002) and not r["dense_count_exceeds_peak"]


def test_committed_evidence_is_self_consistent():
    """Every committed profiles/r0x trace/PMC summary names its configuration and
    build, and a bench line committed beside it quotes the same kernel time within 5 % (the
    trace is a separate, profiled run: profiled clocks sit 2-5 % below un-profiled ones,
    MI355X_MICROARCH.md, and C5's launch is 0.38 ms)."""
    dirs = [os.path.join(ROOT, "profiles", r) for r in ("r02", "r03", "r06")]
    files = [(d, f) for d in dirs if os.path.isdir(d) for f in sorted(os.listdir(d))]
    if not files:
        pytest.skip("no profiles yet")
    for d, f in files:
        if f.startswith(("trace_", "pmc_")) and f.endswith(".json"):
            j = json.load(open(os.path.join(d, f)))
            assert "config" in j and "lib_hash" in j, f
        if f.startswith("bench_") and f.endswith(".json"):
            b = json.load(open(os.path.join(d, f)))
            rl = b["roofline"]
            if "frac_trace" in rl:
                assert rl["frac_trace"] == pytest.approx(rl["frac"], rel=0.05), f


def test_cli_has_every_baseline_mode():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--help"], capture_output=True,
                         text=True, check=True).stdout
    for flag in ("--gpus", "--steps", "--warmup", "--sens", "--lane-change", "--gather", "--cpu-sample",
                 "--global-batch", "--batch", "--host-runs"):
        assert flag in out


@pytest.mark.gpu
def test_gpu_bench_lane_change_line():
    """The C4 bench line on a small batch: one JSON line, statuses equal to the C oracle's."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--lane-change", "2", "--global-batch",
                        "64", "--steps", "1", "--warmup", "1", "--cpu-sample", "64"], capture_output=True,
                       text=True, timeout=110, check=True)
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["config"]["kkt_dim"] == 140 and d["n_gpus"] == 1
    assert d["value"] > 0 and 0 < d["roofline"]["frac"] < 1
    assert d["parity"]["pass"] is True and d["parity"]["instances"] == 64


@pytest.mark.gpu
def test_gpu_bench_c3_small_line():
    """The C3 line on a small global batch, with the host-API median and the CPU legs."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--global-batch", "2048", "--steps", "2",
                        "--warmup", "1", "--cpu-sample", "256", "--host-runs", "2"], capture_output=True,
                       text=True, timeout=110, check=True)
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["scaling"] == "strong" and d["config"]["global_batch"] == 2048
    assert d["success_rate"] == 1.0 and d["host_api"]["median_solves_per_s"] > 0
    assert d["cpu_baseline"]["cores"] == d["cpu_baseline"]["nproc"]
    assert d["summary_statistics"]["ip"]["success_rate"] == 1.0
    assert d["parity"]["pass"] is True and d["parity"]["instances"] == 256
    assert d["parity_fixtures"]["pass"] is True and d["parity_fixtures"]["files"] >= 10
