"""Residency timeline of a C3/C2 SCHUR launch (tools/timeline.hip, MCPX_STAMPS=2).

Writes the bench's own θ (mcp_amd.qp_benchmark.generate_global_slice, seed 1) for a batch,
runs tools/timeline on the GPU and reports where the launch's time goes: pass 1 / pass 2,
the dispatch rounds (when waves start), the completion curve, the number of resident waves
over time, per-SIMD finish times, and which waves end last (their Newton counts and start
times).  Diagnostic: VERDICT r03 "Next round" #2 (the 8,192 shard's lost 21 %).

    python tools/timeline.py [--n 32 --m 16] --batch 8192 65536 [--out gpurun_out/timeline]
"""

from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def hw_fields(hw: np.ndarray, xcc: np.ndarray) -> dict:
    """gfx9 HW_ID: wave 3:0, simd 5:4, cu 11:8, sh 12, se 15:13."""
    return {"wave": hw & 0xF, "simd": (hw >> 4) & 3, "cu": (hw >> 8) & 0xF, "sh": (hw >> 12) & 1,
            "se": (hw >> 13) & 7, "xcc": xcc & 0xF}


def analyse(path: str, B: int) -> dict:
    raw = open(path, "rb").read()
    ms = np.frombuffer(raw[:16], dtype=np.float64)
    rec = np.frombuffer(raw[16:], dtype=np.dtype([("u", "<u8", 5), ("newton", "<i4"), ("status", "<i4")]), count=B)
    start, end = rec["u"][:, 0].astype(np.int64), rec["u"][:, 1].astype(np.int64)
    hw, xcc, pas = rec["u"][:, 2], rec["u"][:, 3], rec["u"][:, 4]
    ok = end > 0
    p1 = ok & (pas == 1)
    t0 = start[ok].min()
    us = lambda t: (t - t0) * 0.01  # 100 MHz → µs
    s1, e1 = us(start[p1]), us(end[p1])
    dur = e1 - s1
    nw = rec["newton"][p1]
    T = e1.max()
    f = hw_fields(hw[p1], xcc[p1])
    simd_key = (((f["xcc"] * 8 + f["se"]) * 2 + f["sh"]) * 16 + f["cu"]) * 4 + f["simd"]
    keys, inv = np.unique(simd_key, return_inverse=True)
    simd_end = np.zeros(len(keys))
    np.maximum.at(simd_end, inv, e1)
    simd_cnt = np.bincount(inv)
    grid = np.linspace(0, T, 401)
    conc = np.array([np.count_nonzero((s1 <= t) & (e1 > t)) for t in grid])
    cmax = conc.max()
    order = np.argsort(e1)
    last = order[-max(1, B // 100):]
    per_step = dur / np.maximum(nw, 1)
    # waves started "at once" (first residency round): start within 5 µs of the first
    first_round = s1 <= s1.min() + 5.0
    out = {
        "B": B,
        "pass1_ms": float(ms[0]), "pass2_ms": float(ms[1]),
        "deferred": int(np.count_nonzero(ok & (pas == 2))),
        "stamp_span_us": float(T),
        "first_round_waves": int(first_round.sum()),
        "resident_max": int(cmax),
        "slots_busy_frac": float(np.trapezoid(conc, grid) / (cmax * T)),
        "complete_us": {q: float(np.quantile(e1, q / 100)) for q in (10, 50, 90, 99, 100)},
        "start_us": {q: float(np.quantile(s1, q / 100)) for q in (10, 50, 90, 99, 100)},
        "simds": int(len(keys)),
        "waves_per_simd": {"min": int(simd_cnt.min()), "mean": float(simd_cnt.mean()), "max": int(simd_cnt.max())},
        "simd_end_us": {q: float(np.quantile(simd_end, q / 100)) for q in (0, 10, 50, 90, 100)},
        "newton": {"mean": float(nw.mean()), "max": int(nw.max()), "p99": float(np.quantile(nw, 0.99))},
        "wave_us": {"mean": float(dur.mean()), "max": float(dur.max())},
        "us_per_step": {"mean": float(per_step.mean()), "first_round": float(per_step[first_round].mean()),
                        "last_1pct": float(per_step[last].mean())},
        "last_1pct": {"newton_mean": float(nw[last].mean()), "start_us_mean": float(s1[last].mean()),
                      "dur_us_mean": float(dur[last].mean())},
        "concurrency": [int(c) for c in conc[::20]],
    }
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=32)
    ap.add_argument("--m", type=int, default=16)
    ap.add_argument("--batch", type=int, nargs="+", default=[8192, 65536])
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "timeline"))
    a = ap.parse_args(argv)
    from mcp_amd.qp_benchmark import generate_global_slice

    os.makedirs(a.out, exist_ok=True)
    exe = os.path.join(ROOT, "tools", "timeline")
    res = []
    for B in a.batch:
        th = generate_global_slice(1, a.n, a.m, 0.0, 0, B)
        tp = os.path.join(a.out, f"theta_{a.n}_{a.m}_{B}.bin")
        with open(tp, "wb") as f:
            f.write(np.array([a.n, a.m, B], dtype=np.int32).tobytes())
            f.write(np.ascontiguousarray(th, dtype=np.float64).tobytes())
        op = os.path.join(a.out, f"tl_{a.n}_{a.m}_{B}.bin")
        subprocess.run([exe, tp, op, str(a.reps)], check=True, timeout=120)
        os.remove(tp)
        r = analyse(op, B)
        r.update(n=a.n, m=a.m)
        print(json.dumps(r), flush=True)
        res.append(r)
    with open(os.path.join(a.out, f"timeline_{a.n}_{a.m}.jsonl"), "w") as f:
        for r in res:
            f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
