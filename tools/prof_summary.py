"""Summarise a tools/gpu_profile.sh run into profiles/<round>/.

    python tools/prof_summary.py gpurun_out/prof_c3 [--dst profiles/r05] [--kernel ipm_solve_kernel]

The source folder holds bench.json (the bench line of the profiled command),
cmd.txt (that command), trace/ (rocprofv3 --kernel-trace --stats of the same
command) and pmc_*/ (one --pmc pass each).  The evidence key, configuration and
build hash come from the bench line's "evidence" record, so bench.py quotes the
summaries only for that configuration and that build of libmcpx.so.

Only dispatches of the full-size launch (largest grid of the kernel) are
averaged: the bench also launches small warm-up / host-API batches.  Writes
kernel_stats_<key>.csv (rocprofv3 --stats, verbatim), trace_<key>.json
(average duration of the full-size dispatches), pmc_<key>.json (per-dispatch
counters: FETCH_SIZE / WRITE_SIZE in KB, SQ_*) and bench_<key>.json.
"""

from __future__ import annotations

import argparse
import csv
import json
import os
import shutil
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def full_size_dispatches(rows, kern: str, grid_key: str):
    rows = [r for r in rows if kern in r["Kernel_Name"]]
    gmax = max(int(r[grid_key]) for r in rows)
    return gmax, [r for r in rows if int(r[grid_key]) == gmax]


def timed_window(cmd: str):
    """(warmup, steps) of the profiled bench command: its timed launches are the
    full-size dispatches [W, W + K) in start order (the host-API runs come after)."""
    import shlex
    import sys

    sys.path.insert(0, ROOT)
    import bench

    toks = shlex.split(cmd)
    a = bench.parse(toks[toks.index("bench.py") + 1:] if "bench.py" in toks else [])
    return a.warmup, a.steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("--dst", default=os.path.join(ROOT, "profiles", "r05"))
    ap.add_argument("--kernel", default="")
    a = ap.parse_args()
    bench = json.loads(open(os.path.join(a.src, "bench.json")).read().strip().splitlines()[-1])
    evid = bench["evidence"]
    key = evid["key"]
    kern = a.kernel or bench["roofline"]["kernel"]
    cmd = open(os.path.join(a.src, "cmd.txt")).read().strip() if os.path.exists(os.path.join(a.src, "cmd.txt")) else ""
    os.makedirs(a.dst, exist_ok=True)
    stamp = {"config": evid["config"], "lib_hash": evid["lib_hash"], "command": cmd}
    shutil.copy(os.path.join(a.src, "bench.json"), os.path.join(a.dst, f"bench_{key}.json"))
    tr = None
    if os.path.exists(os.path.join(a.src, "trace", "run_kernel_trace.csv")):
        shutil.copy(os.path.join(a.src, "trace", "run_kernel_stats.csv"), os.path.join(a.dst, f"kernel_stats_{key}.csv"))
        gmax, full = full_size_dispatches(list(csv.DictReader(open(os.path.join(a.src, "trace", "run_kernel_trace.csv")))),
                                          kern, "Grid_Size_X")
        dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
        if cmd:  # the bench's timed steps only (not its warm-up or host-API launches)
            W, K = timed_window(cmd)
            starts = sorted({int(r["Start_Timestamp"]) for r in full if r["Kernel_Name"] == max(
                {r["Kernel_Name"] for r in full}, key=lambda k: sum(dur(x) for x in full if x["Kernel_Name"] == k))})
            # each launch = one dispatch of every pass; window by the dominant pass's order
            t_lo, t_hi = starts[W], starts[min(W + K, len(starts)) - 1]
            nxt = starts[W + K] if W + K < len(starts) else float("inf")
            full = [r for r in full if t_lo <= int(r["Start_Timestamp"]) < nxt]
        # a launch may be several template instances (the two-pass SCHUR launch: fast pass +
        # deferred re-solve); the dominant one is summarised, the launch total beside it
        by_name = defaultdict(list)
        for r in full:
            by_name[r["Kernel_Name"]].append(dur(r))
        dom = max(by_name, key=lambda k: sum(by_name[k]))
        durs = by_name[dom]
        first = next(r for r in full if r["Kernel_Name"] == dom)
        tr = {"kernel": dom, "Grid_Size": gmax, "dispatches": len(durs),
              "avg_ms": sum(durs) / len(durs), "min_ms": min(durs), "max_ms": max(durs),
              "launch_avg_ms_all_passes": sum(sum(v) for v in by_name.values()) / len(durs),
              "passes": {k: {"dispatches": len(v), "avg_ms": sum(v) / len(v)} for k, v in by_name.items()},
              "VGPR_Count": first.get("VGPR_Count"), "Accum_VGPR_Count": first.get("Accum_VGPR_Count"),
              "SGPR_Count": first.get("SGPR_Count"), "LDS_Block_Size": first.get("LDS_Block_Size"),
              "scratch_bytes": first.get("Scratch_Size") or first.get("Private_Segment_Size"),
              "note": "rocprofv3 --kernel-trace --stats of `command`: the full-size dispatches of its timed steps", **stamp}
        json.dump(tr, open(os.path.join(a.dst, f"trace_{key}.json"), "w"), indent=1)
    pmc = {"kernel": tr["kernel"] if tr else kern}
    for sub in sorted(os.listdir(a.src)):
        f = os.path.join(a.src, sub, "run_counter_collection.csv")
        if not sub.startswith("pmc") or not os.path.exists(f):
            continue
        rows = list(csv.DictReader(open(f)))
        gmax, full = full_size_dispatches(rows, kern, "Grid_Size")
        if tr:
            full = [r for r in full if r["Kernel_Name"] == tr["kernel"]]
        pmc["Grid_Size"] = gmax
        agg = defaultdict(list)
        for r in full:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, v in agg.items():
            pmc[k] = sum(v) / len(v)
            pmc[k + "_dispatches"] = len(v)
    if len(pmc) > 2:
        pmc.update(stamp)
        pmc["note"] = ("rocprofv3 --pmc passes (one per counter group, each its own run of `command` with "
                       "--steps 2 --warmup 0 --cpu-sample 0 --host-runs 0) averaged over the full-size dispatches "
                       "of the dominant kernel; FETCH_SIZE/WRITE_SIZE in KB per dispatch; SQ_WAVE_CYCLES in "
                       "quad-cycles")
        json.dump(pmc, open(os.path.join(a.dst, f"pmc_{key}.json"), "w"), indent=1)
    print(json.dumps(tr), json.dumps(pmc), sep="\n")


if __name__ == "__main__":
    main()
