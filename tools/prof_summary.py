"""Summarise a tools/gpu_profile.sh run (gpurun_out/prof_<tag>/) into profiles/<tag>/.

    python tools/prof_summary.py r01 [--kernel ipm_solve_kernel] [--name c3_schur]

Only dispatches of the full-size launch (largest Grid_Size of the kernel) are
averaged: the bench also launches small warm-up / host-API batches.  Writes
kernel_stats_<name>.csv (rocprofv3 --stats, verbatim), trace_<name>.json
(average duration of the full-size dispatches from the kernel trace) and
pmc_<name>.json (per-dispatch FETCH_SIZE / WRITE_SIZE in KB and SQ_* counters)
and copies bench.json → bench_<name>.json.
"""

from __future__ import annotations

import csv
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    tag = sys.argv[1]
    kern = sys.argv[sys.argv.index("--kernel") + 1] if "--kernel" in sys.argv else "ipm_solve_kernel"
    name = sys.argv[sys.argv.index("--name") + 1] if "--name" in sys.argv else "c3_schur"
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    dst = os.path.join(ROOT, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, f"kernel_stats_{name}.csv"))
    if os.path.exists(os.path.join(src, "bench.json")):
        shutil.copy(os.path.join(src, "bench.json"), os.path.join(dst, f"bench_{name}.json"))
    rows = [r for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_trace.csv"))) if kern in r["Kernel_Name"]]
    gmax = max(int(r["Grid_Size_X"]) for r in rows)
    full = [r for r in rows if int(r["Grid_Size_X"]) == gmax]
    dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
    # a launch may be several template instances of the kernel (the two-pass SCHUR
    # launch: fast pass + deferred re-solve); the dominant one is summarised alone
    by_name = defaultdict(list)
    for r in full:
        by_name[r["Kernel_Name"]].append(dur(r))
    dom = max(by_name, key=lambda k: sum(by_name[k]))
    full = [r for r in full if r["Kernel_Name"] == dom]
    durs = by_name[dom]
    tr = {"kernel": dom, "Grid_Size": gmax, "dispatches": len(durs),
          "avg_ms": sum(durs) / len(durs), "min_ms": min(durs), "max_ms": max(durs),
          "launch_avg_ms_all_passes": sum(sum(v) for v in by_name.values()) / len(durs),
          "passes": {k: {"dispatches": len(v), "avg_ms": sum(v) / len(v)} for k, v in by_name.items()},
          "VGPR_Count": full[0]["VGPR_Count"], "SGPR_Count": full[0]["SGPR_Count"],
          "LDS_Block_Size": full[0]["LDS_Block_Size"],
          "note": "rocprofv3 --kernel-trace of `python3 bench.py --cpu-sample 0`, full-size dispatches only"}
    json.dump(tr, open(os.path.join(dst, f"trace_{name}.json"), "w"), indent=1)
    pmc = {"kernel": tr["kernel"], "Grid_Size": gmax}
    for sub in sorted(os.listdir(src)):
        f = os.path.join(src, sub, "run_counter_collection.csv")
        if not sub.startswith("pmc") or not os.path.exists(f):
            continue
        agg = defaultdict(list)
        for r in csv.DictReader(open(f)):
            if r["Kernel_Name"] == dom and int(r["Grid_Size"]) == gmax:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, v in agg.items():
            pmc[k] = sum(v) / len(v)
            pmc[k + "_dispatches"] = len(v)
    pmc["note"] = ("rocprofv3 --pmc passes (one per counter group) of `python3 bench.py --steps 2 --warmup 0 "
                   "--cpu-sample 0` on 1x MI355X, averaged over the full-size dispatches; FETCH_SIZE/WRITE_SIZE "
                   "in KB per dispatch; SQ_WAVE_CYCLES in quad-cycles")
    json.dump(pmc, open(os.path.join(dst, f"pmc_{name}.json"), "w"), indent=1)
    print(json.dumps(tr), json.dumps(pmc), sep="\n")


if __name__ == "__main__":
    main()
