#!/bin/bash
# One GPU session on the box (run through gpurun), steps in order, the first failure ends it:
#
#   tools/gpu_session.sh <out-dir-name> STEP [STEP ...]
#
#   suite                 the whole -m gpu suite (the driver's round-end check)
#   suite=<f1,f2,...>     -m gpu on the given test files only
#   smoke                 __graft_entry__.smoke()
#   driver                the driver's bench command (bench.py --gpus 1 --steps 20 --warmup 5)
#   bench=<name>:<args>   one bench line, args comma-separated (bench=c4:--lane-change,2)
#   prof=<name>:<args>    tools/gpu_profile.sh: bench line + rocprofv3 trace + PMC passes
#   evid=<name>:<args>    tools/evidence.sh: prof, summaries, then the bench line quoting them
#   timeline=<args>       tools/timeline.py (residency timeline of a SCHUR launch), args comma-separated
#   probe=<name>          tools/parity_probe.py (C3, C2 shapes) on the variant tools/ablib/libmcpx_<name>.so
#   shard                 the per-GPU shards of the strong-scaling configs (C3 2/4/8, C5 512, C4 128)
#
# Outputs go to gpurun_out/<out-dir-name>/ (prof steps: gpurun_out/prof_<name>/).  Every GPU
# step has its own time limit; steps are chained so nothing runs after a failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/${1:?out-dir-name}
shift
mkdir -p "$O"
export TMPDIR=/tmp
T="--timeout 300 --timeout-method thread"
# the tree must be built here, not on the box: a missing module would compile silently for minutes
timeout -k 10 300 python tools/check_prebuilt.py || exit 2
for step in "$@"; do
  echo "[gpu_session] $step $(date +%T)"
  case "$step" in
    suite)
      timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu $T > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 3; }
      tail -2 "$O/pytest_gpu.log" ;;
    suite=*)
      files=${step#suite=}
      timeout -k 10 900 python -u -m pytest ${files//,/ } -x -v -m gpu $T > "$O/pytest_part.log" 2>&1 || { tail -30 "$O/pytest_part.log"; exit 3; }
      tail -2 "$O/pytest_part.log" ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { cat "$O/smoke.log"; exit 4; } ;;
    driver)
      timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench_driver.json" 2> "$O/bench_driver.err" || { tail -20 "$O/bench_driver.err"; exit 5; }
      cut -c1-400 "$O/bench_driver.json" ;;
    bench=*)
      spec=${step#bench=}; name=${spec%%:*}; args=${spec#*:}
      timeout -k 10 400 python bench.py ${args//,/ } > "$O/bench_$name.json" 2> "$O/bench_$name.err" || { tail -20 "$O/bench_$name.err"; exit 6; }
      cut -c1-300 "$O/bench_$name.json" ;;
    prof=*)
      spec=${step#prof=}; name=${spec%%:*}; args=${spec#*:}
      [ "$args" = "$spec" ] && args=""
      bash tools/gpu_profile.sh "$name" ${args//,/ } || exit 7 ;;
    evid=*)
      spec=${step#evid=}; name=${spec%%:*}; args=${spec#*:}
      [ "$args" = "$spec" ] && args=""
      bash tools/evidence.sh "$name" ${args//,/ } || exit 11 ;;
    timeline=*)
      args=${step#timeline=}
      timeout -k 10 300 python -u tools/timeline.py ${args//,/ } --out "$O" > "$O/timeline.log" 2>&1 || { tail -20 "$O/timeline.log"; exit 9; }
      cut -c1-600 "$O/timeline.log" ;;
    probe=*)
      lib=${step#probe=}
      for shape in "32 16 256" "16 8 256"; do
        MCPX_LIB_PATH=tools/ablib/libmcpx_$lib.so timeout -k 10 180 python tools/parity_probe.py $shape >> "$O/parity_probe.txt" 2>&1 || { tail -20 "$O/parity_probe.txt"; exit 10; }
      done
      tail -20 "$O/parity_probe.txt" ;;
    shard)
      for G in 32768 16384 8192; do
        timeout -k 10 300 python bench.py --gpus 1 --global-batch $G --steps 20 --warmup 5 --cpu-sample 0 --host-runs 0 > "$O/bench_g$G.json" 2> "$O/bench_g$G.err" || exit 8
      done
      timeout -k 10 300 python bench.py --sens --global-batch 512 --steps 20 --warmup 5 --cpu-sample 0 > "$O/bench_c5_g512.json" 2> "$O/bench_c5_g512.err" || exit 8
      timeout -k 10 300 python bench.py --lane-change 2 --global-batch 128 --steps 5 --warmup 1 --cpu-sample 0 > "$O/bench_c4_g128.json" 2> "$O/bench_c4_g128.err" || exit 8 ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
echo "[gpu_session] done $(date +%T)"
