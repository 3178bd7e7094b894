cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/icache && export TMPDIR=/tmp
A="--lane-change 10 --steps 1 --warmup 0 --cpu-sample 0 --host-runs 0"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_IFETCH SQ_INSTS_VALU SQ_WAIT_ANY -d gpurun_out/icache/t10_sq -o run --output-format csv -- python3 bench.py $A > gpurun_out/icache/t10_sq.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE -d gpurun_out/icache/t10_sqc -o run --output-format csv -- python3 bench.py $A > gpurun_out/icache/t10_sqc.log 2>&1 &&
A2="--lane-change 2 --steps 1 --warmup 0 --cpu-sample 0 --host-runs 0"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_IFETCH SQ_INSTS_VALU SQ_WAIT_ANY -d gpurun_out/icache/t2_sq -o run --output-format csv -- python3 bench.py $A2 > gpurun_out/icache/t2_sq.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE -d gpurun_out/icache/t2_sqc -o run --output-format csv -- python3 bench.py $A2 > gpurun_out/icache/t2_sqc.log 2>&1
