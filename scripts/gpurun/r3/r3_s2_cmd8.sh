#!/bin/bash
# fp32 / bf16 step profiles (summarised on the box, databases dropped), GEMM PMC counters
set -u
D=gpurun_out/s2j
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/prof_fp32 -o run -- python3 bench.py --steps 10 --warmup 3 --no-bf16-phase > $D/prof_fp32.log 2>&1
echo prof_rc=$?
python3 scripts/rocpd_summary.py /tmp/prof_fp32/run_results.db $D/fp32_stats.csv --steps 10 --marker reduce_records_kernel --top 60 > /dev/null
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/prof_bf16 -o run -- python3 bench.py --amp bf16 --steps 10 --warmup 3 > $D/prof_bf16.log 2>&1
echo prof16_rc=$?
python3 scripts/rocpd_summary.py /tmp/prof_bf16/run_results.db $D/bf16_stats.csv --steps 10 --marker reduce_records_kernel --top 60 > /dev/null
CTR_D=$D bash scripts/gpurun/r3/r3_counters.sh > $D/ctr.log 2>&1
echo ctr_rc=$?
find $D -name "*.db" -delete
du -sh $D
