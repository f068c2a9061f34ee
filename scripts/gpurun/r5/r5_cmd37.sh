#!/bin/bash
# r5c37: counters of the compression pipeline's count / decide_fb / select kernels (25.6 M bucket)
set -u
D=gpurun_out/r5c37
mkdir -p $D
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-include-regex "select|count_kernel|decide_fb|stats_kernel" -d $D/p1 -o run --output-format csv -- python3 bench/kernels.py --only round2 > $D/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAIT_INST_ANY --kernel-include-regex "select|count_kernel|decide_fb|stats_kernel" -d $D/p2 -o run --output-format csv -- python3 bench/kernels.py --only round2 > $D/p2.log 2>&1 || exit 1
find $D -name "*.csv" | head
