#!/bin/bash
# r5c34: two-level arrival counters for the in-grid hand-offs: compression GPU tests,
# pipeline timing in both hand-off modes, kernel trace of the 25.6 M gaussian pipeline
set -u
D=gpurun_out/r5c34
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py > $D/t.log 2>&1
rc=$?; echo test_rc=$rc; tail -5 $D/t.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench/kernels.py --only round2 > $D/launch.txt 2>&1 || exit 1
GKSGD_HANDOFF=lastblock timeout -k 10 300 python3 bench/kernels.py --only round2 > $D/lastblock.txt 2>&1 || exit 1
head -3 $D/launch.txt; head -3 $D/lastblock.txt
GKSGD_HANDOFF=lastblock timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof_lb -o run -- python3 bench/kernels.py --only round2 > $D/prof_lb.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof_l -o run -- python3 bench/kernels.py --only round2 > $D/prof_l.log 2>&1 || exit 1
find $D -name "*kernel_stats.csv" | head
