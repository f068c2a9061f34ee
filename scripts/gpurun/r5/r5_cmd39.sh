#!/bin/bash
# r5c39: fused decide + conditional fallback (final form): compression GPU tests, pipeline timing
# fused / unfused in one call, kernel timeline
set -u
D=gpurun_out/r5c39
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_kernels2_gpu.py > $D/t.log 2>&1
rc=$?; echo test_rc=$rc; grep -E "passed|failed|Error|error" $D/t.log | tail -4 | cut -c1-300; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 300 python3 bench/kernels.py --only round2 > $D/fused$i.txt 2>&1 || exit 1
GKSGD_FB_FUSED=0 timeout -k 10 300 python3 bench/kernels.py --only round2 > $D/unfused$i.txt 2>&1 || exit 1
head -2 $D/fused$i.txt | tail -1; head -2 $D/unfused$i.txt | tail -1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o run -- python3 bench/kernels.py --only round2 > $D/prof.log 2>&1 || exit 1
GKSGD_FB_FUSED=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof0 -o run -- python3 bench/kernels.py --only round2 > $D/prof0.log 2>&1 || exit 1
