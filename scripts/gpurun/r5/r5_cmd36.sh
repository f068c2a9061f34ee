#!/bin/bash
# r5c36: round-batched select (select2_kernel), fused decide + conditional fallback (decide_fb_kernel) + lane-max sketch: compression GPU tests
# (incl. the firing fallback under load), pipeline timing fused / unfused, kernel timeline
set -u
D=gpurun_out/r5c36
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_kernels2_gpu.py > $D/t.log 2>&1
rc=$?; echo test_rc=$rc; grep -E "passed|failed|Error|error" $D/t.log | tail -8 | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench/kernels.py --only round2 > $D/fused.txt 2>&1 || exit 1
GKSGD_FB_FUSED=0 timeout -k 10 300 python3 bench/kernels.py --only round2 > $D/unfused.txt 2>&1 || exit 1
GKSGD_HANDOFF=lastblock timeout -k 10 300 python3 bench/kernels.py --only round2 > $D/fused_lb.txt 2>&1 || exit 1
GKSGD_SELECT_V2=0 timeout -k 10 300 python3 bench/kernels.py --only round2 > $D/sel1.txt 2>&1 || exit 1
head -3 $D/sel1.txt
head -3 $D/fused.txt; head -3 $D/unfused.txt; head -3 $D/fused_lb.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o run -- python3 bench/kernels.py --only round2 > $D/prof.log 2>&1 || exit 1
