#!/bin/bash
# r5c35: lane-max sketch (select reads only lanes that can hold a selected key): compression GPU tests,
# pipeline timing with / without the sketch, kernel timeline of the 25.6 M gaussian pipeline
set -u
D=gpurun_out/r5c35
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_kernels2_gpu.py > $D/t.log 2>&1
rc=$?; echo test_rc=$rc; tail -5 $D/t.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench/kernels.py --only round2 > $D/sketch.txt 2>&1 || exit 1
GKSGD_SELECT_SKETCH=0 timeout -k 10 300 python3 bench/kernels.py --only round2 > $D/nosketch.txt 2>&1 || exit 1
head -4 $D/sketch.txt; head -4 $D/nosketch.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o run -- python3 bench/kernels.py --only round2 > $D/prof.log 2>&1 || exit 1
