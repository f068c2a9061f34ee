#!/bin/bash
# compression kernels: GPU numerics tests + kernel bench + per-kernel profile
set -u
D=gpurun_out/cab
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_kernels2_gpu.py tests/test_graph_gpu.py > $D/tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -3 $D/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench/kernels.py --only compress,round2 --json-out $D/kernels.json > $D/kernels.log 2>&1
rc=$?; echo kernels_rc=$rc; cat $D/kernels.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o prof -- python3 bench/kernels.py --only round2 > $D/prof.log 2>&1
rc=$?; echo prof_rc=$rc; [ $rc -eq 0 ] || exit $rc
python3 scripts/rocpd_summary.py --steps 1 --top 40 $(find $D/prof -name '*.db' | head -1) $D/kernel_summary.txt > $D/sum.log 2>&1; echo sum_rc=$?
find $D/prof -name '*.db' -delete
cut -c1-150 $D/kernel_summary.txt | sed -n 8,30p
