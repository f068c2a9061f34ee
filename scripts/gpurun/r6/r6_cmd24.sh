#!/bin/bash
# r6c24: bf16x6 Winograd (wino_x6.hip): GPU tests vs fp64 / the fp32-MFMA Winograd, then the
# per-shape probe at ResNet-50 bs512 against the fp32-MFMA Winograd
set -u
D=gpurun_out/r6c24
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_wino_x6_gpu.py -x -q --timeout 120 --timeout-method thread > $D/tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -3 $D/tests.log; [ $rc -eq 0 ] || { grep -E "Error|error|assert|Fail" $D/tests.log | head -30; exit $rc; }
timeout -k 10 300 python3 bench/wx6_probe.py --batch 512 > $D/probe.log 2>&1
rc=$?; echo probe_rc=$rc; cat $D/probe.log | head -8
