#!/bin/bash
# r5c9: fp32 GEMMs on the fp32 MFMA vs bf16x6 products (gemm_kern.h X6): time + error vs fp64
set -u
D=gpurun_out/r5c9
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_f32_gpu.py -k "test_gemm_nt_f32 and 1000-64-64" > $D/t.log 2>&1
rc=$?; echo test_rc=$rc; tail -30 $D/t.log | cut -c1-400
timeout -k 10 400 python3 -u bench/x6_probe.py --quick --json-out $D/x6_probe.json > $D/x6_probe.log 2>&1
rc=$?; echo probe_rc=$rc; cat $D/x6_probe.log | cut -c1-600; exit $rc
