#!/bin/bash
# r4 call 34: grad-weight side stream on by default for small batches (auto) -- same-box interleaved A/B at
# the reference batch 32 (auto vs GKSGD_WGRAD_STREAM=0), side-stream e2e test
set -u
D=gpurun_out/r4c34
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_e2e_gpu.py -k side_stream > $D/tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -1 $D/tests.log; [ $rc -eq 0 ] || exit $rc
B="python3 bench.py --batch-size 32 --steps 40 --warmup 10 --no-bf16-phase --ref-batch 0"
for v in auto off auto2 off2; do
  case $v in off*) export GKSGD_WGRAD_STREAM=0 ;; *) unset GKSGD_WGRAD_STREAM ;; esac
  timeout -k 10 300 $B --json-out $D/bs32_$v.json > $D/bs32_$v.log 2>&1
  rc=$?; echo ${v}_rc=$rc; python3 -c "import json;d=json.load(open('$D/bs32_$v.json'));print('$v', d['value'], d['ms_per_step'])"; [ $rc -eq 0 ] || exit $rc
done
