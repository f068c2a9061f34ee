#!/bin/bash
# r4 call 24: Winograd grad-weight with raw dY in LDS (dM formed in registers): rawd / rawds (+ V writes
# spread) vs old (HEAD) on the bs512 shapes; Winograd GPU tests on the rebuilt extension; headline bench
set -u
D=gpurun_out/r4c24
mkdir -p $D
export TMPDIR=/tmp
for v in old rawd rawds old rawd rawds; do
  timeout -k 5 90 ./bench/pbin/wino_probe_$v 512 20 $v 0 2 >> $D/probe.jsonl 2> $D/probe_$v.err || { echo "probe $v failed"; exit 1; }
done
echo probes_ok
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_winograd_gpu.py tests/test_bn_lazy_gpu.py > $D/tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -3 $D/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 --no-bf16-phase --ref-batch 0 --json-out $D/head.json > $D/head.log 2>&1
rc=$?; echo head_rc=$rc; python3 -c "import json;d=json.load(open('$D/head.json'));print('head', d['value'], d['ms_per_step'])"
