#!/bin/bash
# r4 call 33: Winograd grad-weight V rows with bit 5 set stored tile-swapped (conflict-free LDS writes):
# probe A/B (sw vs old) on the bs512 shapes, Winograd GPU tests
set -u
D=gpurun_out/r4c33
mkdir -p $D
export TMPDIR=/tmp
for v in old sw old sw; do
  timeout -k 5 90 ./variants/probe/wino_probe_$v 512 20 $v 0 2 >> $D/probe.jsonl 2> $D/probe_$v.err || { echo "probe $v failed"; exit 1; }
done
echo probes_ok
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_winograd_gpu.py > $D/tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -1 $D/tests.log
