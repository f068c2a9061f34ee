#!/bin/bash
# r6c54: final-tree check of the side-stream GPU tests (bias fork off by default) + smoke
set -u
D=gpurun_out/r6c54
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_e2e_gpu.py tests/test_conv1x1_gpu.py -x -q --timeout 300 --timeout-method thread > $D/tests.log 2>&1
rc=$?; tail -2 $D/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $D/tests.log | head; exit $rc; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1
rc=$?; echo smoke_rc=$rc; tail -1 $D/smoke.log; [ $rc -eq 0 ] || exit $rc
