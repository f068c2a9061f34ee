#!/bin/bash
# r6c50: full GPU suite with the side stream OFF (GKSGD_WGRAD_STREAM=0, the inline path users can select)
set -u
D=gpurun_out/r6c50
mkdir -p $D
export TMPDIR=/tmp
GKSGD_WGRAD_STREAM=0 timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $D/gputests_inline.log 2>&1
rc=$?; echo gputests_inline_rc=$rc; tail -3 $D/gputests_inline.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $D/gputests_inline.log | head -20; exit $rc; }
