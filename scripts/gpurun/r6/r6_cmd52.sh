#!/bin/bash
# r6c52: final HEAD check on the rebuilt extension (TN negative-split quarter rounds): full GPU suite + smoke, default bench,
# and the reference batch eager (the trainer's default execution) gated side vs inline
set -u
D=gpurun_out/r6c52
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $D/gputests.log 2>&1
rc=$?; echo gputests_rc=$rc; tail -3 $D/gputests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $D/gputests.log | head -20; exit $rc; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1
rc=$?; echo smoke_rc=$rc; tail -1 $D/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --json-out $D/bench1.json > $D/bench1.log 2>&1
rc=$?; echo bench1_rc=$rc; [ $rc -eq 0 ] || { tail -20 $D/bench1.log; exit $rc; }
python3 -c "
import json;d=json.load(open('$D/bench1.json'));print({k:d[k] for k in d if k.endswith('value') or k.endswith('ms_per_step') or k.endswith('error')})"
