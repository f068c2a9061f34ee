#!/bin/bash
# r5c6: full GPU suite + smoke + the driver's bench command on the current tree
set -u
D=gpurun_out/r5c6
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest.log 2>&1
rc=$?; echo pytest_rc=$rc; tail -5 $D/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1
rc=$?; echo smoke_rc=$rc; tail -2 $D/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --json-out $D/bench.json > $D/bench.log 2>&1
rc=$?; echo bench_rc=$rc; python3 -c "
import json;d=json.load(open('$D/bench.json'));print({k:d[k] for k in d if k.endswith('value') or k.endswith('ms_per_step')})"
