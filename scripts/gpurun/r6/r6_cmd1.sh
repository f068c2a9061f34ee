#!/bin/bash
# r6c1: new end-to-end precision / momentum-correction GPU tests, the full GPU
# suite under the bf16x6 library default, then the driver bench command with
# the new BASELINE-config model phases (vgg16 / lstm / bert)
set -u
D=gpurun_out/r6c1
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_precision_e2e_gpu.py -x -v --timeout 300 --timeout-method thread > $D/e2e.log 2>&1
rc=$?; echo e2e_rc=$rc; tail -5 $D/e2e.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --json-out $D/bench1.json > $D/bench1.log 2>&1
rc=$?; echo bench1_rc=$rc; [ $rc -eq 0 ] || { tail -20 $D/bench1.log; exit $rc; }
python3 -c "
import json;d=json.load(open('$D/bench1.json'));print({k:d[k] for k in d if k.endswith('value') or k.endswith('ms_per_step') or k.endswith('error') or k.endswith('over_k')})"
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/gputests.log 2>&1
rc=$?; echo gputests_rc=$rc; tail -3 $D/gputests.log; [ $rc -eq 0 ] || exit $rc
