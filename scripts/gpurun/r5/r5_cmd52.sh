#!/bin/bash
# r5c52: final HEAD check -- full GPU suite + smoke + the driver bench command (twice) + BERT + kernel trace of the headline
set -u
D=gpurun_out/r5c52
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 1100 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/gputests.log 2>&1
rc=$?; echo gputests_rc=$rc; tail -3 $D/gputests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1
rc=$?; echo smoke_rc=$rc; tail -1 $D/smoke.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --json-out $D/bench$i.json > $D/bench$i.log 2>&1
  rc=$?; echo bench${i}_rc=$rc; [ $rc -eq 0 ] || { tail -20 $D/bench$i.log; exit $rc; }
  python3 -c "
import json;d=json.load(open('$D/bench$i.json'));print({k:d[k] for k in d if k.endswith('value') or k.endswith('ms_per_step')})"
done
timeout -k 10 600 python3 bench.py --model bert --steps 10 --warmup 3 --no-bf16-phase --json-out $D/bert.json > $D/bert.log 2>&1
rc=$?; echo bert_rc=$rc; [ $rc -eq 0 ] || exit $rc
python3 -c "
import json;d=json.load(open('$D/bert.json'));print({k:d[k] for k in d if k.endswith('value') or k.endswith('ms_per_step')})"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $D/prof -o run -- python3 bench.py --gpus 1 --steps 10 --warmup 5 --no-native-phase --no-bf16-phase --ref-batch 0 --json-out $D/prof_bench.json > $D/prof.log 2>&1
rc=$?; echo prof_rc=$rc
