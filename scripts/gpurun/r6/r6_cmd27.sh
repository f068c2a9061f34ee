#!/bin/bash
# r6c27: HEAD check (container restore) after the deferred shortcut BN and the x6 Winograd (opt-in): full GPU suite +
# smoke, the driver's default bench, fp32 / bf16 headline kernel profiles
set -u
D=gpurun_out/r6c27
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $D/gputests.log 2>&1
rc=$?; echo gputests_rc=$rc; tail -3 $D/gputests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $D/gputests.log | head -20; exit $rc; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1
rc=$?; echo smoke_rc=$rc; tail -1 $D/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --json-out $D/bench1.json > $D/bench1.log 2>&1
rc=$?; echo bench1_rc=$rc; [ $rc -eq 0 ] || { tail -20 $D/bench1.log; exit $rc; }
python3 -c "
import json;d=json.load(open('$D/bench1.json'));print({k:d[k] for k in d if k.endswith('value') or k.endswith('ms_per_step') or k.endswith('error') or k.endswith('ratio')})"
for spec in "fp32 none" "bf16 bf16"; do
  set -- $spec; tag=$1; amp=$2
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof_$tag -o run -- python3 bench.py --gpus 1 --steps 10 --warmup 5 --amp $amp --model-phases none --no-native-phase --no-bf16-phase --ref-batch 0 --json-out $D/$tag.json > $D/prof_$tag.log 2>&1
  rc=$?; echo prof_${tag}_rc=$rc; [ $rc -eq 0 ] || { tail -20 $D/prof_$tag.log; exit $rc; }
  python3 scripts/rocpd_summary.py --marker mc_stats --marker-per-step 1 --steps 10 --title "ResNet-50 bs512 $tag headline, round-6 HEAD (r6c27: deferred shortcut BN)" $(find $D/prof_$tag -name '*.db' | head -1) $D/${tag}_summary.csv > $D/sum_$tag.log 2>&1; echo sum_rc=$?
  find $D/prof_$tag -name '*.db' -delete
  head -12 $D/${tag}_summary.csv | cut -c1-160
done
