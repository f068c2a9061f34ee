#!/bin/bash
# r5m: secondary BASELINE models on the round-5 HEAD (bf16x6 fp32 GEMMs): fp32 phase + bf16 phase per run
set -u
D=gpurun_out/r5m
mkdir -p $D
export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -k 10 400 python -u bench.py "$@" --json-out $D/$name.json > $D/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $D/$name.log; exit $rc; }
  python3 -c "
import json;d=json.load(open('$D/$name.json'));print({k:d[k] for k in d if k.endswith('value') or k.endswith('ms_per_step') or k=='selected_over_k'})"
}
run vgg16 --model vgg16 --steps 20 --warmup 5
run lstm --model lstm --steps 20 --warmup 5
run fcn5net --model fcn5net --steps 50 --warmup 10
run resnet20_bs1024 --model resnet20 --batch-size 1024 --steps 20 --warmup 5
run resnet50_cal --compressor gaussian_cal --steps 20 --warmup 5 --no-native-phase

# the driver's headline command again (box-to-box check against r5c53 / r5c52)
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --json-out $D/bench_head.json > $D/bench_head.log 2>&1
rc=$?; echo bench_head_rc=$rc; [ $rc -eq 0 ] || exit $rc
python3 -c "
import json;d=json.load(open('$D/bench_head.json'));print({k:d[k] for k in d if k.endswith('value') or k.endswith('ms_per_step') or k=='compress_sync_timeouts'})"
echo all_ok
