#!/bin/bash
# secondary BASELINE models on the final round-3 build: fp32 headline phase + bf16 phase per run
set -u
D=gpurun_out/r3m
mkdir -p $D
run() {
  local name=$1; shift
  timeout -k 10 400 python -u bench.py "$@" --json-out $D/$name.json > $D/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $D/$name.log; exit $rc; }
}
run vgg16 --model vgg16 --steps 20 --warmup 5
run lstm --model lstm --steps 20 --warmup 5
run bert --model bert --steps 10 --warmup 5
run fcn5net --model fcn5net --steps 50 --warmup 10
run resnet20_bs1024 --model resnet20 --batch-size 1024 --steps 20 --warmup 5
run resnet50_cal --compressor gaussian_cal --steps 20 --warmup 5
echo all_ok
