#!/bin/bash
# BASELINE.md rows at the reference's own configurations:
# fp32 headline phase + bf16 phase per run, eager and whole-step hipGraph, plus
# a 2-rank gloo rehearsal of the multi-rank path on one GPU.
set -u
D=${REFCFG_D:-gpurun_out/r3j}
mkdir -p $D
run() {
  local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" --json-out $D/$name.json > $D/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $D/$name.log; exit $rc; }
}
run resnet50_bs32 --batch-size 32 --steps 50 --warmup 10
run resnet50_bs32_graph --batch-size 32 --steps 50 --warmup 10 --graph
run resnet20_bs32_topk --model resnet20 --batch-size 32 --compressor topk --steps 100 --warmup 20
run resnet20_bs32_topk_graph --model resnet20 --batch-size 32 --compressor topk --steps 100 --warmup 20 --graph
run resnet20_bs1024_topk --model resnet20 --batch-size 1024 --compressor topk --steps 30 --warmup 10
run vgg16_bs128 --model vgg16 --batch-size 128 --steps 50 --warmup 10
run vgg16_bs128_graph --model vgg16 --batch-size 128 --steps 50 --warmup 10 --graph
run lstm_bs20 --model lstm --batch-size 20 --steps 50 --warmup 10
GKSGD_DIST_BACKEND=gloo run resnet50_bs32_gloo2 --gpus 2 --no-native-rccl --batch-size 32 --steps 20 --warmup 5
echo all_ok
