#!/bin/bash
# r5c8: ResNet-50 bs32 fp32 whole-step HIP graph: grad-weight GEMMs on the side stream inside the
# captured graph (parallel graph branches) vs inline, interleaved A/B/A/B
set -u
D=gpurun_out/r5c8
mkdir -p $D
export TMPDIR=/tmp
B="python3 bench.py --batch-size 32 --steps 60 --warmup 15 --no-bf16-phase --ref-batch 0 --graph"
show() { python3 -c "import json;d=json.load(open('$D/$1.json'));print('$1', d['value'], d['ms_per_step'])"; }
for i in 1 2; do
  timeout -k 10 300 $B --json-out $D/inline$i.json > $D/inline$i.log 2>&1
  rc=$?; echo inline${i}_rc=$rc; show inline$i; [ $rc -eq 0 ] || exit $rc
  GKSGD_WGRAD_STREAM=auto GKSGD_WGRAD_STREAM_GRAPH=1 timeout -k 10 300 $B --json-out $D/side$i.json > $D/side$i.log 2>&1
  rc=$?; echo side${i}_rc=$rc; show side$i; [ $rc -eq 0 ] || { tail -20 $D/side$i.log; exit $rc; }
done
