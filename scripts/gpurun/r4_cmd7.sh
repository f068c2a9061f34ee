#!/bin/bash
# r4 call 7: ResNet-50 bs32 fp32 A/B in one box -- committed choices vs a retune with the split
# candidates (saved, then replayed), side-stream grad-weights, whole-step hipGraph
set -u
D=gpurun_out/r4c7
mkdir -p $D
export TMPDIR=/tmp
B="python3 bench.py --batch-size 32 --steps 40 --warmup 10 --no-bf16-phase --ref-batch 0"
show() { python3 -c "import json;d=json.load(open('$D/$1.json'));print('$1', d['value'], d['ms_per_step'])"; }
timeout -k 10 300 $B --json-out $D/bs32_cached.json > $D/bs32_cached.log 2>&1
rc=$?; echo cached_rc=$rc; show bs32_cached; [ $rc -eq 0 ] || exit $rc
GKSGD_GEMM_RETUNE=1 GKSGD_GEMM_SAVE=$D/choices32.json GKSGD_GEMM_DUMP=$D/dump32.json timeout -k 10 400 $B --json-out $D/bs32_retuned.json > $D/bs32_retuned.log 2>&1
rc=$?; echo retuned_rc=$rc; show bs32_retuned; [ $rc -eq 0 ] || exit $rc
GKSGD_GEMM_CACHE=$D/choices32.json timeout -k 10 300 $B --json-out $D/bs32_replay.json > $D/bs32_replay.log 2>&1
rc=$?; echo replay_rc=$rc; show bs32_replay; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 $B --graph --json-out $D/bs32_graph.json > $D/bs32_graph.log 2>&1
rc=$?; echo graph_rc=$rc; show bs32_graph
