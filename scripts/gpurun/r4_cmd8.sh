#!/bin/bash
# r4 call 8: implicit-GEMM split-K tests; compression per-kernel profile; bs32 retune with the conv
# split candidates; BERT fp32 retune with the interleaved NT kernel (own kernels vs hipBLASLt per shape)
set -u
D=gpurun_out/r4c8
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_f32_gpu.py tests/test_winograd_gpu.py > $D/tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -3 $D/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/profk -o profk -- python3 bench/kernels.py --only round2 > $D/profk.log 2>&1
rc=$?; echo profk_rc=$rc; [ $rc -eq 0 ] || exit $rc
find $D/profk -name '*kernel_stats.csv' -exec cp {} $D/compress_kernel_stats.csv \;
B="python3 bench.py --batch-size 32 --steps 40 --warmup 10 --no-bf16-phase --ref-batch 0"
show() { python3 -c "import json;d=json.load(open('$D/$1.json'));print('$1', d['value'], d['ms_per_step'])"; }
GKSGD_GEMM_RETUNE=1 GKSGD_GEMM_SAVE=$D/choices32.json GKSGD_GEMM_DUMP=$D/dump32.json timeout -k 10 400 $B --json-out $D/bs32_retuned.json > $D/bs32_retuned.log 2>&1
rc=$?; echo retuned_rc=$rc; show bs32_retuned; [ $rc -eq 0 ] || exit $rc
GKSGD_GEMM_CACHE=$D/choices32.json timeout -k 10 300 $B --json-out $D/bs32_replay.json > $D/bs32_replay.log 2>&1
rc=$?; echo replay_rc=$rc; show bs32_replay; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 $B --json-out $D/bs32_cached.json > $D/bs32_cached.log 2>&1
rc=$?; echo cached_rc=$rc; show bs32_cached; [ $rc -eq 0 ] || exit $rc
GKSGD_GEMM_RETUNE=1 GKSGD_GEMM_SAVE=$D/choices_bert.json GKSGD_GEMM_DUMP=$D/dump_bert.json timeout -k 10 500 python3 bench.py --model bert --no-bf16-phase --ref-batch 0 --steps 5 --warmup 3 --json-out $D/bert.json > $D/bert.log 2>&1
rc=$?; echo bert_rc=$rc; show bert
