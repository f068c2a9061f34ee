#!/bin/bash
# r4 call 28: fp32 NT kernel, 32x64 wave tiles: BN-backward epilogue operands prefetched at the start of
# the tile's last K slice -- GEMM / BN-link tests, headline with the cached choices, retune + replay
set -u
D=gpurun_out/r4c28
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_f32_gpu.py tests/test_bnlink_gpu.py tests/test_bn_lazy_gpu.py tests/test_gemm_gpu.py > $D/tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -2 $D/tests.log; [ $rc -eq 0 ] || exit $rc
B="python3 -u bench.py --steps 20 --warmup 5 --no-bf16-phase --ref-batch 0"
timeout -k 10 400 $B --json-out $D/cached.json > $D/cached.log 2>&1
rc=$?; echo cached_rc=$rc; python3 -c "import json;d=json.load(open('$D/cached.json'));print('cached', d['value'], d['ms_per_step'])"; [ $rc -eq 0 ] || exit $rc
GKSGD_GEMM_RETUNE=1 GKSGD_GEMM_SAVE=$D/choices.json GKSGD_GEMM_DUMP=$D/dump.json timeout -k 10 600 $B --json-out $D/retune.json > $D/retune.log 2>&1
rc=$?; echo retune_rc=$rc; python3 -c "import json;d=json.load(open('$D/retune.json'));print('retune', d['value'], d['ms_per_step'])"; [ $rc -eq 0 ] || exit $rc
GKSGD_GEMM_CACHE=$D/choices.json timeout -k 10 400 $B --json-out $D/replay.json > $D/replay.log 2>&1
rc=$?; echo replay_rc=$rc; python3 -c "import json;d=json.load(open('$D/replay.json'));print('replay', d['value'], d['ms_per_step'])"
