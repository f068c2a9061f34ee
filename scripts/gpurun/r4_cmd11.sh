#!/bin/bash
# r4 call 11: compression size probe (fixed vs streaming cost per kernel); bs32 retune with the
# small-batch grad-weight split candidates; full GPU test suite
set -u
D=gpurun_out/r4c11
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $D/probe -o probe -- python3 scripts/debug/compress_size_probe.py > $D/probe.log 2>&1
rc=$?; echo probe_rc=$rc; [ $rc -eq 0 ] || exit $rc
B="python3 bench.py --batch-size 32 --steps 40 --warmup 10 --no-bf16-phase --ref-batch 0"
show() { python3 -c "import json;d=json.load(open('$D/$1.json'));print('$1', d['value'], d['ms_per_step'])"; }
GKSGD_GEMM_RETUNE=1 GKSGD_GEMM_SAVE=$D/choices32.json GKSGD_GEMM_DUMP=$D/dump32.json timeout -k 10 400 $B --json-out $D/bs32_retuned.json > $D/bs32_retuned.log 2>&1
rc=$?; echo retuned_rc=$rc; show bs32_retuned; [ $rc -eq 0 ] || exit $rc
GKSGD_GEMM_CACHE=$D/choices32.json timeout -k 10 300 $B --json-out $D/bs32_replay.json > $D/bs32_replay.log 2>&1
rc=$?; echo replay_rc=$rc; show bs32_replay; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 $B --json-out $D/bs32_cached.json > $D/bs32_cached.log 2>&1
rc=$?; echo cached_rc=$rc; show bs32_cached; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/gputests.log 2>&1
rc=$?; echo gputests_rc=$rc; tail -5 $D/gputests.log
