#!/bin/bash
# r4 call 12: launch hand-offs (decide / finalize as their own 1-workgroup kernels) vs last-block --
# stress tests for both, round-2 compression numbers for both; fp32 NT sweep on the BERT FFN shape
# + counters of its best config
set -u
D=gpurun_out/r4c12
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_kernels2_gpu.py > $D/tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -3 $D/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench/kernels.py --only compress,round2 --json-out $D/k_launch.json > $D/k_launch.log 2>&1
rc=$?; echo klaunch_rc=$rc; grep -i compress $D/k_launch.log; [ $rc -eq 0 ] || exit $rc
GKSGD_HANDOFF=lastblock timeout -k 10 300 python3 bench/kernels.py --only compress,round2 --json-out $D/k_last.json > $D/k_last.log 2>&1
rc=$?; echo klast_rc=$rc; grep -i compress $D/k_last.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace -d $D/probe -o probe -- python3 scripts/debug/compress_size_probe.py > $D/probe.log 2>&1
rc=$?; echo probe_rc=$rc; [ $rc -eq 0 ] || exit $rc
CF="1,2,3,4,7,11,12,13,14,21,22,23,24,101,102,103,104,201,202,203,204,1001,1002,1003,1004,1005,1006,1007,1021,1022,1101,1102,1103"
timeout -k 10 300 python3 bench/gemm_probe.py --op gemm --dtype f32 --C 768 --K 3072 --H 1 --batch 16384 --sweep $CF > $D/sweep_ffn1.jsonl 2>&1
rc=$?; echo sweep_rc=$rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench/gemm_probe.py --op gemm --dtype f32 --C 3072 --K 768 --H 1 --batch 16384 --sweep $CF > $D/sweep_ffn2.jsonl 2>&1
rc=$?; echo sweep2_rc=$rc
python3 - <<'PY'
import json
for f in ("gpurun_out/r4c12/sweep_ffn1.jsonl", "gpurun_out/r4c12/sweep_ffn2.jsonl"):
    rows = [json.loads(l) for l in open(f) if l.startswith("{") and "tflops" in l]
    rows.sort(key=lambda r: -r["tflops"])
    print(f, [(r["cfg"], r["tflops"]) for r in rows[:6]])
PY
