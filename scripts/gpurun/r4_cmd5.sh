#!/bin/bash
# r4 call 5: NT GEMM with interleaved LDS-DMA issue -- correctness, bench (cached choices), retuned bench, phase order
set -u
D=gpurun_out/r4c5
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gemm_f32_gpu.py tests/test_gemm_gpu.py tests/test_conv1x1_gpu.py tests/test_bnlink_gpu.py tests/test_bn_lazy_gpu.py tests/test_linear_gpu.py tests/test_lstm_gpu.py > $D/tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -4 $D/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --json-out $D/bench_cached.json > $D/bench_cached.log 2>&1
rc=$?; echo bench_rc=$rc; python3 -c "import json;d=json.load(open('$D/bench_cached.json'));print('cached', d['value'], d['ms_per_step'], d.get('bf16_value'), d.get('ref_bs32_value'))"; [ $rc -eq 0 ] || exit $rc
GKSGD_GEMM_RETUNE=1 GKSGD_GEMM_SAVE=$D/gemm_choices.json GKSGD_GEMM_DUMP=$D/gemm_dump.json timeout -k 10 900 python3 bench.py --json-out $D/bench_retuned.json > $D/bench_retuned.log 2>&1
rc=$?; echo bench2_rc=$rc; python3 -c "import json;d=json.load(open('$D/bench_retuned.json'));print('retuned', d['value'], d['ms_per_step'], d.get('bf16_value'), d.get('ref_bs32_value'))"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/debug/phase_order_probe.py --order b,s,b,d,b > $D/order.log 2>&1
rc=$?; echo order_rc=$rc; grep phase $D/order.log
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_kernels2_gpu.py > $D/tests_k.log 2>&1
rc=$?; echo testsk_rc=$rc; tail -3 $D/tests_k.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench/kernels.py --only compress --json-out $D/kernels.json > $D/kernels.log 2>&1
rc=$?; echo kernels_rc=$rc; grep compress $D/kernels.log
timeout -k 10 300 python3 bench.py --model lstm --steps 10 --warmup 3 --json-out $D/bench_lstm.json > $D/bench_lstm.log 2>&1
rc=$?; echo lstm_rc=$rc; python3 -c "import json;d=json.load(open('$D/bench_lstm.json'));print('lstm', d['value'], d['ms_per_step'], d.get('bf16_value'))"
