#!/bin/bash
# (1) BN non-temporal A/B, (2) compression pipeline per-kernel profile,
# (3) conv1x1/bn GPU tests + fp32 bench with the fair MIOpen timing (tune dump)
set -u
D=gpurun_out/r3m
mkdir -p $D
export TMPDIR=/tmp
for v in base ntboth ntst; do
  if [ $v = base ]; then unset GKSGD_EXT; else export GKSGD_EXT=variants/$v/_C.so; fi
  timeout -k 10 200 python -u bench/bn_probe.py --dtype f32 --blocks 1024 > $D/bn_$v.log 2>&1 || exit 1
  timeout -k 10 200 python -u bench/bn_probe.py --dtype bf16 --blocks 1024 > $D/bn16_$v.log 2>&1 || exit 1
  echo "bn $v ok"
done
unset GKSGD_EXT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $D/prof_kern -o run -- python3 bench/kernels.py --only compress,round2 --json-out $D/kernels.json > $D/kernels.log 2>&1
echo "kernels rc=$?"
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv1x1_gpu.py tests/test_bn_gpu.py > $D/tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -2 $D/tests.log
[ $rc -eq 0 ] || exit $rc
export GKSGD_GEMM_SAVE=$D/choices.json GKSGD_GEMM_DUMP=$D/tune_dump.json
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --json-out $D/bench.json > $D/bench.log 2>&1
rc=$?; echo bench_rc=$rc; tail -1 $D/bench.log | cut -c1-300
