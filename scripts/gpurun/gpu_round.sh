#!/bin/bash
# One GPU-box session: new-kernel tests, then the secondary BERT / LSTM benches
# (saving the GEMM autotune choices), then a kernel-trace profile of BERT.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r
timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_linear_gpu.py} -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r/tests.log 2>&1 || { tail -30 gpurun_out/r/tests.log; exit 1; }
tail -3 gpurun_out/r/tests.log
for m in ${MODELS:-bert lstm}; do
  GKSGD_GEMM_SAVE=gpurun_out/r/choices_$m.json timeout -k 10 400 python bench.py --model $m --steps 20 --warmup 10 \
    --json-out gpurun_out/r/bench_$m.json > gpurun_out/r/bench_$m.log 2>&1 || { tail -30 gpurun_out/r/bench_$m.log; exit 1; }
  echo "$m $(grep -o '"value": [0-9.]*' gpurun_out/r/bench_$m.json)"
done
if [ -n "${PROF:-}" ]; then
  GKSGD_GEMM_CACHE=gpurun_out/r/choices_$PROF.json timeout -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv \
    -d gpurun_out/r/prof_$PROF -o run -- python3 bench.py --model $PROF --steps 8 --warmup 6 > gpurun_out/r/prof_$PROF.log 2>&1 \
    || { tail -20 gpurun_out/r/prof_$PROF.log; exit 1; }
  echo "profiled $PROF"
fi
