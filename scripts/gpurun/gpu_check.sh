#!/bin/bash
# One GPU-box session: GPU tests, smoke, 1-GPU bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; the script stops at the first
# crash / abort / timeout (exit codes other than 0 and 1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -5 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = test ]; then
  step pytest_gpu 900 python -m pytest tests -m gpu -x -q
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  step bench1 600 python bench.py --steps 20 --warmup 10 --json-out $OUT/bench1.json
fi
if [ "$MODE" = all ] || [ "$MODE" = prof ]; then
  step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 5 --warmup 3
fi
if [ "$MODE" = find ]; then
  step bench_find 900 python bench.py --steps 20 --warmup 10 --cudnn-benchmark --json-out $OUT/bench_find.json
  mkdir -p $OUT/tuning && cp -r tuning/miopen $OUT/tuning/ && ls -la $OUT/tuning/miopen ~/.cache/miopen 2>/dev/null | head -20
  du -sh ~/.cache/miopen 2>/dev/null || true
  step bench_after_find 600 python bench.py --steps 20 --warmup 10 --json-out $OUT/bench_after_find.json
fi
if [ "$MODE" = sweep ]; then
  for bs in ${SWEEP_BS:-128 512}; do
    step bench_bs$bs 600 python bench.py --steps 20 --warmup 10 --batch-size $bs --json-out $OUT/bench_bs$bs.json
  done
  step bench_dense 600 python bench.py --steps 20 --warmup 10 --dense --json-out $OUT/bench_dense.json
fi

# find-db for additional batch sizes: FIND_BS="384 512" bash scripts/gpurun/gpu_check.sh findbs
if [ "$MODE" = findbs ]; then
  for bs in ${FIND_BS:-512}; do
    step find_bs$bs 900 python bench.py --steps 10 --warmup 5 --batch-size $bs --cudnn-benchmark --json-out $OUT/find_bs$bs.json
    step bench_bs$bs 600 python bench.py --steps 20 --warmup 10 --batch-size $bs --json-out $OUT/bench_bs$bs.json
  done
  mkdir -p $OUT/tuning && cp -r tuning/miopen $OUT/tuning/
fi
# targeted: GPU tests of given files + bench A/B + profile
#   TESTS="tests/test_shadow_gpu.py" AB="--no-shadow" bash scripts/gpurun/gpu_check.sh ab
if [ "$MODE" = ab ]; then
  step pytest_sel 600 python -m pytest ${TESTS:-tests/test_shadow_gpu.py} -x -q
  step bench_a 600 python bench.py --steps 20 --warmup 10 --json-out $OUT/bench_a.json
  step bench_b 600 python bench.py --steps 20 --warmup 10 ${AB:---no-shadow} --json-out $OUT/bench_b.json
  step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 5 --warmup 3
fi
# MIOpen solver A/B: the ASM implicit-GEMM bwd/wrw solvers need a zero-fill
# (SubTensorOpWithScalar) of their output before every call.
if [ "$MODE" = solvers ]; then
  step bench_base 600 python bench.py --steps 20 --warmup 10 --json-out $OUT/bench_base.json
  step bench_nobwd 600 env MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_GTC_XDLOPS_NHWC=0 python bench.py --steps 20 --warmup 10 --json-out $OUT/bench_nobwd.json
  step bench_nowrw 600 env MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0 python bench.py --steps 20 --warmup 10 --json-out $OUT/bench_nowrw.json
  step bench_noboth 600 env MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_GTC_XDLOPS_NHWC=0 \
    MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0 python bench.py --steps 20 --warmup 10 --json-out $OUT/bench_noboth.json
fi
# MIOpen kernel-parameter tuning (perf-db) for the bench shapes: exhaustive
# search per convolution, written into the repo's user db (tuning/miopen).
# Progress goes to a growing log under gpurun_out (the call is not idle).
if [ "$MODE" = tune ]; then
  echo "=== tune ($(date +%T))"
  timeout -k 10 ${TUNE_S:-1000} env MIOPEN_FIND_ENFORCE=SEARCH MIOPEN_LOG_LEVEL=5 python bench.py --steps 2 --warmup 1 \
    --cudnn-benchmark --json-out $OUT/tune.json > $OUT/tune.log 2>&1
  echo "tune rc=$?"
  mkdir -p $OUT/tuning && cp -r tuning/miopen $OUT/tuning/ && ls -la $OUT/tuning/miopen
fi
# 1x1 convs as hipBLASLt GEMMs (A/B) + reference per-GPU batch (32)
if [ "$MODE" = gemm ]; then
  step bench_bs32 600 python bench.py --steps 30 --warmup 10 --batch-size 32 --json-out $OUT/bench_bs32.json
fi
# secondary BASELINE configs (1 GPU) + dense comparator
if [ "$MODE" = models ]; then
  for m in ${MODELS:-vgg16 lstm bert fcn5net}; do
    step bench_$m 600 python bench.py --model $m --steps 20 --warmup 5 --json-out $OUT/bench_$m.json
  done
  step bench_dense 600 python bench.py --steps 20 --warmup 10 --dense --json-out $OUT/bench_dense.json
fi
echo done
