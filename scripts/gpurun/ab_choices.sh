#!/bin/bash
# A/B of two conv-kernel autotune caches in one box (alternating runs).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for i in 1 2; do
  for v in ${AB_VARIANTS:-prev new}; do
    timeout -k 10 400 env GKSGD_GEMM_CACHE=tuning/ab_$v.json python bench.py --steps 30 --warmup 10 \
      --json-out gpurun_out/ab/bench_${v}_$i.json > gpurun_out/ab/bench_${v}_$i.log 2>&1 || exit 1
    echo "$v $i $(grep -o '"value": [0-9.]*' gpurun_out/ab/bench_${v}_$i.json)"
  done
done
