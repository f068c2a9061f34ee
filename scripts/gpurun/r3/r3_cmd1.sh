set -o pipefail
mkdir -p gpurun_out/r3
export GKSGD_GEMM_SAVE=gpurun_out/r3/choices.json GKSGD_GEMM_DUMP=gpurun_out/r3/tune_dump.json
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --json-out gpurun_out/r3/bench_fp32.json > gpurun_out/r3/bench_fp32.log 2>&1
rc=$?; echo bench_rc=$rc; tail -3 gpurun_out/r3/bench_fp32.log
[ $rc -eq 0 ] || exit $rc
unset GKSGD_GEMM_SAVE GKSGD_GEMM_DUMP
export GKSGD_GEMM_CACHE=$PWD/gpurun_out/r3/choices.json TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r3/prof_fp32 -o run -- python bench.py --steps 10 --warmup 3 --no-bf16-phase > gpurun_out/r3/prof_fp32.log 2>&1
echo prof_rc=$?; tail -2 gpurun_out/r3/prof_fp32.log
