#!/bin/bash
# Round-2 GPU session: new-kernel tests first, then the whole GPU suite, the
# smoke test and the 1-GPU headline bench.  Every GPU step has its own time
# limit; the script stops at the first crash / abort / timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r2
mkdir -p $OUT
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -4 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for s in ${STEPS:-new all smoke bench}; do
  case $s in
    new) step new_tests 600 python -u -m pytest ${NEW_TESTS:-tests/test_kernels2_gpu.py tests/test_bench_gpu.py} -x -v \
           --timeout 300 --timeout-method thread ;;
    all) step all_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench1 600 python bench.py --steps 20 --warmup 10 --json-out $OUT/bench1.json ;;
    fp32) step bench_fp32 600 python bench.py --steps 10 --warmup 5 --amp none --json-out $OUT/bench_fp32.json ;;
    sweep) for spec in ${SWEEP:-bert:524288000 bert:56000000 bert:28000000 bert:14000000 vgg16:524288000 vgg16:7400000 vgg16:3700000}; do
             m=${spec%%:*}; th=${spec##*:}
             step sweep_${m}_${th} 400 python bench.py --model $m --steps 20 --warmup 10 --threshold $th \
               --json-out $OUT/sweep_${m}_${th}.json
           done ;;
    marker) export GKSGD_ROCTX=1; step marker 600 rocprofv3 --marker-trace --kernel-trace --stats --output-format csv -d $OUT/marker -o run -- \
           python3 bench.py ${MARKER_ARGS:---model bert --steps 4 --warmup 4 --threshold 28000000}; unset GKSGD_ROCTX ;;
    convs) step convs_ours 900 python bench/convs.py --ours --json-out $OUT/convs_ours.json ;;
    ctr) CTR_OUT=$OUT/ctr_wgrad3 PROBE_ARGS="--op wgrad3 --cfg ${TN_CFG:-27} --C 256 --H 14" bash scripts/gpurun/gemm_counters.sh \
           > $OUT/ctr_wgrad3.log 2>&1; tail -40 $OUT/ctr_wgrad3.log
         CTR_OUT=$OUT/ctr_conv3 PROBE_ARGS="--op conv --cfg ${NT_CFG:-124} --C 256 --H 14" bash scripts/gpurun/gemm_counters.sh \
           > $OUT/ctr_conv3.log 2>&1; tail -40 $OUT/ctr_conv3.log ;;
    plan) step plan_bert 600 python bench.py --model bert --steps 20 --warmup 10 --planner mgs --plan-world 8 \
           --json-out $OUT/plan_bert.json
          step bert16 400 python bench.py --model bert --steps 20 --warmup 10 --threshold 7000000 \
           --json-out $OUT/bert16.json ;;
    allbench) for spec in ${ALLBENCH:-"resnet50" "vgg16" "lstm" "bert" "fcn5net" "resnet20 --batch-size 1024" \
                  "resnet20 --batch-size 32" "resnet50 --compressor gaussian_cal" "vgg16 --compressor gaussian_cal" \
                  "bert --compressor gaussian_cal" "lstm --compressor gaussian_cal" "bert --threshold 7000000" \
                  "resnet50 --dense"}; do
             tag=$(echo $spec | tr ' ' '_' | tr -d '-')
             step ab_$tag 400 python bench.py --model $spec --steps 20 --warmup 10 --json-out $OUT/ab_$tag.json
           done ;;
    retune) for m in ${RETUNE_MODELS:-resnet50 bert vgg16 resnet20 lstm}; do
              export GKSGD_GEMM_RETUNE=1 GKSGD_GEMM_SAVE=$OUT/choices_$m.json
              step retune_$m 600 python bench.py --model $m --steps 20 --warmup 10 --json-out $OUT/retune_$m.json
              unset GKSGD_GEMM_RETUNE GKSGD_GEMM_SAVE
            done ;;
    kern) step kernels 600 python bench/kernels.py --only ${KERN_ONLY:-round2,fit} --fit-out $OUT/perf_model_mi355x.json \
           --json-out $OUT/kernels.json ;;
    prof) step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
           python3 bench.py ${PROF_ARGS:---steps 5 --warmup 3} ;;
  esac
done
