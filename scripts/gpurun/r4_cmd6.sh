#!/bin/bash
# r4 call 6: ResNet-50 bs32 fp32 experiments -- eager, side-stream grad-weights, whole-step hipGraph;
# select-kernel prefetch check (compress tests + kernel bench)
set -u
D=gpurun_out/r4c6
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_kernels2_gpu.py tests/test_winograd_gpu.py tests/test_gemm_f32_gpu.py > $D/tests_k.log 2>&1
rc=$?; echo testsk_rc=$rc; tail -3 $D/tests_k.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench/kernels.py --only compress,round2 --json-out $D/kernels.json > $D/kernels.log 2>&1
rc=$?; echo kernels_rc=$rc; grep -i compress $D/kernels.log
B="python3 bench.py --batch-size 32 --steps 40 --warmup 10 --no-bf16-phase --ref-batch 0"
GKSGD_GEMM_RETUNE=1 GKSGD_GEMM_SAVE=$D/choices32.json GKSGD_GEMM_DUMP=$D/dump32.json timeout -k 10 400 $B --json-out $D/bs32_eager.json > $D/bs32_eager.log 2>&1
rc=$?; echo eager_rc=$rc; python3 -c "import json;d=json.load(open('$D/bs32_eager.json'));print('eager', d['value'], d['ms_per_step'])"; [ $rc -eq 0 ] || exit $rc
export GKSGD_GEMM_CACHE=$D/choices32.json
GKSGD_WGRAD_STREAM=1 timeout -k 10 300 $B --json-out $D/bs32_stream.json > $D/bs32_stream.log 2>&1
rc=$?; echo stream_rc=$rc; python3 -c "import json;d=json.load(open('$D/bs32_stream.json'));print('stream', d['value'], d['ms_per_step'])"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 $B --graph --json-out $D/bs32_graph.json > $D/bs32_graph.log 2>&1
rc=$?; echo graph_rc=$rc; python3 -c "import json;d=json.load(open('$D/bs32_graph.json'));print('graph', d['value'], d['ms_per_step'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $D/prof -o prof -- python3 bench.py --batch-size 32 --steps 10 --warmup 5 --no-bf16-phase --ref-batch 0 > $D/prof.log 2>&1
rc=$?; echo prof_rc=$rc; [ $rc -eq 0 ] || exit $rc
python3 scripts/rocpd_summary.py --marker reduce_records_kernel --steps 10 $(find $D/prof -name '*.db' | head -1) $D/prof_summary.txt > $D/sum.log 2>&1; echo sum_rc=$?
head -14 $D/prof_summary.txt
