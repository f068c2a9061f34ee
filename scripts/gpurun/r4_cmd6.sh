#!/bin/bash
# r4 call 6: ResNet-50 bs32 fp32 experiments -- eager, side-stream grad-weights, whole-step hipGraph;
# select-kernel prefetch check (compress tests + kernel bench)
set -u
D=gpurun_out/r4c6
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_kernels2_gpu.py > $D/tests_k.log 2>&1
rc=$?; echo testsk_rc=$rc; tail -3 $D/tests_k.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench/kernels.py --only compress,round2 --json-out $D/kernels.json > $D/kernels.log 2>&1
rc=$?; echo kernels_rc=$rc; grep -i compress $D/kernels.log
B="python3 bench.py --batch-size 32 --steps 40 --warmup 10 --no-bf16-phase --ref-batch 0"
timeout -k 10 300 $B --json-out $D/bs32_eager.json > $D/bs32_eager.log 2>&1
rc=$?; echo eager_rc=$rc; python3 -c "import json;d=json.load(open('$D/bs32_eager.json'));print('eager', d['value'], d['ms_per_step'])"; [ $rc -eq 0 ] || exit $rc
GKSGD_WGRAD_STREAM=1 timeout -k 10 300 $B --json-out $D/bs32_stream.json > $D/bs32_stream.log 2>&1
rc=$?; echo stream_rc=$rc; python3 -c "import json;d=json.load(open('$D/bs32_stream.json'));print('stream', d['value'], d['ms_per_step'])"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 $B --graph --json-out $D/bs32_graph.json > $D/bs32_graph.log 2>&1
rc=$?; echo graph_rc=$rc; python3 -c "import json;d=json.load(open('$D/bs32_graph.json'));print('graph', d['value'], d['ms_per_step'])"
