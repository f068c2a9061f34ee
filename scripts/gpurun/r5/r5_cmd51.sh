#!/bin/bash
# r5c51: fused decide/fallback restricted to launch hand-offs, half co-resident grid: compression GPU tests,
# pipeline timing fused / unfused, the driver's bench command
set -u
D=gpurun_out/r5c51
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_kernels2_gpu.py tests/test_dist_gpu.py tests/test_bench_gpu.py > $D/t.log 2>&1
rc=$?; echo test_rc=$rc; tail -2 $D/t.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 300 python3 bench/kernels.py --only round2 > $D/fused$i.txt 2>&1 || exit 1
GKSGD_FB_FUSED=0 timeout -k 10 300 python3 bench/kernels.py --only round2 > $D/unfused$i.txt 2>&1 || exit 1
head -2 $D/fused$i.txt | tail -1; head -2 $D/unfused$i.txt | tail -1
done
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --json-out $D/bench.json > $D/bench.log 2>&1
rc=$?; echo bench_rc=$rc; [ $rc -eq 0 ] || { tail -20 $D/bench.log; exit $rc; }
python3 -c "
import json;d=json.load(open('$D/bench.json'));print({k:d[k] for k in d if k.endswith('value') or k.endswith('ms_per_step')})"
