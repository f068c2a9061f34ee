#!/bin/bash
# r5c14: the driver's bench command with bf16x6 fp32 GEMMs as default (all phases); tuning choices saved
set -u
D=gpurun_out/r5c14
mkdir -p $D
export TMPDIR=/tmp
GKSGD_GEMM_SAVE=$D/choices.json timeout -k 10 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 --json-out $D/bench.json > $D/bench.log 2>&1
rc=$?; echo bench_rc=$rc; [ $rc -eq 0 ] || { tail -30 $D/bench.log; exit $rc; }
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --json-out $D/bench2.json > $D/bench2.log 2>&1
rc=$?; echo bench2_rc=$rc
python3 -c "
import json
for n in ('bench','bench2'):
    d=json.load(open('$D/%s.json'%n)); print(n, {k:d[k] for k in d if k.endswith('value') or k.endswith('ms_per_step')})"
