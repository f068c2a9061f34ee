#!/bin/bash
# r5c1: native RCCL bootstrap tests (non-blocking init, shared communicator,
# init deadline without a peer) + a default bench line
set -o pipefail
mkdir -p gpurun_out/r5c1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "rccl or share or gaussian or decide or select or count" > gpurun_out/r5c1/pytest.log 2>&1 && \
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --json-out gpurun_out/r5c1/bench.json > gpurun_out/r5c1/bench.log 2>&1
rc=$?
tail -5 gpurun_out/r5c1/pytest.log
tail -3 gpurun_out/r5c1/bench.log | cut -c1-600
exit $rc
