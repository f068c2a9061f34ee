#!/bin/bash
# Whole-step hipGraph vs eager at the launch-bound ResNet-20 bs32 config under
# HIP-runtime / stream settings (ms per step of bench.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/g2
run() {  # tag env... -- args
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --model resnet20 --batch-size 32 --steps 50 --warmup 20 ${GARGS:-} \
    > gpurun_out/g2/$tag.log 2>&1 || { echo "$tag failed"; tail -n 5 gpurun_out/g2/$tag.log; exit 1; }
  echo "$tag $(tail -n 1 gpurun_out/g2/$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
}
run eager X=1
run eager_inline GKSGD_COMM_STREAM=0
GARGS=--graph run graph X=1
GARGS=--graph run graph_inline GKSGD_COMM_STREAM=0
GARGS=--graph run graph_pc1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=1
GARGS=--graph run graph_inline_pc1 GKSGD_COMM_STREAM=0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=1
GARGS=--graph run graph_pc0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
