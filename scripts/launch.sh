#!/bin/bash
# Launch compressed data-parallel training, one process per MI355X GPU.
#
# Parity: reference run.sh:1-16 (reads exp_configs/$dnn.conf, then mpirun with
# UCX/NCCL env).  Here: configs/$dnn.conf + torch.distributed.run on one node
# (RCCL over xGMI).  Every variable can be overridden from the environment:
#   dnn=resnet50 nworkers=8 density=0.001 compressor=gaussian scripts/launch.sh
set -euo pipefail
cd "$(dirname "$0")/.."
dnn="${dnn:-resnet20}"
source "configs/$dnn.conf"
nworkers="${nworkers:-2}"
density="${density:-1}"
compressor="${compressor:-gaussian}"
nstepsupdate="${nstepsupdate:-1}"
threshold="${threshold:-524288000}"
saved_dir="${saved_dir:-./logs/iclr}"
master_port="${master_port:-29500}"
extra_flags="${extra_flags:-}"
export HSA_ENABLE_IPC_MODE_LEGACY="${HSA_ENABLE_IPC_MODE_LEGACY:-0}"
export NCCL_DEBUG="${NCCL_DEBUG:-WARN}"
# dedicated high-priority comm stream + one RCCL channel per xGMI link
export NCCL_MIN_NCHANNELS="${NCCL_MIN_NCHANNELS:-8}"
exec python -m torch.distributed.run --nnodes=1 --nproc-per-node "$nworkers" \
  --master-addr 127.0.0.1 --master-port "$master_port" \
  -m gaussiank_sgd_amd.train.dist_trainer \
  --dnn "$dnn" --dataset "$dataset" --max-epochs "$max_epochs" --batch-size "$batch_size" \
  --nworkers "$nworkers" --lr "$lr" --nsteps-update "$nstepsupdate" --density "$density" \
  --compressor "$compressor" --threshold "$threshold" --saved-dir "$saved_dir" $extra_flags "$@"
