#!/bin/bash
# r4 call 4: bf16-after-bs32 slowdown probe; compression pipeline timing + per-kernel profile; fp32 BERT profile
set -u
D=gpurun_out/r4c4
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 300 python3 scripts/debug/phase_order_probe.py --order b,s,b,d,b > $D/order.log 2>&1
rc=$?; echo order_rc=$rc; grep phase $D/order.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench/kernels.py --only compress,round2 --json-out $D/kernels.json > $D/kernels.log 2>&1
rc=$?; echo kernels_rc=$rc; tail -20 $D/kernels.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/profk -o prof -- python3 bench/kernels.py --only compress > $D/profk.log 2>&1
rc=$?; echo profk_rc=$rc; [ $rc -eq 0 ] || exit $rc
python3 scripts/rocpd_summary.py $(find $D/profk -name '*.db' | head -1) $D/compress_kernels.txt > /dev/null 2>&1; echo sumk=$?
find $D/profk -name '*.db' -delete
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $D/profb -o prof -- python3 bench.py --model bert --steps 5 --warmup 3 --no-bf16-phase --ref-batch 0 > $D/profb.log 2>&1
rc=$?; echo profb_rc=$rc; [ $rc -eq 0 ] || exit $rc
python3 scripts/rocpd_summary.py --marker attn_f32_fwd --marker-per-step 12 --steps 5 $(find $D/profb -name '*.db' | head -1) $D/bert_f32_summary.txt > /dev/null 2>&1; echo sumb_rc=$?
find $D/profb -name '*.db' -delete
head -14 $D/bert_f32_summary.txt
