#!/bin/bash
# r5c16: full GPU suite + smoke on the split GEMM build with bf16x6; fp32 (bf16x6) headline kernel profile
set -u
D=gpurun_out/r5c16
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/gputests.log 2>&1
rc=$?; echo gputests_rc=$rc; tail -3 $D/gputests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1
rc=$?; echo smoke_rc=$rc; tail -2 $D/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $D/prof -o prof -- python3 bench.py --steps 10 --warmup 5 --no-bf16-phase --ref-batch 0 > $D/prof.log 2>&1
rc=$?; echo prof_rc=$rc; [ $rc -eq 0 ] || exit $rc
python3 scripts/rocpd_summary.py --marker reduce_records_kernel --steps 10 $(find $D/prof -name '*.db' | head -1) $D/prof_summary.txt > $D/sum.log 2>&1; echo sum_rc=$?
head -40 $D/prof_summary.txt | cut -c1-250
