#!/bin/bash
# r4 call 26: full GPU test suite on the current build, then the fp32 headline kernel profile and a
# default-options bench line (headline + bf16 + reference-batch phases)
set -u
D=gpurun_out/r4c26
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $D/gputests.log 2>&1
rc=$?; echo gputests_rc=$rc; tail -3 $D/gputests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $D/prof -o prof -- python3 bench.py --steps 10 --warmup 5 --no-bf16-phase --ref-batch 0 > $D/prof.log 2>&1
rc=$?; echo prof_rc=$rc; [ $rc -eq 0 ] || exit $rc
python3 scripts/rocpd_summary.py --marker reduce_records_kernel --steps 10 $(find $D/prof -name '*.db' | head -1) $D/prof_summary.txt > $D/sum.log 2>&1; echo sum_rc=$?
head -14 $D/prof_summary.txt
timeout -k 10 600 python3 -u bench.py --json-out $D/default.json > $D/default.log 2>&1
rc=$?; echo default_rc=$rc; tail -1 $D/default.log | cut -c1-400
