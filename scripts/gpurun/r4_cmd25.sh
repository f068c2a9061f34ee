#!/bin/bash
# r4 call 25: LDS-transpose block totals in the count tail, decide and finalize (u32 scans, eq scan only with an exact-key slot)
# -- compression tests (both hand-off forms), round-2 numbers, size probe timeline
set -u
D=gpurun_out/r4c25
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_kernels2_gpu.py > $D/tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -3 $D/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench/kernels.py --only compress,round2 --json-out $D/k_launch.json > $D/k_launch.log 2>&1
rc=$?; echo klaunch_rc=$rc; grep -i compress $D/k_launch.log; [ $rc -eq 0 ] || exit $rc
GKSGD_HANDOFF=lastblock timeout -k 10 300 python3 bench/kernels.py --only round2 --json-out $D/k_last.json > $D/k_last.log 2>&1
rc=$?; echo klast_rc=$rc; grep -i compress $D/k_last.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace -d $D/probe -o probe -- python3 scripts/debug/compress_size_probe.py > $D/probe.log 2>&1
rc=$?; echo probe_rc=$rc
