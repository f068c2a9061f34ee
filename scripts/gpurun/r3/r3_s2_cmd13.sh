#!/bin/bash
# full GPU suite, smoke(), reference-config bench rows with the Winograd build
set -u
D=gpurun_out/s2p
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $D/tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -2 $D/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1
rc=$?; echo smoke_rc=$rc; tail -1 $D/smoke.log
[ $rc -eq 0 ] || exit $rc
REFCFG_D=$D/refcfg bash scripts/gpurun/r3/r3_refcfg.sh
