#!/bin/bash
# r5c54: finalize / decide in the stats / count passes' last blocks with launch hand-offs
# (GKSGD_STEP_INGRID=1, new default) vs their own launches (=0): compression GPU tests,
# interleaved pipeline timing, kernel timelines
set -u
D=gpurun_out/r5c54
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_kernels2_gpu.py > $D/t.log 2>&1
rc=$?; echo test_rc=$rc; tail -3 $D/t.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
GKSGD_STEP_INGRID=1 timeout -k 10 300 python3 bench/kernels.py --only round2 > $D/ingrid$i.txt 2>&1 || exit 1
GKSGD_STEP_INGRID=0 timeout -k 10 300 python3 bench/kernels.py --only round2 > $D/launch$i.txt 2>&1 || exit 1
head -3 $D/ingrid$i.txt | tail -2; head -3 $D/launch$i.txt | tail -2
done
GKSGD_STEP_INGRID=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof1 -o run -- python3 bench/kernels.py --only round2 > $D/prof1.log 2>&1 || exit 1
GKSGD_STEP_INGRID=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof0 -o run -- python3 bench/kernels.py --only round2 > $D/prof0.log 2>&1 || exit 1
for p in prof1 prof0; do
  db=$(find $D/$p -name '*.db' | head -1)
  echo "## $p"; python3 scripts/compress_timeline.py $db
  find $D/$p -name '*.db' -delete
done
