#!/bin/bash
# r5c2: batched weight re-layouts (prep.hip): GPU tests, bs32 eager bench (with / without), bs32 kernel profile
set -u
D=gpurun_out/r5c2
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_weight_prep_gpu.py tests/test_bn_gpu.py tests/test_bnlink_gpu.py \
  tests/test_winograd_gpu.py tests/test_conv1x1_gpu.py tests/test_kernels_gpu.py tests/test_graph_gpu.py -k "not stress" > $D/pytest.log 2>&1
rc=$?; tail -4 $D/pytest.log; [ $rc -eq 0 ] || exit $rc
B="python3 bench.py --batch-size 32 --steps 40 --warmup 10 --no-bf16-phase --ref-batch 0"
timeout -k 10 300 $B --json-out $D/bs32_eager.json > $D/bs32_eager.log 2>&1
rc=$?; echo eager_rc=$rc; python3 -c "import json;d=json.load(open('$D/bs32_eager.json'));print('eager', d['value'], d['ms_per_step'])"; [ $rc -eq 0 ] || exit $rc
GKSGD_WEIGHT_PREP=0 timeout -k 10 300 $B --json-out $D/bs32_eager_noprep.json > $D/bs32_eager_noprep.log 2>&1
rc=$?; echo noprep_rc=$rc; python3 -c "import json;d=json.load(open('$D/bs32_eager_noprep.json'));print('noprep', d['value'], d['ms_per_step'])"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 $B --json-out $D/bs32_eager2.json > $D/bs32_eager2.log 2>&1
rc=$?; echo eager2_rc=$rc; python3 -c "import json;d=json.load(open('$D/bs32_eager2.json'));print('eager2', d['value'], d['ms_per_step'])"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $D/prof -o prof -- python3 bench.py --batch-size 32 --steps 10 --warmup 5 --no-bf16-phase --ref-batch 0 > $D/prof.log 2>&1
rc=$?; echo prof_rc=$rc; [ $rc -eq 0 ] || exit $rc
python3 scripts/rocpd_summary.py --marker reduce_records_kernel --steps 10 $(find $D/prof -name '*.db' | head -1) $D/prof_summary.txt > $D/sum.log 2>&1; echo sum_rc=$?
find $D/prof -name '*.db' -delete
head -14 $D/prof_summary.txt
GKSGD_BN_FIN_FUSE=0 timeout -k 10 300 $B --json-out $D/bs32_eager_nofin.json > $D/bs32_eager_nofin.log 2>&1
rc=$?; echo nofin_rc=$rc; python3 -c "import json;d=json.load(open('$D/bs32_eager_nofin.json'));print('nofin', d['value'], d['ms_per_step'])"
