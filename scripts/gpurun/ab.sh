#!/bin/bash
# Same-box A/B of two extension builds (the working tree's _C.so vs
# variants/old/_C.so), interleaved new/old/new/old so drift shows up:
#   AB_CMDS: ';'-separated commands (each run under both builds)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${AB_OUT:-gpurun_out/ab}
mkdir -p $OUT
IFS=';' read -ra CMDS <<< "${AB_CMDS:-python bench.py --steps 20 --warmup 10}"
i=0
for c in "${CMDS[@]}"; do
  i=$((i+1))
  for v in new old new2 old2; do
    case $v in old*) export GKSGD_EXT=variants/old/_C.so ;; *) unset GKSGD_EXT ;; esac
    timeout -k 10 300 $c > $OUT/c${i}_$v.log 2>&1 || { echo "c$i $v failed"; tail -n 5 $OUT/c${i}_$v.log; exit 1; }
    echo "c$i $v $(tail -n 1 $OUT/c${i}_$v.log | cut -c1-${AB_CUT:-160})"
  done
done
