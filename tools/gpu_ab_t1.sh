#!/bin/bash
# T=1 A/B of build/ab/liballl_A.so vs liballl_B.so at M and C5 (bench lines without the CPU
# baseline or the round-robin line).  usage: bash tools/gpu_ab_t1.sh <rounds>
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=${1:-2}
for cfg in M C5; do
  echo "== $cfg"
  bash tools/ab_bench.sh $R --config $cfg --no-rr-line --stream-line none --event-iters 0 || exit $?
done
