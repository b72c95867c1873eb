#!/bin/bash
# Round-robin A/B at one config: the in-tree library and build/ab variants.
# usage: bash tools/gpu_rr_ab_cfg.sh <tag> <config> <threads> <variant>...
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=$1; CFG=$2; TH=$3; shift 3
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 200 python tools/rr_bench.py --config $CFG --threads $TH --iters 20 --warmup 20 > $O/rr_base.json 2> $O/rr_base.err
rc=$?; echo "base rc=$rc"; cat $O/rr_base.json; [ $rc -ne 0 ] && exit $rc
for v in "$@"; do
  ALLL_LIB_AB=build/ab/liballl_$v.so timeout -k 10 200 python tools/rr_bench.py --config $CFG --threads $TH --iters 20 --warmup 20 > $O/rr_$v.json 2> $O/rr_$v.err
  rc=$?; echo "$v rc=$rc"; cat $O/rr_$v.json; [ $rc -ne 0 ] && exit $rc
done
exit 0
