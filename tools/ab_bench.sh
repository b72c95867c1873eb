#!/bin/bash
# A/B timing of two builds of liballl.so on one box: build/ab/liballl_A.so vs liballl_B.so,
# alternating bench.py runs of config M (no CPU baseline; VARIANTS="A B C" for more builds).
# usage: bash tools/ab_bench.sh [rounds] [bench args]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=${1:-3}; shift
mkdir -p gpurun_out
for i in $(seq $R); do
  for v in ${VARIANTS:-A B}; do
    ALLL_LIB_AB=build/ab/liballl_$v.so timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > gpurun_out/ab_$v$i.json 2> gpurun_out/ab_$v$i.err || exit $?
    python3 -c "
import json; d=json.load(open('gpurun_out/ab_$v$i.json'))
print('$v$i iters/s %.0f  phases %s  eval %.1f us b2b %s'%(d['resample_iters_per_s'],
 {k:round(v*1e3,1) for k,v in d['phase_ms'].items()}, d['roofline']['eval_ms_in_loop']*1e3, d['roofline'].get('eval_ms_back_to_back')))"
  done
done
