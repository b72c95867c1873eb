#!/bin/bash
# A/B timing of one build under different environment settings, alternating bench.py runs.
# usage: ENVS="ALLL_X=1 ALLL_X=2:ALLL_Y=3" bash tools/ab_env.sh [rounds] [bench args]
# (a variant may set several variables, separated by ":")
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=${1:-3}; shift
mkdir -p gpurun_out
for i in $(seq $R); do
  for v in ${ENVS:?}; do
    env ${v//:/ } timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > gpurun_out/abe_$v.$i.json 2> gpurun_out/abe_$v.$i.err || exit $?
    python3 -c "
import json; d=json.load(open('gpurun_out/abe_$v.$i.json'))
print('$v #$i iters/s %.0f  phases %s  eval %.1f us frac %.3f'%(d['resample_iters_per_s'],
 {k:round(v*1e3,1) for k,v in d['phase_ms'].items()}, d['roofline']['eval_ms_in_loop']*1e3, d['roofline']['frac']))"
  done
done
