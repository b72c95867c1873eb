#!/bin/bash
# Full gpu test suite with the working-tree library, then A/B bench rounds of build/ab/liballl_{A,B}.so
# on the given configs.  usage: bash tools/gpu_ab_cfg.sh "<configs>" [rounds] [skip-tests]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
CFGS=${1:-M}; R=${2:-2}
if [ -z "$3" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1
  rc=$?; tail -3 gpurun_out/pytest_ab.log; [ $rc -eq 0 ] || exit $rc
fi
for c in $CFGS; do
  for i in $(seq $R); do
    for v in ${VARIANTS:-A B}; do
      ALLL_LIB_AB=build/ab/liballl_$v.so timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --steps 40 --warmup 5 --event-iters 0 \
          > gpurun_out/ab_${c}_$v$i.json 2> gpurun_out/ab_${c}_$v$i.err || { echo "bench $c $v rc=$?"; tail -5 gpurun_out/ab_${c}_$v$i.err; exit 1; }
      python3 -c "
import json; d=json.load(open('gpurun_out/ab_${c}_$v$i.json'))
print('$c $v$i it/s %.0f  phases %s  frac %.3f'%(d['resample_iters_per_s'] or 0,
 {k:round(v*1e3,1) for k,v in d['phase_ms'].items()}, d['roofline']['frac']))"
    done
  done
done
