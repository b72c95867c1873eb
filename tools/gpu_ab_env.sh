#!/bin/bash
# T = 1 bench lines under environment variants on one box (one process per variant, alternating
# `reps` times): usage: bash tools/gpu_ab_env.sh <tag> "<configs>" "<VAR=a VAR=b ...>" [reps] [extra bench args]
# (a variant "-" runs with no extra variable)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${1:-ab}; CFGS=${2:-M}; VARS=${3:--}; REPS=${4:-2}; EXTRA=${5:-}
O=gpurun_out/$T
mkdir -p $O
for rep in $(seq 1 $REPS); do
  for c in $CFGS; do
    for v in $VARS; do
      if [ "$v" = "-" ]; then E=(); else E=("$v"); fi
      env "${E[@]}" timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --no-rr-line --stream-line none --event-iters 0 $EXTRA \
          > $O/ab_${c}_${v}_$rep.json 2> $O/ab_${c}_${v}_$rep.err
      rc=$?; [ $rc -eq 0 ] || { echo "$c $v rc=$rc"; tail -3 $O/ab_${c}_${v}_$rep.err; exit $rc; }
      python3 -c "
import json; d=json.load(open('$O/ab_${c}_${v}_$rep.json')); p=d['phase_ms']
print('$c $v run $rep: %.0f it/s  mis %.1f us  xchg %.1f  eval %.1f  match %s' % (d['resample_iters_per_s'], p['mis_ms']*1e3, p['exchange_ms']*1e3, p['eval_ms']*1e3, (d.get('trajectory_check') or {}).get('match')))"
    done
  done
done
