#!/bin/bash
# Sweep of LFMIS tuning knobs on config M (in-loop phase times from the kernels' stamps).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
OUT=gpurun_out/sweep_mis.txt
: > $OUT
run() {
  echo "== $*" >> $OUT
  env "$@" timeout -k 10 120 python bench.py --no-cpu-baseline --steps 30 --warmup 3 --event-iters 0 $BENCH_ARGS 2>/dev/null \
    | python3 -c "import json,sys; d=json.load(sys.stdin); p=d['phase_ms']; print('iters/s %.0f eval %.1f mis %.1f res %.1f total %.1f' % (d['resample_iters_per_s'], p['eval_ms']*1e3, p['mis_ms']*1e3, p['resample_ms']*1e3, p['total_ms']*1e3))" >> $OUT || { echo "run failed" >> $OUT; exit 1; }
}
run X=0
BENCH_ARGS="--atomic-claims" run X=atomic
for g in 2 3 5 6; do BENCH_ARGS="--grid-rounds $g" run G=$g; done
for sh in 11 13 14; do run ALLL_BKT_SHIFT=$sh; done
for rt in 4 6 8 16; do run ALLL_RUN_TILES=$rt; done
for lds in 24 40 56 100 150; do run ALLL_RESOLVE_LDS=$lds; done
cat $OUT
