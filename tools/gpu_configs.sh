#!/bin/bash
# bench line per configuration (and the atomic round-0 variant) for regression checks
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
OUT=gpurun_out/configs.txt
: > $OUT
for cfg in ${CONFIGS:-M C2 C3 C5}; do
  for v in ${VARIANTS:-default --atomic-claims}; do
    echo "== $cfg $v" >> $OUT
    [ "$v" = default ] && v=""
    timeout -k 10 400 python bench.py --no-cpu-baseline --event-iters 0 --config $cfg $v 2>/dev/null \
      | python3 -c "import json,sys; d=json.load(sys.stdin); p=d['phase_ms']; print('iters/s %.0f eval %.1f mis %.1f res %.1f total %.1f frac %.3f viol %d rounds %d' % (d['resample_iters_per_s'], p['eval_ms']*1e3, p['mis_ms']*1e3, p['resample_ms']*1e3, p['total_ms']*1e3, d['roofline']['frac'], d['violated_last'], d['lfmis_rounds_max']))" >> $OUT || { echo failed >> $OUT; exit 1; }
  done
done
cat $OUT
