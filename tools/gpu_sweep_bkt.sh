#!/bin/bash
# Sweep of the bucketed round-0 shape (ALLL_RUN_TILES x ALLL_BKT_SHIFT) on config M.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for rt in ${RTS:-5 10 16}; do for sh in ${SHS:-12 13 14}; do
  ALLL_RUN_TILES=$rt ALLL_BKT_SHIFT=$sh timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 > gpurun_out/sw.json 2>/dev/null || exit $?
  python3 -c "
import json; d=json.load(open('gpurun_out/sw.json'))
print('rt $rt sh $sh iters/s %.0f mis %.1f us'%(d['resample_iters_per_s'], d['phase_ms']['mis_ms']*1e3))"
done; done
