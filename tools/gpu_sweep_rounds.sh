#!/bin/bash
# Sweep of the full-grid LFMIS round count (bench --grid-rounds 3/4/5) on config M, then an A/B
# of build/ab/liballl_A.so against liballl_WR3.so (WAVE_ROUND_MIN = 3).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for i in 1 2; do
 for g in 3 4 5; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 200 --grid-rounds $g > gpurun_out/gr_$g.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/gr_$g.json')); print('G=$g', round(d['resample_iters_per_s']), {k:round(v*1e3,1) for k,v in d['phase_ms'].items()})"
 done
done
VARIANTS="A WR3" bash tools/ab_bench.sh 2 --steps 200
