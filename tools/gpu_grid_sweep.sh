#!/bin/bash
# Grid LFMIS rounds before the one-workgroup tail: G = 3, 4 (default), 5 at M and C2, alternating.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for i in 1 2; do
  for g in 3 4 5; do
    for c in M C2; do
      timeout -k 10 200 python bench.py --no-cpu-baseline --config $c --grid-rounds $g --steps 40 --warmup 5 --event-iters 0 \
          > gpurun_out/gs_${c}_$g.$i.json 2> gpurun_out/gs_${c}_$g.$i.err || exit $?
      python3 -c "
import json; d=json.load(open('gpurun_out/gs_${c}_$g.$i.json'))
print('$c G=$g #$i iters/s %.0f phases %s'%(d['resample_iters_per_s'], {k:round(v*1e3,1) for k,v in d['phase_ms'].items()}))"
    done
  done
done
