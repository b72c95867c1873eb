#!/bin/bash
# Sweep of the T = 1 grid rounds before the one-workgroup tail (bench.py --grid-rounds),
# alternating the values twice per config.  Lines go to gpurun_out/rounds_<cfg>_<G>_<i>.json.
# usage: bash tools/gpu_sweep_rounds.sh "<M rounds>" "<C5 rounds>"
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
run() {
  local cfg=$1 g=$2 i=$3
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-rr-line --stream-line none --event-iters 0 --config $cfg --grid-rounds $g \
      > gpurun_out/rounds_${cfg}_${g}_$i.json 2> gpurun_out/rounds_${cfg}_${g}_$i.err || exit $?
  python3 -c "
import json; d=json.load(open('gpurun_out/rounds_${cfg}_${g}_$i.json'))
print('$cfg G=$g run $i: %.0f it/s  mis %.1f us' % (d['resample_iters_per_s'], d['phase_ms']['mis_ms'] * 1e3))"
}
for i in 1 2; do
  for g in $1; do run M $g $i; done
  for g in $2; do run C5 $g $i; done
done
