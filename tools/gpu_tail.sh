#!/bin/bash
# LDS tail: full GPU parity suite with the working tree's build, then A/B of HEAD (A) vs working
# tree (B) on M, C2, C5, and the working tree at G = 3 / 4 grid rounds.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/pytest_tail.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_tail.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_bench.sh 3 --config M --steps 40 --warmup 5 --event-iters 0 || exit $?
bash tools/ab_bench.sh 2 --config C2 --steps 40 --warmup 5 --event-iters 0 || exit $?
bash tools/ab_bench.sh 2 --config C5 --steps 40 --warmup 5 --event-iters 0 || exit $?
for g in 3 4; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --config M --grid-rounds $g --steps 40 --warmup 5 --event-iters 0 \
      > gpurun_out/tg_$g.json 2> gpurun_out/tg_$g.err || exit $?
  python3 -c "
import json; d=json.load(open('gpurun_out/tg_$g.json'))
print('M G=$g iters/s %.0f phases %s'%(d['resample_iters_per_s'], {k:round(v*1e3,1) for k,v in d['phase_ms'].items()}))"
done
