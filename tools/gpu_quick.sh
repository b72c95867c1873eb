#!/bin/bash
# Quick GPU check: a pytest selection (-k expression, -m gpu), then bench lines for the given
# configs (in-loop phase times).  usage: bash tools/gpu_quick.sh "<pytest -k expr>" "M C5 ..." [tag]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${3:-q}
if [ -n "$1" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$1" \
      > gpurun_out/pytest_$TAG.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
fi
for c in $2; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --steps 40 --warmup 5 --event-iters 0 \
      > gpurun_out/bench_${TAG}_$c.json 2> gpurun_out/bench_${TAG}_$c.err
  rc=$?; [ $rc -eq 0 ] || { echo "bench $c rc=$rc"; tail -5 gpurun_out/bench_${TAG}_$c.err; exit $rc; }
  python3 -c "
import json,sys; d=json.load(open('gpurun_out/bench_${TAG}_$c.json'))
print('$c', 'it/s %.0f'%(d['resample_iters_per_s'] or 0), 'ms/step %.4f'%d['ms_per_step'], {k:round(v*1e3,1) for k,v in d['phase_ms'].items()}, 'frac %.3f'%d['roofline']['frac'])"
done
