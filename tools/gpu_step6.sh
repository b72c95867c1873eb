#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu6.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu6.log
[ $rc -ne 0 ] && exit $rc
SWEEP_GRIDS=256 timeout -k 10 600 python tools/eval_sweep.py 2>&1 | tee gpurun_out/sweep6.txt
for cfg in M C5; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --config $cfg > gpurun_out/bench6_$cfg.json 2> gpurun_out/bench6_$cfg.err || exit $?
  python -c "import json,sys; d=json.load(open('gpurun_out/bench6_$cfg.json')); print('$cfg', d['value'], d['resample_iters_per_s'], d['phase_ms'], d['roofline']['kernel'], d['roofline']['achieved'], d['roofline']['eval_ms_back_to_back'], d['lfmis_rounds_max'])"
done
