#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu6.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu6.log
[ $rc -ne 0 ] && exit $rc
for v in "" "--no-ranged"; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline $v > gpurun_out/bench6$v.json 2> gpurun_out/bench6$v.err || exit $?
  python -c "import json,sys; d=json.load(open('gpurun_out/bench6$v.json')); print('$v', d['value'], d['resample_iters_per_s'], d['phase_ms'], d['roofline']['kernel'], d['roofline']['achieved'], d['roofline']['eval_ms_back_to_back'], d['lfmis_rounds_max'])"
done
for cfg in C2 C5; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --config $cfg > gpurun_out/bench6_$cfg.json 2> gpurun_out/bench6_$cfg.err || exit $?
  python -c "import json,sys; d=json.load(open('gpurun_out/bench6_$cfg.json')); print('$cfg', d['value'], d['resample_iters_per_s'], d['phase_ms'], d['roofline']['kernel'], d['roofline']['achieved'], d['roofline']['eval_ms_back_to_back'], d['lfmis_rounds_max'])"
done
