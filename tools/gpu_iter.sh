#!/bin/bash
# Development loop on one MI355X: parity tests, then a bench line of config M.
# usage: bash tools/gpu_iter.sh <tag> [pytest selection]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-it}; SEL=${2:-tests/test_gpu_parity.py}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest $SEL -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; python3 -c "
import json,sys; d=json.load(open('gpurun_out/bench_$TAG.json'))
print('iters/s %.0f  ms/step %.4f  phases %s  eval frac %.3f (%.1f us)'%(d['resample_iters_per_s'],d['ms_per_step'],
 {k:round(v*1e3,1) for k,v in d['phase_ms'].items()}, d['roofline']['frac'], d['roofline']['eval_ms_in_loop']*1e3))"
exit $rc
