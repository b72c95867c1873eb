#!/bin/bash
# Full round-end rehearsal on one MI355X: every GPU test, smoke(), the default bench line
# (with the CPU baseline), then the rocprofv3 profile of config M (tools/gpu_profile.sh).
# usage: bash tools/gpu_full.sh <tag>
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r1}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/pytest_gpu_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_$TAG.json; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_profile.sh ${TAG}_M M
