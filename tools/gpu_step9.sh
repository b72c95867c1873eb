#!/bin/bash
# GPU tests, default bench line, then the rocprofv3 profile of config M.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu9.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu9.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench9.json 2> gpurun_out/bench9.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench9.json; tail -3 gpurun_out/bench9.err
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_profile.sh r1_M M
