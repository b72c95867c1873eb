#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m "gpu and slow" -x -q > gpurun_out/pytest_gpu_slow.log 2>&1
rc=$?; echo "pytest slow rc=$rc"; tail -15 gpurun_out/pytest_gpu_slow.log
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_profile.sh r1a --steps 30 --warmup 3 --profile-iters 5
