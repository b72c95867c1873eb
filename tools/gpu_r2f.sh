#!/bin/bash
# Round-2 final evidence (r2f kernels): the full GPU parity suite, then the r2c evidence set
# (traces + eval PMC for M, C4, C5, R; eval issue counters; C2/C3; one-rank RCCL; default line).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/pytest_r2f.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_r2f.log; [ $rc -eq 0 ] || exit $rc
TAG=r2f bash tools/gpu_r2c.sh
