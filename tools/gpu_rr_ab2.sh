#!/bin/bash
# round-robin GPU tests, then the A/B of tools/gpu_rr_ab.sh.  usage: bash tools/gpu_rr_ab2.sh <tag> <variant>...
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=$1
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_gpu_round_robin.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/$T/pytest_rr.log 2>&1
rc=$?; echo "pytest rr rc=$rc"; tail -2 gpurun_out/$T/pytest_rr.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_rr_ab.sh "$@"
