#!/bin/bash
# Round-robin fixpoint check: the RR GPU tests of the fixpoint modes (or the -k expression given),
# M throughput for T = 16 and 4, then (PROF=1) a kernel trace at T = 16.
# usage: bash tools/gpu_rr_fp.sh <tag> [pytest -k expression]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-fp}; K=${2:-fp}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_round_robin.py -x -q --timeout 120 --timeout-method thread -k "$K" > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -6 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/rr_bench.py --config M --threads 16,4 --iters 5 > gpurun_out/rr_$TAG.json 2>&1
rc=$?; tail -3 gpurun_out/rr_$TAG.json; [ $rc -eq 0 ] || exit $rc
if [ "${PROF:-0}" = 1 ]; then bash tools/gpu_rr_prof.sh rrprof_$TAG 16 || exit $?; fi
