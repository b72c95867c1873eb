#!/bin/bash
# GPU tests (all, including the CLI and 10M-clause parity) then the default bench line.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 700 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu8.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu8.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench8.json 2> gpurun_out/bench8.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench8.json; tail -5 gpurun_out/bench8.err
exit $rc
