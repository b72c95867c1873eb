#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -k "hybrid or bench or big or baseline" > gpurun_out/pytest_sweep.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_sweep.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python tools/eval_sweep.py 2>&1 | tee gpurun_out/sweep.txt
