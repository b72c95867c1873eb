#!/bin/bash
# Round-2 first GPU pass: the whole -m gpu suite (C4 excluded, it has its own step in
# gpu_r2b.sh), smoke, then gpu_r2b.sh.  Every GPU step is bounded; the script stops at the
# first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    -k "not C4_3sat_128M" > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_r2b.sh
