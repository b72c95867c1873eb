#!/bin/bash
# Round-0 lose marks by epoch tag: full GPU parity suite with the working tree's
# build, then A/B of HEAD (A) vs working tree (B) on M, C2 and C5.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/pytest_tag.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_tag.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_bench.sh 3 --config M --steps 40 --warmup 5 --event-iters 0 || exit $?
bash tools/ab_bench.sh 2 --config C2 --steps 40 --warmup 5 --event-iters 0 || exit $?
bash tools/ab_bench.sh 2 --config C5 --steps 40 --warmup 5 --event-iters 0 || exit $?
