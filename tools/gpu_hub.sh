#!/bin/bash
# Hub spread check: parity on the hot-variable instances, then C5 A/B of ALLL_HUB_SPREAD
# (0 off, 4 round-0 scatter only, 5 + k_claim rounds, 7 + wave rounds) and a C5 kernel trace.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "powerlaw or C5 or hub or atomic_claims" > gpurun_out/pytest_hub.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_hub.log; [ $rc -eq 0 ] || exit $rc
ENVS="ALLL_HUB_SPREAD=0 ALLL_HUB_SPREAD=4 ALLL_HUB_SPREAD=5 ALLL_HUB_SPREAD=7" bash tools/ab_env.sh 2 --config C5 --steps 40 --warmup 5 --event-iters 0 || exit $?
BENCH_ARGS="--config C5" bash tools/gpu_timeline.sh && python3 tools/timeline.py $(find gpurun_out/tl -name "*kernel_trace.csv" | head -1) 14
