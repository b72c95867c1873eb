#!/bin/bash
# Owner-slot mixing A/B on C5 (vmix owner slots vs identity owner slots, buckets keep vmix),
# parity of the hot-variable instances with identity owner slots first.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
ALLL_OWNER_VMIX=0 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "powerlaw or C5 or atomic_claims" > gpurun_out/pytest_omix.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_omix.log; [ $rc -eq 0 ] || exit $rc
ENVS="ALLL_OWNER_VMIX=1 ALLL_OWNER_VMIX=0 ALLL_OWNER_VMIX=0:ALLL_NO_VMIX=1" bash tools/ab_env.sh 3 --config C5 --steps 40 --warmup 5 --event-iters 0 || exit $?
ALLL_OWNER_VMIX=0 BENCH_ARGS="--config C5" bash tools/gpu_timeline.sh && python3 tools/timeline.py $(find gpurun_out/tl -name "*kernel_trace.csv" | head -1) 14
