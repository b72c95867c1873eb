#!/bin/bash
# kernel timeline of one loop iteration (rocprofv3 kernel trace of a short bench run)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/tl
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl -o run -- \
    python3 bench.py --no-cpu-baseline --steps 20 --warmup 2 --event-iters 0 $BENCH_ARGS > gpurun_out/tl.json 2>&1 || exit $?
python3 tools/timeline.py $(find gpurun_out/tl -name "*kernel_trace.csv" | head -1) 12
