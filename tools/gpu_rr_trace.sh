#!/bin/bash
# Kernel trace of the round robin at one config (steady state).  usage: bash tools/gpu_rr_trace.sh <tag> <config> <T>
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rr_trace -o run -- \
    python3 tools/rr_bench.py --config $2 --threads $3 --iters 2 --warmup 20 > $O/rr_trace.json 2> $O/rr_trace.err
rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
python3 tools/rr_passes.py $O/rr_trace | tail -40
