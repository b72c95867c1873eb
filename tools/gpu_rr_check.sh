#!/bin/bash
# Round-robin check of a tree: the round-robin GPU tests, steady-state throughput at M (and C2)
# over T, the default bench line without the CPU baseline (both trajectory checks).
# usage: bash tools/gpu_rr_check.sh <tag> [pytest -k expression]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-rr}; K=${2:-}
O=gpurun_out/$T
mkdir -p $O
if [ -n "$K" ]; then KA=(-k "$K"); else KA=(); fi
fatal() { case $1 in 0) ;; *) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_round_robin.py -v -x --timeout 300 --timeout-method thread \
    "${KA[@]}" > $O/pytest_rr.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR" $O/pytest_rr.log | head; tail -2 $O/pytest_rr.log; fatal $rc pytest
timeout -k 10 300 python tools/rr_bench.py --config M --threads 16,4 --warmup 20 --iters 20 > $O/rr_M.json 2> $O/rr_M.err
rc=$?; cat $O/rr_M.json; fatal $rc rrM
timeout -k 10 300 python tools/rr_bench.py --config C2 --threads 16 --warmup 20 --iters 20 > $O/rr_C2.json 2> $O/rr_C2.err
rc=$?; cat $O/rr_C2.json; fatal $rc rrC2
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err
rc=$?; tail -2 $O/bench.err; python tools/bench_brief.py $O/bench.json; fatal $rc bench
