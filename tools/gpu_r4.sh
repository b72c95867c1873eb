#!/bin/bash
# Round-4 GPU check: default bench line (with the oracle trajectory check), the full GPU parity
# suite (up to 10 failures reported), smoke, then round-robin throughput at M and a kernel trace
# of it.  Stops after a crash or a time limit.  usage: bash tools/gpu_r4.sh <tag>
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r4}
O=gpurun_out/$T
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 400 python bench.py --no-rr-line > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; cat $O/bench.json | head -c 3000; echo; fatal $rc bench
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=10 --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR" $O/pytest.log | head -20; tail -3 $O/pytest.log; fatal $rc pytest
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $O/smoke.log; fatal $rc smoke
timeout -k 10 300 python tools/rr_bench.py --config M --threads 16,4 --iters 10 --warmup 2 > $O/rr_M.json 2> $O/rr_M.err
rc=$?; echo "rr rc=$rc"; cat $O/rr_M.json; fatal $rc rr
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rr_trace -o run -- \
    python3 tools/rr_bench.py --config M --threads 16 --iters 3 --warmup 1 > $O/rr_trace.json 2> $O/rr_trace.err
rc=$?; echo "rr trace rc=$rc"; fatal $rc rrtrace
timeout -k 10 400 python bench.py > $O/bench_full.json 2> $O/bench_full.err
rc=$?; echo "bench (with the round-robin line) rc=$rc"; fatal $rc bench_full
exit 0
