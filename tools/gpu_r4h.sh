#!/bin/bash
# Round-robin tests, RR throughput at M / C5, the round robin under torch's bundled runtime, bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${1:-r4h}
O=gpurun_out/$T
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_round_robin.py tests/test_gpu_multirank.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/pytest_rr.log 2>&1
rc=$?; echo "pytest rr rc=$rc"; tail -2 $O/pytest_rr.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/rr_bench.py --config M --threads 16,4 --iters 20 --warmup 20 > $O/rr_M.json 2> $O/rr_M.err
rc=$?; echo "rr M rc=$rc"; cat $O/rr_M.json; fatal $rc rrM
timeout -k 10 200 python tools/rr_bench.py --config C5 --threads 16 --iters 20 --warmup 20 > $O/rr_C5.json 2> $O/rr_C5.err
rc=$?; echo "rr C5 rc=$rc"; cat $O/rr_C5.json; fatal $rc rrC5
timeout -k 10 100 python tools/rr_hang.py --torch --iters 14 > $O/hang_torch.log 2>&1
rc=$?; echo "rr under torch's runtime rc=$rc"; tail -3 $O/hang_torch.log; fatal $rc hang
exit 0
