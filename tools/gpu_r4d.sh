#!/bin/bash
# Round-4 round-robin check: the round-robin parity tests, throughput at M (T=16, 4), a kernel
# trace of it, then the default bench line (with its round-robin line and CPU baseline).
# Stops after a crash or a time limit.  usage: bash tools/gpu_r4d.sh <tag>
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r4d}
O=gpurun_out/$T
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_round_robin.py -m gpu -v --maxfail=5 --timeout 200 --timeout-method thread > $O/pytest_rr.log 2>&1
rc=$?; echo "pytest rr rc=$rc"; grep -E "FAILED|ERROR" $O/pytest_rr.log | head -20; tail -3 $O/pytest_rr.log; fatal $rc pytest
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/rr_bench.py --config M --threads 16,4 --iters 10 --warmup 2 > $O/rr_M.json 2> $O/rr_M.err
rc=$?; echo "rr rc=$rc"; cat $O/rr_M.json; fatal $rc rr
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rr_trace -o run -- \
    python3 tools/rr_bench.py --config M --threads 16 --iters 3 --warmup 1 > $O/rr_trace.json 2> $O/rr_trace.err
rc=$?; echo "rr trace rc=$rc"; fatal $rc rrtrace
python -c "import csv,glob,sys; f=glob.glob(sys.argv[1]+\"/**/*kernel_stats.csv\",recursive=True); [print(r[\"Name\"][:60], r[\"Calls\"], r[\"AverageNs\"]) for r in csv.DictReader(open(f[0]))][:0] if f else print(\"no stats\")" $O/rr_trace | head -30
timeout -k 10 300 python bench.py > $O/bench_full.json 2> $O/bench_full.err
rc=$?; echo "bench (with the round-robin line) rc=$rc"; tail -5 $O/bench_full.err; head -c 1500 $O/bench_full.json; fatal $rc bench_full
exit 0
