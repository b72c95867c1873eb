#!/bin/bash
# Round-robin check + A/B of the grid-round count, then the default bench line.
# usage: bash tools/gpu_r4e.sh <tag>
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r4e}
O=gpurun_out/$T
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_round_robin.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/pytest_rr.log 2>&1
rc=$?; echo "pytest rr rc=$rc"; tail -2 $O/pytest_rr.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/rr_bench.py --config M --threads 16,4 --iters 10 --warmup 2 > $O/rr_M.json 2> $O/rr_M.err
rc=$?; echo "rr rc=$rc"; cat $O/rr_M.json; fatal $rc rr
for v in g2 g3; do
  ALLL_LIB_AB=build/ab/liballl_$v.so timeout -k 10 120 python tools/rr_bench.py --config M --threads 16 --iters 10 --warmup 2 > $O/rr_$v.json 2> $O/rr_$v.err
  rc=$?; echo "$v rc=$rc"; cat $O/rr_$v.json; fatal $rc $v
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rr_trace -o run -- \
    python3 tools/rr_bench.py --config M --threads 16 --iters 3 --warmup 1 > $O/rr_trace.json 2> $O/rr_trace.err
rc=$?; echo "rr trace rc=$rc"; fatal $rc rrtrace
timeout -k 10 400 python bench.py > $O/bench_full.json 2> $O/bench_full.err
rc=$?; echo "bench rc=$rc"; tail -4 $O/bench_full.err; head -c 600 $O/bench_full.json; echo
python -c "import json,sys; d=json.load(open(sys.argv[1])); print(json.dumps({k: d.get(k) for k in ('value','ms_per_step','trajectory_check','gpu_same_mis_as_cpu_baseline')})[:1500])" $O/bench_full.json
exit $rc
