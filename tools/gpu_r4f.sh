#!/bin/bash
# Round-4 gate: the full GPU parity suite, smoke, a steady-state round-robin trace at M (T=16,
# iterations 41-43) and the default bench line.  Stops after a crash or a time limit.
# usage: bash tools/gpu_r4f.sh <tag>
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r4f}
O=gpurun_out/$T
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=10 --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR" $O/pytest.log | head -20; tail -2 $O/pytest.log; fatal $rc pytest
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $O/smoke.log; fatal $rc smoke
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rr_trace -o run -- \
    python3 tools/rr_bench.py --config M --threads 16 --iters 3 --warmup 40 > $O/rr_trace.json 2> $O/rr_trace.err
rc=$?; echo "rr trace rc=$rc"; fatal $rc rrtrace
timeout -k 10 200 python tools/rr_bench.py --config M --threads 16,4 --iters 20 --warmup 40 > $O/rr_M.json 2> $O/rr_M.err
rc=$?; echo "rr rc=$rc"; cat $O/rr_M.json; fatal $rc rr
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; tail -3 $O/bench.err
python -c "import json,sys; d=json.load(open(sys.argv[1])); print(json.dumps({k: d.get(k) for k in ('value','ms_per_step','phase_ms','trajectory_check')})[:1200]); g=d.get('gpu_same_mis_as_cpu_baseline') or {}; print(g.get('resample_iters_per_s'), (g.get('trajectory_check') or {}).get('match'))" $O/bench.json
exit $rc
