#!/bin/bash
# Kernel attributes set at create: the full GPU suite, then the round robin at M under torch's
# bundled HIP runtime (the stall of DESIGN.md §10), then the default bench line.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${1:-r4g}
O=gpurun_out/$T
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=10 --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR" $O/pytest.log | head -20; tail -2 $O/pytest.log; fatal $rc pytest
[ $rc -ne 0 ] && exit $rc
timeout -k 10 100 python tools/rr_hang.py --torch --iters 14 > $O/hang_torch.log 2>&1
rc=$?; echo "rr under torch's runtime rc=$rc"; tail -4 $O/hang_torch.log; fatal $rc hang
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; tail -2 $O/bench.err
python -c "import json,sys; d=json.load(open(sys.argv[1])); g=d.get('gpu_same_mis_as_cpu_baseline') or {}; print(d['resample_iters_per_s'], d['trajectory_check']['match'], g.get('resample_iters_per_s'), (g.get('trajectory_check') or {}).get('match'))" $O/bench.json
exit $rc
