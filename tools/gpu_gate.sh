#!/bin/bash
# GPU gate of a tree: the full GPU parity suite, smoke(), the default bench line (both
# trajectory checks), and the one-rank RCCL exchange path.  Stops after a crash, an abort or a
# time limit.  usage: bash tools/gpu_gate.sh <tag> [pytest -k expression]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-gate}; K=${2:-}
O=gpurun_out/$T
mkdir -p $O
if [ -n "$K" ]; then KA=(-k "$K"); else KA=(); fi
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --maxfail=10 --timeout 300 --timeout-method thread "${KA[@]}" \
    > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR" $O/pytest.log | head -20; tail -2 $O/pytest.log; fatal $rc pytest
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $O/smoke.log; fatal $rc smoke
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; tail -2 $O/bench.err; fatal $rc bench
python tools/bench_brief.py $O/bench.json
timeout -k 10 300 python bench.py --rccl-self --no-cpu-baseline --steps 20 --warmup 3 > $O/bench_rccl_self.json \
    2> $O/bench_rccl_self.err
rc=$?; echo "rccl-self rc=$rc"; fatal $rc rcclself
python tools/bench_brief.py $O/bench_rccl_self.json
exit $rc
