#!/bin/bash
# Round-4 final gate: full GPU suite, smoke, the default bench line, the RCCL one-rank exchange
# path and the round robin under torch's bundled runtime.  usage: bash tools/gpu_r4i.sh <tag>
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r4i}
O=gpurun_out/$T
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=10 --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR" $O/pytest.log | head -20; tail -2 $O/pytest.log; fatal $rc pytest
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $O/smoke.log; fatal $rc smoke
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; tail -2 $O/bench.err; fatal $rc bench
python -c "import json,sys; d=json.load(open(sys.argv[1])); g=d.get('gpu_same_mis_as_cpu_baseline') or {}; print(d['resample_iters_per_s'], d['ms_per_step'], d['trajectory_check']['match'], d['roofline']['frac'], g.get('resample_iters_per_s'), (g.get('trajectory_check') or {}).get('match'), (d.get('cpu_baseline') or {}).get('value'))" $O/bench.json
timeout -k 10 300 python bench.py --rccl-self --no-cpu-baseline --steps 20 --warmup 3 > $O/bench_rccl_self.json 2> $O/bench_rccl_self.err
rc=$?; echo "rccl-self rc=$rc"; fatal $rc rcclself
timeout -k 10 100 python tools/rr_hang.py --torch --iters 14 > $O/rr_torch.log 2>&1
rc=$?; echo "rr under torch's runtime rc=$rc"; tail -2 $O/rr_torch.log
exit $rc
