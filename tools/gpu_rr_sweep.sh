#!/bin/bash
# Round-robin GPU tests, then throughput over T at M, C2 and C5 (steady state after 20
# warm-up iterations).  usage: bash tools/gpu_rr_sweep.sh <tag>
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${1:-rrs}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_round_robin.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/pytest_rr.log 2>&1
rc=$?; echo "pytest rr rc=$rc"; tail -2 $O/pytest_rr.log; [ $rc -ne 0 ] && exit $rc
for cfg in M C2 C5; do
  timeout -k 10 300 python tools/rr_bench.py --config $cfg --threads 4,16,64 --iters 20 --warmup 20 > $O/rr_$cfg.json 2> $O/rr_$cfg.err
  rc=$?; echo "$cfg rc=$rc"; cat $O/rr_$cfg.json; [ $rc -ne 0 ] && exit $rc
done
exit 0
