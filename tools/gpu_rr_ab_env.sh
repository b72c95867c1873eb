#!/bin/bash
# Round-robin throughput at M under environment variants (one process per variant, alternating
# twice): usage: bash tools/gpu_rr_ab_env.sh <tag> "<VAR=a VAR=b ...>" [threads]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${1:-ab}; VARS=${2:-}; TH=${3:-16}
O=gpurun_out/$T
mkdir -p $O
for rep in 1 2; do
  for v in $VARS; do
    env $v timeout -k 10 200 python tools/rr_bench.py --config M --threads $TH --warmup 20 --iters 20 \
        > $O/ab_${v}_$rep.json 2> $O/ab_${v}_$rep.err
    rc=$?; [ $rc -eq 0 ] || { echo "$v rc=$rc"; tail -3 $O/ab_${v}_$rep.err; exit $rc; }
    echo "$v $rep $(cat $O/ab_${v}_$rep.json)"
  done
done
