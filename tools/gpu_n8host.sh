#!/bin/bash
# Rehearsal of the 8-GPU configs on one GPU: `bench.py --gpus 8` with 8 ranks on the one
# device (ALLL_BENCH_SAME_DEVICE=1) over the host-staged gloo exchange, every rank laying out
# and evaluating its own clause shard; the line checks itself against the committed oracle
# trajectory of the config.  usage: bash tools/gpu_n8host.sh <tag> "<configs>" [steps] [warmup]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${1:-n8}; CFGS=${2:-C4 C5}; S=${3:-3}; W=${4:-1}
O=gpurun_out/$T
mkdir -p $O
for c in $CFGS; do
  ALLL_BENCH_SAME_DEVICE=1 timeout -k 10 900 python bench.py --gpus 8 --config $c --exchange-impl host \
      --steps $S --warmup $W --no-cpu-baseline --event-iters 0 > $O/bench_${c}_n8host.json 2> $O/bench_${c}_n8host.err
  rc=$?; echo "$c rc=$rc"; tail -3 $O/bench_${c}_n8host.err
  case $rc in 0) ;; *) exit $rc;; esac
  python tools/bench_brief.py $O/bench_${c}_n8host.json
done
