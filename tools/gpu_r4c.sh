#!/bin/bash
# Round-4 evidence: M kernel trace + eval traffic PMC (tools/gpu_profile.sh), the LFMIS
# per-kernel PMC floor table at M, C4 / C5 traces, per-config bench lines, the 8-rank
# same-device create rehearsal at C4 and the default bench line.  Stops after a crash or a
# time limit.  usage: bash tools/gpu_r4c.sh <tag>
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r4c}
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; [ $1 -eq 0 ] || echo "step $2 rc=$1"; }
bash tools/gpu_profile.sh ${T}_M M --steps 20 --warmup 5; fatal $? profM
bash tools/gpu_pmc_mis.sh ${T} M > gpurun_out/pmc_mis_${T}.log 2>&1; fatal $? pmcmis
bash tools/gpu_profile.sh ${T}_C5 C5 --steps 20 --warmup 5; fatal $? profC5
bash tools/gpu_profile.sh ${T}_C4 C4 --steps 10 --warmup 3; fatal $? profC4
bash tools/gpu_quick.sh "" "C2 C3 R" $T; fatal $? quick
# 8 ranks of a sharded C4 run on this one GPU (host exchange): alll_create with every rank
# laying out its own shard, 8 processes sharing the box's CPU share
ALLL_BENCH_SAME_DEVICE=1 timeout -k 10 600 python bench.py --gpus 8 --config C4 --exchange-impl host \
    --steps 2 --warmup 1 --no-cpu-baseline --event-iters 0 > gpurun_out/bench_${T}_C4_n8host.json \
    2> gpurun_out/bench_${T}_C4_n8host.err; fatal $? c4n8
timeout -k 10 400 python bench.py > gpurun_out/bench_${T}.json 2> gpurun_out/bench_${T}.err; fatal $? bench
cat gpurun_out/bench_${T}.json | head -c 2500
exit 0
