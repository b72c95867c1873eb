#!/bin/bash
# Round-4 evidence, part 2: C4 trace + eval traffic, C2 / C3 / R bench lines, the 8-rank
# same-device C4 create rehearsal (every rank lays out its own shard; host exchange) and the
# default bench line.  usage: bash tools/gpu_r4c2.sh <tag>
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r4c}
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; [ $1 -eq 0 ] || echo "step $2 rc=$1"; }
bash tools/gpu_profile.sh ${T}_C4 C4 --steps 10 --warmup 3; fatal $? profC4
bash tools/gpu_quick.sh "" "C2 C3 R" $T; fatal $? quick
ALLL_BENCH_SAME_DEVICE=1 timeout -k 10 600 python bench.py --gpus 8 --config C4 --exchange-impl host \
    --steps 2 --warmup 1 --no-cpu-baseline --event-iters 0 > gpurun_out/bench_${T}_C4_n8host.json \
    2> gpurun_out/bench_${T}_C4_n8host.err; fatal $? c4n8
timeout -k 10 400 python bench.py > gpurun_out/bench_${T}.json 2> gpurun_out/bench_${T}.err; fatal $? bench
head -c 1500 gpurun_out/bench_${T}.json
exit 0
