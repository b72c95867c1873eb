#!/bin/bash
# Round-end evidence set: kernel traces + eval traffic PMC for M, C4,
# C5, R, the eval issue/wait/TA counters at M, the one-rank RCCL bench line, per-config bench
# lines and the default bench line (with the CPU baseline).  Stops at the first failing step.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:?set TAG, e.g. TAG=r3b}
bash tools/gpu_profile.sh ${T}_M M --steps 20 --warmup 5 || exit $?
bash tools/gpu_profile.sh ${T}_C4 C4 --steps 10 --warmup 3 || exit $?
bash tools/gpu_profile.sh ${T}_C5 C5 --steps 20 --warmup 5 || exit $?
bash tools/gpu_profile.sh ${T}_R R --steps 20 --warmup 5 || exit $?
bash tools/gpu_pmc_eval2.sh || exit $?
bash tools/gpu_quick.sh "" "C2 C3" $T || exit $?
timeout -k 10 200 python bench.py --rccl-self --no-cpu-baseline --steps 40 --warmup 5 --event-iters 0 \
    > gpurun_out/bench_${T}_rccl_self.json 2> gpurun_out/bench_${T}_rccl_self.err || exit $?
timeout -k 10 400 python bench.py > gpurun_out/bench_${T}.json 2> gpurun_out/bench_${T}.err || exit $?
cat gpurun_out/bench_${T}.json
