#!/bin/bash
# Round-2 final evidence: kernel traces + eval traffic PMC for M, C4, C5, R, the default bench
# line, and per-config bench lines.  Stops at the first failing step.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
bash tools/gpu_profile.sh r2b_M M --steps 20 --warmup 5 || exit $?
bash tools/gpu_profile.sh r2b_C4 C4 --steps 10 --warmup 3 || exit $?
bash tools/gpu_profile.sh r2b_C5 C5 --steps 20 --warmup 5 || exit $?
bash tools/gpu_profile.sh r2b_R R --steps 20 --warmup 5 || exit $?
bash tools/gpu_quick.sh "" "C2 C3" r2b || exit $?
timeout -k 10 400 python bench.py > gpurun_out/bench_r2b.json 2> gpurun_out/bench_r2b.err || exit $?
cat gpurun_out/bench_r2b.json
