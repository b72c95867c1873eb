#!/bin/bash
# Round-robin evidence: throughput sweep over T at M and at the 100k CPU-baseline sample, and a
# kernel trace at M, T = 16.  usage: bash tools/gpu_rr_evidence.sh <tag>
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:?tag}
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/rr_bench.py --config M --threads 4,16,64,256 --iters 5 > gpurun_out/rr_${TAG}_M.json 2>&1 || exit $?
timeout -k 10 200 python -u tools/rr_bench.py --config R --threads 4,16 --iters 50 > gpurun_out/rr_${TAG}_R.json 2>&1 || exit $?
cat gpurun_out/rr_${TAG}_M.json gpurun_out/rr_${TAG}_R.json
bash tools/gpu_rr_prof.sh rrprof_$TAG 16
