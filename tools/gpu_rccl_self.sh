#!/bin/bash
# The multi-GPU exchange path over a one-rank RCCL communicator (library loaded before torch)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --rccl-self --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/bench_rccl_self.json 2> gpurun_out/bench_rccl_self.err
rc=$?; echo "rccl-self rc=$rc"; tail -3 gpurun_out/bench_rccl_self.err
python -c "import json; d=json.load(open('gpurun_out/bench_rccl_self.json')); print(d['resample_iters_per_s'], d['config']['exchange'], d['graphs'], d['phase_ms'])"
exit $rc
