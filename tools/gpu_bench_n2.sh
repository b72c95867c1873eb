#!/bin/bash
# rehearsal of the 2-rank bench path on one GPU (RCCL refuses two ranks on one device, so this
# exercises the agreed fallback to the host-staged gloo exchange)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
ALLL_BENCH_SAME_DEVICE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 10 --warmup 2 --config C2 \
  > gpurun_out/bench_n2.json 2> gpurun_out/bench_n2.err
rc=$?; echo "rc=$rc"; cat gpurun_out/bench_n2.json; tail -8 gpurun_out/bench_n2.err
