#!/bin/bash
# Round-2 checks: C4 parity at full size, the bench line, the N=2 self-launch rehearsal on one
# GPU (host exchange) and the loud failure of --gpus 2 without it.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 420 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 400 --timeout-method thread \
    -k "C4_3sat_128M or M_3sat_10M" > gpurun_out/pytest_c4.log 2>&1
rc=$?; echo "pytest C4 rc=$rc"; tail -5 gpurun_out/pytest_c4.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/bench_r2b.json 2> gpurun_out/bench_r2b.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_r2b.json | head -c 1500; echo; [ $rc -eq 0 ] || exit $rc
ALLL_BENCH_SAME_DEVICE=1 timeout -k 10 300 python bench.py --gpus 2 --exchange-impl host --no-cpu-baseline --steps 10 --warmup 2 --event-iters 0 \
    > gpurun_out/bench_n2host.json 2> gpurun_out/bench_n2host.err
rc=$?; echo "bench n2 host rc=$rc"; head -c 600 gpurun_out/bench_n2host.json; echo; tail -3 gpurun_out/bench_n2host.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --gpus 2 --no-cpu-baseline --steps 10 --warmup 2 --event-iters 0 \
    > gpurun_out/bench_n2rccl.json 2> gpurun_out/bench_n2rccl.err
echo "bench n2 rccl on a 1-GPU box (expected to fail loudly): rc=$?"; tail -4 gpurun_out/bench_n2rccl.err
exit 0
