#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_round_robin.py -x -q --timeout 120 --timeout-method thread -k "fp and not cap" > gpurun_out/pytest_fp1.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_fp1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/rr_bench.py --config M --threads 16,4 --iters 5 > gpurun_out/rr_fp1.json 2>&1
rc=$?; cat gpurun_out/rr_fp1.json | tail -5; exit $rc
