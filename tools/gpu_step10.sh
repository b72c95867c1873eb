#!/bin/bash
# parity tests (fast subset first), then bench on M with and without the bucketed round 0
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q > gpurun_out/pytest_gpu10.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_gpu10.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench10.json 2> gpurun_out/bench10.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench10.json; tail -3 gpurun_out/bench10.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof10 -o run -- python3 bench.py --no-cpu-baseline --steps 20 > gpurun_out/bench10p.json 2>&1
rc=$?; echo "prof rc=$rc"; python3 tools/prof_summary.py gpurun_out/prof10 M 2>&1 | head -16
