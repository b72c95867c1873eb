#!/bin/bash
# first GPU check: smoke -> gpu tests (not slow) -> short bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -m pytest tests -m "gpu and not slow" -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench1.json 2> gpurun_out/bench1.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench1.json; tail -5 gpurun_out/bench1.err
exit $rc
