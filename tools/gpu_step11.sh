#!/bin/bash
# default bench line (with CPU baseline) + rocprofv3 profile of config M
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench11.json 2> gpurun_out/bench11.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench11.json; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_profile.sh r1_M M
