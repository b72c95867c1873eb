#!/bin/bash
# Round-2 evidence: rocprofv3 kernel trace + eval traffic PMC for M, C4, C5, then PMC counters of
# the LFMIS kernels at M.  Stops at the first failing step.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_profile.sh r2_M M --steps 20 --warmup 5 || exit $?
bash tools/gpu_profile.sh r2_C4 C4 --steps 10 --warmup 3 || exit $?
bash tools/gpu_profile.sh r2_C5 C5 --steps 20 --warmup 5 || exit $?
bash tools/gpu_pmc_mis.sh r2 M || exit $?
