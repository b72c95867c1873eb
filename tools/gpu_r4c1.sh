#!/bin/bash
# Round-4 evidence, part 1: M and C5 kernel traces + eval traffic PMC (tools/gpu_profile.sh) and
# the LFMIS per-kernel PMC passes (tools/gpu_pmc_mis.sh) at M and C5.  usage: bash tools/gpu_r4c1.sh <tag>
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r4c}
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; [ $1 -eq 0 ] || echo "step $2 rc=$1"; }
bash tools/gpu_profile.sh ${T}_M M --steps 20 --warmup 5; fatal $? profM
bash tools/gpu_pmc_mis.sh ${T} M > gpurun_out/pmc_mis_${T}_M.log 2>&1; fatal $? pmcmisM
bash tools/gpu_profile.sh ${T}_C5 C5 --steps 20 --warmup 5; fatal $? profC5
bash tools/gpu_pmc_mis.sh ${T} C5 > gpurun_out/pmc_mis_${T}_C5.log 2>&1; fatal $? pmcmisC5
exit 0
