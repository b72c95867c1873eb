cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/pytest_full_s4.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_full_s4.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_quick.sh "" "M C5" s4
