cd "${GRAFT_REPO_ROOT:-/root/repo}"
for i in 1 2; do for g in ${GRIDS:-2048 1024 512}; do
  ALLL_FP_GRID=$g timeout -k 10 120 python -u tools/rr_bench.py --config M --threads 16,4 --iters 5 2>&1 | sed "s/^/grid=$g /"
done; done
