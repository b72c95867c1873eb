cd "${GRAFT_REPO_ROOT:-/root/repo}"
for g in 4 6 8 10; do
  echo "G=$g"; timeout -k 10 200 python bench.py --no-cpu-baseline --event-iters 0 --config C5 --grid-rounds $g 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); p=d['phase_ms']; print('iters/s %.0f mis %.1f rounds %d' % (d['resample_iters_per_s'], p['mis_ms']*1e3, d['lfmis_rounds_max']))"
done
