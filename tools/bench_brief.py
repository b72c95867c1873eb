"""One line per bench JSON file: iterations/s, ms per step, phases, trajectory checks, roofline,
round-robin line, streaming line and CPU baseline.  usage: python tools/bench_brief.py <bench.json>..."""
import json
import sys

for path in sys.argv[1:]:
    try:
        d = json.loads(open(path).read().strip().splitlines()[-1])
    except (OSError, ValueError, IndexError) as e:
        print(f"{path}: unreadable ({e})")
        continue
    ph = d.get("phase_ms") or {}
    rf = d.get("roofline") or {}
    rr = d.get("gpu_same_mis_as_cpu_baseline") or {}
    tc = (d.get("trajectory_check") or {}).get("match")
    rtc = (rr.get("trajectory_check") or {}).get("match")
    sl = d.get("stream_line") or {}
    slc = (sl.get("check") or {}).get("match")
    print(f"{path}: {d.get('config', {}).get('workload', '?')[:3]} n={d.get('n_gpus')} "
          f"it/s={d.get('resample_iters_per_s') or 0:.1f} ms/step={d.get('ms_per_step') or 0:.4f} "
          f"eval/xchg/mis/res={ph.get('eval_ms', 0):.4f}/{ph.get('exchange_ms', 0):.4f}/{ph.get('mis_ms', 0):.4f}/"
          f"{ph.get('resample_ms', 0):.4f} match={tc} frac={rf.get('frac', 0):.3f} "
          f"(loop {rf.get('frac_in_loop') or 0:.3f}) rr_it/s={rr.get('resample_iters_per_s')} rr_match={rtc} "
          f"stream_it/s={sl.get('resample_iters_per_s')} stream_match={slc} "
          f"cpu={(d.get('cpu_baseline') or {}).get('value')}")
