"""Summarise a tools/gpu_profile.sh output directory: per-kernel stats from the kernel trace
and per-launch HBM bytes of the eval kernel from the PMC passes (gfx950 correction: FETCH_SIZE
reads half the bytes of a wide coalesced stream -- MI355X_MICROARCH.md §HBM -- so it is doubled;
WRITE_SIZE is used as reported).  Writes <dir>/pmc_eval_traffic.json."""
import csv
import glob
import json
import os
import statistics
import sys

d = sys.argv[1]
config = sys.argv[2] if len(sys.argv) > 2 else "M"


def rows(pattern):
    out = []
    for f in glob.glob(os.path.join(d, pattern), recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


stats = rows("trace/**/*kernel_stats.csv")
print("== kernel stats (rocprofv3 --kernel-trace --stats)")
for r in sorted(stats, key=lambda r: -float(r.get("TotalDurationNs", 0)))[:20]:
    print(f"{r['Name'][:60]:60s} calls={r['Calls']:>6s} avg_ns={float(r['AverageNs']):12.1f} "
          f"total_ms={float(r['TotalDurationNs'])/1e6:9.3f} pct={float(r['Percentage']):6.2f}")

res = {}
for name in ("FETCH_SIZE", "WRITE_SIZE", "TCC_HIT_sum", "TCC_MISS_sum"):
    vals = {}
    for r in rows(f"pmc_*/**/*counter_collection.csv"):
        if r.get("Counter_Name") == name and "k_eval" in r.get("Kernel_Name", ""):
            vals.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
    for k, v in vals.items():
        res.setdefault(k, {})[name] = statistics.median(v)
print("== PMC (median per launch)")
for k, v in res.items():
    print(k[:80], v)
    if "FETCH_SIZE" in v and "WRITE_SIZE" in v:
        fetch_b = 2 * v["FETCH_SIZE"] * 1024
        write_b = v["WRITE_SIZE"] * 1024
        v["hbm_bytes_per_launch"] = fetch_b + write_b
        print(f"   corrected HBM bytes/launch: read {fetch_b/1e6:.1f} MB + write {write_b/1e6:.1f} MB")
    if "TCC_HIT_sum" in v:
        v["l2_hit_rate"] = v["TCC_HIT_sum"] / max(1.0, v["TCC_HIT_sum"] + v["TCC_MISS_sum"])
        print(f"   L2 hit rate {v['l2_hit_rate']:.3f}")
# bench-format record (bench.py --traffic-json): the roofline's kernel, the evaluation alone
# (k_eval_hybrid / k_eval_ragged / ...: not the fused k_eval_scatter, whose bytes include the
# round-0 scatter); the other kernels stay under per_kernel
out = {"config": config, "n_gpus": 1, "per_kernel": res}
main = [k for k in res if "hbm_bytes_per_launch" in res[k]]
alone = [k for k in main if "k_eval_scatter" not in k]
if alone:
    main = alone
if main:
    k = max(main, key=lambda k: res[k]["hbm_bytes_per_launch"])
    out.update(kernel=k, hbm_bytes_per_launch=res[k]["hbm_bytes_per_launch"],
               fetch_bytes=2 * res[k]["FETCH_SIZE"] * 1024, write_bytes=res[k]["WRITE_SIZE"] * 1024,
               correction="FETCH_SIZE x2 (gfx950 wide-stream undercount), KiB units")
    for r in stats:
        if r["Name"].startswith(k.split("(")[0]):
            out["trace_avg_ns"] = float(r["AverageNs"])
            out["trace_calls"] = int(r["Calls"])
json.dump(out, open(os.path.join(d, "pmc_eval_traffic.json"), "w"), indent=1)
print(json.dumps({k: v for k, v in out.items() if k != "per_kernel"}))
