"""Per-kernel floor table of the loop's kernels: rocprofv3 kernel-trace durations next to the
PMC counters of the same kernels (tools/gpu_pmc_mis.sh passes), the measured HBM-side bytes per
launch and the bandwidth they imply, as a fraction of the 6.3 TB/s a streaming kernel reaches
on MI355X (MI355X_MICROARCH.md) and of the 8 TB/s peak.

FETCH_SIZE is doubled (gfx950 wide-stream correction, MI355X_MICROARCH.md §HBM); WRITE_SIZE is
taken as reported.  Both count Infinity-Cache hits, so for a kernel whose data stays in the
256 MB MALL they over-state HBM traffic: the "MB/launch" column is an upper bound.

usage: python tools/floor_table.py <pmc dir> <trace dir> [--md]
"""
import collections
import csv
import glob
import statistics
import sys

ACHIEVABLE = 6.3e12
PEAK = 8.0e12


def short(name):
    return name.split("(")[0].replace("void alll::", "").replace("alll::", "")


def counters(d):
    res = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{d}/p*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            res[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: statistics.median(v) for c, v in d2.items()} for k, d2 in res.items()}


def durations(d):
    out = {}
    for f in glob.glob(f"{d}/**/*kernel_stats.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            out[short(r["Name"])] = (int(r["Calls"]), float(r["AverageNs"]) / 1e3)
    return out


def main():
    pmc, tr = counters(sys.argv[1]), durations(sys.argv[2])
    md = "--md" in sys.argv
    rows = []
    for k, c in pmc.items():
        if k not in tr:
            continue
        calls, us = tr[k]
        fetch = 2 * c.get("FETCH_SIZE", 0.0) * 1024
        write = c.get("WRITE_SIZE", 0.0) * 1024
        byt = fetch + write
        bw = byt / (us * 1e-6) if us > 0 else 0.0
        cyc = c.get("SQ_WAVE_CYCLES", 0.0)
        wait = c.get("SQ_WAIT_ANY", 0.0) / cyc if cyc else float("nan")
        rows.append((us * calls, k, calls, us, fetch / 1e6, write / 1e6, bw / 1e12, bw / ACHIEVABLE, bw / PEAK, wait,
                     c.get("SQ_INSTS_VALU", 0.0), c.get("SQ_INSTS_VMEM_RD", 0.0) + c.get("SQ_INSTS_VMEM_WR", 0.0),
                     byt / ACHIEVABLE * 1e6))
    rows.sort(reverse=True)
    hdr = ("kernel", "calls", "avg us", "fetch MB", "write MB", "TB/s", "of 6.3", "of 8", "wait frac", "VALU",
           "VMEM", "floor us")
    if md:
        print("| " + " | ".join(hdr) + " |")
        print("|" + "---|" * len(hdr))
    else:
        print(("{:28s}" + " {:>9s}" * (len(hdr) - 1)).format(*hdr))
    for r in rows:
        _, k, calls, us, f, w, tbs, fa, fp, wait, valu, vmem, floor = r
        vals = (k, str(calls), f"{us:.1f}", f"{f:.2f}", f"{w:.2f}", f"{tbs:.2f}", f"{fa:.2f}", f"{fp:.2f}",
                f"{wait:.2f}", f"{valu:.0f}", f"{vmem:.0f}", f"{floor:.1f}")
        if md:
            print("| " + " | ".join(vals) + " |")
        else:
            print(("{:28s}" + " {:>9s}" * (len(hdr) - 1)).format(*vals))


if __name__ == "__main__":
    main()
