#!/usr/bin/env python3
"""Join tools/kbench.py's group list with a rocprofv3 kernel trace: per (launch, split) the
median per-launch GPU time (all kernels of the launch, e.g. GEMM + split-K finalize)."""
import csv
import json
import statistics
import sys


def main(trace_csv, groups_json):
    rows = list(csv.DictReader(open(trace_csv)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    meta = json.load(open(groups_json))
    reps = meta["reps"]
    # cut at marker kernels
    segs, cur = [], None
    for r in rows:
        if "spin_kernel" in r["Kernel_Name"]:
            if cur is not None:
                segs.append(cur)
            cur = []
        elif cur is not None:
            cur.append(r)
    out = []
    for gi, g in enumerate(meta["groups"]):
        seg = segs[gi] if gi < len(segs) else []
        n = len(seg) // reps if reps else 0
        per = []
        for k in range(reps):
            ks = seg[k * n:(k + 1) * n]
            if ks:
                per.append(sum(int(x["End_Timestamp"]) - int(x["Start_Timestamp"]) for x in ks) / 1e3)
        names = sorted({x["Kernel_Name"][:60] for x in seg})
        med = statistics.median(per) if per else float("nan")
        out.append((g["launch"], g["fn"], g["split"], n, med, names))
        print(f"{g['launch']:3d} {g['fn']:24s} split={g['split']:2d} kernels/launch={n} {med:8.2f} us  {names[0] if names else ''}")
    tot = {}
    for l, fn, s, n, med, _ in out:
        tot.setdefault(l, {})[s] = med
    best = sum(min(v.values()) for v in tot.values())
    auto = sum(v.get(0, min(v.values())) for v in tot.values())
    print(f"sum(auto split) = {auto:.1f} us   sum(best split) = {best:.1f} us")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
