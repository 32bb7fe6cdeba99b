#!/usr/bin/env python3
"""Per-dispatch table of a rocprofv3 --pmc run (run_counter_collection.csv): one row per kernel
dispatch of the LAST training step of bench.py --no-graph, in launch order, with every counter
of the pass and derived columns when their inputs are present:

  l2_hit%    TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum)
  rd_MB      memory-side read bytes, 64*(TCC_EA0_RDREQ - TCC_EA0_RDREQ_32B) + 32*TCC_EA0_RDREQ_32B
             (the gfx950 halving of FETCH_SIZE for wide streaming reads is in
             MI355X_MICROARCH.md §HBM — treat rd_MB as a relative measure between variants)
  mfma%      SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE * 256 CUs)

    python tools/pmc_dispatch.py gpurun_out/l2a [--last N] [--kernel SUBSTR]
"""
import argparse
import collections
import csv
import glob
import os


def load(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    disp = collections.OrderedDict()
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = int(row["Dispatch_Id"])
                e = disp.setdefault(k, {"name": row["Kernel_Name"], "grid": int(row["Grid_Size"]),
                                        "vgpr": int(row["VGPR_Count"]), "agpr": int(row.get("Accum_VGPR_Count", 0) or 0),
                                        "lds": int(row["LDS_Block_Size"]), "c": {}})
                e["c"][row["Counter_Name"]] = e["c"].get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
    return [disp[k] for k in sorted(disp)]


def short(name):
    n = name.split("(")[0]
    for pre in ("void ", "vae::", "(anonymous namespace)::"):
        n = n.replace(pre, "")
    return n[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--last", type=int, default=80)
    ap.add_argument("--kernel", default="")
    ap.add_argument("--dedupe", action="store_true")
    a = ap.parse_args()
    rows = [r for r in load(a.dir) if a.kernel in r["name"]]
    if a.dedupe:       # bench.py times each call 20x back to back after the step: keep one of each run
        out = []
        for r in rows:
            if out and out[-1]["name"] == r["name"] and out[-1]["grid"] == r["grid"]:
                continue
            out.append(r)
        rows = out
    rows = rows[-a.last:]
    keys = sorted({k for r in rows for k in r["c"]})
    print(f"{'kernel':60s} {'grid':>8s} {'vgpr':>4s} " + " ".join(f"{k[:14]:>14s}" for k in keys) + "  derived")
    for r in rows:
        c = r["c"]
        der = []
        if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
            tot = c["TCC_HIT_sum"] + c["TCC_MISS_sum"]
            der.append(f"l2_hit {100 * c['TCC_HIT_sum'] / tot:5.1f}%" if tot else "l2_hit -")
        if "TCC_EA0_RDREQ_sum" in c and "TCC_EA0_RDREQ_32B_sum" in c:
            rd = 64 * (c["TCC_EA0_RDREQ_sum"] - c["TCC_EA0_RDREQ_32B_sum"]) + 32 * c["TCC_EA0_RDREQ_32B_sum"]
            der.append(f"rd {rd / 1e6:7.2f} MB")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c and "GRBM_GUI_ACTIVE" in c and c["GRBM_GUI_ACTIVE"]:
            der.append(f"mfma {100 * c['SQ_VALU_MFMA_BUSY_CYCLES'] / (c['GRBM_GUI_ACTIVE'] * 256):5.1f}%")
        print(f"{short(r['name']):60s} {r['grid']:8d} {r['vgpr']:4d} " +
              " ".join(f"{c.get(k, 0):14.0f}" for k in keys) + "  " + "  ".join(der))


if __name__ == "__main__":
    main()
