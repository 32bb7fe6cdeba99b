#!/usr/bin/env python3
"""HBM traffic per launch from rocprofv3 --pmc passes (FETCH_SIZE pass + WRITE_SIZE pass).

    python tools/pmc_traffic.py --fetch DIR_C --write DIR_D --out profiles/r1_pmc.json

Each DIR holds the run_counter_collection.csv of one `rocprofv3 --pmc ...` run of bench.py
(scripts/gpu_pmc.sh).  Per MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are in KiB
(rocprofv3 derived counters); on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced
streaming read, so it is doubled; WRITE_SIZE is taken as is.  Values are averaged over the
dispatches of each kernel symbol; bench.py looks the dominant kernel up by its device symbol.
"""
import argparse
import collections
import csv
import glob
import json
import os


def per_kernel(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    acc = collections.defaultdict(list)
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row["Counter_Name"] != counter:
                    continue
                name = row["Kernel_Name"]
                acc[name].append(float(row["Counter_Value"]))
    return {k: (sum(v) / len(v), len(v)) for k, v in acc.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    fe = per_kernel(a.fetch, "FETCH_SIZE")
    wr = per_kernel(a.write, "WRITE_SIZE")
    out = {"source": "rocprofv3 --pmc FETCH_SIZE (x2, gfx950 correction) + --pmc WRITE_SIZE, KiB -> bytes",
           "kernels": {}}
    for k in sorted(set(fe) | set(wr)):
        f_kib, nf = fe.get(k, (0.0, 0))
        w_kib, nw = wr.get(k, (0.0, 0))
        out["kernels"][k] = {
            "fetch_bytes_per_launch": round(2 * f_kib * 1024),
            "write_bytes_per_launch": round(w_kib * 1024),
            "hbm_bytes_per_launch": round(2 * f_kib * 1024 + w_kib * 1024),
            "dispatches": [nf, nw],
        }
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    json.dump(out, open(a.out, "w"), indent=1)
    print(f"{len(out['kernels'])} kernels -> {a.out}")


if __name__ == "__main__":
    main()
