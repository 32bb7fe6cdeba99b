#!/usr/bin/env python3
"""rocprofv3 --kernel-trace --stats output of one bench command -> a per-kernel JSON summary stamped
with the build it measured (bench.py pairs a call's kernels with a summary of the same build only).

    python3 tools/prof_summary.py --dir gpurun_out/TAG_prof --out profiles/r4_v0_kstats.json \
        --config "bench.py --steps 20 ..."

Per kernel (full demangled name as rocprofv3 writes it): calls, average / min / max duration (us)
and the share of kernel time, from the *_kernel_stats.csv under --dir.
"""
import argparse
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import build_identity  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--config", default="")
    args = ap.parse_args()
    files = glob.glob(os.path.join(args.dir, "**", "*kernel_stats.csv"), recursive=True)
    if not files:
        sys.exit(f"no *kernel_stats.csv under {args.dir}")
    kernels = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            kernels[r["Name"]] = {"calls": int(r["Calls"]), "avg_us": round(float(r["AverageNs"]) / 1e3, 3),
                                  "min_us": round(float(r["MinNs"]) / 1e3, 3),
                                  "max_us": round(float(r["MaxNs"]) / 1e3, 3),
                                  "pct": round(float(r["Percentage"]), 3)}
    digest, head = build_identity()
    out = {"config": args.config, "source": files, "digest": digest, "head": head,
           "kernels": dict(sorted(kernels.items(), key=lambda kv: -kv[1]["pct"]))}
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    json.dump(out, open(args.out, "w"), indent=1)
    print(f"{len(kernels)} kernels -> {args.out} (digest {digest}, head {head})")


if __name__ == "__main__":
    main()
