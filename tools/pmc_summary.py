#!/usr/bin/env python3
"""Per-kernel PMC summary of one bench configuration from separate rocprofv3 --pmc passes
(scripts/gpu_r2_measure.sh: pass A = SQ counters, B = GRBM_GUI_ACTIVE + MFMA MOPS + FETCH_SIZE,
C = WRITE_SIZE + TCC hit/miss).

    python3 tools/pmc_summary.py --dirs gpurun_out/m1_pa gpurun_out/m1_pb gpurun_out/m1_pc \
        --out profiles/r2_v1_pmc.json

Per kernel symbol, averaged over its dispatches:
  hbm_bytes_per_launch = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes; MI355X_MICROARCH.md §HBM: on
                         gfx950 FETCH_SIZE reports half the bytes of a wide coalesced read)
  mfma_busy            = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)
                         (GRBM_GUI_ACTIVE is summed over the 8 XCDs; busy cycles over all SIMDs)
  mfma_flops           = SQ_INSTS_VALU_MFMA_MOPS_BF16 x 512 (rocprof's MOP unit)
  wait_frac            = SQ_WAIT_ANY / SQ_WAVE_CYCLES
plus a whole-run total (all dispatches of the vae library) for the step-level MFMA-busy figure.
Counts from a --pmc run (serialised dispatches, no graphs) — durations are NOT bench timings.
"""
import argparse
import collections
import csv
import glob
import json
import os


def load(dirs):
    per = collections.defaultdict(lambda: collections.defaultdict(list))   # kernel -> counter -> values
    dur = collections.defaultdict(dict)                                      # kernel -> dispatch -> ns
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    k = row["Kernel_Name"]
                    per[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
                    dur[k][(d, row["Dispatch_Id"])] = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
    return per, dur


def build_identity():
    """(digest, head) of the measured build: vae_build_digest() of the in-tree libvaehip.so (the
    digest of the csrc sources it was compiled from; bench.py only pairs a summary with a library of
    the same digest) and the git HEAD the tree was sent from (GIT_HEAD, set by the caller — the GPU
    box's copy of the tree has no .git; `git rev-parse` where it does)."""
    import ctypes
    import subprocess
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    try:
        lib = ctypes.CDLL(os.path.join(repo, "pytorch-vae_amd", "vae_amd", "libvaehip.so"))
        lib.vae_build_digest.restype = ctypes.c_char_p
        digest = lib.vae_build_digest().decode()
    except Exception:
        digest = None
    head = os.environ.get("GIT_HEAD") or None
    if head is None:
        try:
            head = subprocess.run(["git", "rev-parse", "--short", "HEAD"], capture_output=True, text=True,
                                  cwd=repo).stdout.strip() or None
        except Exception:
            head = None
    return digest, head


def mean(v):
    return sum(v) / len(v) if v else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dirs", nargs="+", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--config", default="")
    args = ap.parse_args()
    per, dur = load(args.dirs)
    out, tot = {}, collections.Counter()
    for k, c in per.items():
        if k.startswith(("at::", "void at::", "__amd_rocclr")) or "at::native" in k or "at::cuda" in k:
            continue                      # torch's own kernels (fills, RNG, the bench's spin)
        fetch, write = mean(c.get("FETCH_SIZE", [])), mean(c.get("WRITE_SIZE", []))
        grbm, busy = mean(c.get("GRBM_GUI_ACTIVE", [])), mean(c.get("SQ_VALU_MFMA_BUSY_CYCLES", []))
        mops = mean(c.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", []))
        wait, wcyc = mean(c.get("SQ_WAIT_ANY", [])), mean(c.get("SQ_WAVE_CYCLES", []))
        e = {"dispatches": max(len(v) for v in c.values()),
             "pmc_run_avg_us": round(mean(list(dur[k].values())) / 1e3, 2)}
        if fetch is not None and write is not None:
            e["hbm_bytes_per_launch"] = int((2 * fetch + write) * 1024)
            e["fetch_bytes_x2"] = int(2 * fetch * 1024)
            e["write_bytes"] = int(write * 1024)
        if grbm and busy is not None:
            e["mfma_busy"] = round(busy / (grbm / 8 * 1024), 4)
        if mops is not None:
            e["mfma_flops"] = mops * 512
        if wait is not None and wcyc:
            e["wait_frac"] = round(wait / wcyc, 3)
        if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
            h, m = mean(c["TCC_HIT_sum"]), mean(c["TCC_MISS_sum"])
            e["l2_hit"] = round(h / (h + m), 3) if h + m else None
        out[k] = e
        for name in ("GRBM_GUI_ACTIVE", "SQ_VALU_MFMA_BUSY_CYCLES"):
            if name in c:
                tot[name] += sum(c[name])
    digest, head = build_identity()
    summary = {"config": args.config, "sources": args.dirs, "digest": digest, "head": head,
               "all_vae_dispatches_mfma_busy": (round(tot["SQ_VALU_MFMA_BUSY_CYCLES"] /
                                                     (tot["GRBM_GUI_ACTIVE"] / 8 * 1024), 4)
                                               if tot["GRBM_GUI_ACTIVE"] else None),
               "kernels": dict(sorted(out.items(), key=lambda kv: -kv[1]["pmc_run_avg_us"] * kv[1]["dispatches"]))}
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    json.dump(summary, open(args.out, "w"), indent=1)
    print(f"{len(out)} kernels -> {args.out}; MFMA busy over all vae dispatches: {summary['all_vae_dispatches_mfma_busy']}")


if __name__ == "__main__":
    main()
