#!/usr/bin/env python3
"""Every kernel the timed steps run, mapped to the passing GPU tests that pin it.

    python3 tools/kernel_coverage.py [--kstats profiles/r6_*kstats*.json] [--coverage profiles/r6_coverage_*.json]

Inputs:
  * rocprofv3 kernel summaries of bench.py runs (tools/prof_summary.py: one per BASELINE
    configuration), the kernels the benchmark timed;
  * coverage records written by the GPU tests (gpurun_out/kernel_coverage_<config>.json, copied to
    profiles/): for each kernel the step launched (vae_launch_log), the passing checks / tests of
    the calls that launch it — tests/test_gpu_stepcheck.py (the VanillaVAE family: every op
    teacher-forced in fp64 at the bench shapes) and tests/test_gpu_bf16_shapes.py (VQ-VAE B=128,
    big_ae B=64: every gradient against the fp32 oracle under the autocast bar).

Prints, per summary, each library kernel with the tests that pin it, and exits non-zero when a kernel
of a summary has none (torch's own kernels of the bench's setup are not the library's and are listed
apart).  A summary is matched with the coverage records of its own configuration (its bench
arguments: --arch / --batch).  Library kernels launched fewer times than the summary's warmup + timed
steps ran outside the step — the plan's setup and restore copies, bench.py's per-call timing of the
op-by-op prologue — and are listed apart."""
import argparse
import glob
import json
import os
import re
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# bench.py configuration -> coverage record tag (the GPU test's config of the same workload)
CONFIG_TAG = {("vanilla", 64): "vanilla_64", ("betaH", 32): "betaH_32", ("iwae", 64): "iwae_64",
              ("vq", 128): "vq_128", ("ae_big", 64): "ae_big_64"}


def workload(d):
    toks = str(d.get("config") or "").split()
    arch, batch, steps, warmup = "vanilla", 64, 0, 0
    for i, t in enumerate(toks[:-1]):
        if t == "--arch":
            arch = toks[i + 1]
        elif t == "--batch":
            batch = int(toks[i + 1])
        elif t == "--steps":
            steps = int(toks[i + 1])
        elif t == "--warmup":
            warmup = int(toks[i + 1])
    return arch, batch, steps + warmup


def is_library_kernel(name: str) -> bool:
    return ("vae::" in name or name.startswith("(anonymous namespace)::") or "_ZN3vae" in name
            or "anonymous namespace" in name) and "at::" not in name


def norm(name: str) -> str:
    return re.sub(r"\s+", " ", name).strip()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kstats", nargs="*", default=None)
    ap.add_argument("--coverage", nargs="*", default=None)
    ap.add_argument("--round", default="r6")
    args = ap.parse_args()
    kst = args.kstats or sorted(glob.glob(os.path.join(REPO, "profiles", f"{args.round}_*kstats*.json")))
    cov_files = args.coverage or sorted(glob.glob(os.path.join(REPO, "profiles", f"{args.round}_coverage_*.json")))
    cov = {}
    for f in cov_files:
        d = json.load(open(f))
        tag = re.sub(r"^.*coverage_", "", os.path.basename(f)).replace(".json", "")
        m = cov.setdefault(tag, {})
        for k, tests in d.get("coverage", {}).items():
            if tests:
                m.setdefault(norm(k), set()).add(d.get("test", f))
    bad = 0
    for f in kst:
        d = json.load(open(f))
        arch, batch, steps = workload(d)
        wl = (arch, batch)
        tag = CONFIG_TAG.get(wl)
        m = cov.get(tag, {}) if tag else {}
        kern = d.get("kernels", {})
        # a kernel launched fewer times than the warmup + timed steps is not part of the step: bench.py's
        # per-call timing pass (the op-by-op prologue calls) and the plan's setup / restore copies
        setup = [k for k in kern if is_library_kernel(k) and kern[k].get("calls", steps) < steps]
        lib = [k for k in kern if is_library_kernel(k) and k not in setup]
        other = [k for k in kern if not is_library_kernel(k)]
        print(f"== {os.path.relpath(f, REPO)}  ({wl[0]} B={wl[1]}; digest {d.get('digest')}; coverage {tag})")
        for k in lib:
            tests = sorted(m.get(norm(k), []))
            if not tests:
                bad += 1
            print(f"  {'ok ' if tests else 'NO '} {k[:100]}")
            for t in tests:
                print(f"        {t}")
        for k in setup:
            print(f"  --  {k[:100]}  ({kern[k].get('calls')} launches < {steps} warmup + timed steps: outside the step)")
        if other:
            print(f"  (not library kernels, bench setup: {len(other)})")
    if not kst:
        print("no kernel summaries found")
        return 1
    print(f"{bad} library kernel(s) without a passing test")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
