#!/usr/bin/env python3
"""Per-kernel resources of the built objects (diagnostic): VGPRs, AGPRs, static LDS and the
resulting waves per SIMD, read from the gfx950 code objects embedded in build/*.o.

    python3 tools/kres.py [filter-substring]
"""
import glob
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/llvm/bin"
BUILD = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "pytorch-vae_amd", "csrc", "build")


def code_object(obj, tmp):
    fat = os.path.join(tmp, "fat.bin")
    subprocess.run([f"{LLVM}/llvm-objcopy", "--dump-section", f".hip_fatbin={fat}", obj, os.path.join(tmp, "x.o")],
                   check=True, capture_output=True)
    co = os.path.join(tmp, "co.o")
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", "--input=" + fat, "--output=" + co,
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950"], check=True, capture_output=True)
    return co


def kernels(co):
    out = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True, text=True).stdout
    for blk in out.split("- .agpr_count:")[1:]:
        def f(key):
            m = re.search(r"\." + key + r":\s+(\S+)", blk)
            return m.group(1) if m else None
        yield {"name": f("name"), "vgpr": int(f("vgpr_count") or 0), "agpr": int(re.match(r"\s*(\d+)", blk).group(1)),
               "lds": int(f("group_segment_fixed_size") or 0), "scratch": int(f("private_segment_fixed_size") or 0), "sgpr": int(f("sgpr_count") or 0)}


def main():
    flt = sys.argv[1] if len(sys.argv) > 1 else ""
    seen = set()
    with tempfile.TemporaryDirectory() as tmp:
        for obj in sorted(glob.glob(os.path.join(BUILD, "vae_*.o"))):
            for k in kernels(code_object(obj, tmp)):
                if flt not in (k["name"] or "") or k["name"] in seen:
                    continue
                seen.add(k["name"])
                regs = ((k["vgpr"] + 7) // 8) * 8 + ((k["agpr"] + 7) // 8) * 8 if k["agpr"] else ((k["vgpr"] + 7) // 8) * 8
                w_reg = min(8, 512 // max(regs, 1))
                w_lds = min(8, (163840 // max(k["lds"], 1)) * 4 // 4) if k["lds"] else 8
                name = subprocess.run(["c++filt", k["name"]], capture_output=True, text=True).stdout.strip()
                print(f"{k['vgpr']:4d}v {k['agpr']:3d}a {k['lds']:6d}B {k['scratch']:4d}S  waves/SIMD<=reg {w_reg} lds-wg/CU {w_lds}  {name[:150]}")


if __name__ == "__main__":
    main()
