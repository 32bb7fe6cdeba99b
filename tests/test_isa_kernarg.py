"""ISA check of kernarg_prefetch (vae_common.hpp), CPU only: the disassembled gfx950 code objects
of the built library, every prefetch block's destination SGPRs disjoint from its base-address
SGPRs.

Round-5 fault (profiles/r5_notes.md): with plain "=s" outputs the compiler could give a prefetch
destination one of the base registers, so a returning load overwrote the base of the next and the
fp32 Autoencoder test hit an illegal address.  The outputs are early-clobber ("=&s") since; this
test reads the machine code itself, so a change of constraint or compiler that brings the overlap
back fails here, before any GPU run."""
import os
import re
import subprocess
from concurrent.futures import ThreadPoolExecutor

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(REPO, "pytorch-vae_amd", "csrc", "build")
LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"

# s_load_dword s6, s[0:1], 0x40
LOAD = re.compile(r"s_load_dword\s+s(\d+),\s*s\[(\d+):(\d+)\],\s*0x([0-9a-f]+)")


def prefetch_blocks(asm: str):
    """Runs of kernarg-prefetch loads: consecutive `s_load_dword sD, s[a:b], k*64` lines (k = 1, 2,
    ...) closed by `s_waitcnt lgkmcnt(0)`.  Returns [(base lo, base hi, [dest regs])]."""
    blocks, cur = [], None
    for line in asm.splitlines():
        m = LOAD.search(line)
        if m:
            d, lo, hi, off = int(m.group(1)), int(m.group(2)), int(m.group(3)), int(m.group(4), 16)
            if cur is not None and (lo, hi) == cur[0] and off == 64 * (len(cur[1]) + 1):
                cur[1].append(d)
                continue
            cur = ((lo, hi), [d]) if off == 64 else None
            continue
        if cur is not None and "s_waitcnt" in line and "lgkmcnt(0)" in line:
            blocks.append((cur[0][0], cur[0][1], cur[1]))
        cur = None
    return blocks


def overlaps(blocks):
    return [(lo, hi, ds) for lo, hi, ds in blocks if any(lo <= d <= hi for d in ds)]


def test_parser_flags_an_aliased_destination():
    good = "s_load_dword s6, s[0:1], 0x40\n s_load_dword s7, s[0:1], 0x80\n s_waitcnt lgkmcnt(0)\n"
    bad = "s_load_dword s6, s[0:1], 0x40\n s_load_dword s1, s[0:1], 0x80\n s_waitcnt lgkmcnt(0)\n"
    assert prefetch_blocks(good) == [(0, 1, [6, 7])] and not overlaps(prefetch_blocks(good))
    assert overlaps(prefetch_blocks(bad)) == [(0, 1, [6, 1])]


def _disasm(obj: str, tmp: str) -> str:
    base = os.path.join(tmp, os.path.basename(obj))
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={base}.fb", obj, f"{base}.null"],
                   check=True, capture_output=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={base}.fb",
                    f"--targets={TARGET}", f"--output={base}.co"], check=True, capture_output=True)
    r = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", f"{base}.co"], check=True,
                       capture_output=True, text=True)
    return r.stdout


@pytest.mark.timeout(600)
def test_every_kernarg_prefetch_block_keeps_its_base(tmp_path):
    if not os.path.isdir(BUILD):
        pytest.skip("library not built (make -C pytorch-vae_amd/csrc)")
    objs = sorted(os.path.join(BUILD, f) for f in os.listdir(BUILD)
                  if f.endswith(".o") and f.startswith("vae_") and not f.startswith("probe_"))
    if not objs:
        pytest.skip("no objects in build/")
    with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        asms = list(ex.map(lambda o: _disasm(o, str(tmp_path)), objs))
    total, bad = 0, []
    for o, asm in zip(objs, asms):
        blocks = prefetch_blocks(asm)
        total += len(blocks)
        bad += [(os.path.basename(o),) + b for b in overlaps(blocks)]
    assert not bad, bad
    assert total >= 100, f"only {total} prefetch blocks found: the scan no longer matches the code"
