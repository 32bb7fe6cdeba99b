"""The C-ABI library loads (no GPU work) and exports exactly what include/vaehip.h declares."""
import ctypes
import os
import re

from vae_amd import _lib as L

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "vaehip.h")


def declared_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^(?:int|int32_t|int64_t|const char\*)\s+(vae_\w+)\(", src, flags=re.M)))


def test_library_loads_and_abi_version():
    lib = L.load()
    assert lib.vae_abi_version() == L.ABI_VERSION


def test_every_declared_symbol_is_exported_and_bound():
    lib = ctypes.CDLL(L.LIB_PATH)
    decl = declared_functions()
    assert len(decl) >= 18
    for name in decl:
        assert hasattr(lib, name), name
    assert sorted(L.EXPORTED) == decl


def test_struct_sizes_match_header_layout():
    # field order mirrors vaehip.h; a mismatch would shift every pointer after it
    assert ctypes.sizeof(L.Xform) == 6 * 4 + 10 * 8 + 2 * 4 + 3 * 8      # ... dgamma_out, dbeta_out, table
    assert L.ConvArgs.wt.offset > L.ConvArgs.x_xf.offset


def test_bad_arguments_fail_loudly_without_gpu():
    lib = L.load()
    a = L.ConvArgs()  # all zero: bad geometry, rejected before any launch
    rc = lib.vae_conv2d_fwd(ctypes.byref(a), None)
    assert rc != 0
    assert b"conv2d_fwd" in lib.vae_last_error()


def test_activation_backward_epilogue_without_aux_is_rejected():
    """A NULL pre-activation pointer in a backward epilogue is an argument error, not a fault."""
    lib = L.load()
    a = L.ConvArgs(dtype=L.F32, n=1, h=4, w=4, c=8, k=8, p=2, q=2, r=3, stride=2, pad=1)
    a.dy = 1 << 20
    a.wt = 1 << 20
    a.dx = 1 << 20
    a.dx_epi = L.Xform(kind=L.X_ACT, channels=8, slope=0.01)
    rc = lib.vae_conv2d_bwd_data(ctypes.byref(a), None)
    assert rc == -1 and b"aux" in lib.vae_last_error()


def test_build_digest_names_the_sources():
    """vae_build_digest() = sha256 (16 hex) of the csrc sources + vaehip.h the library was built
    from (Makefile); profiles/ summaries carry it and bench.py pairs them by it."""
    import glob
    import hashlib
    lib = L.load()
    d = lib.vae_build_digest().decode()
    assert re.fullmatch(r"[0-9a-f]{16}", d)
    csrc = os.path.join(os.path.dirname(HEADER), "..", "pytorch-vae_amd", "csrc")
    files = sorted(glob.glob(os.path.join(csrc, "*.hip")) + glob.glob(os.path.join(csrc, "*.hpp")),
                   key=lambda p: os.path.basename(p)) + [HEADER]
    h = hashlib.sha256(b"".join(open(f, "rb").read() for f in files)).hexdigest()[:16]
    assert d == h, "libvaehip.so is stale: rebuild (make -C pytorch-vae_amd/csrc)"


def test_launch_log_without_gpu():
    """The launch log records nothing for a call rejected before launching, and reports the
    size of an empty listing."""
    lib = L.load()
    assert lib.vae_launch_log(1) == 0
    a = L.ConvArgs()
    assert lib.vae_conv2d_fwd(ctypes.byref(a), None) != 0
    assert lib.vae_launch_log(0) == 0
    assert lib.vae_launch_log_names(None, 0) == 1
