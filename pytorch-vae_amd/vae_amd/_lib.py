"""ctypes binding of libvaehip.so (include/vaehip.h).

The library is the product: there is no CPU or PyTorch fallback.  Loading fails loudly
when the shared object is missing, and every call raises ``VaeHipError`` with the
library's message when it returns non-zero.  torch is imported first so the process has a
single HIP runtime (torch's bundled libamdhip64, which the library binds by soname).
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_float, c_int32, c_int64, c_void_p

import torch  # noqa: F401  (must precede the library: one HIP runtime per process)

LIB_NAME = "libvaehip.so"
LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), LIB_NAME)
# diagnostics: VAE_HIP_LIB=probe loads the phase-timestamp build (make -C pytorch-vae_amd/csrc probe);
# any other value V loads libvaehip_V.so (a build-flag variant for A/B timing)
if os.environ.get("VAE_HIP_LIB"):
    LIB_PATH = LIB_PATH.replace("libvaehip.so", "libvaehip_%s.so" % os.environ["VAE_HIP_LIB"])
ABI_VERSION = 25

F32, BF16 = 0, 1
X_NONE, X_ACT, X_BN_ACT, X_BN_DY = 0, 1, 2, 3
LOSS_VANILLA, LOSS_BETA_H, LOSS_BETA_B, LOSS_IWAE, LOSS_VQ = 0, 1, 2, 3, 4


class VaeHipError(RuntimeError):
    pass


class Xform(ctypes.Structure):
    _fields_ = [("kind", c_int32), ("channels", c_int32), ("slope", c_float), ("count", c_float),
                ("eps", c_float), ("momentum", c_float),
                ("sum", c_void_p), ("sumsq", c_void_p), ("shift", c_void_p), ("gamma", c_void_p),
                ("beta", c_void_p), ("dgamma", c_void_p), ("dbeta", c_void_p), ("aux", c_void_p),
                ("running_mean", c_void_p), ("running_var", c_void_p),
                ("reps", c_int32), ("rstride", c_int32), ("dgamma_out", c_void_p), ("dbeta_out", c_void_p),
                ("table", c_void_p)]


class BnArgs(ctypes.Structure):
    _fields_ = [("mode", c_int32), ("xf", Xform), ("table", c_void_p), ("db", c_void_p)]


class ConvArgs(ctypes.Structure):
    _fields_ = [("dtype", c_int32), ("n", c_int32), ("h", c_int32), ("w", c_int32), ("c", c_int32),
                ("k", c_int32), ("p", c_int32), ("q", c_int32), ("r", c_int32), ("stride", c_int32),
                ("pad", c_int32), ("x_nchw_f32", c_int32),
                ("x", c_void_p), ("x_xf", Xform), ("wt", c_void_p), ("bias", c_void_p), ("y", c_void_p),
                ("y_sum", c_void_p), ("y_sumsq", c_void_p), ("sum_reps", c_int32), ("sum_rstride", c_int32),
                ("residual", c_void_p), ("residual_xf", Xform),
                ("dy", c_void_p), ("dy_xf", Xform), ("dx", c_void_p), ("dx_epi", Xform),
                ("dx_dgamma", c_void_p), ("dx_dbeta", c_void_p), ("dw", c_void_p), ("db", c_void_p),
                ("split_k", c_int32), ("workspace", c_void_p), ("workspace_bytes", c_int64),
                ("bn_finalize", POINTER(BnArgs)), ("bn_counter", c_void_p), ("wt_t", c_void_p),
                ("dw_inner", c_int32), ("deterministic", c_int32), ("defer_reduce", c_int32)]


class LinearArgs(ctypes.Structure):
    _fields_ = [("dtype", c_int32), ("m", c_int32), ("n", c_int32), ("k", c_int32),
                ("x", c_void_p), ("x_xf", Xform), ("wt", c_void_p), ("bias", c_void_p), ("y", c_void_p),
                ("y_f32", c_int32), ("dy", c_void_p), ("dy_f32", c_int32), ("dx", c_void_p), ("dx_epi", Xform),
                ("dx_dgamma", c_void_p),
                ("dx_dbeta", c_void_p), ("sum_reps", c_int32), ("sum_rstride", c_int32),
                ("dw", c_void_p), ("db", c_void_p),
                ("mulv", c_void_p), ("eps", c_void_p), ("kl_coef", c_void_p), ("dmulv", c_void_p),
                ("samples", c_int32), ("workspace", c_void_p), ("workspace_bytes", c_int64),
                ("bn_finalize", POINTER(BnArgs)), ("bn_counter", c_void_p), ("deterministic", c_int32)]


class HeadArgs(ctypes.Structure):
    _fields_ = [("dtype", c_int32), ("n", c_int32), ("h", c_int32), ("w", c_int32), ("c", c_int32),
                ("x", c_void_p), ("x_xf", Xform), ("wt", c_void_p), ("bias", c_void_p),
                ("target", c_void_p), ("samples", c_int32), ("recon", c_void_p), ("sse", c_void_p),
                ("coef", c_void_p), ("dx", c_void_p), ("dx_epi", Xform), ("dx_dgamma", c_void_p),
                ("dx_dbeta", c_void_p), ("sum_reps", c_int32), ("sum_rstride", c_int32),
                ("dw", c_void_p), ("db", c_void_p), ("grad_recon", c_void_p),
                ("workspace", c_void_p), ("workspace_bytes", c_int64),
                ("bn_finalize", POINTER(BnArgs)), ("bn_counter", c_void_p), ("elbo", c_void_p),
                ("deterministic", c_int32), ("defer_reduce", c_int32)]


class ElboArgs(ctypes.Structure):
    _fields_ = [("kind", c_int32), ("batch", c_int32), ("samples", c_int32), ("latent", c_int32),
                ("img_elems", c_int32), ("kld_weight", c_float), ("beta", c_float), ("gamma", c_float),
                ("c_max", c_float), ("c_stop_iter", c_float), ("iter", c_void_p), ("mulv", c_void_p),
                ("sse", c_void_p), ("out", c_void_p), ("per_img", c_void_p), ("head_coef", c_void_p),
                ("kl_coef", c_void_p), ("vq_sse", c_void_p), ("vq_beta", c_float), ("vq_elems", c_float)]


SLAB_MAX = 32                      # vaehip.h VAE_SLAB_MAX


class GradSlab(ctypes.Structure):
    """vaehip.h vae_grad_slab: dst[j] = sum_{r < rows} slab[r * ld + j], j < count."""
    _fields_ = [("dst", c_void_p), ("count", c_int64), ("slab", c_void_p), ("rows", c_int32), ("ld", c_int64)]


class AdamArgs(ctypes.Structure):
    """vaehip.h vae_adam_args (vae_adam_step_ex: Adam with the deferred slab reductions and loss)."""
    _fields_ = [("n", c_int64), ("p", c_void_p), ("g", c_void_p), ("m", c_void_p), ("v", c_void_p),
                ("step", c_void_p), ("lr", c_void_p), ("beta1", ctypes.c_double), ("beta2", ctypes.c_double),
                ("eps", c_float), ("weight_decay", c_float), ("p_lowp", c_void_p), ("nslab", c_int32),
                ("slab", GradSlab * SLAB_MAX), ("has_elbo", c_int32), ("elbo", ElboArgs)]


class VqArgs(ctypes.Structure):
    _fields_ = [("dtype", c_int32), ("rows", c_int32), ("dim", c_int32), ("codes", c_int32),
                ("lat", c_void_p), ("lat_xf", Xform), ("codebook", c_void_p), ("indices", c_void_p),
                ("q", c_void_p), ("sse", c_void_p), ("beta", c_float), ("dq", c_void_p), ("loss_grad", c_void_p),
                ("dlat", c_void_p), ("dcodebook", c_void_p)]


class ReconArgs(ctypes.Structure):
    _fields_ = [("dtype", c_int32), ("n", c_int32), ("h", c_int32), ("w", c_int32), ("c", c_int32),
                ("y", c_void_p), ("target", c_void_p), ("recon", c_void_p), ("sse", c_void_p), ("dy", c_void_p),
                ("grad_scale", c_float), ("grad_recon", c_void_p), ("ld", c_int32)]


class BnApplyArgs(ctypes.Structure):
    """vaehip.h vae_bn_apply_args (a materialised lrelu(BN(y)) / BN-backward gradient)."""
    _fields_ = [("dtype", c_int32), ("rows", c_int64), ("channels", c_int32), ("x", c_void_p), ("xf", Xform),
                ("db", c_void_p), ("out", c_void_p)]


class ReconLossArgs(ctypes.Structure):
    """vaehip.h vae_recon_loss_args (the Autoencoder's centre-weighted MSE / MS-SSIM)."""
    _fields_ = [("kind", c_int32), ("n", c_int32), ("c", c_int32), ("h", c_int32), ("w", c_int32),
                ("recon", c_void_p), ("target", c_void_p), ("mask", c_void_p), ("window", c_float * 16),
                ("window_size", c_int32), ("levels", c_int32), ("level_weights", c_float * 8),
                ("normalize", c_int32), ("size_average", c_int32), ("grad", c_void_p), ("grad_scale", c_float),
                ("out", c_void_p), ("sse", c_void_p), ("per_img", c_void_p), ("workspace", c_void_p),
                ("workspace_bytes", c_int64)]


RLOSS_CENTER, RLOSS_MSSIM = 0, 1


class RecordArgs(ctypes.Structure):
    _fields_ = [("batch", c_int32), ("samples", c_int32), ("img_elems", c_int32), ("nterms", c_int32),
                ("step", c_int32), ("src_terms", c_void_p), ("terms", c_void_p), ("per_img", c_void_p),
                ("per", c_void_p), ("img", c_void_p), ("recon", c_void_p), ("best", c_void_p), ("at", c_void_p),
                ("hi_img", c_void_p), ("hi_recon", c_void_p), ("lo_img", c_void_p), ("lo_recon", c_void_p)]


class SwapDesc(ctypes.Structure):
    _fields_ = [("src", c_void_p), ("dst", c_void_p), ("a", c_int32), ("rs", c_int32), ("b", c_int32),
                ("src_dtype", c_int32)]


SWAP_MAX = 16
PAD_MAX = 4


class PadDesc(ctypes.Structure):
    _fields_ = [("rows", c_int64), ("c", c_int32), ("cp", c_int32), ("src", c_void_p), ("dst", c_void_p)]


class KeepRange(ctypes.Structure):
    _fields_ = [("off", c_int64), ("bytes", c_int64)]


class StepBeginArgs(ctypes.Structure):
    _fields_ = [("zero", c_void_p), ("bytes", c_int64), ("step", c_void_p), ("dtype", c_int32),
                ("n", c_int32), ("c", c_int32), ("h", c_int32), ("w", c_int32), ("cp", c_int32),
                ("x", c_void_p), ("y", c_void_p), ("npad", c_int32), ("pad", PadDesc * PAD_MAX),
                ("nswap", c_int32), ("swap", SwapDesc * SWAP_MAX), ("nkeep", c_int32),
                ("keep", KeepRange * 32)]


class LatentArgs(ctypes.Structure):
    _fields_ = [("dtype", c_int32), ("batch", c_int32), ("samples", c_int32), ("latent", c_int32),
                ("in_features", c_int32), ("out_features", c_int32),
                ("x", c_void_p), ("x_xf", Xform), ("w1", c_void_p), ("b1", c_void_p), ("mulv", c_void_p),
                ("eps", c_void_p), ("z", c_void_p), ("w2", c_void_p), ("b2", c_void_p), ("h", c_void_p),
                ("dh", c_void_p), ("kl_coef", c_void_p), ("dmulv", c_void_p), ("dw2", c_void_p), ("db2", c_void_p),
                ("dx", c_void_p), ("dx_epi", Xform), ("dx_dgamma", c_void_p), ("dx_dbeta", c_void_p),
                ("sum_reps", c_int32), ("sum_rstride", c_int32), ("dw1", c_void_p), ("db1", c_void_p),
                ("eps_step", c_void_p), ("eps_seed", ctypes.c_uint64), ("eps_gen", c_int32)]

# name -> (argtypes)
_SIGS = {
    "vae_abi_version": [],
    "vae_last_error": [],
    "vae_build_digest": [],
    "vae_launch_log": [c_int32],
    "vae_launch_log_names": [ctypes.c_char_p, c_int64],
    "vae_conv2d_fwd": [POINTER(ConvArgs), c_void_p],
    "vae_conv2d_bwd_data": [POINTER(ConvArgs), c_void_p],
    "vae_conv2d_bwd_filter": [POINTER(ConvArgs), c_void_p],
    "vae_convT2d_fwd": [POINTER(ConvArgs), c_void_p],
    "vae_convT2d_bwd_data": [POINTER(ConvArgs), c_void_p],
    "vae_convT2d_bwd_filter": [POINTER(ConvArgs), c_void_p],
    "vae_convT2d_bwd": [POINTER(ConvArgs), c_void_p],
    "vae_convT2d_fwd_recon": [POINTER(ConvArgs), POINTER(ReconArgs), c_void_p],
    "vae_linear_fwd": [POINTER(LinearArgs), c_void_p],
    "vae_linear_bwd_data": [POINTER(LinearArgs), c_void_p],
    "vae_linear_bwd_filter": [POINTER(LinearArgs), c_void_p],
    "vae_head_fwd": [POINTER(HeadArgs), c_void_p],
    "vae_head_bwd_data": [POINTER(HeadArgs), c_void_p],
    "vae_head_bwd_filter": [POINTER(HeadArgs), c_void_p],
    "vae_head_bwd": [POINTER(HeadArgs), c_void_p],
    "vae_bn_finalize": [POINTER(BnArgs), c_void_p],
    "vae_reparam_fwd": [c_int32, c_int32, c_int32, c_int32, c_void_p, c_void_p, c_void_p, c_void_p],
    "vae_elbo_fwd": [POINTER(ElboArgs), c_void_p],
    "vae_vq_fwd": [POINTER(VqArgs), c_void_p],
    "vae_vq_bwd": [POINTER(VqArgs), c_void_p],
    "vae_recon_fwd": [POINTER(ReconArgs), c_void_p],
    "vae_recon_bwd": [POINTER(ReconArgs), c_void_p],
    "vae_adam_step": [c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, ctypes.c_double,
                      ctypes.c_double, c_float, c_float, c_void_p, c_void_p],
    "vae_cast_bf16": [c_int64, c_void_p, c_void_p, c_void_p],
    "vae_deferred_reset": [],
    "vae_deferred_take": [POINTER(GradSlab), c_int32, POINTER(ElboArgs), POINTER(c_int32)],
    "vae_adam_step_ex": [POINTER(AdamArgs), c_void_p],
    "vae_step_begin": [c_void_p, c_int64, c_void_p, c_void_p],
    "vae_step_record": [POINTER(RecordArgs), c_void_p],
    "vae_swap_axes": [c_int32, c_void_p, c_void_p],
    "vae_nchw_to_nhwc_pad": [c_int32, c_int32, c_int32, c_int32, c_int32, c_int32, c_void_p, c_void_p, c_void_p],
    "vae_pad_channels": [c_int32, c_int64, c_int32, c_int32, c_void_p, c_void_p, c_void_p],
    "vae_unpad_accumulate": [c_int64, c_int32, c_int32, c_void_p, c_void_p, c_void_p],
    "vae_conv2d_workspace_size": [POINTER(ConvArgs), c_int32, POINTER(ctypes.c_size_t)],
    "vae_convT2d_workspace_size": [POINTER(ConvArgs), c_int32, POINTER(ctypes.c_size_t)],
    "vae_linear_workspace_size": [POINTER(LinearArgs), c_int32, POINTER(ctypes.c_size_t)],
    "vae_head_workspace_size": [POINTER(HeadArgs), c_int32, POINTER(ctypes.c_size_t)],
    "vae_conv_bwd_filter_batch": [c_int32, c_void_p, c_void_p, c_void_p, c_int64, c_void_p],
    "vae_conv_bwd_filter_batch_workspace_size": [c_int32, c_void_p, c_void_p, POINTER(ctypes.c_size_t)],
    "vae_step_begin_ex": [POINTER(StepBeginArgs), c_void_p],
    "vae_latent_fc_fwd": [POINTER(LatentArgs), c_void_p],
    "vae_latent_dec_fwd": [POINTER(LatentArgs), c_void_p],
    "vae_latent_dec_bwd": [POINTER(LatentArgs), c_void_p],
    "vae_latent_fc_bwd": [POINTER(LatentArgs), c_void_p],
    "vae_recon_loss": [POINTER(ReconLossArgs), c_void_p],
    "vae_bn_apply": [POINTER(BnApplyArgs), c_void_p],
    "vae_recon_loss_workspace_size": [POINTER(ReconLossArgs), POINTER(ctypes.c_size_t)],
}
EXPORTED = tuple(_SIGS)

_lib = None


def load(path: str = LIB_PATH):
    """Load the shared library (no GPU work).  Raises if it is missing or the ABI differs."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise VaeHipError(f"{path} not found — build it with `make -C pytorch-vae_amd/csrc` "
                          f"(or __graft_entry__.build()); there is no fallback path")
    lib = ctypes.CDLL(path)
    for name, argtypes in _SIGS.items():
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = (ctypes.c_char_p if name in ("vae_last_error", "vae_build_digest") else
                      c_int64 if name == "vae_launch_log_names" else c_int32)
    if lib.vae_abi_version() != ABI_VERSION:
        raise VaeHipError(f"libvaehip ABI {lib.vae_abi_version()} != expected {ABI_VERSION}")
    _lib = lib
    return lib


def call(name: str, *args):
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.vae_last_error().decode(errors="replace")
        raise VaeHipError(f"{name} failed (rc={rc}): {msg}")


OP_FWD, OP_BWD_DATA, OP_BWD_FILTER, OP_BWD = 0, 1, 2, 3          # vaehip.h enum vae_op
LAYER_CONV2D, LAYER_CONVT2D = 0, 1                               # vaehip.h enum vae_layer_kind

# entry point -> (its workspace query, op)
WS_QUERY = {
    "vae_conv2d_fwd": ("vae_conv2d_workspace_size", OP_FWD),
    "vae_conv2d_bwd_data": ("vae_conv2d_workspace_size", OP_BWD_DATA),
    "vae_conv2d_bwd_filter": ("vae_conv2d_workspace_size", OP_BWD_FILTER),
    "vae_convT2d_fwd": ("vae_convT2d_workspace_size", OP_FWD),
    "vae_convT2d_bwd_data": ("vae_convT2d_workspace_size", OP_BWD_DATA),
    "vae_convT2d_bwd_filter": ("vae_convT2d_workspace_size", OP_BWD_FILTER),
    "vae_convT2d_bwd": ("vae_convT2d_workspace_size", OP_BWD),
    "vae_linear_fwd": ("vae_linear_workspace_size", OP_FWD),
    "vae_linear_bwd_data": ("vae_linear_workspace_size", OP_BWD_DATA),
    "vae_linear_bwd_filter": ("vae_linear_workspace_size", OP_BWD_FILTER),
    "vae_head_fwd": ("vae_head_workspace_size", OP_FWD),
    "vae_head_bwd_data": ("vae_head_workspace_size", OP_BWD_DATA),
    "vae_head_bwd_filter": ("vae_head_workspace_size", OP_BWD_FILTER),
    "vae_head_bwd": ("vae_head_workspace_size", OP_BWD),
}


def deferred_take():
    """The weight-gradient reductions (and the loss) the calls since the last take / reset deferred
    (vaehip.h vae_deferred_take): ([GradSlab], ElboArgs or None).  Clears the list."""
    lib = load()
    out = (GradSlab * SLAB_MAX)()
    el = ElboArgs()
    has = c_int32(0)
    n = lib.vae_deferred_take(out, SLAB_MAX, ctypes.byref(el), ctypes.byref(has))
    if n > SLAB_MAX:
        raise VaeHipError(f"{n} deferred reductions > {SLAB_MAX}")
    return [GradSlab.from_buffer_copy(out[i]) for i in range(n)], (el if has.value else None)


def workspace_size(fn: str, arg) -> int:
    """Workspace bytes the entry point `fn` needs for `arg` (a ConvArgs / LinearArgs / HeadArgs
    filled as for the call; its workspace fields are ignored).  Runs no kernel."""
    q, op = WS_QUERY[fn]
    out = ctypes.c_size_t(0)
    call(q, ctypes.byref(arg), op, ctypes.byref(out))
    return int(out.value)


def ptr(t) -> int | None:
    """Device pointer of a tensor (None for None)."""
    if t is None:
        return None
    return t.data_ptr()


def stream_ptr() -> int:
    return torch.cuda.current_stream().cuda_stream


def dtype_code(dt: torch.dtype) -> int:
    if dt == torch.float32:
        return F32
    if dt == torch.bfloat16:
        return BF16
    raise VaeHipError(f"unsupported dtype {dt}")


class FilterBatch:
    """Argument block of one vae_conv_bwd_filter_batch call: the weight-gradient calls
    (vae_conv2d_bwd_filter / vae_convT2d_bwd_filter, each with its ConvArgs) of one backward
    segment, run as grouped launches (vaehip.h).  Keeps the item structs alive."""

    FNS = {"vae_conv2d_bwd_filter": LAYER_CONV2D, "vae_convT2d_bwd_filter": LAYER_CONVT2D}

    def __init__(self, calls):
        self.calls = list(calls)                   # [(fn, byref(ConvArgs))]
        n = len(self.calls)
        self.kinds = (c_int32 * n)(*[self.FNS[fn] for fn, _ in self.calls])
        self.items = (c_void_p * n)(*[ctypes.addressof(ref._obj) for _, ref in self.calls])
        self.workspace, self.workspace_bytes = None, 0
        self.side = False            # run on the plan's side stream (net.run_calls)
        # scalar-argument calls that read this batch's output (vae_unpad_accumulate of a padded
        # gradient): run right behind it on the same stream, whichever stream that is
        self.after = []

    @property
    def args(self):
        return [ref._obj for _, ref in self.calls]

    def workspace_size(self) -> int:
        out = ctypes.c_size_t(0)
        call("vae_conv_bwd_filter_batch_workspace_size", len(self.calls), self.kinds, self.items, ctypes.byref(out))
        return int(out.value)

    def __call__(self, stream):
        call("vae_conv_bwd_filter_batch", len(self.calls), self.kinds, self.items, self.workspace,
             self.workspace_bytes, stream)
        for fn, args in self.after:
            call(fn, *args, stream)


def recon_loss_args(kind: int, n: int, c: int, h: int, w: int, *, mask=None, window=None, levels: int = 5,
                    level_weights=(0.0448, 0.2856, 0.3001, 0.2363, 0.1333), normalize: bool = True) -> "ReconLossArgs":
    """A vae_recon_loss argument block with the loss's constants filled in (pointers left to the caller):
    kind RLOSS_CENTER with `mask` ([h][w] device tensor), or RLOSS_MSSIM with the 1-D `window`
    (models.MSSIM's normalised window, host floats)."""
    a = ReconLossArgs(kind=kind, n=n, c=c, h=h, w=w, size_average=1, grad_scale=1.0)
    if kind == RLOSS_CENTER:
        a.mask = mask.data_ptr()
    else:
        win = [float(v) for v in window]
        a.window_size = len(win)
        for i, v in enumerate(win):
            a.window[i] = v
        a.levels = levels
        for i, v in enumerate(level_weights):
            a.level_weights[i] = float(v)
        a.normalize = int(normalize)
    return a


def recon_loss_workspace(a: "ReconLossArgs") -> int:
    out = ctypes.c_size_t(0)
    call("vae_recon_loss_workspace_size", ctypes.byref(a), ctypes.byref(out))
    return int(out.value)
