"""Helpers for the GPU tests: NHWC/NCHW moves and BatchNorm transform descriptors built
from torch tensors, so single C-ABI entry points can be checked against PyTorch-CPU fp32."""
import torch

from vae_amd import _lib as L


def nhwc(t_nchw, dtype):
    return t_nchw.permute(0, 2, 3, 1).contiguous().to(device="cuda", dtype=dtype)


def to_nchw(t_nhwc):
    return t_nhwc.float().permute(0, 3, 1, 2).contiguous().cpu()


class BNState:
    """A pre-BN NHWC tensor y plus BN params and the producer-side sums the kernels read."""

    def __init__(self, y_nchw, shift=None, seed=0, dtype=torch.float32):
        g = torch.Generator().manual_seed(seed)
        C = y_nchw.shape[1]
        self.y_nchw = y_nchw
        self.gamma = 0.8 + 0.4 * torch.rand(C, generator=g)
        self.beta = (torch.rand(C, generator=g) * 2 - 1) * 0.1
        self.shift = shift if shift is not None else torch.zeros(C)
        d = (y_nchw - self.shift.view(1, -1, 1, 1)).double()
        self.sum = d.sum(dim=(0, 2, 3)).float()
        self.sumsq = (d * d).sum(dim=(0, 2, 3)).float()
        self.count = y_nchw.numel() // C
        self.dev = {k: getattr(self, k).cuda() for k in ("gamma", "beta", "shift", "sum", "sumsq")}
        self.y_dev = nhwc(y_nchw, dtype)

    def act_ref(self):
        """lrelu(BN_train(y)) in PyTorch, NCHW fp32 CPU."""
        yb = torch.nn.functional.batch_norm(self.y_nchw, None, None, self.gamma, self.beta, True, 0.1, 1e-5)
        return torch.nn.functional.leaky_relu(yb, 0.01)

    def xf(self, kind=L.X_BN_ACT, aux=None, dgamma=None, dbeta=None):
        C = self.gamma.numel()
        x = L.Xform(kind=kind, channels=C, slope=0.01, count=float(self.count), eps=1e-5, momentum=0.1)
        x.sum = self.dev["sum"].data_ptr()
        x.sumsq = self.dev["sumsq"].data_ptr()
        x.shift = self.dev["shift"].data_ptr()
        x.gamma = self.dev["gamma"].data_ptr()
        x.beta = self.dev["beta"].data_ptr()
        if kind in (L.X_BN_DY,):
            x.dgamma = dgamma.data_ptr()
            x.dbeta = dbeta.data_ptr()
        if aux is not None:
            x.aux = aux.data_ptr()
        return x


def rel(a, b):
    a = a.double().flatten()
    b = b.double().flatten()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def tol(dtype):
    return 2e-5 if dtype == torch.float32 else 2e-2


def give_workspace(a, *fns):
    """Query the workspace the calls `fns` need for args `a` (vae_*_workspace_size), allocate
    it and point `a` at it; returns the buffer (keep it alive until the calls are done)."""
    need = max(L.workspace_size(fn, a) for fn in fns)
    ws = torch.empty(max(1, (need + 3) // 4), device="cuda")
    a.workspace = ws.data_ptr()
    a.workspace_bytes = ws.numel() * 4
    return ws


def launched(fn):
    """Run fn() with the library's launch log on; return the names of the kernels it launched."""
    import ctypes
    from vae_amd import _lib as L
    lib = L.load()
    lib.vae_launch_log(1)
    try:
        fn()
    finally:
        lib.vae_launch_log(0)
    need = lib.vae_launch_log_names(None, 0)
    buf = ctypes.create_string_buffer(int(need))
    lib.vae_launch_log_names(buf, need)
    return buf.value.decode()
