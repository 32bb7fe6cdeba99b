"""Debug: where does the bf16 MFMA head backward's dx differ from autograd?"""
import ctypes, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "pytorch-vae_amd"), os.path.join(REPO, "tests")]
import torch
import torch.nn.functional as F
from vae_amd import _lib as L
from gpu_util import BNState

torch.manual_seed(6)
N, C, H = 2, 32, 64
y_prev = torch.randn(N, C, H, H)
gam = 0.8 + 0.4 * torch.rand(C); bet = torch.rand(C) * 0.2 - 0.1
w = torch.randn(3, C, 3, 3) * 0.1
b = torch.randn(3) * 0.1
tgt = torch.rand(N, 3, H, H)
z = F.batch_norm(y_prev, None, None, gam, bet, True, 0.1, 1e-5).requires_grad_()
rec = torch.tanh(F.conv2d(F.leaky_relu(z, 0.01), w, b, padding=1))
loss = F.mse_loss(rec, tgt); loss.backward()
dtype = torch.bfloat16
bn = BNState(y_prev, dtype=dtype); bn.gamma, bn.beta = gam, bet
bn.dev["gamma"], bn.dev["beta"] = gam.cuda(), bet.cuda()
wd = w.permute(0, 2, 3, 1).contiguous().cuda(); bd = b.cuda(); tg = tgt.cuda()
recon = torch.empty(N, 3, H, H, device="cuda"); sse = torch.zeros(N, device="cuda")
coef = torch.full((N,), 2.0 / rec.numel(), device="cuda")
dx = torch.zeros(N, H, H, C, device="cuda", dtype=dtype)
dgp = torch.zeros(C, device="cuda"); dbp = torch.zeros(C, device="cuda")
dw = torch.zeros(wd.shape, device="cuda"); db = torch.zeros(3, device="cuda")
a = L.HeadArgs(dtype=L.dtype_code(dtype), n=N, h=H, w=H, c=C, samples=1)
a.x = bn.y_dev.data_ptr(); a.x_xf = bn.xf(); a.wt = wd.data_ptr(); a.bias = bd.data_ptr(); a.target = tg.data_ptr()
a.recon = recon.data_ptr(); a.sse = sse.data_ptr(); a.coef = coef.data_ptr()
a.dx = dx.data_ptr(); a.dx_epi = bn.xf(aux=bn.y_dev); a.dx_dgamma = dgp.data_ptr(); a.dx_dbeta = dbp.data_ptr()
a.dw = dw.data_ptr(); a.db = db.data_ptr()
st = torch.cuda.current_stream().cuda_stream
L.call("vae_head_fwd", ctypes.byref(a), st)
L.call("vae_head_bwd_data", ctypes.byref(a), st)
torch.cuda.synchronize()
got = dx.float().permute(0, 3, 1, 2).cpu()
ref = z.grad
err = (got - ref).abs()
scale = ref.abs().max()
bad = err > 0.05 * scale
print("max rel", float(err.max() / scale), "bad count", int(bad.sum()), "of", bad.numel())
idx = bad.nonzero()
if len(idx):
    print("bad n:", torch.bincount(idx[:, 0]).tolist())
    print("bad c:", torch.bincount(idx[:, 1], minlength=C).tolist())
    print("bad h:", torch.bincount(idx[:, 2], minlength=H).tolist())
    print("bad w:", torch.bincount(idx[:, 3], minlength=H).tolist())
    for k in idx[:10].tolist():
        n, c, h, ww = k
        print(k, float(got[n, c, h, ww]), float(ref[n, c, h, ww]))
