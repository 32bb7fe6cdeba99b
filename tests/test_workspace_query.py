"""Workspace queries of the C ABI (vaehip.h vae_*_workspace_size) — CPU only: a
query runs the entry point's own planning with the launches switched off, so it needs no device,
and a call whose workspace is short fails in planning, before anything is launched.

Shapes are the VanillaVAE B=64 layers (models/vanilla_vae.py:25-75): the deep-K / small-M encoder
tail and the linears split K over workgroups (fp32 partial slabs in the workspace), the big-M
early layers do not."""
import ctypes

import pytest

from vae_amd import _lib as L

FAKE = 1 << 24          # aligned, never dereferenced (nothing launches)


def _conv(n, h, c, k, stride=2, r=3, pad=1, dtype=None):
    p = h // stride
    a = L.ConvArgs(dtype=L.BF16 if dtype is None else dtype, n=n, h=h, w=h, c=c, k=k, p=p, q=p, r=r,
                   stride=stride, pad=pad)
    a.x = a.wt = a.y = FAKE
    a.x_xf = L.Xform(kind=L.X_NONE, channels=c)
    return a


def _need(fn, a):
    return L.workspace_size(fn, a)


def test_split_k_layers_need_workspace_and_big_layers_none():
    deep = _conv(64, 4, 256, 512)            # encoder.4: M = 64*2*2 = 256 rows, K = 2304
    wide = _conv(64, 64, 8, 32)              # encoder.0 (padded RGB): M = 64*32*32 rows
    nd, nw = _need("vae_conv2d_fwd", deep), _need("vae_conv2d_fwd", wide)
    assert nd > 0 and nd % 4 == 0
    assert nd >= 2 * 256 * 512 * 4          # at least two fp32 partial slabs of the output
    assert nw == 0


def test_query_is_deterministic_and_ignores_workspace_fields():
    a = _conv(64, 4, 256, 512)
    n0 = _need("vae_conv2d_fwd", a)
    a.workspace, a.workspace_bytes = FAKE, 7
    assert _need("vae_conv2d_fwd", a) == n0
    assert a.workspace_bytes == 7            # the caller's struct is not modified


def test_short_workspace_is_an_error_not_a_silent_downgrade():
    lib = L.load()
    a = _conv(64, 4, 256, 512)
    need = _need("vae_conv2d_fwd", a)
    a.workspace, a.workspace_bytes = FAKE, need - 4
    rc = lib.vae_conv2d_fwd(ctypes.byref(a), None)
    assert rc == -1
    msg = lib.vae_last_error()
    assert b"workspace" in msg and str(need).encode() in msg


def test_explicit_split_without_workspace_is_rejected():
    lib = L.load()
    a = _conv(64, 4, 256, 512)
    a.split_k = 4
    rc = lib.vae_conv2d_fwd(ctypes.byref(a), None)
    assert rc == -1 and b"split_k" in lib.vae_last_error()


def test_staged_weight_copy_counts_in_the_need():
    """convT2d_fwd without a caller-supplied swapped weight copy (wt_t) stages it at the end of the
    workspace: the need includes its bf16 bytes; with wt_t it does not."""
    a = _conv(64, 4, 256, 128)               # decoder.1 convT 256 -> 128 at 4x4 -> 8x8
    a.p = a.q = 8
    n_stage = _need("vae_convT2d_fwd", a)
    a.wt_t = FAKE
    n_given = _need("vae_convT2d_fwd", a)
    wbytes = 128 * 9 * 256 * 2
    assert n_stage >= n_given + wbytes


@pytest.mark.parametrize("op", ["vae_head_bwd", "vae_head_bwd_filter"])
def test_head_filter_partials_need_workspace(op):
    a = L.HeadArgs(dtype=L.BF16, n=64, h=64, w=64, c=32, samples=1)
    a.x = a.wt = a.bias = a.target = a.recon = a.sse = a.coef = a.dx = a.dw = a.db = FAKE
    a.dx_dgamma = a.dx_dbeta = FAKE
    a.x_xf = L.Xform(kind=L.X_BN_ACT, channels=32, count=1.0, slope=0.01)     # lrelu(BN(x)), as in the net
    a.dx_epi = L.Xform(kind=L.X_BN_ACT, channels=32, count=1.0, slope=0.01)
    for f in ("sum", "sumsq", "gamma", "beta", "aux"):
        setattr(a.x_xf, f, FAKE)
        setattr(a.dx_epi, f, FAKE)
    n = _need(op, a)
    assert n > 0 and n % (64 * 4) == 0          # one fp32 row of partials per workgroup
    assert _need("vae_head_fwd", a) == 0


def test_bad_op_is_rejected():
    lib = L.load()
    a = _conv(4, 8, 8, 8)
    out = ctypes.c_size_t(0)
    assert lib.vae_conv2d_workspace_size(ctypes.byref(a), 9, ctypes.byref(out)) == -1


def _bn(kind, c):
    x = L.Xform(kind=kind, channels=c, count=1.0, slope=0.01, eps=1e-5)
    for f in ("sum", "sumsq", "gamma", "beta", "dgamma", "dbeta", "aux"):
        setattr(x, f, FAKE)
    return x


def test_filter_batch_workspace():
    """vae_conv_bwd_filter_batch: the bf16 3x3 layers with a BN-backward dy run as one grid whose
    K-sliced layers write partial slabs (the batch's own workspace); any other item runs as its own
    call with a region of its own, so a batch of those needs the sum of the items' needs.  A short
    workspace fails in planning."""
    fin = _conv(64, 32, 32, 32)                  # final_layer ConvT 32 -> 32, 32x32 -> 64x64
    fin.p = fin.q = 64
    fin.dy = fin.dw = FAKE
    fin.x_xf, fin.dy_xf = _bn(L.X_BN_ACT, 32), _bn(L.X_BN_DY, 32)
    enc = _conv(64, 16, 64, 128)                 # encoder.2 conv 64 -> 128
    enc.dy = enc.dw = FAKE
    enc.x_xf, enc.dy_xf = _bn(L.X_BN_ACT, 64), _bn(L.X_BN_DY, 128)
    b = L.FilterBatch([("vae_convT2d_bwd_filter", ctypes.byref(fin)), ("vae_conv2d_bwd_filter", ctypes.byref(enc))])
    need = b.workspace_size()
    assert need > 0 and need % 256 == 0           # K-slice partial slabs of the grouped grid
    lib = L.load()
    rc = lib.vae_conv_bwd_filter_batch(2, b.kinds, b.items, FAKE, need - 4, None)
    assert rc == -1 and b"workspace" in lib.vae_last_error()
    # fp32 items do not group: each keeps its standalone plan and region
    f32 = []
    for a in (fin, enc):
        c = L.ConvArgs.from_buffer_copy(a)
        c.dtype = L.F32
        f32.append(c)
    n1, n2 = _need("vae_convT2d_bwd_filter", f32[0]), _need("vae_conv2d_bwd_filter", f32[1])
    b32 = L.FilterBatch([("vae_convT2d_bwd_filter", ctypes.byref(f32[0])), ("vae_conv2d_bwd_filter", ctypes.byref(f32[1]))])
    r = lambda v: (v + 255) // 256 * 256
    assert b32.workspace_size() == r(n1) + r(n2)


def _vq_items():
    """VQ-VAE B=128 residual-stack weight gradients (models/vq_vae.py:57-70): the 3x3 256 -> 256
    conv and the 1x1 256 -> 256 conv on the 16x16 latent grid, bf16, no BatchNorm — standalone
    items of a batch (each keeps its own plan, slab and region)."""
    c3 = _conv(128, 16, 256, 256, stride=1, r=3, pad=1)
    c1 = _conv(128, 16, 256, 256, stride=1, r=1, pad=0)
    for a in (c3, c1):
        a.dy = a.dw = FAKE
        a.dy_xf = L.Xform(kind=L.X_NONE, channels=256)
    return c3, c1


def test_filter_batch_nested_queries_leave_no_state():
    """Round-5 fault (profiles/r5_notes.md): a workspace query nested inside the batch collector
    recorded the query's fake slab pointer.  The collector queries each standalone item's need with
    the thread's query state saved around it (vae_wgrad_batch.hip item_need): the batch need is the
    sum of the items' own needs, every standalone query gives the same answer before and after a
    batch query, and a real call after the queries is planned for real (a short workspace fails in
    planning instead of being taken for a query)."""
    lib = L.load()
    c3, c1 = _vq_items()
    r = lambda v: (v + 255) // 256 * 256
    n3, n1 = _need("vae_conv2d_bwd_filter", c3), _need("vae_conv2d_bwd_filter", c1)
    assert n3 > 0                                 # the 3x3 weight gradient slices K into slabs
    items = [("vae_conv2d_bwd_filter", ctypes.byref(c3)), ("vae_conv2d_bwd_filter", ctypes.byref(c1))]
    b = L.FilterBatch(items)
    need = b.workspace_size()
    assert need == r(n3) + r(n1)
    for _ in range(3):                            # repeated: no state carried from one query to the next
        assert b.workspace_size() == need
        assert _need("vae_conv2d_bwd_filter", c3) == n3 and _need("vae_conv2d_bwd_filter", c1) == n1
    # a grouped VanillaVAE layer beside them: slabs after the standalone regions
    fin = _conv(64, 32, 32, 32)
    fin.p = fin.q = 64
    fin.dy = fin.dw = FAKE
    fin.x_xf, fin.dy_xf = _bn(L.X_BN_ACT, 32), _bn(L.X_BN_DY, 32)
    mixed = L.FilterBatch(items + [("vae_convT2d_bwd_filter", ctypes.byref(fin))])
    nm = mixed.workspace_size()
    assert nm >= need
    assert mixed.workspace_size() == nm
    # the query state is off again: real calls with a short workspace are rejected in planning
    # (a leaked query flag would return 0 here without looking at the workspace)
    for bb, nn in ((b, need), (mixed, nm)):
        rc = lib.vae_conv_bwd_filter_batch(len(bb.kinds), bb.kinds, bb.items, FAKE, nn - 256, None)
        assert rc == -1 and b"workspace" in lib.vae_last_error()
    c3.workspace, c3.workspace_bytes = FAKE, n3 - 4
    assert lib.vae_conv2d_bwd_filter(ctypes.byref(c3), None) == -1
    assert b"workspace" in lib.vae_last_error()


def _head_with_elbo(n, batch, latent=128):
    a = L.HeadArgs(dtype=L.BF16, n=n, h=64, w=64, c=32, samples=1)
    a.x = a.wt = a.bias = a.target = a.recon = a.sse = a.dx = a.dw = a.db = FAKE
    a.dx_dgamma = a.dx_dbeta = FAKE
    a.x_xf = L.Xform(kind=L.X_BN_ACT, channels=32, count=1.0, slope=0.01)
    a.dx_epi = L.Xform(kind=L.X_BN_ACT, channels=32, count=1.0, slope=0.01)
    for f in ("sum", "sumsq", "gamma", "beta", "aux"):
        setattr(a.x_xf, f, FAKE)
        setattr(a.dx_epi, f, FAKE)
    e = L.ElboArgs(kind=L.LOSS_VANILLA, batch=batch, samples=1, latent=latent, img_elems=3 * 64 * 64)
    e.iter = e.mulv = e.sse = e.out = e.per_img = e.head_coef = e.kl_coef = FAKE
    a.coef = FAKE                                 # (the query plans the unfused call)
    need = _need("vae_head_bwd", a)
    a.coef = None                                 # fused: the seed coefficient comes from the loss
    a.workspace, a.workspace_bytes = FAKE, need
    a.elbo = ctypes.addressof(e)
    return a, e


@pytest.mark.parametrize("n,batch,latent", [(2048, 2048, 128), (64, 32, 128), (64, 64, 0), (64, 0, 128)])
def test_fused_elbo_head_rejects_bad_shapes(n, batch, latent):
    """the ELBO fused into the head backward (vae_head_args.elbo) keeps per-row KL terms in
    a 1024-entry LDS array; it takes vae_elbo_fwd's shape checks (batch in 1..1024, latent > 0) and
    the loss must describe the head's own batch — rejected before anything launches."""
    lib = L.load()
    a, e = _head_with_elbo(n, batch, latent)
    rc = lib.vae_head_bwd(ctypes.byref(a), None)
    assert rc == -2, (rc, lib.vae_last_error())
    assert b"fused ELBO" in lib.vae_last_error()
