"""Op-by-op, teacher-forced check of one bf16 training step of the VanillaVAE family at the shapes
bench.py times (every timed bf16 kernel pinned at its benched shape).

After ONE step of the exact bench path (engine.TrainStep: one HIP graph with vae_step_begin_ex,
the on-device eps draw, the fused bottleneck kernels, the ELBO in the head backward, the batched
weight gradients and Adam), every buffer the step wrote is still on the device.  Each op is then
recomputed on the CPU in fp64 from the GPU's OWN inputs to that op (teacher forcing: the stored
bf16 activations and gradients, the bf16 weight copy Adam read, the fp32 master parameters), with
the kernels' operand rounding mirrored (a transformed operand, lrelu(BN(y)) or the BatchNorm-
backward a*g + b*y + c, is rounded to bf16 before the product, as the kernels stage it), and
compared with the GPU's output of that op:

  * bf16 outputs (activations, data gradients): elementwise |got - ref| <= 2^-7 |ref| + 2e-3 rms(ref)
    (output rounding 2^-9 plus the rare operand-rounding flip), relative norm <= 4e-3; elements
    whose LeakyReLU branch is ambiguous (|z| below 1e-4 of max|z|, where fp32 vs fp64 statistics
    can pick the other branch) are counted and excluded;
  * fp32 outputs (weight gradients, mu|logvar, loss terms): max|got - ref| / max|ref| <= 2e-3 and
    relative norm <= 1e-3 (VERDICT r5 #2's bar for the grouped weight gradients); loss terms 1e-5;
  * Adam: the torch.optim.Adam formula on the GPU's own gradients, |dp| <= 1e-6 (|p| + lr).

The reference semantics are the reference's modules' (models/vanilla_vae.py:25-146,
beta_vae.py:129-152, iwae.py:95-160, experiment.py:308-311 Adam); the oracle tests pin the same
formulas to reference-generated vectors (tests/test_oracle_golden.py).  Each check names the plan
call whose output it verifies, so the test can map every kernel the step launched (vae_launch_log)
to the checks that pin it."""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn.functional as F

SLOPE, BN_EPS, MOM = 0.01, 1e-5, 0.1
D64 = torch.float64


def bf(t: torch.Tensor) -> torch.Tensor:
    """Round to bf16 (round-to-nearest-even, as the kernels' conversions), back to fp64."""
    return t.to(torch.bfloat16).to(D64)


def cpu64(t: torch.Tensor) -> torch.Tensor:
    return t.detach().to("cpu", D64)


def nchw(t: torch.Tensor) -> torch.Tensor:
    """A GPU NHWC map -> CPU NCHW fp64."""
    return cpu64(t).permute(0, 3, 1, 2).contiguous()


def lrelu(x):
    return torch.where(x > 0, x, x * SLOPE)


@dataclass
class Check:
    name: str
    call: Tuple[str, int]              # (plan call fn, its occurrence) whose output this verifies
    ok: bool
    detail: Dict[str, float] = field(default_factory=dict)


class BN:
    """Train-mode BatchNorm of a stored pre-BN map y (NCHW fp64) with the fp32 master gamma / beta.

    Teacher-forced statistics: `fsum` = the producer's own replicated sums (StepPlan.bnfwd:
    [2][reps][C] of y - shift, shift the producing conv's bias) give the mean / variance the
    consuming kernels used; `bsum` (StepPlan.bnbwd: sum g*xhat, sum g) the BatchNorm-backward's.
    Without them the statistics come from the stored tensors (fp64)."""

    def __init__(self, y, gamma, beta, fsum=None, shift=None):
        self.y = y
        self.M = y.shape[0] * y.shape[2] * y.shape[3]
        if fsum is not None:
            s0, s1 = fsum[0] / self.M, fsum[1] / self.M
            self.mean = s0 + shift
            self.var = torch.clamp(s1 - s0 * s0, min=0.0)
        else:
            self.mean = y.mean((0, 2, 3))
            self.var = y.var((0, 2, 3), unbiased=False)
        self.invstd = 1.0 / torch.sqrt(self.var + BN_EPS)
        self.gamma, self.beta = gamma, beta
        v = lambda t: t.view(1, -1, 1, 1)
        self.xhat = (y - v(self.mean)) * v(self.invstd)
        self.z = v(gamma) * self.xhat + v(beta)

    def act(self):
        """The consumer's operand: bf16(lrelu(BN(y)))."""
        return bf(lrelu(self.z))

    def ambiguous(self):
        return self.z.abs() < 1e-5 * self.z.abs().max()

    def lrelu_back(self, dact):
        """dL/dz from dL/d lrelu(z)."""
        return torch.where(self.z > 0, dact, dact * SLOPE)

    def dy(self, g, bsum=None):
        """dL/dy from g = dL/dz (BatchNorm backward, batch statistics), rounded to bf16 as the
        consuming kernel stages it: a*g + b*y + c.  bsum: the producer's (sum g*xhat, sum g)."""
        v = lambda t: t.view(1, -1, 1, 1)
        if bsum is not None:
            mgx, mg = bsum[0] / self.M, bsum[1] / self.M
        else:
            mg = g.mean((0, 2, 3))
            mgx = (g * self.xhat).mean((0, 2, 3))
        a = self.gamma * self.invstd
        b = -a * self.invstd * mgx
        c = -a * (mg - self.mean * self.invstd * mgx)
        return bf(v(a) * g + v(b) * self.y + v(c))

    def dgamma(self, g):
        return (g * self.xhat).sum((0, 2, 3))

    def dbeta(self, g):
        return g.sum((0, 2, 3))


def cmp_bf16(got, ref, mask=None):
    """A bf16 output: relative norm <= 3e-3 (its rounding is 2^-9 relative per element) and
    max |got - ref| <= 2^-7 max |ref| (two bf16 ulps at the largest magnitude); elements whose
    LeakyReLU branch is ambiguous (mask) are excluded and counted."""
    n_amb = 0
    if mask is not None:
        n_amb = int(mask.sum())
        keep = ~mask
        got, ref = got[keep], ref[keep]
    d = got - ref
    rn = float(d.norm() / ref.norm().clamp_min(1e-30))
    rm = float(d.abs().max() / ref.abs().max().clamp_min(1e-30))
    ok = rn <= 3e-3 and rm <= 2.0 ** -7 and n_amb <= 1e-3 * (ref.numel() + n_amb)
    return ok, {"relnorm": rn, "relmax": rm, "ambiguous": n_amb, "elements": ref.numel() + n_amb}


def cmp_f32(got, ref, relmax_bar=2e-3, relnorm_bar=1e-3):
    rm = float((got - ref).abs().max() / ref.abs().max().clamp_min(1e-30))
    rn = float((got - ref).norm() / ref.norm().clamp_min(1e-30))
    return rm <= relmax_bar and rn <= relnorm_bar, {"relmax": rm, "relnorm": rn, "elements": ref.numel()}


def conv_grads(kind, x, w, dy, stride, pad, op=0):
    """(dx, dw) of conv2d / conv_transpose2d by fp64 autograd."""
    x = x.clone().requires_grad_(True)
    w = w.clone().requires_grad_(True)
    y = (F.conv2d(x, w, None, stride, pad) if kind == "conv" else
         F.conv_transpose2d(x, w, None, stride, pad, op))
    y.backward(dy)
    return x.grad, w.grad


class StepCheck:
    """Checks one step of a VanillaVAE-family StepPlan (bf16, the TrainStep engine's plan:
    latent_fused, pad_rgb; elbo_in_head for vanilla / BetaVAE-H, vae_elbo_fwd for IWAE)."""

    def __init__(self, net, plan, pre_params, pre_lowp, pre_running, post_params, post_lowp, post_running,
                 lr, loss, kld_weight, beta=4.0):
        self.net, self.plan = net, plan
        self.lr, self.loss, self.M_N, self.beta = lr, loss, kld_weight, beta
        lay = net.layout
        self.P = {k: cpu64(v) for k, v in lay.export_reference(pre_params).items()}        # fp32 master
        self.W = {k: cpu64(v) for k, v in lay.export_reference(pre_lowp.float()).items()}  # bf16 copy
        self.G = {k: cpu64(v) for k, v in lay.export_reference(plan.grads).items()}        # GPU grads
        self.pre_params, self.post_params = pre_params, post_params
        self.post_lowp = post_lowp
        self.pre_running, self.post_running = pre_running, post_running
        self.checks: List[Check] = []
        self.h = net.hidden_dims
        self.B, self.S = plan.B, plan.S
        # which call produced each BatchNorm's forward sums (the conv / convT feeding it) and its
        # backward sums (the data gradient whose epilogue applies its LeakyReLU backward)
        h, nd = self.h, len(self.h) - 1
        self._stat_call = {f"encoder.{i}.1": ("vae_conv2d_fwd", i) for i in range(len(h))}
        self._stat_call.update({f"decoder.{i}.1": ("vae_convT2d_fwd", i) for i in range(nd)})
        self._stat_call["final_layer.1"] = ("vae_convT2d_fwd", nd)
        self._bstat_call = {"final_layer.1": ("vae_head_bwd", 0), f"decoder.{nd - 1}.1": ("vae_convT2d_bwd", 0),
                            f"encoder.{len(h) - 1}.1": ("vae_latent_fc_bwd", 0)}
        self._bstat_call.update({f"decoder.{i}.1": ("vae_convT2d_bwd_data", nd - 2 - i) for i in range(nd - 1)})
        self._bstat_call.update({f"encoder.{i}.1": ("vae_conv2d_bwd_data", len(h) - 2 - i) for i in range(len(h) - 1)})

    def add(self, name, call, res):
        ok, det = res
        self.checks.append(Check(name, call, bool(ok), det))

    def bn(self, y, prefix):
        """The BatchNorm `prefix` of stored map y with the producer's own statistics (teacher forcing),
        and a check of those statistics against the stored tensor's."""
        fs = cpu64(self.plan.bnfwd[prefix]).sum(1)                      # [2][C]
        conv = prefix[:-2] + ".0.bias"
        bn = BN(y, self.P[prefix + ".weight"], self.P[prefix + ".bias"], fs, self.P[conv])
        sh = self.P[conv].view(1, -1, 1, 1)
        want = torch.stack([(y - sh).sum((0, 2, 3)), ((y - sh) ** 2).sum((0, 2, 3))])
        # (the producer sums its fp32 accumulators before the bf16 store: relative 1e-3 is that rounding)
        self.add(f"{prefix} forward statistics", self._stat_call.get(prefix, ("?", 0)),
                 cmp_f32(fs, want, 5e-3, 2e-3))
        return bn

    def bsum(self, prefix, bn, g):
        """The producer's BatchNorm-backward sums of `prefix`, checked against the stored gradient."""
        bs = cpu64(self.plan.bnbwd[prefix]).sum(1)                      # [sum g*xhat, sum g][C]
        self.add(f"{prefix} backward statistics", self._bstat_call.get(prefix, ("?", 0)),
                 cmp_f32(bs, torch.stack([bn.dgamma(g), bn.dbeta(g)]), 1e-2, 5e-3))
        return bs

    # -------------------------------------------------------------------------------- forward
    def run(self):
        p, h, B, S = self.plan, self.h, self.B, self.S
        BS = B * S
        x = cpu64(p.x)
        # step head: the image as 8 zero-padded bf16 NHWC channels (vae_step_begin_ex)
        x8 = cpu64(p.x8)
        want8 = torch.zeros_like(x8)
        want8[..., :3] = bf(x.permute(0, 2, 3, 1))
        self.add("x8 (padded NHWC image)", ("vae_step_begin_ex", 0),
                 (bool(torch.equal(x8, want8)), {"max_abs": float((x8 - want8).abs().max())}))
        # encoder
        enc = [nchw(t) for t in p.enc]
        bns = []
        inp = bf(x)
        for i in range(len(h)):
            pre = f"encoder.{i}"
            ref = F.conv2d(inp, self.W[pre + ".0.weight"], self.P[pre + ".0.bias"], 2, 1)
            self.add(f"{pre} conv fwd", ("vae_conv2d_fwd", i), cmp_bf16(enc[i], ref))
            bns.append(self.bn(enc[i], pre + ".1"))
            inp = bns[-1].act()
        # running statistics (first forward consumer of each BatchNorm)
        self._check_running([(f"encoder.{i}.1", enc[i]) for i in range(len(h))], "encoder")
        # fc_mu | fc_var (vae_latent_fc_fwd)
        act4 = inp.flatten(1)
        mu = act4 @ self.W["fc_mu.weight"].t() + self.P["fc_mu.bias"]
        lv = act4 @ self.W["fc_var.weight"].t() + self.P["fc_var.bias"]
        mulv = cpu64(p.mulv)
        self.add("fc_mu|fc_var", ("vae_latent_fc_fwd", 0), cmp_f32(mulv, torch.cat([mu, lv], 1)))
        # reparameterization with the on-device eps draw, decoder_input (vae_latent_dec_fwd)
        gmu, glv = mulv[:, :mulv.shape[1] // 2], mulv[:, mulv.shape[1] // 2:]
        eps = cpu64(p.eps).view(BS, -1)
        n = eps.numel()
        em, es = float(eps.mean()), float(eps.std())
        self.add("eps ~ N(0,1) (device draw)", ("vae_latent_dec_fwd", 0),
                 (abs(em) < 6.0 / math.sqrt(n) and abs(es - 1.0) < 6.0 / math.sqrt(2 * n) + 1e-3 and
                  bool(torch.isfinite(eps).all()), {"mean": em, "std": es, "n": n}))
        mu_r, lv_r = gmu.repeat_interleave(S, 0), glv.repeat_interleave(S, 0)
        z = cpu64(p.z).float().double()
        zr = mu_r + eps * torch.exp(0.5 * lv_r)
        self.add("reparameterize z", ("vae_latent_dec_fwd", 0), cmp_bf16(z, zr))
        h0_ref = bf(z) @ self.W["decoder_input.weight"].t() + self.P["decoder_input.bias"]
        h0 = nchw(p.h0)
        self.add("decoder_input", ("vae_latent_dec_fwd", 0), cmp_bf16(h0.flatten(1), h0_ref))
        # decoder ConvT stack
        r = h[::-1]
        outs = [nchw(t) for t in p.dec] + [nchw(p.fin)]
        names = [f"decoder.{i}" for i in range(len(r) - 1)] + ["final_layer"]
        dbns = []
        inp = h0
        for i, pre in enumerate(names):
            ref = F.conv_transpose2d(inp, self.W[pre + ".0.weight"], self.P[pre + ".0.bias"], 2, 1, 1)
            self.add(f"{pre} convT fwd", ("vae_convT2d_fwd", i), cmp_bf16(outs[i], ref))
            dbns.append(self.bn(outs[i], pre + ".1"))
            inp = dbns[-1].act()
        self._check_running([(pre + ".1", outs[i]) for i, pre in enumerate(names)], "decoder")
        # head: Conv2d(32 -> 3) + tanh, SSE (vae_head_fwd)
        wh = bf(self.P["final_layer.3.weight"])
        pre_t = F.conv2d(inp, wh, self.P["final_layer.3.bias"], 1, 1)
        recon = cpu64(p.recon)
        self.add("head conv + tanh (recon)", ("vae_head_fwd", 0), cmp_bf16(recon, torch.tanh(pre_t)))
        xt = x.repeat_interleave(S, 0)
        sse = cpu64(p.sse)
        self.add("per-image SSE", ("vae_head_fwd", 0),
                 cmp_f32(sse, ((recon - xt) ** 2).sum((1, 2, 3)), 1e-5, 1e-5))
        # ELBO terms from the GPU's sse and mu|logvar (vae_head_bwd's reduction or vae_elbo_fwd)
        elbo_call = ("vae_head_bwd", 0) if p.elbo_in_head else ("vae_elbo_fwd", 0)
        head_coef, kl_coef, want_out = self._elbo(sse, gmu, glv)
        got_out = cpu64(p.out)[:3]
        self.add("ELBO loss terms", elbo_call, cmp_f32(got_out, want_out, 1e-5, 1e-5))
        if not p.elbo_in_head:
            self.add("ELBO backward coefficients", elbo_call,
                     cmp_f32(torch.cat([cpu64(p.head_coef), cpu64(p.kl_coef)]), torch.cat([head_coef, kl_coef]),
                             1e-4, 1e-5))
        # ------------------------------------------------------------------------- backward
        # head backward: seed coef * (recon - x)(1 - recon^2), bf16 operand; dW (fp32)
        seed = bf(head_coef.view(-1, 1, 1, 1) * (recon - xt) * (1 - recon * recon))
        dact, dwh = conv_grads("conv", inp, wh, seed, 1, 1)
        g_fin = nchw(p.g_fin)
        fbn = dbns[-1]
        self.add("head bwd data (g final_layer)", ("vae_head_bwd", 0),
                 cmp_bf16(g_fin, fbn.lrelu_back(dact), fbn.ambiguous()))
        self.add("head bwd filter (final_layer.3.weight)", ("vae_head_bwd", 0),
                 cmp_f32(self.G["final_layer.3.weight"], dwh))
        self.add("head bwd bias (final_layer.3.bias)", ("vae_head_bwd", 0),
                 cmp_f32(self.G["final_layer.3.bias"], seed.sum((0, 2, 3)), 2e-3, 1e-3))
        # decoder backward, last block first: data gradients through each BN-backward
        g_outs = [nchw(t) for t in p.g_dec] + [g_fin]
        g_h0 = nchw(p.g_h0)
        wgrad_refs = {}
        for i in reversed(range(len(names))):
            pre = names[i]
            bs = self.bsum(pre + ".1", dbns[i], g_outs[i])
            dy = dbns[i].dy(g_outs[i], bs)
            x_in = dbns[i - 1].act() if i > 0 else h0
            dx, dw = conv_grads("convT", x_in, self.W[pre + ".0.weight"], dy, 2, 1, 1)
            wgrad_refs[pre + ".0.weight"] = dw
            call = ("vae_convT2d_bwd", 0) if i == len(names) - 1 else ("vae_convT2d_bwd_data", len(names) - 2 - i)
            if i > 0:
                self.add(f"{pre} convT bwd data", call,
                         cmp_bf16(g_outs[i - 1], dbns[i - 1].lrelu_back(dx), dbns[i - 1].ambiguous()))
            else:
                self.add(f"{pre} convT bwd data (d decoder_input)", call, cmp_bf16(g_h0, dx))
            self._bn_param_grads(pre + ".1", bs)
        # bottleneck backward (vae_latent_dec_bwd / vae_latent_fc_bwd)
        gh = g_h0.flatten(1)
        self.add("decoder_input.weight grad", ("vae_latent_dec_bwd", 0),
                 cmp_f32(self.G["decoder_input.weight"], gh.t() @ bf(z)))
        self.add("decoder_input.bias grad", ("vae_latent_dec_bwd", 0),
                 cmp_f32(self.G["decoder_input.bias"], gh.sum(0)))
        dz = gh @ self.W["decoder_input.weight"]                        # [BS, D]
        std_r = torch.exp(0.5 * lv_r)
        kc = kl_coef.view(-1, 1)
        dmu = (dz + kc * mu_r).view(B, S, -1).sum(1)
        dlv = (dz * eps * 0.5 * std_r + kc * 0.5 * (torch.exp(lv_r) - 1.0)).view(B, S, -1).sum(1)
        dmulv = torch.cat([dmu, dlv], 1)
        self.add("d mu|logvar", ("vae_latent_dec_bwd", 0), cmp_f32(cpu64(p.dmulv).view(B, -1), dmulv))
        gd = cpu64(p.dmulv).view(B, -1)
        g16 = bf(gd)                     # (the bottleneck kernels stage d[mu|logvar] as a bf16 operand)
        self.add("fc_mu.weight grad", ("vae_latent_fc_bwd", 0),
                 cmp_f32(self.G["fc_mu.weight"], g16[:, :gd.shape[1] // 2].t() @ act4))
        self.add("fc_var.weight grad", ("vae_latent_fc_bwd", 0),
                 cmp_f32(self.G["fc_var.weight"], g16[:, gd.shape[1] // 2:].t() @ act4))
        self.add("fc_mu|fc_var bias grad", ("vae_latent_fc_bwd", 0),
                 cmp_f32(torch.cat([self.G["fc_mu.bias"], self.G["fc_var.bias"]]), gd.sum(0)))
        wcat = torch.cat([self.W["fc_mu.weight"], self.W["fc_var.weight"]], 0)
        dact4 = (g16 @ wcat).view_as(bns[-1].y)
        g_enc = [nchw(t) for t in p.g_enc]
        self.add("fc bwd data (g encoder.4)", ("vae_latent_fc_bwd", 0),
                 cmp_bf16(g_enc[-1], bns[-1].lrelu_back(dact4), bns[-1].ambiguous()))
        # encoder backward
        for i in reversed(range(len(h))):
            pre = f"encoder.{i}"
            bs = self.bsum(pre + ".1", bns[i], g_enc[i])
            dy = bns[i].dy(g_enc[i], bs)
            x_in = bns[i - 1].act() if i > 0 else bf(x)
            dx, dw = conv_grads("conv", x_in, self.W[pre + ".0.weight"], dy, 2, 1)
            wgrad_refs[pre + ".0.weight"] = dw
            if i > 0:
                self.add(f"{pre} conv bwd data", ("vae_conv2d_bwd_data", len(h) - 1 - i),
                         cmp_bf16(g_enc[i - 1], bns[i - 1].lrelu_back(dx), bns[i - 1].ambiguous()))
            self._bn_param_grads(pre + ".1", bs)
        # every conv / convT weight gradient (the grouped launch vae_conv_bwd_filter_batch)
        for k, ref in wgrad_refs.items():
            call = ("vae_convT2d_bwd", 0) if k == "final_layer.0.weight" else ("vae_conv_bwd_filter_batch", 0)
            self.add(f"{k} grad", call, cmp_f32(self.G[k], ref))
        self._check_adam()
        return self.checks

    # -------------------------------------------------------------------------------- pieces
    def _elbo(self, sse, mu, lv):
        """(head_coef [BS], kl_coef [BS], [loss, Reconstruction_Loss, KLD]) in fp64."""
        B, S = self.B, self.S
        E = 3 * self.net.img_size ** 2
        kld = -0.5 * (1 + lv - mu * mu - torch.exp(lv)).sum(1)                  # [B]
        if self.loss == "iwae":
            lw = sse.view(B, S) / E + self.M_N * kld.view(B, 1)
            w = torch.softmax(lw, 1)
            wl = (w * lw).sum(1, keepdim=True)
            g = w * (1 + lw - wl) / B                                           # dL/dlw
            out = torch.stack([wl.mean(), sse.sum() / E / (B * S), -kld.mean()])
            return (g * 2.0 / E).flatten(), (g * self.M_N).flatten(), out
        recon = sse.sum() / (B * E)
        km = kld.mean()
        if self.loss == "vanilla":
            loss, klc, rep = recon + self.M_N * km, self.M_N, -km
        else:                                                                 # BetaVAE-H
            loss, klc, rep = recon + self.beta * self.M_N * km, self.beta * self.M_N, km
        hc = torch.full((B,), 2.0 / (B * E), dtype=D64)
        return hc, torch.full((B,), klc / B, dtype=D64), torch.stack([loss, recon, rep])

    def _bn_param_grads(self, prefix, bs):
        """dL/dgamma, dL/dbeta as the weight-gradient call of the conv feeding the BatchNorm publishes
        them (StepPlan.bwd_extras; the full-resolution ConvT's own call for final_layer.1): the sums
        the backward produced (checked against the stored gradient by bsum)."""
        call = ("vae_convT2d_bwd", 0) if prefix == "final_layer.1" else ("vae_conv_bwd_filter_batch", 0)
        self.add(f"{prefix}.weight grad (dgamma)", call, cmp_f32(self.G[prefix + ".weight"], bs[0], 1e-5, 1e-5))
        self.add(f"{prefix}.bias grad (dbeta)", call, cmp_f32(self.G[prefix + ".bias"], bs[1], 1e-5, 1e-5))

    def _check_running(self, pairs, tag):
        lay = self.net.layout
        pre, post = cpu64(self.pre_running), cpu64(self.post_running)
        worst = 0.0
        for prefix, y in pairs:
            b = lay.bn_by_prefix[prefix]
            C = b.channels
            m0, v0 = pre[b.offset:b.offset + C], pre[b.offset + C:b.offset + 2 * C]
            m1, v1 = post[b.offset:b.offset + C], post[b.offset + C:b.offset + 2 * C]
            # the batch statistics the kernels used: the producer's own sums (checked against the
            # stored tensor by bn()), unbiased variance for the running estimate (nn.BatchNorm2d)
            M = y.shape[0] * y.shape[2] * y.shape[3]
            fs = cpu64(self.plan.bnfwd[prefix]).sum(1)
            s0, s1 = fs[0] / M, fs[1] / M
            mean = s0 + self.P[prefix[:-2] + ".0.bias"]
            var = torch.clamp(s1 - s0 * s0, min=0.0) * M / (M - 1)
            wm, wv = (1 - MOM) * m0 + MOM * mean, (1 - MOM) * v0 + MOM * var
            worst = max(worst, float((m1 - wm).abs().max() / wm.abs().max().clamp_min(1e-30)),
                        float((v1 - wv).abs().max() / wv.abs().max()))
        self.add(f"{tag} BatchNorm running statistics", ("vae_conv2d_fwd" if tag == "encoder" else "vae_convT2d_fwd", 1),
                 (worst <= 1e-5, {"relmax": worst}))

    def _check_adam(self):
        """torch.optim.Adam (experiment.py:308-311), first step from zero state, on the GPU's grads."""
        g = cpu64(self.plan.grads)
        p0, p1 = cpu64(self.pre_params), cpu64(self.post_params)
        b1, b2, eps = 0.9, 0.999, 1e-8
        m, v = (1 - b1) * g, (1 - b2) * g * g
        want = p0 - self.lr / (1 - b1) * m / (torch.sqrt(v) / math.sqrt(1 - b2) + eps)
        err = float(((p1 - want).abs() / (p0.abs() + self.lr)).max())
        self.add("Adam parameters", ("adam", 0), (err <= 1e-6, {"max_scaled_err": err}))
        lowp = self.post_lowp.detach().cpu()
        want_lp = self.post_params.detach().cpu().to(torch.bfloat16)
        eq = float((lowp == want_lp).double().mean())
        self.add("Adam bf16 weight copy", ("adam", 0), (eq == 1.0, {"equal_fraction": eq}))


def run_bench_step(arch: str, batch: int, seed: int = 1265, segments: int = 1, defer: bool = True):
    """One step of bench.py's plan for `arch` at `batch` (graph-replayed TrainStep, on-device eps),
    with the pre/post state snapshots StepCheck needs and the kernels every call launched.
    segments > 1: the weight gradients batched per backward segment as the data-parallel step cuts
    it into gradient buckets (dp.plan_buckets; TrainStep's default of two at N > 1)."""
    from vae_amd import _lib as L
    from vae_amd.engine import FusedAdam, TrainStep
    from vae_amd.net import StepPlan, VAENet, call_one
    from gpu_util import launched
    S = 5 if arch == "iwae" else 1
    loss = {"vanilla": "vanilla", "betaH": "betaH", "iwae": "iwae"}[arch]
    kld = {"vanilla": 1e-8, "betaH": 2.5e-4, "iwae": 2.5e-4}[arch]
    lr = {"vanilla": 0.005, "betaH": 0.005, "iwae": 0.007}[arch]
    gen = torch.Generator().manual_seed(seed)
    net = VAENet(latent_dim=128, dtype=torch.bfloat16, device="cuda", generator=gen)
    plan = StepPlan(net, batch, loss=loss, kld_weight=kld, samples=S)
    if segments > 1:
        from vae_amd.dp import plan_buckets
        ends = [b[0] for b in plan_buckets(plan.bwd_calls_raw, plan.grads, net.layout, segments)]
        assert len(ends) == segments, ends
        plan.batch_wgrads(ends)
    opt = FusedAdam(net, lr=lr)
    g = torch.Generator(device="cuda").manual_seed(seed)
    plan.x.copy_(torch.rand(plan.x.shape, generator=g, device="cuda"))
    step = TrainStep(net, plan, opt, graph=True, device_eps=seed, defer_reductions=defer)
    assert step.device_eps and plan.latent_fused and plan.pad_rgb
    pre = (net.params.clone(), net.lowp.clone(), net.running.clone())
    names_step = launched(step)                 # capture (warm-up step + restore) and one replay
    torch.cuda.synchronize()
    post = (net.params.clone(), net.lowp.clone(), net.running.clone())
    chk = StepCheck(net, plan, pre[0], pre[1], pre[2], post[0], post[1], post[2], lr, loss, kld)
    checks = chk.run()
    # the kernels of every call (each call launched once more with the log on; after the checks)
    sp = L.stream_ptr()
    per_call: Dict[Tuple[str, int], str] = {}
    seen: Dict[str, int] = {}
    for fn, ref in plan.fwd_calls[step._begin[1]:] + plan.bwd_calls:
        k = seen.get(fn, 0)
        seen[fn] = k + 1
        per_call[(fn, k)] = launched(lambda: call_one(fn, ref, sp))
    per_call[("vae_step_begin_ex", 0)] = launched(lambda: L.call("vae_step_begin_ex", step._begin[0], sp))
    if step.deferred:       # (the default one-rank step: slab reductions and loss inside the optimizer launch)
        per_call[("adam", 0)] = launched(lambda: opt.apply_deferred(plan.grads, step._slabs, step._elbo, sp))
    else:
        per_call[("adam", 0)] = launched(lambda: opt.apply(plan.grads, sp, refresh_swaps=False))
    # what TrainStep's capture ran besides the step (it restores the state the warm-up step changed
    # and refreshes the bf16 weight copies: net.sync_lowp) — not part of the replayed step
    per_call[("restore", 0)] = launched(net.sync_lowp)
    torch.cuda.synchronize()
    return checks, names_step, per_call


def kernel_names(text: str) -> List[str]:
    """Demangled kernel names of a vae_launch_log_names listing."""
    out = []
    for line in text.splitlines():
        f = line.split("\t")
        if f and f[0]:
            out.append(f[1] if len(f) > 1 and f[1] else f[0])
    return out


def coverage(checks: List[Check], names_step: str, per_call: Dict[Tuple[str, int], str]):
    """kernel -> names of the PASSING checks of the calls that launch it; and the kernels of the step
    no passing check covers."""
    ok_by_call: Dict[Tuple[str, int], List[str]] = {}
    for c in checks:
        if c.ok:
            ok_by_call.setdefault(c.call, []).append(c.name)
    cov: Dict[str, List[str]] = {}
    for call, text in per_call.items():
        if call[0] == "restore":
            continue
        for k in kernel_names(text):
            cov.setdefault(k, [])
            cov[k] += ok_by_call.get(call, [])
    restore = set(kernel_names(per_call.get(("restore", 0), "")))
    # every kernel the step launched belongs to a call of the step (or to the capture's restore)
    step_kernels = [k for k in kernel_names(names_step) if k in cov or k not in restore]
    missing = [k for k in step_kernels if not cov.get(k)]
    return cov, step_kernels, missing
