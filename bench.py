#!/usr/bin/env python3
"""Benchmark: train images/sec of the VanillaVAE training step on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--dtype bf16|f32] [--arch vanilla|betaH|iwae|vq]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

With --gpus N > 1 and no RANK in the environment, this process starts the N rank processes
itself (before anything touches the GPU) and waits for them; rank r runs on device
r % device_count.  Ranks on distinct devices exchange gradients over RCCL; when there are
fewer devices than ranks (a 1-GPU box) they share devices and fall back to gloo, because RCCL
needs one device per rank.  --selftest replaces the training step with a CPU stand-in (the
gradient exchange only) to check the launcher, the barrier/max-over-ranks timing and the
output line without a GPU (tests/test_bench_launcher.py).

Workload (BASELINE.json configs[1]): VanillaVAE latent_dim=128, 64x64x3 synthetic images, batch 64
per GPU (weak scaling, data parallel over ranks, RCCL gradient all-reduce), bf16 MFMA with fp32
accumulation / statistics / optimizer.  A "step" = forward + ELBO + backward + [all-reduce] + Adam
(experiment.py:45-86 + :308-311), inputs already resident in HBM, the whole step replayed from
HIP graphs.  Prints ONE JSON line on rank 0.

roofline: the dominant kernel of the step (largest time per step, measured with HIP events on the
stream it runs on, each launch isolated behind a spin kernel so the events bracket only it) with
its algorithmic FLOPs/bytes per launch; `traffic` comes from the committed
rocprofv3 --pmc summary in profiles/ when present.
cpu_baseline: the oracle (oracle/vae_oracle.py, a PyTorch-CPU fp32 restatement pinned against the
reference) timed on this host's cores on a bounded sample of the same workload.
"""
from __future__ import annotations

import argparse
import glob
import json
import math
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [REPO, os.path.join(REPO, "pytorch-vae_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "train images/sec (node) VanillaVAE 64×64 bs=64 at 1/2/4/8 GPU; ELBO match"
MFMA_PEAK_TFLOPS = {"bf16": 2500.0, "f32": 157.3}   # dense, MI355X_MICROARCH.md
HBM_PEAK_GBS = 8000.0
# a profile summary pairs with a call only when its kernels' rocprof time (average per launch x
# launches in the call) is within this fraction of the call's event-timed duration
PAIR_TOL = 0.15
# the fork's Autoencoder configs (models/autoencoder.py; hidden_dims of configs/*ae*.yaml)
AE_WIDTHS = {"ae_big": [128, 256, 512, 1024, 2048], "ae_vbig": [256, 512, 1024, 2048, 4096],
             "ae_vvbig": [512, 1024, 2048, 4096, 4096]}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=64, help="per-GPU batch")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--no-dropin", action="store_true", help="skip the drop-in path leg (model.forward + "
                    "loss_function + backward + torch.optim.Adam through VAEXperiment.training_step)")
    ap.add_argument("--arch", default="vanilla", choices=["vanilla", "betaH", "iwae", "vq"] + sorted(AE_WIDTHS),
                    help="vq: BASELINE.json configs[4], VQ-VAE B=128 (pass --batch 128); ae_big / ae_vbig / "
                         "ae_vvbig: the Autoencoder of configs/big_ae.yaml / patient_vbig_ae.yaml / "
                         "patient_vvbig_ae.yaml (MSE, no KL)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--buckets", type=int, default=2,
                    help="N > 1: gradient buckets (all-reduces) per step; with more than one the weight "
                         "gradients closing each bucket but the last overlap the next backward segment")
    ap.add_argument("--no-overlap", action="store_true", help="N > 1: no overlap stream (TrainStep(overlap=False))")
    ap.add_argument("--comm-bf16", action="store_true",
                    help="N > 1: all-reduce the gradients in bf16 (TrainStep(comm_dtype=torch.bfloat16); opt-in)")
    ap.add_argument("--force-buckets", action="store_true",
                    help="run the bucketed all-reduce path even at one rank (under torch.distributed.run)")
    ap.add_argument("--host-comm", action="store_true",
                    help="N > 1: issue the bucket all-reduces from the host between segment graphs instead "
                         "of capturing them (RCCL) into the step's one graph (engine.TrainStep(graph_comm))")
    ap.add_argument("--concurrent", choices=["auto", "on", "off"], default="auto",
                    help="weight gradients on a side stream beside the data-gradient chain; auto = off: the "
                         "VanillaVAE family measured 0.88 vs 0.77 ms (r1: the graph's per-call fork/join edges cost "
                         "more than the overlap gains), VQ-VAE 3.436 on vs 3.330 off at r4 (it was 9.96 -> 8.51 ms "
                         "in r1, before the image-tile kernels filled the chip on their own)")
    ap.add_argument("--wg-overlap", action="store_true",
                    help="the decoder's weight gradients as their own batch on a side stream in the graph "
                         "(StepPlan(wg_overlap=True)), beside the encoder's data gradients")
    ap.add_argument("--no-defer", action="store_true",
                    help="keep the slab reductions as launches of their own (TrainStep(defer_reductions=False))")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--kernel-breakdown", action="store_true", help="print per-kernel times to stderr")
    ap.add_argument("--selftest", action="store_true",
                    help="CPU stand-in step (launcher / timing / output contract check; no GPU)")
    return ap.parse_args()


# ----------------------------------------------------------------------------- rank launcher
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int) -> int:
    """Start n rank processes of this script (torchrun-style env) and wait for them.  Runs in a
    parent that never touched the GPU; if one rank fails the others are stopped (by PID)."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    return rc


# ----------------------------------------------------------------------------- kernels
def conv_cost(fn, a, dsz):
    """(flops, bytes) per launch by the counting rules of BASELINE.md §3 / SURVEY §8(d)."""
    R = a.r
    n, h, w, c, k, p, q = a.n, a.h, a.w, a.c, a.k, a.p, a.q
    if fn.startswith("vae_conv2d"):
        macs = n * p * q * k * c * R * R
        x_b, y_b = n * h * w * c * (4 if a.x_nchw_f32 else dsz), n * p * q * k * dsz
    else:  # transposed: 2*N*Cin*Hin*Win*Cout*R*S
        macs = n * h * w * c * k * R * R
        x_b, y_b = n * h * w * c * dsz, n * p * q * k * dsz
    w_b = k * c * R * R * dsz
    if fn.endswith("_fwd"):
        return 2 * macs, x_b + w_b + y_b
    if fn.endswith("_bwd_data"):
        return 2 * macs, y_b + w_b + x_b
    if fn.endswith("_bwd"):                                  # both: dy + its pre-BN y, x, W -> dx, dW
        return 4 * macs, 2 * y_b + 2 * x_b + w_b + k * c * R * R * 4
    return 2 * macs, x_b + y_b + k * c * R * R * 4          # bwd_filter writes fp32 dW


def linear_cost(fn, a, dsz):
    macs = a.m * a.n * a.k
    if fn.endswith("_fwd"):
        return 2 * macs, a.m * a.k * dsz + a.n * a.k * dsz + a.m * a.n * (4 if a.y_f32 else dsz)
    if fn.endswith("_bwd_data"):
        return 2 * macs, a.m * a.n * (4 if a.dy_f32 else dsz) + a.n * a.k * dsz + a.m * a.k * dsz
    return 2 * macs, a.m * a.n * (4 if a.dy_f32 else dsz) + a.m * a.k * dsz + a.n * a.k * 4


def head_cost(fn, a, dsz):
    macs = a.n * a.h * a.w * 3 * a.c * 9
    x_b = a.n * a.h * a.w * a.c * dsz
    img = a.n * 3 * a.h * a.w * 4
    if fn == "vae_head_fwd":
        return 2 * macs, x_b + 2 * img          # reads x, target; writes recon
    if fn == "vae_head_bwd_data":
        return 2 * macs, 2 * img + x_b + x_b    # recon, target, y (epilogue) -> dx
    if fn == "vae_head_bwd":
        return 4 * macs, 2 * img + x_b + x_b + 3 * a.c * 9 * 4   # data + filter in one pass
    return 2 * macs, x_b + 2 * img + 3 * a.c * 9 * 4


def vq_cost(fn, a, dsz):
    if fn == "vae_vq_fwd":       # distance GEMM rows x codes x dim (+ argmin, gather)
        return 2 * a.rows * a.codes * a.dim, 2 * a.rows * a.dim * dsz + a.codes * a.dim * 4 + a.rows * 8
    return 0, 3 * a.rows * a.dim * dsz + a.rows * 8 + a.codes * a.dim * 4


def kernel_costs(plan, dsz):
    from vae_amd import _lib as L
    out = []
    for fn, ref in plan.fwd_calls + plan.bwd_calls:
        if fn == "vae_convT2d_fwd_recon":           # (conv args, recon args): the ConvT + Tanh/MSE
            a, rc = ref[0]._obj, ref[1]._obj
            f, b = conv_cost("vae_convT2d_fwd", a, dsz)
            img = rc.n * rc.c * rc.h * rc.w * 4
            out.append((fn, ref, f, b + 2 * img + (rc.n * rc.h * rc.w * 8 * dsz if rc.dy else 0)))
            continue
        if isinstance(ref, tuple) or ref is None:
            out.append((fn, None, 0, 0))
            continue
        if isinstance(ref, L.FilterBatch):          # several layers' weight gradients in one call
            fb = [conv_cost(f, r._obj, dsz) for f, r in ref.calls]
            out.append((fn, ref, sum(c[0] for c in fb), sum(c[1] for c in fb)))
            continue
        a = ref._obj
        if isinstance(a, L.ConvArgs):
            f, b = conv_cost(fn, a, dsz)
        elif isinstance(a, L.LinearArgs):
            f, b = linear_cost(fn, a, dsz)
        elif isinstance(a, L.HeadArgs):
            f, b = head_cost(fn, a, dsz)
        elif isinstance(a, L.VqArgs):
            f, b = vq_cost(fn, a, dsz)
        elif isinstance(a, L.BnApplyArgs):          # materialised transform: read (+ aux), write
            f, b = 0, a.rows * a.channels * dsz * (3 if a.xf.kind == L.X_BN_DY else 2)
        elif isinstance(a, L.ReconLossArgs):        # recon, target read; dL/drecon written
            f, b = 0, 3 * a.n * a.c * a.h * a.w * 4
        else:
            f, b = 0, 0
        out.append((fn, ref, f, b))
    return out


def time_kernels(plan, reps=20):
    """Per-launch duration of every call of the step: `reps` back-to-back launches of the call
    bracketed by HIP events on the stream it runs on, queued behind a spin kernel so host launch
    latency is not measured; average per launch.  (The calls accumulate into the plan's gradient
    buffers; this runs after the timed region and its loss terms were read.)"""
    from vae_amd.net import call_one
    from vae_amd.engine import begin_args
    st = torch.cuda.current_stream()
    sp = st.cuda_stream
    # the leading image / weight padding calls run inside vae_step_begin_ex in the trained step
    # (engine.begin_args), not as launches of their own: not timed here (0 us)
    nbegin = begin_args(plan, torch.zeros(1, dtype=torch.int64, device="cuda"))[1]
    res = []
    for i, (fn, ref) in enumerate(plan.fwd_calls + plan.bwd_calls):
        if i < nbegin:
            res.append((fn, ref, 0.0))
            continue
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(400000)               # spin: everything below is queued behind it
        e0.record(st)
        for _ in range(reps):
            call_one(fn, ref, sp)
        e1.record(st)
        torch.cuda.synchronize()
        res.append((fn, ref, e0.elapsed_time(e1) * 1e3 / reps))   # µs per launch
    return res


def call_kernels(fn, ref):
    """The device kernels one call of the step launches, as (mangled, demangled, launches): the call
    is run once more with the library's launch log on (vaehip.h vae_launch_log) — what rocprofv3
    and the PMC summaries key their rows by; `launches` is how many times the call launches that
    kernel (a grouped call may run one kernel several times).  (Runs after the timed region, like
    time_kernels.)"""
    import ctypes
    from vae_amd import _lib as L
    from vae_amd.net import call_one
    lib = L.load()
    lib.vae_launch_log(1)
    try:
        call_one(fn, ref, torch.cuda.current_stream().cuda_stream)
    finally:
        lib.vae_launch_log(0)
    need = lib.vae_launch_log_names(None, 0)
    buf = ctypes.create_string_buffer(int(need))
    lib.vae_launch_log_names(buf, need)
    out = []
    for line in buf.value.decode(errors="replace").splitlines():
        f = line.split("\t")
        m, d = f[0], (f[1] if len(f) > 1 and f[1] else f[0])
        out.append((m, d, int(f[2]) if len(f) > 2 else 1))     # (mangled, demangled, launches)
    return out


def _row_of(kernel, names):
    """The row of `names` (profile keys) that is this kernel (mangled or demangled form), or None."""
    m, d = kernel[0], kernel[1]
    for k in names:
        if k in (m, d):
            return k
    return None


def _profiles(pattern, arch):
    """profiles/ files of this arch (VQ-VAE / wide-AE runs carry "vq" / "ae_big" in the name),
    newest round/version first (natural order of the r<round>_v<version> prefix)."""
    import re
    tag = arch if arch == "vq" or arch in AE_WIDTHS else None
    paths = [p for p in glob.glob(os.path.join(REPO, "profiles", pattern))
             if (re.search(tag + r"(_|\.|$)", os.path.basename(p)) if tag else
                 not re.search(r"(^|_)(vq|ae)_", os.path.basename(p)))]     # (not "iwae_")
    key = lambda p: [int(t) if t.isdigit() else t for t in re.split(r"(\d+)", os.path.basename(p))]
    return sorted(paths, key=key, reverse=True)


def _profile_workload(d):
    """(arch, batch) a profile summary was measured on, from the bench arguments it records
    (tools/pmc_summary.py / prof_summary.py --config; none given = the default VanillaVAE B=64)."""
    toks = str(d.get("config") or "").split()
    arch, batch = "vanilla", None
    for i, t in enumerate(toks[:-1]):
        if t == "--arch":
            arch = toks[i + 1]
        elif t == "--batch":
            batch = int(toks[i + 1])
    return arch, batch if batch is not None else 64


def _matching_profile(pattern, arch, kernels, digest, batch=None):
    """Newest profiles/ summary measured on THIS build (its `digest` equals the loaded library's
    vae_build_digest, i.e. the same csrc sources) and on this workload (arch and batch: the same
    kernels of another batch size move other bytes) that holds EVERY kernel of the call; else None
    with the reason."""
    why = "no profiles/%s summary" % pattern
    why_wl = None                                   # (a summary of this build, another workload)
    want = (arch, batch if batch is not None else 64)
    for path in _profiles(pattern, arch):
        try:
            d = json.load(open(path))
        except Exception:
            continue
        if d.get("digest") != digest:
            why = f"no {pattern} summary of this build (digest {digest})"
            continue
        if _profile_workload(d) != want:
            why_wl = f"no {pattern} summary of this build for {want[0]} batch {want[1]}"
            continue
        rows = {k: _row_of(k_, d.get("kernels", {})) for k_ in kernels for k in [k_[1]]}
        if any(v is None for v in rows.values()):
            why = f"{os.path.relpath(path, REPO)} lacks " + ", ".join(k for k, v in rows.items() if v is None)
            continue
        return path, d, rows
    return None, None, why_wl or why


def pmc_traffic(kernels, digest, arch="vanilla", batch=None):
    """HBM bytes per launch of a call = the sum over ITS kernels (tools/pmc_summary.py: 2 x
    FETCH_SIZE + WRITE_SIZE, MI355X_MICROARCH.md §HBM) from a PMC summary of this very build that
    holds all of them; otherwise None (with the reason)."""
    path, d, rows = _matching_profile("*pmc*.json", arch, kernels, digest, batch)
    if path is None:
        return None, rows
    n_of = {k[1]: (k[2] if len(k) > 2 else 1) for k in kernels}
    per = {k: d["kernels"][r].get("hbm_bytes_per_launch") for k, r in rows.items()}
    if any(v is None for v in per.values()):
        return None, f"{os.path.relpath(path, REPO)}: no FETCH_SIZE/WRITE_SIZE for every kernel"
    # bytes of the CALL: each kernel's per-launch bytes times its launches in the call
    per = {k: v * n_of.get(k, 1) for k, v in per.items()}
    # the same summary's SQ / TCC counters of each kernel (tools/pmc_summary.py): MFMA busy
    # (SQ_VALU_MFMA_BUSY_CYCLES over GRBM_GUI_ACTIVE x CUs), wave-cycle fraction parked in waits
    # (SQ_WAIT_ANY / SQ_WAVE_CYCLES) and the L2 hit rate (TCC_HIT / (TCC_HIT + TCC_MISS))
    counters = {k: {c: d["kernels"][r].get(c) for c in ("mfma_busy", "wait_frac", "l2_hit")} for k, r in rows.items()}
    return {"bytes": sum(per.values()), "bytes_per_kernel": per, "launches": n_of, "counters": counters,
            "file": os.path.relpath(path, REPO), "digest": d.get("digest"), "head": d.get("head")}, None


def step_traffic(calls, digest, arch="vanilla", batch=None):
    """HBM bytes of one whole step from the PMC summary of this build: per call, the per-launch
    bytes of its kernels times their launches in the call (a kernel shared by several calls
    contributes its average once per launch, so the sum over the step's calls is the step total).  (None, reason) when any kernel is missing."""
    kernels = [k for ks in calls for k in ks]
    path, d, rows = _matching_profile("*pmc*.json", arch, kernels, digest, batch)
    if path is None:
        return None, rows
    total = 0.0
    for ks in calls:
        for k in ks:
            v = d["kernels"][_row_of(k, d["kernels"])].get("hbm_bytes_per_launch")
            if v is None:
                return None, f"{os.path.relpath(path, REPO)}: no FETCH_SIZE/WRITE_SIZE for {k[1]}"
            total += v * (k[2] if len(k) > 2 else 1)
    return {"bytes": int(total), "file": os.path.relpath(path, REPO)}, None


def rocprof_times(kernels, digest, arch="vanilla", batch=None):
    """Average duration (us) of a call's kernels in a rocprofv3 --kernel-trace --stats summary of
    this build (tools/prof_summary.py), or None (with the reason)."""
    path, d, rows = _matching_profile("*kstats*.json", arch, kernels, digest, batch)
    if path is None:
        return None, rows
    n_of = {k[1]: (k[2] if len(k) > 2 else 1) for k in kernels}
    per = {k: d["kernels"][r]["avg_us"] for k, r in rows.items()}
    # time of the CALL: each kernel's average launch times its launches in the call
    return {"avg_us": per, "launches": n_of, "sum_avg_us": round(sum(v * n_of.get(k, 1) for k, v in per.items()), 2),
            "file": os.path.relpath(path, REPO), "head": d.get("head")}, None


# ----------------------------------------------------------------------------- CPU baseline
def host_cpus():
    """CPUs this process may actually use: os.cpu_count() (the whole machine), the affinity mask,
    and the cgroup CPU quota (cgroup v2 cpu.max, v1 cfs_quota/period) — on the GPU box the job's
    share is a quota far below the machine's count."""
    info = {"os_cpu_count": os.cpu_count()}
    try:
        info["affinity"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        pass
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            quota = q / per if q > 0 else None
        except (OSError, ValueError):
            pass
    if quota is not None:
        info["cgroup_quota_cpus"] = round(quota, 2)
    usable = min(v for v in (info.get("affinity"), quota, os.cpu_count()) if v)
    info["usable"] = max(1, int(usable))
    return info


def cpu_baseline(batch, seconds, arch="vanilla", threads=None):
    """The oracle's fp32 step (fwd + loss + bwd + Adam) on the host cores, bounded sample.
    threads: torch intra-op threads; default: every CPU this process may use (host_cpus: the
    smallest of os.cpu_count(), the affinity mask and the cgroup quota — the GPU box shows the
    whole machine's 256 CPUs to os.cpu_count() but holds a job to its share)."""
    from oracle import vae_oracle as O
    prev = torch.get_num_threads()
    cpus = host_cpus()
    torch.set_num_threads(threads or cpus["usable"])
    threads = torch.get_num_threads()
    vq = arch == "vq"
    ae = AE_WIDTHS.get(arch)
    sd = O.make_params(O.vq_param_spec() if vq else (O.ae_param_spec(hidden_dims=ae) if ae else O.vanilla_param_spec()),
                       1265)
    P = {k: (v.clone().requires_grad_(True) if not k.endswith(("running_mean", "running_var", "num_batches_tracked"))
             else v.clone()) for k, v in sd.items()}
    leaves = [v for v in P.values() if v.requires_grad]
    m = [torch.zeros_like(v) for v in leaves]
    v2 = [torch.zeros_like(v) for v in leaves]
    x, eps = O.make_inputs(batch, 128, 1265)

    def step(it):
        stats = {}
        if vq:
            hd = O.VQ_HIDDEN
            q, vq_loss, _, _ = O.vq_quantize(O.vq_encode(P, x, hd), P["vq_layer.embedding.weight"], 0.25)
            rec = O.vq_decode(P, q, hd)
            loss = torch.nn.functional.mse_loss(rec, x) + vq_loss
        elif ae:
            rec = O.vanilla_decode(P, O.ae_encode(P, x, ae, True, stats), ae, True, stats)
            loss = O.ae_loss(rec, x)["loss"]
        else:
            hd = O.DEFAULT_HIDDEN
            mu, lv = O.vanilla_encode(P, x, hd, True, stats)
            z = O.reparameterize(mu, lv, eps)
            rec = O.vanilla_decode(P, z, hd, True, stats)
            loss = O.vanilla_loss(rec, x, mu, lv, 1e-8)["loss"]
        for t in leaves:
            t.grad = None
        loss.backward()
        with torch.no_grad():
            for i, t in enumerate(leaves):
                O.adam_step(t, t.grad, m[i], v2[i], it, 0.005)

    step(1)
    n, t0 = 0, time.perf_counter()
    while True:
        step(n + 2)
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds or n >= 200:
            break
    name = "VQVAE" if vq else (f"Autoencoder {ae}" if ae else "VanillaVAE")
    torch.set_num_threads(prev)
    lim = ", ".join(f"{k} {v}" for k, v in cpus.items() if k != "usable")
    return {"value": round(n * batch / el, 2), "unit": "images/s", "cores": threads, "kind": "port",
            "host_cpus": cpus,
            "sample": f"oracle {name} fp32 train step (fwd+loss+bwd+Adam), B={batch}, {n} steps / {el:.1f}s "
                      f"on {threads} threads (usable CPUs {cpus['usable']}: {lim})"}


# ----------------------------------------------------------------------------- main
def timed_loop(step, args, distributed, sync):
    """W untimed steps, then exactly K timed steps bracketed by barrier + device sync on both
    sides; returns the max over ranks of the timed region (seconds)."""
    for _ in range(args.warmup):
        step()
    sync()
    if distributed:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    sync()
    if distributed:
        dist.barrier()
    sync()
    elapsed = time.perf_counter() - t0
    if distributed:
        dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed


def selftest(args, distributed):
    """The launcher / timing / output contract without a GPU: the step is a gloo all-reduce of a
    gradient-sized buffer (3,937,635 fp32, VanillaVAE) — the only cross-rank work of the real step."""
    if distributed:
        dist.init_process_group("gloo")
    rank, world = (dist.get_rank(), dist.get_world_size()) if distributed else (0, 1)
    grads = torch.full((3937635,), float(rank + 1))

    def step():
        if distributed:
            dist.all_reduce(grads)
            grads.div_(world)

    elapsed = timed_loop(step, args, distributed, lambda: None)
    if rank == 0:
        print(json.dumps({"metric": "selftest (CPU stand-in step: gradient all-reduce only)",
                          "value": round(world * args.batch * args.steps / elapsed, 1), "unit": "images/s",
                          "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
                          "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
                          "selftest": True, "grad_mean_ok": bool(torch.allclose(grads, torch.full_like(grads, (world + 1) / 2))),
                          "config": {"workload": "selftest", "per_gpu_batch": args.batch,
                                     "global_batch": world * args.batch, "parallelism": f"dp{world}"}}), flush=True)
    if distributed:
        dist.barrier()
        dist.destroy_process_group()


def dropin_leg(args, dtype, steps=None, warmup=3, engine="graph"):
    """The drop-in path a reference user runs (vae_amd.run / experiment.fit, the counterpart of
    run.py -> VAEXperiment.training_step), timed like the headline (same batch, synchronised
    region).  engine="graph" (their default): experiment.GraphedSteps — the BaseVAE model's fused
    step replayed from HIP graphs with the experiment's logging on the device and the torch
    optimizer's state; engine="eager": the model's forward, loss_function (vae_elbo_fwd on the
    GPU), loss.backward() (the fused HIP backward behind autograd) and torch.optim.Adam.  Returns
    its img/s."""
    from vae_amd.experiment import GraphedSteps, VAEXperiment
    from vae_amd.models import vae_models
    arch = {"vanilla": ("VanillaVAE", {}), "betaH": ("BetaVAE", {"loss_type": "H", "beta": 4}),
            "iwae": ("IWAE", {"num_samples": 5}), "vq": ("VQVAE", None)}[args.arch]
    if arch[1] is None:
        model = vae_models["VQVAE"](in_channels=3, embedding_dim=64, num_embeddings=512, dtype=dtype,
                                    device="cuda", seed=1265)
    else:
        model = vae_models[arch[0]](in_channels=3, latent_dim=128, dtype=dtype, device="cuda", seed=1265, **arch[1])
    model.train()
    lr = 0.007 if args.arch == "iwae" else 0.005
    exp = VAEXperiment(model, {"LR": lr, "weight_decay": 0.0, "kld_weight": 2.5e-4})
    opt = exp.configure_optimizers()[0]
    g = torch.Generator(device="cuda").manual_seed(1265)
    x = torch.rand(args.batch, 3, 64, 64, generator=g, device="cuda")
    batch = (x, torch.zeros(args.batch, device="cuda"), [f"{i}.png" for i in range(args.batch)])
    steps = steps or max(10, min(args.steps, 50))
    gs = GraphedSteps(exp, opt) if engine == "graph" else None

    def one(i):
        if gs is not None:
            gs(batch, i)
            return
        opt.zero_grad(set_to_none=True)
        loss = exp.training_step(batch, i)
        loss.backward()
        opt.step()
    for i in range(warmup):
        one(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        one(i)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if gs is not None:
        gs.flush()
    path = ("experiment.fit(engine='graph') step: GraphedSteps (fused HIP-graph step, torch Adam state shared, "
            "logging on the device)" if gs is not None else
            "VAEXperiment.training_step -> loss.backward -> torch.optim.Adam (eager; loss_function on the GPU ELBO kernel)")
    return {"value": round(args.batch * steps / el, 1), "unit": "images/s", "ms_per_step": round(el / steps * 1e3, 4),
            "steps": steps, "path": path, "loss": float(exp.logged["loss"])}


def main():
    args = parse()
    if "RANK" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))          # parent: never touches the GPU
    # (--force-buckets under torch.distributed.run with one rank: the RCCL path at world size 1)
    distributed = "RANK" in os.environ and (int(os.environ.get("WORLD_SIZE", "1")) > 1 or args.force_buckets)
    if args.selftest:
        return selftest(args, distributed)
    ndev = max(1, torch.cuda.device_count())
    comm = "none"
    if distributed:
        local = int(os.environ.get("LOCAL_RANK", "0"))
        world_env = int(os.environ["WORLD_SIZE"])
        dev = local % ndev
        torch.cuda.set_device(dev)
        if world_env > ndev:
            # fewer devices than ranks: RCCL cannot place two ranks on one device
            dist.init_process_group("gloo")
            comm = f"gloo ({world_env} ranks on {ndev} device(s))"
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
            comm = "rccl"
        rank, world = dist.get_rank(), dist.get_world_size()
    else:
        rank, world = 0, 1
        torch.cuda.set_device(0)
    from vae_amd import _lib as L  # noqa: F401
    from vae_amd.engine import FusedAdam, TrainStep
    from vae_amd.net import StepPlan, VAENet

    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    dsz = 2 if args.dtype == "bf16" else 4
    gen = torch.Generator().manual_seed(1265)                     # same init on every rank
    S = 5 if args.arch == "iwae" else 1
    if args.arch == "vq":
        from vae_amd.vq import VQNet, VQStepPlan
        net = VQNet(dtype=dtype, device="cuda", generator=gen)
        plan = VQStepPlan(net, args.batch, concurrent=args.concurrent == "on")
        opt = FusedAdam(net, lr=0.005)                             # configs/vae/vq_vae.yaml LR
    elif args.arch in AE_WIDTHS:
        # models.Autoencoder's fused step: the VanillaVAE plan with the fc_var half pinned at zero and
        # eps = 0 (z = fc(h)), MSE only (M_N = 0); configs/big_ae.yaml LR
        net = VAENet(latent_dim=128, hidden_dims=AE_WIDTHS[args.arch], dtype=dtype, device="cuda", generator=gen)
        for nm in ("fc_var.weight", "fc_var.bias"):
            sp = net.layout.by_name[nm]
            net.params[sp.offset:sp.offset + sp.numel].zero_()
        net.sync_lowp()
        plan = StepPlan(net, args.batch, loss="vanilla", kld_weight=0.0, concurrent=args.concurrent == "on")
        opt = FusedAdam(net, lr=0.005)
    else:
        net = VAENet(latent_dim=128, dtype=dtype, device="cuda", generator=gen)
        loss = {"vanilla": "vanilla", "betaH": "betaH", "iwae": "iwae"}[args.arch]
        kld = {"vanilla": 1e-8, "betaH": 2.5e-4, "iwae": 2.5e-4}[args.arch]
        lr = {"vanilla": 0.005, "betaH": 0.005, "iwae": 0.007}[args.arch]
        plan = StepPlan(net, args.batch, loss=loss, kld_weight=kld, samples=S, concurrent=args.concurrent == "on",
                        wg_overlap=args.wg_overlap)
        opt = FusedAdam(net, lr=lr)
    # synthetic data resident in HBM (per-rank seed 1265+rank): U[0,1) images, N(0,1) eps
    g = torch.Generator(device="cuda").manual_seed(1265 + rank)
    plan.x.copy_(torch.rand(plan.x.shape, generator=g, device="cuda"))
    # eps: drawn inside the step every step on the device (the reference's randn_like,
    # vanilla_vae.py:116) where the fused bottleneck does it; otherwise a resident N(0,1) draw
    ae = args.arch in AE_WIDTHS
    step = TrainStep(net, plan, opt, graph=not args.no_graph, device_eps=None if ae or args.arch == "vq" else 1265 + rank,
                     graph_comm=not args.host_comm, force_buckets=args.force_buckets, nbuckets=args.buckets,
                     defer_reductions=not args.no_defer, overlap=not args.no_overlap,
                     comm_dtype=torch.bfloat16 if args.comm_bf16 else torch.float32)
    if hasattr(plan, "eps") and not ae and not step.device_eps:
        plan.eps.copy_(torch.randn(plan.eps.shape, generator=g, device="cuda"))

    elapsed = timed_loop(step, args, distributed, torch.cuda.synchronize)
    loss_terms = step.loss_terms()                  # rank mean (sync_dist) when distributed
    finite = all(math.isfinite(v) for v in loss_terms)

    if rank != 0:
        if distributed:
            dist.barrier()
            dist.destroy_process_group()
        return

    # ---- dominant kernel: per-launch time with HIP events on the step's stream
    times = time_kernels(plan)
    costs = kernel_costs(plan, dsz)
    rows, rows_ref = [], []
    for (fn, ref, us), (_, _, fl, by) in zip(times, costs):
        rows.append((us, fn, fl, by))
        rows_ref.append(ref)
    if args.kernel_breakdown:
        for us, fn, fl, by in rows:
            print(f"{fn:28s} {us:9.2f} us  {fl / 1e9:8.3f} GF  {by / 1e6:8.2f} MB  "
                  f"{(fl / us / 1e6) if us else 0:8.1f} TF/s  {(by / us / 1e3) if us else 0:8.1f} GB/s",
                  file=sys.stderr)
    idx = max(range(len(rows)), key=lambda i: rows[i][0])
    us, fn, fl, by = rows[idx]
    ai = fl / by if by else 0.0
    peak_tf = MFMA_PEAK_TFLOPS[args.dtype]
    ridge = peak_tf * 1e12 / (HBM_PEAK_GBS * 1e9)
    if ai >= ridge:
        roof = {"bound": "mfma", "achieved": round(fl / (us * 1e-6) / 1e12, 3), "peak": peak_tf, "unit": "TFLOP/s"}
    else:
        roof = {"bound": "hbm", "achieved": round(by / (us * 1e-6) / 1e9, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s"}
    roof["frac"] = round(roof["achieved"] / roof["peak"], 4)
    from vae_amd import _lib as L
    digest = L.load().vae_build_digest().decode()
    kernels = call_kernels(fn, rows_ref[idx])
    tr, why_tr = pmc_traffic(kernels, digest, args.arch, args.batch)
    roof["traffic"] = tr["bytes"] if tr else None
    roof["traffic_ratio"] = round(tr["bytes"] / by, 3) if tr and by else None
    roof["traffic_source"] = tr if tr else {"missing": why_tr}
    roof["kernel"] = f"{fn} (call #{idx} of the step; its kernels: {', '.join(k[1] for k in kernels) or 'n/a'})"
    roof["us_per_launch"] = round(us, 2)
    rp, why_rp = rocprof_times(kernels, digest, args.arch, args.batch)
    if rp and abs(rp["sum_avg_us"] - us) > PAIR_TOL * us:
        # the profile's kernels do not account for this call's measured time: not the same work
        # (another plan or launch count), so neither its times nor its counters are evidence here
        why = (f"{rp['file']}: rocprof sum {rp['sum_avg_us']} us vs {us:.2f} us event time "
               f"(> {PAIR_TOL:.0%} apart)")
        rp, why_rp = None, why
        roof["traffic"] = roof["traffic_ratio"] = None
        roof["traffic_source"] = {"missing": why}
    roof["rocprof"] = rp if rp else {"missing": why_rp}
    roof["build_digest"] = digest
    roof["algorithmic"] = {"flops": fl, "bytes": by, "ai_flop_per_byte": round(ai, 1)}
    step_kernel_us = sum(r[0] for r in rows)
    # the step-level attainable time — every kernel at its own roofline bound,
    # max(flops / MFMA peak, bytes / HBM peak), summed — over the measured step time; and the
    # literal MFMA fraction, all of the step's flops over the measured step at the bf16/fp32 peak
    attain_us = sum(max(fl_ / (peak_tf * 1e6), by_ / (HBM_PEAK_GBS * 1e3)) for _, _, fl_, by_ in rows)
    step_flops = sum(r[2] for r in rows)

    cpu = cpu1 = None
    if not args.no_cpu_baseline and world == 1:     # the CPU baseline is an N=1 figure (rank 0)
        cpu = cpu_baseline(args.batch, args.cpu_seconds, args.arch)
        cpu1 = cpu_baseline(args.batch, args.cpu_seconds * 0.6, args.arch, threads=1)

    ms = elapsed / args.steps * 1e3
    value = world * args.batch * args.steps / elapsed
    step_roof = {"attainable_us": round(attain_us, 2), "step_us": round(ms * 1e3, 2),
                 "frac": round(attain_us / (ms * 1e3), 4),
                 "mfma_frac": round(step_flops / (ms * 1e-3) / (peak_tf * 1e12), 4),
                 "step_gflop": round(step_flops / 1e9, 3)}
    # the whole step's counter traffic against its algorithmic bytes
    step_bytes = sum(r[3] for r in rows)
    st_tr, why_st = step_traffic([call_kernels(f_, r_) for (_, f_, _, _), r_ in zip(rows, rows_ref)], digest, args.arch, args.batch)
    step_roof["algorithmic_bytes"] = int(step_bytes)
    step_roof["traffic"] = st_tr["bytes"] if st_tr else None
    step_roof["traffic_ratio"] = round(st_tr["bytes"] / step_bytes, 3) if st_tr and step_bytes else None
    step_roof["traffic_source"] = st_tr["file"] if st_tr else {"missing": why_st}
    dropin = dropin_eager = None
    if world == 1 and not args.no_dropin and args.arch not in AE_WIDTHS:
        dropin = dropin_leg(args, dtype, steps=max(20, min(args.steps, 100)))
        dropin_eager = dropin_leg(args, dtype, engine="eager")
    line = {
        "metric": METRIC if args.arch == "vanilla" else f"train images/sec {args.arch} 64x64 bs={args.batch} (1 GPU config)",
        "value": round(value, 1),
        "unit": "images/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": ("synthetic: U[0,1) 64x64x3 images resident in HBM, N(0,1) eps drawn on the device inside every "
                 "step (Philox4x32-10 + Box-Muller in the bottleneck kernel), random-init weights" if step.device_eps else
                 "synthetic: U[0,1) 64x64x3 images" + ("" if ae or args.arch == "vq" else " + N(0,1) eps") +
                 " resident in HBM, random-init weights"),
        "config": {"workload": ("VQVAE embedding_dim=64 num_embeddings=512 64x64 train step (fwd+loss+bwd+Adam)"
                                if args.arch == "vq" else
                                f"Autoencoder hidden_dims={AE_WIDTHS[args.arch]} latent_dim=128 64x64 train step "
                                "(fwd+MSE+bwd+Adam)" if args.arch in AE_WIDTHS else
                                f"{'VanillaVAE' if args.arch == 'vanilla' else args.arch} latent_dim=128 "
                                f"64x64 train step (fwd+ELBO+bwd+Adam){' IWAE K=5' if S > 1 else ''}"),
                   "per_gpu_batch": args.batch, "global_batch": world * args.batch,
                   "parallelism": f"dp{world}", "graph": not args.no_graph,
                   "comm": comm + (" (in-graph)" if getattr(step, "graph_comm", False) else "") +
                           (f", {len(step.buckets)} buckets" if step.comm is not None else "") +
                           (", overlapped" if getattr(step, "overlap", False) else "") +
                           (", bf16 gradients" if getattr(step, "comm_dtype", None) == torch.bfloat16 else ""),
                   "devices_used": min(world, ndev)},
        "elbo": ({"loss": loss_terms[0], "Reconstruction_Loss": loss_terms[1], "finite": finite}
                 if args.arch in AE_WIDTHS else      # (the Autoencoder's loss is the MSE alone)
                 {"loss": loss_terms[0], "Reconstruction_Loss": loss_terms[1],
                  ("VQ_Loss" if args.arch == "vq" else "KLD"): loss_terms[2], "finite": finite}),
        "sum_kernel_us_isolated": round(step_kernel_us, 1),
        "roofline": roof,
        "step_roofline": step_roof,
        "dropin": dropin,
        "dropin_eager": dropin_eager,
        "cpu_baseline": cpu,
        "cpu_baseline_1thread": cpu1,
    }
    print(json.dumps(line), flush=True)
    if distributed:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
