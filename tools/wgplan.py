#!/usr/bin/env python3
"""Offline model of the grouped weight-gradient planner (vae_wgrad_batch.hip, `plan_at` and the XCD
runs) for the VanillaVAE batch, to compare plans under the planner's cost model with per-layer costs
measured by tools/wgprobe.py (diagnostic; no GPU).

    python3 tools/wgplan.py [--batch 64] [--probe gpurun_out/r6p_wgprobe.json]

Prints, per layer: class, K-steps, slices, units per item, items and the modelled item time; then per
XCD run the modelled end time (LPT order, 64 slots per XCD)."""
import argparse
import json
import math

KP64 = 64
PRO, REFILL, EPI, STORE_EPI = 6.0, 2.0, 3.0, 1.5
SLOTS = 512


def layers(n, latent_hw=2, hidden=(32, 64, 128, 256, 512)):
    """(name, kind, M, J, U pixels, du, dv) of the nine 3x3 weight gradients of the VanillaVAE batch,
    in batch order (decoder ConvTs last layer first, then the encoder convs deepest first)."""
    out = []
    # decoder ConvT i: (h, C_in) -> (2h, C_out); U = x (input side), V = dy
    dec = [(16, 64, 32), (8, 128, 64), (4, 256, 128), (2, 512, 256)]
    for h, ci, co in dec:
        out.append((f"convT {h}x{h}x{ci}", "T", ci, co, n * h * h, False, True))
    enc = [(4, 256, 512), (8, 128, 256), (16, 64, 128), (32, 32, 64), (64, 8, 32)]
    for h, ci, co in enc:
        p = h // 2
        out.append((f"conv {h}x{h}x{ci}", "C", co, ci, n * p * p, True, ci != 8))
    return out


def klass(M, J, du, dv, step64x128, step64x64, bw):
    mn = min(M, J)
    if mn < 64:
        cu, cv = min(M, 32), min(J, 32)
        kp = 64
        tiles = math.ceil(M / 32) * math.ceil(J / 32)
        by = kp * 2.0 * (cu * (2 if du else 1) + 9.0 * cv * (2 if dv else 1))
        return "all", kp, tiles, 1.2 + by / bw
    if J >= 128:
        return "64x128", KP64, math.ceil(M / 64) * math.ceil(J / 128) * 9, step64x128
    return "64x64", KP64, math.ceil(M / 64) * math.ceil(J / 64) * 9, step64x64


def plan(L, T, epi_all, defer=True):
    items, rows = 0, []
    for (name, kind, M, J, npix, du, dv), (cls, kp, tiles, su) in L:
        epi = epi_all if cls == "all" else EPI
        steps = math.ceil(npix / kp)
        body = T - PRO - epi
        sl = max(1, min(steps, math.ceil(steps * su / max(body, 0.5))))
        ks = math.ceil(steps / sl)
        slices = math.ceil(npix / (ks * kp))
        tpi = 1
        if slices == 1:
            unit = ks * su + (STORE_EPI if defer else epi)
            tpi = max(1, min(tiles, int((T - PRO + REFILL) / (unit + REFILL))))
        ni = math.ceil(slices * tiles / tpi)
        items += ni
        rows.append((name, cls, steps, slices, ks, tpi, ni, tiles, su, epi if slices > 1 or not defer else STORE_EPI))
    return items, rows


def item_us(ks, tpi, su, epi):
    return PRO + tpi * (ks * su + epi) + (tpi - 1) * REFILL


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--s128", type=float, default=2.1)
    ap.add_argument("--s64", type=float, default=1.33)
    ap.add_argument("--bw", type=float, default=51200.0)
    ap.add_argument("--epi-all", type=float, default=5.5)
    ap.add_argument("--true", default=None, help="json {layer index: us per K-step} measured")
    args = ap.parse_args()
    L = [(l, klass(l[2], l[3], l[5], l[6], args.s128, args.s64, args.bw)) for l in layers(args.batch)]
    lo, hi = 1.0, 1.0
    while plan(L, hi, args.epi_all)[0] > SLOTS:
        hi *= 2
    for _ in range(24):
        mid = (lo + hi) / 2
        if plan(L, mid, args.epi_all)[0] > SLOTS:
            lo = mid
        else:
            hi = mid
    n, rows = plan(L, hi, args.epi_all)
    true = {int(k): v for k, v in json.load(open(args.true)).items()} if args.true else {}
    print(f"T = {hi:.2f} us, {n} items")
    tot = 0.0
    for i, (name, cls, steps, slices, ks, tpi, ni, tiles, su, epi) in enumerate(rows):
        m = item_us(ks, tpi, su, epi)
        t = item_us(ks, tpi, true[i], epi) if i in true else None
        tot += ni * (t if t else m)
        print(f"  L{i} {name:18s} {cls:6s} steps {steps:4d} slices {slices:3d} ks {ks:3d} tpi {tpi:3d} items {ni:4d}"
              f"  model {m:6.2f} us" + (f"  true {t:6.2f}" if t else ""))
    print(f"  work {tot:.0f} slot-us, {tot / SLOTS:.1f} us per slot")


def simulate(L, T, epi_all, true, per_xcd_cap=None, order="lpt"):
    """Item list as vae_wgrad_batch.hip builds it at target T, cut into 8 XCD runs of equal modelled
    time (at most per_xcd_cap items each when given), each run list-scheduled on 64 slots in LPT
    order with the `true` per-step costs: returns (items, makespan)."""
    import heapq
    n, rows = plan(L, T, epi_all)
    lst = []
    for i, (name, cls, steps, slices, ks, tpi, ni, tiles, su, epi) in enumerate(rows):
        units = slices * tiles
        for it in range(ni):
            u = min(tpi, units - it * tpi)
            lst.append((item_us(ks, u, su, epi), item_us(ks, u, true.get(i, su), epi)))
    tot = sum(m for m, _ in lst)
    runs, e = [], 0
    for x in range(8):
        cum, cnt, r = 0.0, 0, []
        while e < len(lst) and (x == 7 or cum < tot / 8) and (per_xcd_cap is None or cnt < per_xcd_cap):
            cum += lst[e][0]; r.append(lst[e]); e += 1; cnt += 1
        runs.append(r)
    if e < len(lst):
        return n, float("inf")
    span = 0.0
    for r in runs:
        r = sorted(r, key=lambda t: -t[0]) if order == "lpt" else r
        slots = [0.0] * 64
        for _, t in r:
            s = heapq.heappop(slots)
            heapq.heappush(slots, s + t)
        span = max(span, max(slots))
    return n, span


if __name__ == "__main__":
    main()
