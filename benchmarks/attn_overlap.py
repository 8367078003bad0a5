#!/usr/bin/env python3
"""Do a mixed step's two attention kernels overlap?  Flash prefill over the step's prompt
chunks (compute-bound) and paged decode over its decode rows (HBM-bound) at the serving shapes
(Llama-3-8B heads, 6 prompts x 643 new tokens over 930 keys; 128 decode rows x 1000 keys), timed
back to back on one stream vs on two streams (both launch orders) and, with --splits, on two
streams restricted to disjoint CU sets; cold KV (rotated copies), HIP events, medians of
interleaved rounds.  ``unified``: one flash launch over both, the decode rows as one-token
sequences in the same heaviest-first tile list.  (A flash-occupancy-cap arm -- unused LDS so a decode workgroup fits beside
one flash workgroup per CU -- measured 190 us vs 178 serial and was removed.)

    python benchmarks/attn_overlap.py [--md out.md]
"""
from __future__ import annotations

import argparse
import math
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from llm_kubernetes_minikube_sharp4dev_amd import ops  # noqa: E402

DEV = "cuda"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--md", default=None)
    ap.add_argument("--rounds", type=int, default=15)
    ap.add_argument("--splits", default="", type=lambda v: [int(x) for x in v.split(",") if x])
    a = ap.parse_args()
    Hq, Hkv, D, BS = 32, 8, 128, 16
    # decode rows: 128 x 1000 keys, its own blocks
    Bd, ctx_d = 128, 1000
    nb_d = (ctx_d + BS - 1) // BS
    # prefill: 6 prompts, 643 new of 930 keys
    Bp, q, ctx_p = 6, 643, 930
    nb_p = (ctx_p + BS - 1) // BS
    NB = Bd * nb_d + Bp * nb_p + 1
    copies = []
    for _ in range(2):  # two KV caches so consecutive rounds do not hit the same bytes in MALL
        kc = torch.randn(NB, Hkv, BS, D, device=DEV, dtype=torch.bfloat16)
        copies.append((kc, torch.randn_like(kc)))
    perm = torch.randperm(NB - 1, device=DEV).int()
    bt_d = torch.zeros(Bd, 8192 // BS, dtype=torch.int32, device=DEV)
    bt_d[:, :nb_d] = perm[: Bd * nb_d].view(Bd, nb_d)
    bt_p = perm[Bd * nb_d: Bd * nb_d + Bp * nb_p].view(Bp, nb_p).contiguous()
    qd = torch.randn(Bd, Hq, D, device=DEV, dtype=torch.bfloat16)
    cl_d = torch.full((Bd,), ctx_d, dtype=torch.int32, device=DEV)
    qp = torch.randn(Bp * q, Hq * D, device=DEV, dtype=torch.bfloat16)
    cu = torch.arange(0, Bp * q + 1, q, dtype=torch.int32, device=DEV)
    cl_p = torch.full((Bp,), ctx_p, dtype=torch.int32, device=DEV)
    ts, tq = ops.prefill_tiles([q] * Bp, [ctx_p] * Bp, Hq // Hkv, True)
    tiles = (torch.from_numpy(ts).to(DEV), torch.from_numpy(tq).to(DEV))
    out_p = torch.empty_like(qp)
    out_d = torch.empty_like(qd)
    # unified: ONE flash launch over [prompt rows | decode rows], the decode rows as q_len-1
    # sequences (causal with past = ctx - 1), tiles of both kinds in one heaviest-first list
    W = bt_d.shape[1]
    bt_u = torch.zeros(Bp + Bd, W, dtype=torch.int32, device=DEV)
    bt_u[:Bp, :nb_p] = bt_p
    bt_u[Bp:] = bt_d
    q_u = torch.cat([qp, qd.view(Bd, Hq * D)])
    cu_u = torch.cat([cu, cu[-1] + torch.arange(1, Bd + 1, dtype=torch.int32, device=DEV)])
    cl_u = torch.cat([cl_p, cl_d])
    tsu, tqu = ops.prefill_tiles([q] * Bp + [1] * Bd, [ctx_p] * Bp + [ctx_d] * Bd, Hq // Hkv, True)
    tiles_u = (torch.from_numpy(tsu).to(DEV), torch.from_numpy(tqu).to(DEV))
    # other orders of the same tile list: decode tiles (seq >= Bp) interleaved one-for-one with
    # the prompt tiles, and prompt tiles first
    isd = tsu >= Bp
    dpos, ppos = np.nonzero(isd)[0], np.nonzero(~isd)[0]
    inter = []
    for i in range(max(len(dpos), len(ppos))):
        if i < len(ppos):
            inter.append(ppos[i])
        if i < len(dpos):
            inter.append(dpos[i])
    orders = {"unified_inter": np.asarray(inter), "unified_pfirst": np.concatenate([ppos, dpos])}
    for k2 in (2, 4):  # k prompt tiles per decode tile
        o2, di = [], 0
        for i, pi in enumerate(ppos):
            o2.append(pi)
            if i % k2 == k2 - 1 and di < len(dpos):
                o2.append(dpos[di])
                di += 1
        o2.extend(dpos[di:])
        orders[f"unified_p{k2}d1"] = np.asarray(o2)
    tiles_o = {k: (torch.from_numpy(tsu[o]).to(DEV), torch.from_numpy(tqu[o]).to(DEV)) for k, o in orders.items()}
    out_u = torch.empty_like(q_u)
    cu_dd = torch.arange(0, Bd + 1, dtype=torch.int32, device=DEV)
    tsd, tqd = ops.prefill_tiles([1] * Bd, [ctx_d] * Bd, Hq // Hkv, True)
    tiles_dd = (torch.from_numpy(tsd).to(DEV), torch.from_numpy(tqd).to(DEV))
    out_dd = torch.empty(Bd, Hq * D, device=DEV, dtype=torch.bfloat16)
    side = torch.cuda.Stream()
    sc = 1 / math.sqrt(D)
    it = [0]

    def flash(kv):
        ops.flash_prefill(qp, kv[0], kv[1], cu, Hq, Hkv, D, sc, True, block_tables=bt_p, ctx_lens=cl_p,
                          tiles=tiles, out=out_p)

    def decode(kv):
        ops.paged_decode(qd, kv[0], kv[1], bt_d, cl_d, sc, out=out_d)

    def unified(kv):
        ops.flash_prefill(q_u, kv[0], kv[1], cu_u, Hq, Hkv, D, sc, True, block_tables=bt_u, ctx_lens=cl_u,
                          tiles=tiles_u, out=out_u)

    def unified_o(kv, name):
        ops.flash_prefill(q_u, kv[0], kv[1], cu_u, Hq, Hkv, D, sc, True, block_tables=bt_u, ctx_lens=cl_u,
                          tiles=tiles_o[name], out=out_u)

    def decode_flash(kv):
        ops.flash_prefill(qd.view(Bd, Hq * D), kv[0], kv[1], cu_dd, Hq, Hkv, D, sc, True, block_tables=bt_d,
                          ctx_lens=cl_d, tiles=tiles_dd, out=out_dd)

    def arm(name):
        if name in extra:
            return masked_arm(*extra[name])
        kv = copies[it[0] % 2]
        it[0] += 1
        if name == "flash":
            flash(kv)
        elif name == "decode":
            decode(kv)
        elif name == "unified":
            unified(kv)
        elif name in tiles_o:
            unified_o(kv, name)
        elif name == "decode_flash":
            decode_flash(kv)
        elif name == "serial":
            flash(kv)
            decode(kv)
        else:  # two streams: the first named kernel on the current stream, the other on the side
            first, second = (flash, decode) if name == "2s_flash_first" else (decode, flash)
            ev = torch.cuda.Event()
            ev.record()
            side.wait_event(ev)
            first(kv)
            with torch.cuda.stream(side):
                second(kv)
            ev2 = torch.cuda.Event()
            ev2.record(side)
            torch.cuda.current_stream().wait_event(ev2)

    # CU-partitioned arms: flash and decode on two streams restricted to disjoint CU sets
    # (hipExtStreamCreateWithCUMask), K CUs for decode; "lo" = CUs [0, K), "il" = every
    # (256 / K)-th CU
    L = ops.lib()
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    nw = (ncu + 31) // 32

    def words(cus):
        w = [0] * nw
        for c in cus:
            w[c // 32] |= 1 << (c % 32)
        return w

    masked = {}
    for K in a.splits:
        for lay in ("lo", "il"):
            if lay == "lo":
                dec = list(range(K))
            else:
                step = ncu / K
                dec = sorted({int(i * step) for i in range(K)})
            fl = [c for c in range(ncu) if c not in set(dec)]
            masked[(K, lay)] = (torch.cuda.ExternalStream(L.cu_mask_stream(words(dec))),
                                torch.cuda.ExternalStream(L.cu_mask_stream(words(fl))))

    def masked_arm(K, lay, which):
        sd, sf = masked[(K, lay)]
        kv = copies[it[0] % 2]
        it[0] += 1
        cur = torch.cuda.current_stream()
        ev = torch.cuda.Event()
        ev.record(cur)
        joins = []
        if which in ("both", "decode"):
            sd.wait_event(ev)
            with torch.cuda.stream(sd):
                decode(kv)
            e = torch.cuda.Event()
            e.record(sd)
            joins.append(e)
        if which in ("both", "flash"):
            sf.wait_event(ev)
            with torch.cuda.stream(sf):
                flash(kv)
            e = torch.cuda.Event()
            e.record(sf)
            joins.append(e)
        for e in joins:
            cur.wait_event(e)

    arms = ["flash", "decode", "decode_flash", "serial", "2s_flash_first", "2s_decode_first", "unified", *tiles_o]
    extra = {}
    for (K, lay) in masked:
        for which in ("both", "decode", "flash"):
            name = f"mask{K}{lay}_{which}"
            arms.append(name)
            extra[name] = (K, lay, which)
    for n in arms:
        arm(n)
    torch.cuda.synchronize()
    # the unified launch equals the two kernels' outputs
    kv = copies[0]
    flash(kv)
    decode(kv)
    unified(kv)
    decode_flash(kv)
    torch.cuda.synchronize()
    err_p = (out_u[: Bp * q].float() - out_p.float()).abs().max().item()
    err_d = (out_u[Bp * q:].float() - out_d.view(Bd, -1).float()).abs().max().item()
    err_dd = (out_dd.float() - out_d.view(Bd, -1).float()).abs().max().item()
    print(f"unified vs separate: prefill max|d| {err_p:.3g}, decode max|d| {err_d:.3g}; decode_flash {err_dd:.3g}",
          flush=True)
    ts_ = {n: [] for n in arms}
    for _ in range(a.rounds):
        for n in arms:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            arm(n)
            e1.record()
            e1.synchronize()
            ts_[n].append(e0.elapsed_time(e1) * 1e3)
    med = {n: statistics.median(v) for n, v in ts_.items()}
    lines = ["| arm | us |", "|---|---|"] + [f"| {n} | {med[n]:.1f} |" for n in arms]
    if masked:
        lines.append(f"\nCU masks of the decode streams: " + "; ".join(
            f"{K}{lay}: {L.stream_cu_mask(masked[(K, lay)][0].cuda_stream, nw)}" for (K, lay) in list(masked)[:2]))
    lines.append(f"\nsum of the two alone {med['flash'] + med['decode']:.1f} us, max {max(med['flash'], med['decode']):.1f} us")
    print("\n".join(lines), flush=True)
    if a.md:
        with open(a.md, "w") as f:
            f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
