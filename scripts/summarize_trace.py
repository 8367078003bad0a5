#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace (run_kernel_trace.csv) over bench.py's timed window
as a markdown table: per-kernel time share, call count, mean duration, GPU busy fraction and
the idle-gap histogram.

The window is bounded by the two ``lk_window_mark_kernel`` launches bench.py makes under
``LK_TRACE_WINDOW=1`` (csrc/marker.hip): exactly the timed steps, no warm-up, no drain.
Without markers in the trace it falls back to the last WINDOW seconds.

    python scripts/summarize_trace.py run_kernel_trace.csv [WINDOW_S] > profiles/x.md
"""
import collections
import csv
import os
import sys

BY_GRID = os.environ.get("SUMMARY_BY_GRID") == "1"

# coarse classes for the budget table (first match wins)
CLASSES = [
    ("decode GEMM (wsgemm / skinny, weight streaming)", ("wsgemm", "skinny", "ws_linear")),
    ("prefill GEMM (gemm_kernel / gemm1w, MFMA)", ("gemm_kernel", "gemm1w", "reduce1w")),
    ("hipBLASLt / rocBLAS", ("Cijk", "rocblas")),
    ("flash prefill + cascade", ("flash_prefill",)),
    ("paged decode attention", ("paged_decode", "decode_reduce", "split_reduce")),
    ("norms (rms/layer)", ("rmsnorm", "layernorm")),
    ("rope + KV write", ("rope", "kv_write")),
    ("sampling / select", ("sample", "select", "argmax", "gumbel")),
    ("kNN", ("knn", "score_topk", "topk")),
    ("activations / elementwise", ("act", "silu", "gelu", "elementwise", "vectorized", "copy")),
]


def _cls(name):
    for label, keys in CLASSES:
        if any(k in name for k in keys):
            return label
    return "other"


def window(rows, window_s):
    """(t0, t1, how): the marker-bounded timed window, else the last window_s seconds."""
    marks = sorted(int(r["Start_Timestamp"]) for r in rows if "lk_window_mark" in r["Kernel_Name"])
    if len(marks) >= 2:
        return marks[0], marks[-1], "between the lk_window_mark kernels (bench.py timed window)"
    end = max(int(r["End_Timestamp"]) for r in rows)
    return end - window_s * 1e9, end, f"last {window_s:.1f} s of the trace (no window markers)"


def main(path, window_s, top=int(os.environ.get("SUMMARY_TOP", "25"))):
    rows = list(csv.DictReader(open(path)))
    t0, t1, how = window(rows, window_s)
    window_s = (t1 - t0) / 1e9
    agg = collections.defaultdict(lambda: [0, 0])
    ev = []
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s < t0 or e > t1 or "lk_window_mark" in r["Kernel_Name"]:
            continue
        name = r["Kernel_Name"].replace("(anonymous namespace)", "anon").split("(")[0][:100]
        ev.append((s, e, name))
        if BY_GRID:  # one row per (kernel, grid): separates the GEMM shapes of one template
            grid = r.get("Grid_Size") or "x".join(r.get(f"Grid_Size_{a}", "?") for a in "XYZ")
            name += f" grid={grid}"
        a = agg[name]
        a[0] += e - s
        a[1] += 1
    ev.sort()
    busy, gaps, big = 0, [], []
    cs, ce, cn = ev[0]
    for s, e, n in ev[1:]:
        if s > ce:
            busy += ce - cs
            gaps.append(s - ce)
            if s - ce >= 1e5:  # itemise every idle gap >= 100 us: (gap, before, after, when)
                big.append((s - ce, cn, n, (ce - t0) / 1e9))
            cs, ce = s, e
        else:
            ce = max(ce, e)
        cn = n if e >= ce else cn
    busy += ce - cs
    tot = sum(v[0] for v in agg.values())
    print(f"Window: {window_s:.2f} s, {how}; GPU busy {busy / 1e6:.0f} ms "
          f"({100 * busy / (window_s * 1e9):.1f} %), {len(ev)} kernels\n")
    print("| kernel | total ms | share | calls | mean us |\n|---|---|---|---|---|")
    for k, (t, n) in sorted(agg.items(), key=lambda x: -x[1][0])[:top]:
        print(f"| `{k}` | {t / 1e6:.1f} | {100 * t / tot:.1f} % | {n} | {t / n / 1e3:.1f} |")
    b = collections.Counter()
    bt = collections.Counter()
    for g in gaps:
        k = "<5us" if g < 5e3 else "5-20us" if g < 2e4 else "20-100us" if g < 1e5 else "0.1-1ms" if g < 1e6 else ">1ms"
        b[k] += 1
        bt[k] += g
    byc = collections.defaultdict(float)
    for k, (t, n) in agg.items():
        byc[_cls(k)] += t
    print("\n| class | total ms | share |\n|---|---|---|")
    for k, t in sorted(byc.items(), key=lambda x: -x[1]):
        print(f"| {k} | {t / 1e6:.1f} | {100 * t / tot:.1f} % |")
    print("\n| idle gap | count | total ms |\n|---|---|---|")
    for k in ["<5us", "5-20us", "20-100us", "0.1-1ms", ">1ms"]:
        print(f"| {k} | {b[k]} | {bt[k] / 1e6:.1f} |")
    # every kernel that is not ours (PyTorch eager ops, runtime copies): what still runs outside
    # the HIP kernel library inside the timed steps
    foreign = {k: v for k, v in agg.items() if "anon::" not in k and "lk_" not in k}
    if foreign:
        print("\n| kernel outside the HIP library | calls | total ms |\n|---|---|---|")
        for k, (t, n) in sorted(foreign.items(), key=lambda x: -x[1][0]):
            print(f"| `{k[:90]}` | {n} | {t / 1e6:.2f} |")
    if big:
        print(f"\nIdle gaps >= 100 us ({len(big)}, {sum(g for g, *_ in big) / 1e6:.1f} ms), largest first:\n")
        print("| gap us | at s | last kernel before | first kernel after |\n|---|---|---|---|")
        for g, a, n, at in sorted(big, reverse=True)[:40]:
            print(f"| {g / 1e3:.0f} | {at:.3f} | `{a[:60]}` | `{n[:60]}` |")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 4.0)
