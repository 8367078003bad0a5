#!/usr/bin/env python3
"""Attention phase of each layer in a rocprofv3 kernel trace: from the first attention kernel after
a GEMM to the last one before the next GEMM.  In a mixed serving step the prefill rows' flash
kernel and the decode rows' paged-decode kernels run side by side (two streams); this splits the
phase's wall time into both-running / flash-only / decode-only / neither, so it shows which of the
two is the critical path.

    python scripts/attn_phase.py run_kernel_trace.csv [--md out.md]

Only the timed window between the lk_window_mark kernels (bench.py LK_TRACE_WINDOW=1) is used
when the marks are present.
"""
from __future__ import annotations

import argparse
import csv
import statistics

GEMM = ("gemm1w_kernel", "gemm_kernel", "wsgemm", "reduce1w", "Cijk_")
FLASH = ("flash_prefill_kernel",)
DECODE = ("paged_decode_kernel", "decode_reduce_kernel")


def _kind(name: str) -> str:
    if any(k in name for k in FLASH):
        return "flash"
    if any(k in name for k in DECODE):
        return "decode"
    if any(k in name for k in GEMM):
        return "gemm"
    return "other"


def _union(iv):
    out = []
    for s, e in sorted(iv):
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def _len(iv):
    return sum(e - s for s, e in iv)


def _inter(a, b):
    i = j = 0
    out = []
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if s < e:
            out.append([s, e])
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return out


def phases(rows):
    marks = sorted(int(r["Start_Timestamp"]) for r in rows if "lk_window_mark" in r["Kernel_Name"])
    t0, t1 = (marks[0], marks[-1]) if len(marks) >= 2 else (0, 1 << 62)
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), _kind(r["Kernel_Name"]))
                for r in rows if t0 <= int(r["Start_Timestamp"]) <= t1 and "lk_window_mark" not in r["Kernel_Name"])
    cur, out = None, []
    for s, e, k in ks:
        if k in ("flash", "decode"):
            if cur is None:
                cur = {"flash": [], "decode": [], "start": s, "end": e}
            cur[k].append((s, e))
            cur["end"] = max(cur["end"], e)
        elif k == "gemm" and cur is not None:
            cur["next_gemm"] = s
            out.append(cur)
            cur = None
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--md", default=None)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ph = phases(rows)
    lines = []
    for label, sel in (("mixed (flash + decode)", lambda p: p["flash"] and p["decode"]),
                       ("flash only", lambda p: p["flash"] and not p["decode"]),
                       ("decode only", lambda p: p["decode"] and not p["flash"])):
        ps = [p for p in ph if sel(p)]
        if not ps:
            continue
        wall = both = fo = do = 0
        walls, fl, dl = [], [], []
        for p in ps:
            w = p["next_gemm"] - p["start"]
            f, d = _union(p["flash"]), _union(p["decode"])
            b = _len(_inter(f, d))
            wall += w
            both += b
            fo += _len(f) - b
            do += _len(d) - b
            walls.append(w / 1e3)
            fl.append(_len(f) / 1e3)
            dl.append(_len(d) / 1e3)
        idle = wall - both - fo - do
        lines += [f"### {label}: {len(ps)} phases, {wall / 1e6:.1f} ms wall",
                  "",
                  "| | ms | share of phase wall |", "|---|---|---|",
                  f"| both running | {both / 1e6:.1f} | {100 * both / wall:.1f} % |",
                  f"| flash only | {fo / 1e6:.1f} | {100 * fo / wall:.1f} % |",
                  f"| decode only | {do / 1e6:.1f} | {100 * do / wall:.1f} % |",
                  f"| neither (launch gaps, small kernels) | {idle / 1e6:.1f} | {100 * idle / wall:.1f} % |",
                  "",
                  f"median per phase: wall {statistics.median(walls):.1f} us, flash busy "
                  f"{statistics.median(fl):.1f} us, decode busy {statistics.median(dl):.1f} us", ""]
    text = "\n".join(lines)
    print(text)
    if a.md:
        with open(a.md, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
