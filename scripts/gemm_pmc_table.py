#!/usr/bin/env python3
"""Effective clock and MFMA busy of GEMM dispatches from rocprofv3 ``--pmc ... --kernel-trace``
runs (scripts/gpu_gemm_power.sh):

    python scripts/gemm_pmc_table.py gpurun_out/pwr/<label>_<impl> ... [--md out.md]

Per run: one call = every kernel launched as often as the one with the largest total time (a
  column-split GEMM's two launches; the library's GEMM + silu_mul), dispatches after the first 5
  (warm-up), per-call sums of the mean duration (kernel trace) and counters, effective clock = GRBM_GUI_ACTIVE / 8 XCDs / duration
  (MI355X_MICROARCH.md 'DVFS give-back'), MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x
  GRBM_GUI_ACTIVE / 8), barrier / wait share = SQ_WAIT_ANY / SQ_WAVE_CYCLES.
The label carries the shape (q6144_4096_4096 = N, K, M), so TF/s is computed here."""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import os
import statistics


def _one(pattern):
    f = glob.glob(pattern, recursive=True)
    return f[0] if f else None


def load(d):
    cc = _one(os.path.join(d, "**", "*counter_collection.csv"))
    kt = _one(os.path.join(d, "**", "*kernel_trace.csv"))
    if cc is None:
        return None
    dur = {}
    names = {}
    if kt:
        with open(kt) as fh:
            for r in csv.DictReader(fh):
                dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
                names[r["Dispatch_Id"]] = r["Kernel_Name"]
    ctr = collections.defaultdict(dict)
    with open(cc) as fh:
        for r in csv.DictReader(fh):
            did = r["Dispatch_Id"]
            names.setdefault(did, r["Kernel_Name"])
            c = ctr[did]
            c[r["Counter_Name"]] = c.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            if did not in dur and r.get("Start_Timestamp") and r.get("End_Timestamp"):
                dur[did] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    by_kernel = collections.defaultdict(list)
    for did in sorted(ctr, key=int):
        if did in dur:
            by_kernel[names[did]].append(did)
    if not by_kernel:
        return None
    # one call = every kernel launched as often as the top one (a column-split GEMM is two
    # launches, the library's SwiGLU projection GEMM + silu_mul): durations summed per call,
    # counters summed over the call's kernels
    top = max(by_kernel, key=lambda k: sum(dur[d] for d in by_kernel[k]))
    parts = [k for k in by_kernel if len(by_kernel[k]) == len(by_kernel[top])]
    per = {k: (by_kernel[k][5:] or by_kernel[k]) for k in parts}
    mean = lambda key: sum(statistics.fmean(ctr[d].get(key, 0.0) for d in ds) for ds in per.values())  # noqa: E731
    us = sum(statistics.fmean(dur[d] for d in ds) for ds in per.values())
    cyc = mean("GRBM_GUI_ACTIVE") / 8
    return {
        "kernel": " + ".join(k[:40] for k in parts)[:90], "dispatches": len(per[top]), "us": us,
        "clock_ghz": cyc / (us * 1e3) if us else 0.0,
        "mfma_busy": mean("SQ_VALU_MFMA_BUSY_CYCLES") / (1024 * cyc) if cyc else 0.0,
        "wait_share": mean("SQ_WAIT_ANY") / max(1.0, mean("SQ_WAVE_CYCLES")),
        "mfma_insts": mean("SQ_INSTS_MFMA"),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--md", default=None)
    a = ap.parse_args()
    lines = ["| run | kernel | us (profiled) | TF/s | eff. clock GHz | MFMA busy | busy x clock | SQ_WAIT_ANY share |",
             "|---|---|---|---|---|---|---|---|"]
    for d in a.dirs:
        r = load(d)
        label = os.path.basename(d.rstrip("/"))
        if r is None:
            lines.append(f"| {label} | (no data) | | | | | | |")
            continue
        tf = ""
        parts = label.split("_")
        try:
            n, k, m = int(parts[1]), int(parts[2]), int(parts[3])
            tf = f"{2 * m * n * k / (r['us'] * 1e-6) / 1e12:.0f}"
        except (IndexError, ValueError):
            pass
        lines.append(f"| {label} | `{r['kernel']}` | {r['us']:.1f} | {tf} | {r['clock_ghz']:.2f} | "
                     f"{100 * r['mfma_busy']:.1f} % | {r['mfma_busy'] * r['clock_ghz']:.3f} | "
                     f"{100 * r['wait_share']:.1f} % |")
    out = "\n".join(lines) + "\n"
    print(out)
    if a.md:
        with open(a.md, "w") as f:
            f.write(out)


if __name__ == "__main__":
    main()
