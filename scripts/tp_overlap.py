#!/usr/bin/env python3
"""Compute / communication overlap of TP prefill in one rank's rocprofv3 kernel trace
(scripts/gpu_tp_overlap.sh): for every all-reduce(+norm) kernel of the xGMI library
(``xgmi_*`` kernels), the fraction of its duration during which a GEMM kernel of the same
process ran on another queue -- the chunked post-attention pipeline of models/llama.py
(_post_attn_pipelined) puts chunk i's tail beside chunk i+1's GEMMs.  Decode steps' tails (in
hipGraphs, on the compute stream) have nothing to overlap and are reported separately by size.

    python scripts/tp_overlap.py run_kernel_trace.csv > overlap.md
"""
import collections
import csv
import sys


def main(path):
    rows = list(csv.DictReader(open(path)))
    ks = []
    for r in rows:
        name = r["Kernel_Name"]
        ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, r.get("Queue_Id") or r.get("Stream_Id") or "",
                   int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0)))
    gemms = sorted((s, e, q) for s, e, n, q, _ in ks if ("gemm" in n and "xgmi" not in n))
    ars = [(s, e, n, q, g) for s, e, n, q, g in ks if "xgmi" in n]
    # GEMM intervals merged per queue for the overlap integral
    def covered(s, e, q):
        tot = 0
        for gs, ge, gq in gemms:
            if ge <= s:
                continue
            if gs >= e:
                break
            if gq != q:
                tot += min(e, ge) - max(s, gs)
        return min(tot, e - s)

    by = collections.defaultdict(lambda: [0, 0, 0])
    queues = collections.Counter(q for _, _, _, q, _ in ars)
    for s, e, n, q, g in ars:
        short = n.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
        k = (short, g, q)
        by[k][0] += 1
        by[k][1] += e - s
        by[k][2] += covered(s, e, q)
    print(f"# TP collective / GEMM overlap: {path}\n")
    print(f"{len(ars)} xGMI collective kernels on queues {dict(queues)}; {len(gemms)} GEMM kernels\n")
    gq = collections.Counter(q for _, _, q in gemms)
    print(f"GEMM kernels by queue: {dict(gq)}\n")
    print("| collective kernel | grid | queue | calls | total us | us beside a GEMM (other queue) | overlapped |")
    print("|---|---|---|---|---|---|---|")
    tot = ov = 0
    for (n, g, q), (c, d, o) in sorted(by.items(), key=lambda kv: -kv[1][1]):
        tot += d
        ov += o
        print(f"| `{n}` | {g} | {q} | {c} | {d / 1e3:.1f} | {o / 1e3:.1f} | {100.0 * o / max(1, d):.1f} % |")
    print(f"\nAll collectives: {tot / 1e3:.1f} us, {ov / 1e3:.1f} us of it beside a GEMM ({100.0 * ov / max(1, tot):.1f} %)")


if __name__ == "__main__":
    main(sys.argv[1])
