#!/usr/bin/env python3
"""Where the GPU sits idle: every gap between consecutive kernels (all queues merged) of a
rocprofv3 kernel trace over the last WINDOW seconds, grouped by the (previous kernel ->
next kernel) pair, largest total first.  A gap that recurs once per engine step shows up as
one pair with ~steps occurrences.

    python scripts/trace_gaps.py run_kernel_trace.csv 6.0 [min_gap_us=20] > gaps.md
"""
import collections
import csv
import sys


def short(name: str) -> str:
    n = name.replace("(anonymous namespace)", "anon").split("(")[0]
    return n.replace("void ", "")[:70]


def main(path, window_s, min_us=20.0):
    rows = list(csv.DictReader(open(path)))
    end = max(int(r["End_Timestamp"]) for r in rows)
    t0 = end - window_s * 1e9
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]))
                for r in rows if int(r["Start_Timestamp"]) >= t0)
    pairs = collections.defaultdict(lambda: [0, 0.0, 0.0])
    hist = collections.Counter()
    busy_end, prev = ev[0][1], ev[0][2]
    total_gap = 0.0
    for s, e, name in ev[1:]:
        gap = (s - busy_end) / 1e3
        if gap > 0:
            total_gap += gap
            b = "<5" if gap < 5 else "5-20" if gap < 20 else "20-100" if gap < 100 else "100-1000" if gap < 1000 else ">1000"
            hist[b] += 1
            if gap >= min_us:
                p = pairs[(prev, name)]
                p[0] += 1
                p[1] += gap
                p[2] = max(p[2], gap)
        if e >= busy_end:
            busy_end, prev = e, name
    span = (ev[-1][1] - ev[0][0]) / 1e3
    print(f"Window {window_s} s: {len(ev)} kernels, span {span / 1e3:.1f} ms, idle {total_gap / 1e3:.1f} ms "
          f"({100 * total_gap / span:.2f} %)\n")
    print("| gap us | count |\n|---|---|")
    for b in ("<5", "5-20", "20-100", "100-1000", ">1000"):
        print(f"| {b} | {hist[b]} |")
    print(f"\nGaps >= {min_us} us by (previous kernel -> next kernel):\n")
    print("| previous kernel | next kernel | count | total ms | mean us | max us |\n|---|---|---|---|---|---|")
    for (a, b), (n, tot, mx) in sorted(pairs.items(), key=lambda kv: -kv[1][1])[:30]:
        print(f"| `{a}` | `{b}` | {n} | {tot / 1e3:.2f} | {tot / n:.1f} | {mx:.1f} |")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]), float(sys.argv[3]) if len(sys.argv) > 3 else 20.0)
