#!/usr/bin/env python3
"""Where the device idles in a rocprofv3 kernel trace: for every gap > MIN_US in the last
WINDOW seconds, the kernels just before and after it (stream-merged order), grouped by that
(before, after) pair with counts and total idle time.

    python scripts/gap_context.py run_kernel_trace.csv 4.0 100 [END_SKIP_S] > gaps.md

END_SKIP_S drops the trace's last seconds (bench.py's post-window drain) before the window.
"""
import collections
import csv
import sys


def short(n):
    return n.replace("(anonymous namespace)", "anon").split("(")[0].replace("void ", "")[:70]


def main(path, window_s, min_us, end_skip_s=0.0):
    rows = list(csv.DictReader(open(path)))
    end = max(int(r["End_Timestamp"]) for r in rows) - end_skip_s * 1e9
    t0 = end - window_s * 1e9
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]))
                for r in rows if t0 <= int(r["Start_Timestamp"]) <= end)
    busy = sum(e - s for s, e, _ in ev)  # upper bound (overlapping kernels double-count)
    print(f"window {window_s} s ending {end_skip_s} s before the trace end: {len(ev)} kernels\n")
    agg = collections.defaultdict(lambda: [0, 0.0])
    ce, cn = ev[0][1], ev[0][2]
    for s, e, n in ev[1:]:
        if s > ce and (s - ce) / 1e3 >= min_us:
            a = agg[(cn, n)]
            a[0] += 1
            a[1] += (s - ce) / 1e3
        if e > ce:
            ce, cn = e, n
    print(f"gaps >= {min_us} us in the last {window_s} s, by (kernel before, kernel after)\n")
    print("| before | after | gaps | idle ms |\n|---|---|---|---|")
    for (b, a), (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:25]:
        print(f"| `{b}` | `{a}` | {c} | {t / 1e3:.1f} |")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]), float(sys.argv[3]), float(sys.argv[4]) if len(sys.argv) > 4 else 0.0)
