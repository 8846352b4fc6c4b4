"""Per-dispatch-shape breakdown of a rocprofv3 kernel trace.

Groups the dispatches in run_kernel_trace.csv by (kernel, grid size) and prints count,
total and average duration, so one can see where an iteration kernel spends its time
per pyramid level / pass length.  Usage: python tools/trace_breakdown.py <trace.csv> [filter]
"""
import csv
import re
import sys
from collections import defaultdict


def short(name):
    name = re.sub(r"\(.*\)$", "", name)
    return name.replace("tvl1k::", "").replace("void ", "")


def main():
    path = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    groups = defaultdict(lambda: [0, 0.0])
    kern = defaultdict(lambda: [0, 0.0])
    for row in csv.DictReader(open(path)):
        n = short(row["Kernel_Name"])
        dur = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3  # us
        kern[n][0] += 1
        kern[n][1] += dur
        if filt and filt not in n:
            continue
        key = (n, int(row["Grid_Size_X"]) * int(row["Grid_Size_Y"]) * int(row["Grid_Size_Z"]))
        groups[key][0] += 1
        groups[key][1] += dur
    print(f"{'kernel':44s} {'calls':>6s} {'total ms':>9s} {'avg us':>8s}")
    for n, (c, t) in sorted(kern.items(), key=lambda kv: -kv[1][1]):
        print(f"{n[:44]:44s} {c:6d} {t / 1e3:9.2f} {t / c:8.1f}")
    if filt:
        print(f"\n{'kernel':44s} {'threads':>9s} {'calls':>6s} {'total ms':>9s} {'avg us':>8s}")
        for (n, g), (c, t) in sorted(groups.items(), key=lambda kv: (kv[0][0], -kv[0][1])):
            print(f"{n[:44]:44s} {g:9d} {c:6d} {t / 1e3:9.2f} {t / c:8.1f}")


if __name__ == "__main__":
    main()
