"""Inter-kernel gaps of one solve from a rocprofv3 kernel trace.

usage: gap_trace.py kernel_trace.csv
Splits the idle time between consecutive kernels on the solve's queue by what the second
kernel follows: a residual check (k_reduce: the host's read and its next launch) or any
other kernel (dispatch of a launch already queued)."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows = [r for r in rows if "k_" in r["Kernel_Name"] or "kb_" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the last solve: from the last k_convert to the end
starts = [i for i, r in enumerate(rows) if "k_convert" in r["Kernel_Name"]]
rows = rows[starts[-1]:]
gap = defaultdict(list)
for a, b in zip(rows, rows[1:]):
    g = (int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1000.0
    kind = "after k_reduce" if "k_reduce" in a["Kernel_Name"] else "after other"
    gap[kind].append(g)
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows) / 1e6
wall = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e6
print(f"kernels {len(rows)}  wall {wall:.2f} ms  busy {busy:.2f} ms  idle {wall - busy:.2f} ms")
for k, v in sorted(gap.items()):
    v.sort()
    print(f"{k:15s} n {len(v):4d}  total {sum(v) / 1000:.3f} ms  median {v[len(v) // 2]:.1f} us  "
          f"p90 {v[int(len(v) * 0.9)]:.1f} us  max {v[-1]:.1f} us")
