"""Per-kernel VALU utilisation from tools/pmc_single.sh: SQ_INSTS_VALU x 2 cycles (one wave64
VALU instruction issues over 2 cycles, MI355X_MICROARCH.md) / (1024 SIMDs x GRBM_GUI_ACTIVE/8).
Usage: python tools/valu_util.py gpurun_out/prof_<tag>"""
import csv
import glob
import sys
from collections import defaultdict


def short(name):
    return name.split("(")[0].replace("void ", "").replace("tvl1k::", "")


d = sys.argv[1]
acc = defaultdict(lambda: defaultdict(float))
n = defaultdict(set)
for f in glob.glob(f"{d}/pmc_valu/*counter_collection.csv"):
    for row in csv.DictReader(open(f)):
        k = short(row["Kernel_Name"])
        acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
        n[k].add(row.get("Dispatch_Id", row.get("Correlation_Id")))
dur = defaultdict(float)
for f in glob.glob(f"{d}/trace/*kernel_trace.csv"):
    for row in csv.DictReader(open(f)):
        dur[short(row["Kernel_Name"])] += (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9
print(f"{'kernel':42s} {'disp':>5s} {'VALU/disp':>11s} {'SALU/VALU':>9s} {'clk GHz':>7s} {'VALU util':>9s}")
for k, c in sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_INSTS_VALU", 0)):
    nd = len(n[k])
    gui = c.get("GRBM_GUI_ACTIVE", 0) / 8.0
    valu = c.get("SQ_INSTS_VALU", 0)
    util = valu * 2 / (1024 * gui) if gui else float("nan")
    clk = gui / dur[k] / 1e9 * (len(n[k]) and 1) if dur.get(k) else float("nan")
    print(f"{k:42s} {nd:5d} {valu / max(nd, 1):11.4g} {c.get('SQ_INSTS_SALU', 0) / max(valu, 1):9.3f} "
          f"{clk:7.2f} {util:9.3f}")
