#!/usr/bin/env python3
"""Per-kernel averages of every counter in rocprofv3 --pmc runs (one directory per pass):
    python tools/pmc_probe.py DIR [DIR ...]
Prints, per kernel, each counter's mean per dispatch, and for the SQ stall counters the
split of wave cycles (WAIT_ANY: parked on s_waitcnt / barrier; WAIT_INST_ANY: issue
stalls; ACTIVE_INST_ANY: issuing; all quad-cycles, MI355X_MICROARCH.md 'rocprofv3 PMC')."""
import collections
import csv
import glob
import os
import sys


def main():
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.defaultdict(lambda: collections.defaultdict(int))
    for d in sys.argv[1:]:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"].split("(")[0][:60]
                tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
                cnt[k][r["Counter_Name"]] += 1
    for k in sorted(tot):
        m = {c: tot[k][c] / cnt[k][c] for c in tot[k]}
        print(k)
        for c in sorted(m):
            print(f"  {c:28s} {m[c]:16.4g}")
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            parts = [c for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                                 "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS",
                                 "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_MISC", "SQ_INST_CYCLES_VMEM")
                     if c in m]
            print("  fraction of wave cycles: " +
                  ", ".join(f"{c[3:]} {m[c] / wc:.3f}" for c in parts))


if __name__ == "__main__":
    main()
