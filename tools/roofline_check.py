#!/usr/bin/env python3
"""Recompute the bench line's roofline fraction by hand from committed profiles (VERDICT r1:
the BENCH `frac` must agree within 5 % with what the rocprofv3 kernel stats + PMC counters
give).  frac_by_hand = PMC HBM bytes per iteration-pass launch (FETCH_SIZE x 2 + WRITE_SIZE,
profiles/traffic.json) / the iteration class's average duration in the kernel-stats CSV of the
same single-pair run / 8 TB/s.
Usage: python tools/roofline_check.py profiles/r2/kernel_stats_single_pair.csv profiles/r2/bench_c2_default.json"""
import csv
import json
import sys

stats, bench = sys.argv[1], sys.argv[2]
traffic = json.load(open(sys.argv[3] if len(sys.argv) > 3 else "profiles/traffic.json"))
kern = set(traffic["iterate_kernels"])
tot_ns = calls = 0
for r in csv.DictReader(open(stats)):
    n = r["Name"].split("(")[0].replace("void ", "").replace("tvl1k::", "")
    if n in kern:
        tot_ns += float(r["TotalDurationNs"])
        calls += int(r["Calls"])
avg_us = tot_ns / calls / 1e3
by_hand = traffic["iterate_hbm_bytes_per_launch"] / (avg_us * 1e-6) / 8e12
line = json.loads(open(bench).read().strip().splitlines()[-1])
r = line["roofline"]
print(f"iteration class: {calls} launches in the kernel stats, avg {avg_us:.2f} us; "
      f"PMC bytes/launch {traffic['iterate_hbm_bytes_per_launch']:,}")
print(f"frac by hand (PMC bytes / rocprof avg / 8 TB/s): {by_hand:.4f}")
print(f"bench frac (live accounting {r['bytes_per_launch']:,} B / HIP-event avg "
      f"{r['avg_launch_us']} us): {r['frac']}")
print(f"ratio bench / by hand: {r['frac'] / by_hand:.4f}  (within 5 %: {abs(r['frac'] / by_hand - 1) <= 0.05})")
if traffic.get("iterate_valu_frac") is not None:
    print(f"VALU issue utilisation of the class (SQ_INSTS_VALU x 2 / (1024 x GRBM_GUI_ACTIVE / 8)): "
          f"{traffic['iterate_valu_frac']}")
