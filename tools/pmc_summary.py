#!/usr/bin/env python3
"""Summarise a tools/profile.sh run: per-kernel durations (kernel trace) and PMC
counters (per-dispatch sums / averages).  FETCH_SIZE is doubled per
MI355X_MICROARCH.md (gfx950 reports 1/2 of the bytes of wide coalesced streams);
WRITE_SIZE is taken as is.  Both are in KB in rocprofv3's derived counters.
Usage: python tools/pmc_summary.py gpurun_out/prof_<tag> [kernel-substring ...] [--batch]
  --batch: the batched kernels of tvl1_calc_batch (kb_iterate_roll + kb_warp_iter as the
           iteration class, kb_warp_ring as the warp class; tools/pmc_strips.sh)
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name):
    return name.split("(")[0].replace("void ", "").replace("tvl1k::", "")


def main():
    d = sys.argv[1]
    args = [a for a in sys.argv[2:] if not a.startswith("--") and not a.endswith(".json")]
    batch = "--batch" in sys.argv
    pre = "kb_" if batch else "k_"
    want = args or [pre + "iterate", pre + "warp"]
    rows = list(csv.DictReader(open(os.path.join(d, "trace", "run_kernel_trace.csv"))))
    dur = defaultdict(list)
    for r in rows:
        dur[short(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    print(f"{'kernel':40s} {'calls':>6s} {'total ms':>9s} {'avg us':>8s}")
    for k, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        print(f"{k:40s} {len(v):6d} {sum(v)/1e6:9.2f} {sum(v)/len(v)/1e3:8.1f}")
    ctr = defaultdict(lambda: defaultdict(float))
    calls = defaultdict(lambda: defaultdict(int))
    for f in glob.glob(os.path.join(d, "pmc_*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            ctr[k][r["Counter_Name"]] += float(r["Counter_Value"])
            calls[k][r["Counter_Name"]] += 1
    out = {}
    for k in ctr:
        if not any(w in k for w in want):
            continue
        c = ctr[k]
        n = max(calls[k].values())
        tot_ns = sum(dur.get(k, [0])) or 1
        avg_ns = tot_ns / max(1, len(dur.get(k, [1])))
        res = {"dispatches": n, "avg_us_trace": round(avg_ns / 1e3, 2)}
        if "FETCH_SIZE" in c:
            fb = 2 * c["FETCH_SIZE"] * 1024 / calls[k]["FETCH_SIZE"]
            res["fetch_bytes_per_dispatch_x2"] = round(fb)
        if "WRITE_SIZE" in c:
            wb = c["WRITE_SIZE"] * 1024 / calls[k]["WRITE_SIZE"]
            res["write_bytes_per_dispatch"] = round(wb)
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            res["hbm_bytes_per_dispatch"] = round(fb + wb)
            res["hbm_GBs_at_trace_avg"] = round((fb + wb) / avg_ns, 1)
        for name in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY",
                     "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU", "GRBM_GUI_ACTIVE"):
            if name in c:
                res[name + "_per_dispatch"] = round(c[name] / calls[k][name])
        if "SQ_WAVE_CYCLES" in c and "SQ_WAIT_ANY" in c:
            res["wait_any_frac"] = round(c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"], 3)
        if "SQ_WAVE_CYCLES" in c and "SQ_ACTIVE_INST_VALU" in c:
            res["valu_active_frac"] = round(c["SQ_ACTIVE_INST_VALU"] / c["SQ_WAVE_CYCLES"], 3)
        out[k] = res
    # kernel classes as bench.py / tvl1_stats report them: every iteration pass
    # (k_iterate_roll + k_iterate_tb of the hybrid) and every warpBackward
    classes = {}
    # (k_warp_iter, warpBackward fused with a warp's first pass, is an iteration pass)
    for cls, prefix in (("iterate", pre + "iterate"), ("warp", pre + "warp")):
        ks = [k for k in out if k.startswith(prefix) or (cls == "iterate" and k.startswith(pre + "warp_iter"))]
        if cls == "warp":
            ks = [k for k in ks if not k.startswith(pre + "warp_iter")]
        if not ks:
            continue
        n = sum(out[k]["dispatches"] for k in ks)
        tot_ns = sum(sum(dur.get(k, [])) for k in ks)
        ndur = sum(len(dur.get(k, [])) for k in ks)
        res = {"kernels": ks, "dispatches": n, "avg_us_trace": round(tot_ns / max(1, ndur) / 1e3, 2)}
        if all("hbm_bytes_per_dispatch" in out[k] for k in ks):
            hb = sum(out[k]["hbm_bytes_per_dispatch"] * out[k]["dispatches"] for k in ks) / n
            res["hbm_bytes_per_dispatch"] = round(hb)
            res["hbm_GBs_at_trace_avg"] = round(hb / (tot_ns / max(1, ndur)), 1)
            res["hbm_frac_of_8TBs"] = round(hb / (tot_ns / max(1, ndur)) / 8000.0, 4)
        # VALU issue utilisation: SQ_INSTS_VALU x 2 cycles / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)
        if all("SQ_INSTS_VALU" in ctr[k] and "GRBM_GUI_ACTIVE" in ctr[k] for k in ks):
            valu = sum(ctr[k]["SQ_INSTS_VALU"] for k in ks)
            gui = sum(ctr[k]["GRBM_GUI_ACTIVE"] for k in ks) / 8.0
            res["valu_frac"] = round(valu * 2 / (1024 * gui), 4) if gui else None
        classes[cls] = res
    out["classes"] = classes
    print(json.dumps(out, indent=1))
    # profiles/traffic.json for bench.py's roofline.traffic
    it = classes.get("iterate", {})
    if "--emit-traffic" in sys.argv and "hbm_bytes_per_dispatch" in it:
        path = sys.argv[sys.argv.index("--emit-traffic") + 1]
        json.dump({"iterate_hbm_bytes_per_launch": it["hbm_bytes_per_dispatch"],
                   "iterate_avg_us_trace": it["avg_us_trace"],
                   "iterate_hbm_frac_of_8TBs": it.get("hbm_frac_of_8TBs"),
                   "iterate_valu_frac": it.get("valu_frac"),
                   "iterate_kernels": it["kernels"], "dispatches": it["dispatches"],
                   "warp_hbm_bytes_per_launch": classes.get("warp", {}).get("hbm_bytes_per_dispatch"),
                   "source": d, "method": "rocprofv3 --pmc FETCH_SIZE (x2, gfx950) + WRITE_SIZE, "
                   "separate passes, average over every iteration-pass dispatch of " +
                   ("one strip batch at a time (tools/pmc_strips.sh)" if batch else
                    "one pair alone (tools/pmc_single.sh)") +
                   "; valu_frac from the SQ_INSTS_VALU pass"},
                  open(path, "w"), indent=1)


if __name__ == "__main__":
    main()
