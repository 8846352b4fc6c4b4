#!/usr/bin/env python3
"""Cost-weighted issue model of the TV-L1 iteration kernels.

Three inputs, all committed under profiles/:
  * the emitted gfx950 ISA of a kernel (tools/issue_model.py --dump-isa), from which the
    per-step instruction counts of each wavefront role's hot loop are taken by class;
  * the PMC counters of one C2 pair alone (tools/pmc_issue.sh -> --collect), per kernel and
    grid size (= per pyramid level): the dynamic instruction counts by class, SQ_WAVES,
    the wave-cycle split and GRBM_GUI_ACTIVE;
  * the issue cost of each instruction class measured on the chip (tools/issue_rate.hip).

Modes:
  --collect DIR          rocprofv3 output of tools/pmc_issue.sh -> CSV on stdout
  --dump-isa OUT         compile the engine device-only and write the ISA of the kernels the
                         model reads (k_warp_iter<6,0,128,1,2>, kb_warp_iter<6,0,2>)
  --model                the report (defaults: profiles/r6/issue/*)
"""
import argparse
import csv
import glob
import json
import os
import re
import subprocess
import sys
import tempfile
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
LLVM = Path("/opt/rocm/lib/llvm/bin")


def short(name):
    return name.split("(")[0].replace("void ", "").replace("tvl1k::", "").strip()


# ----------------------------------------------------------------------------- collect
def level_tagger(spec):
    """spec "substr:levels:warps": dispatches of a kernel whose name holds substr come
    `warps` per level, coarsest level first, `levels` levels per solve (k_warp_iter: one
    launch per warp, TVL1_SPEC=0).  Two levels can share a grid size (C2's levels 0 and 1
    both run 1000 blocks), so the level is taken from the dispatch's ordinal in its file."""
    sub, levels, warps = spec.split(":")
    levels, warps = int(levels), int(warps)
    seen = defaultdict(dict)   # file -> dispatch id -> ordinal

    def tag(fname, kernel, did):
        if sub not in kernel:
            return ""
        m = seen[fname]
        if did not in m:
            m[did] = len(m)
        return "L%d" % (levels - 1 - (m[did] % (levels * warps)) // warps)
    return tag


def collect(d, spec="k_warp_iter<:5:30"):
    """Per (kernel, grid size, level): dispatches, mean duration (kernel trace) and the mean
    of every counter per dispatch over the --pmc passes of tools/pmc_issue.sh."""
    tag = level_tagger(spec)
    dur = defaultdict(list)
    for f in glob.glob(os.path.join(d, "trace", "*kernel_trace.csv")):
        rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Dispatch_Id"]))
        for r in rows:
            k = short(r["Kernel_Name"])
            grid = int(r["Grid_Size_X"]) * int(r.get("Grid_Size_Y") or 1) * int(r.get("Grid_Size_Z") or 1)
            key = (k, grid, tag(f, k, r["Dispatch_Id"]))   # counters report the whole grid
            dur[key].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    val = defaultdict(lambda: defaultdict(float))
    cnt = defaultdict(lambda: defaultdict(set))
    for f in glob.glob(os.path.join(d, "pmc_*", "*counter_collection.csv")):
        pas = Path(f).parent.name
        rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Dispatch_Id"]))
        for r in rows:
            k = short(r["Kernel_Name"])
            key = (k, int(r["Grid_Size"]), tag(f, k, r["Dispatch_Id"]))
            name = r["Counter_Name"]
            # a counter read in two passes (SQ_INSTS_VALU, GRBM_GUI_ACTIVE) is averaged over both
            val[key][name] += float(r["Counter_Value"])
            cnt[key][name].add((pas, r["Dispatch_Id"]))
    names = sorted({n for k in val for n in val[k]})
    w = csv.writer(sys.stdout)
    w.writerow(["kernel", "grid", "level", "dispatches", "avg_dur_ns"] + names)
    for key in sorted(val, key=lambda k: (k[0], k[2], -k[1])):
        ds = dur.get(key, [])
        row = [key[0], key[1], key[2], len(ds), round(sum(ds) / len(ds), 1) if ds else ""]
        for n in names:
            c = len(cnt[key][n])
            row.append(round(val[key][n] / c, 2) if c else "")
        w.writerow(row)


# ----------------------------------------------------------------------------- ISA
ISA_KERNELS = {
    # mangled-name fragment -> file name: the C2 pair's iteration class (k_warp_iter + the
    # streaming and blocked passes it runs) and the production strips' fused first pass
    "11k_warp_iterILi6ELi0ELi128ELi1ELi2E": "k_warp_iter_6_0_128_1_2.s",
    "14k_iterate_rollILb0ELi4ELi2ELi0E": "k_iterate_roll_0_4_2_0.s",
    "14k_iterate_rollILb0ELi2ELi4ELi0E": "k_iterate_roll_0_2_4_0.s",
    "14k_iterate_rollILb0ELi2ELi2ELi0E": "k_iterate_roll_0_2_2_0.s",
    "18k_iterate_roll_midILi0E": "k_iterate_roll_mid_0.s",
    "13k_iterate_tb4ILi0ELi3E": "k_iterate_tb4_0_3.s",
    "12kb_warp_iterILi6ELi0ELi2E": "kb_warp_iter_6_0_2.s",
    "15kb_iterate_rollILi4ELi2ELi0E": "kb_iterate_roll_4_2_0.s",
    "15kb_iterate_rollILi4ELi1ELi0E": "kb_iterate_roll_4_1_0.s",
    "15kb_iterate_rollILi2ELi1ELi0E": "kb_iterate_roll_2_1_0.s",
    "15kb_iterate_rollILi2ELi2ELi0E": "kb_iterate_roll_2_2_0.s",
}
# the C2 iteration class as rocprofv3 names it -> its ISA file
CLASS_KERNELS = {
    "k_warp_iter<6, 0, 128, 1, 2>": "k_warp_iter_6_0_128_1_2.s",
    "k_iterate_roll<false, 4, 2, 0>": "k_iterate_roll_0_4_2_0.s",
    "k_iterate_roll<false, 2, 4, 0>": "k_iterate_roll_0_2_4_0.s",
    "k_iterate_roll<false, 2, 2, 0>": "k_iterate_roll_0_2_2_0.s",
    "k_iterate_roll_mid<0>": "k_iterate_roll_mid_0.s",   # r6: absent from runs before it
    "k_iterate_tb4<0, 3>": "k_iterate_tb4_0_3.s",
}
# the production strips' batched iteration class (the kernels that hold 98 % of its time)
STRIP_CLASS_KERNELS = {
    "kb_warp_iter<6, 0, 2>": "kb_warp_iter_6_0_2.s",
    "kb_iterate_roll<4, 2, 0>": "kb_iterate_roll_4_2_0.s",
    "kb_iterate_roll<4, 1, 0>": "kb_iterate_roll_4_1_0.s",
    "kb_iterate_roll<2, 1, 0>": "kb_iterate_roll_2_1_0.s",
    "kb_iterate_roll<2, 2, 0>": "kb_iterate_roll_2_2_0.s",
}


def compact(lines):
    """llvm-objdump lines of one kernel -> 'offset<TAB>mnemonic<TAB>operands[ -> target]'."""
    sym = lines[0].split()
    base = int(sym[0], 16)
    out = [sym[1]]
    for l in lines[1:]:
        m = re.match(r"\t(\S+)\s*(.*?)\s*// ([0-9A-F]+):[^<]*(<[^+>]+(\+0x([0-9a-f]+))?>)?", l)
        if not m:
            continue
        t = ""
        if m.group(4):
            t = " -> %x" % (int(m.group(6), 16) if m.group(6) else 0)
        out.append("%x\t%s\t%s%s" % (int(m.group(3), 16) - base, m.group(1), m.group(2), t))
    return out


def dump_isa(out, so=ROOT / "fibsem-optflow_amd/lib/libtvl1_hip.so"):
    """The shipped code: both translation units' gfx950 objects of the built library."""
    sys.path.insert(0, str(ROOT / "tools"))
    import kernel_resources as kr
    out = Path(out)
    out.mkdir(parents=True, exist_ok=True)
    lines = []
    with tempfile.TemporaryDirectory() as t:
        for o in kr.so_objects(so, t):
            lines += subprocess.run([str(LLVM / "llvm-objdump"), "-d", "--no-show-raw-insn", str(o)],
                                    check=True, capture_output=True, text=True).stdout.split("\n")
    for sub, fname in ISA_KERNELS.items():
        start = next(i for i, l in enumerate(lines) if re.match(r"^[0-9a-f]+ <_ZN5tvl1k" + sub, l))
        end = next((i for i in range(start + 1, len(lines)) if re.match(r"^[0-9a-f]+ <", lines[i])),
                   len(lines))
        body = compact([l for l in lines[start:end] if l.strip()])
        (out / fname).write_text("\n".join(body) + "\n")
        print(f"{fname}: {len(body) - 1} instructions")


# ----------------------------------------------------------------------------- ISA loops
def load_isa(path):
    """(addr, mnemonic, operands, branch target) per instruction of a compact ISA dump."""
    ins = []
    for l in Path(path).read_text().split("\n")[1:]:
        if not l.strip():
            continue
        p = l.split("\t")
        rest, t = (p[2] if len(p) > 2 else ""), None
        if " -> " in rest:
            rest, tt = rest.split(" -> ")
            t = int(tt, 16)
        ins.append((int(p[0], 16), p[1], rest, t))
    return ins


# A forward branch inside a loop skips the region up to its target.  The region is rare (the
# branch taken) when it holds one of these: exact-division / sqrt fallbacks, the out-of-window
# global gather, the constants' stores (store_c), issue-priority steps.
RARE = ("v_div_fixup", "v_div_scale", "v_div_fmas", "global_load", "flat_load", "buffer_store",
        "s_setprio")


def hot_path(ins, h, latch):
    """Instruction indices of one trip of the loop headed at h (its last back edge at latch)
    along its common path.  Rules: an unconditional branch is followed (backwards too: the
    compiler lays some of a trip's blocks out of order); a conditional branch out of the loop
    or backwards is not taken (out-of-line code is cold: the x = 0 column forms, the loop
    exit); a forward conditional branch inside the loop skips a rare region (RARE) or a short
    edge-form region (< 60 instructions without f64 adds: the y = 0 / y = H-1 / last-band
    forms), and does not skip the residual's f64 accumulation or the LDS gather (>= 60
    instructions with LDS reads).  The trip ends when the path returns to h."""
    idx = {a: i for i, (a, _, _, _) in enumerate(ins)}
    i, path, seen = h, [], set()
    while True:
        if i in seen:
            raise RuntimeError(f"hot path of the loop at {h} revisits {i}")
        seen.add(i)
        a, mn, r, t = ins[i]
        path.append(i)
        if t is not None and (mn.startswith("s_cbranch") or mn == "s_branch"):
            ti = idx[t]
            if mn == "s_branch":
                if ti == h:
                    break
                i = ti
                continue
            if ti == h and i > h:   # the loop's conditional back edge: the next trip
                break
            if ti <= i or ti > latch or ti < h:
                i += 1
                continue
            mns = [x[1] for x in ins[i + 1:ti]]
            if any(m.startswith(RARE) for m in mns):
                take = True
            elif any(m.startswith("v_add_f64") for m in mns):
                take = False
            elif len(mns) >= 60 and any(m.startswith("ds_read") for m in mns):
                take = False
            else:
                take = True
            i = ti if take else i + 1
            continue
        i += 1
        if i == h:
            break
    return path


def role_loops(ins):
    """The three role loops of k_warp_iter / kb_warp_iter (the loops with an s_barrier, outside
    the entry block), as {role: per-trip mnemonic counts}; a trip is 3 steps (the step loops
    are unrolled by 3).  Producer: the loop with the most LDS reads (the gather); stage 2: the
    one with the residual's f64 adds; stage 1: the other."""
    idx = {a: i for i, (a, _, _, _) in enumerate(ins)}
    heads = defaultdict(int)
    for i, (a, mn, r, t) in enumerate(ins):
        if t is not None and t < a and (mn.startswith("s_cbranch") or mn == "s_branch"):
            heads[idx[t]] = max(heads[idx[t]], i)
    loops = []
    for h, l in sorted(heads.items()):
        if h < 100 or l - h < 300 or any(h0 <= h <= l0 for h0, l0 in loops):
            continue
        if not any(ins[k][1] == "s_barrier" for k in range(h, l + 1)):
            continue
        loops.append((h, l))
    counts = []
    for h, l in loops:
        c = defaultdict(int)
        for i in hot_path(ins, h, l):
            c[ins[i][1]] += 1
        counts.append(dict(c))
    assert len(counts) == 3, f"expected 3 role loops, found {len(counts)}"
    lds = [sum(v for m, v in c.items() if m.startswith("ds_read")) for c in counts]
    f64 = [sum(v for m, v in c.items() if m.startswith("v_add_f64")) for c in counts]
    prod = max(range(3), key=lambda k: lds[k])
    s2 = max((k for k in range(3) if k != prod), key=lambda k: f64[k])
    s1 = next(k for k in range(3) if k not in (prod, s2))
    return {"producer": counts[prod], "stage1": counts[s1], "stage2": counts[s2]}


# ----------------------------------------------------------------------------- costs
def load_rates(path):
    """tools/issue_rate.hip's table: name -> {waves per SIMD: (per wave, per SIMD)}."""
    out = {}
    for l in Path(path).read_text().split("\n"):
        if l.startswith("#") or "/SIMD:" not in l:
            continue
        name = l[:l.index(" 1/SIMD:")].strip()
        vals = re.findall(r"(\d)/SIMD:\s+([\d.]+) /wave\s+([\d.]+) /SIMD", l)
        out[name] = {int(w): (float(a), float(b)) for w, a, b in vals}
    return out


# mnemonic -> the measured row that prices it.  Full-rate VALU (2.5 cycles per wave-instruction
# per SIMD as measured), half rate (4.2-4.6), transcendental (8.2), packed f32 (8.7).  Rows:
# tools/issue_rate.hip.  v_cndmask_b32_e32's own row is an artefact of the probe (its VCC
# operand); it is priced as the e64 form.
PRICE_RULES = [
    (r"^v_(rcp|rsq|sqrt|exp|log|sin|cos)_f32", "v_rcp_f32"),
    (r"^v_pk_", "v_pk_add_f32"),
    (r"^v_cvt_f64_f32", "v_cvt_f64_f32"),
    (r"^v_(add|mul|fma)_f64", "v_add_f64"),
    (r"^v_readfirstlane", "v_readfirstlane_b32"),
    (r"_dpp$", "v_add_f32_dpp wave_shr:1"),
    (r"^v_cndmask", "v_cndmask_b32"),
    (r"^v_cmp.*_e64$", "v_cmp_gt_f32_e64"),
    (r"^v_cmp", "v_cmp_gt_f32_e32"),
    (r"^v_(max|min)", "v_max_f32"),
    (r"^v_med3", "v_med3_f32"),
    (r"^v_(floor|trunc|fract|rndne|ceil)", "v_floor_f32"),
    (r"^v_cvt_(i32|u32)_f32", "v_cvt_i32_f32"),
    (r"^v_cvt", "v_cvt_f32_i32"),
    (r"^v_(lshl_add|add_lshl|lshl_or|and_or|or3|xad|add3)", "v_lshl_add_u32"),
    (r"^v_(mad|mul)_u32_u24|^v_mad_", "v_mad_u32_u24"),
    (r"^v_(lshl|lshr|ashr)", "v_lshlrev_b32"),
    (r"^v_ldexp|^v_frexp", "v_ldexp_f32"),
    (r"^v_mov_b64", "v_mov_b64"),
    (r"^v_mul_f32_e64", "v_mul_f32_e64 (neg)"),
    (r"^v_fmac", "v_fmac_f32"),
    (r"^v_fma_f32", "v_fma_f32"),
    (r"^v_(add|sub|subrev)_f32", "v_add_f32"),
    (r"^v_mul_f32", "v_mul_f32"),
    (r"^v_(add|sub|subrev)_(u32|co_u32|i32)", "v_add_u32"),
    (r"^v_(and|or|xor|not|bfi|bfe)_b32", "v_and_b32"),
    (r"^v_mov_b32", "v_mov_b32"),
]
DEFAULT_HALF = "v_max_f32"   # anything else a VALU: priced at half rate, and listed


def price_key(mn):
    for pat, key in PRICE_RULES:
        if re.search(pat, mn):
            return key
    return DEFAULT_HALF


def is_valu(mn):
    return mn.startswith("v_") and not mn.startswith(("v_readlane", "v_writelane")) or \
        mn.startswith(("v_readlane", "v_writelane"))


# ----------------------------------------------------------------------------- geometry
C2_LEVELS = {"L0": (6144, 4096), "L1": (4915, 3277), "L2": (3932, 2621), "L3": (3146, 2097),
             "L4": (2517, 1678)}


def warp_iter_steps(W, H, blocks, bw=128, k=2):
    """(blocks, producer steps, stage steps) summed over the launch's blocks: bands of bw - 2k
    output px, segments of ceil(H / segs) rows; a segment's stages run 3 * thirds steps,
    its producers 3 (thirds + 1) (warp_iter_seg)."""
    bands = (W + bw - 2 * k - 1) // (bw - 2 * k)
    segs = blocks // bands
    seg = -(-H // segs)
    prod = stage = n = 0
    for s_ in range(segs):
        ys, ye = s_ * seg, min(s_ * seg + seg, H)
        if ys >= H:
            continue
        r0 = max(ys - k, 0)
        thirds = (ye + k - r0 + 2) // 3
        prod += bands * 3 * (thirds + 1)
        stage += bands * 3 * thirds
        n += bands
    return n, prod, stage


def model(isa_path, pmc_path, rates_path, roles_path=None, kernel="k_warp_iter<6, 0, 128, 1, 2>",
          levels=C2_LEVELS):
    """The report as a dict (see --model)."""
    ins = load_isa(isa_path)
    roles = role_loops(ins)
    rates = load_rates(rates_path)
    simd_cost = {k: v[8][1] for k, v in rates.items()}   # 8 waves per SIMD: throughput
    wave_cost = {k: v[1][0] for k, v in rates.items()}   # one wave alone: its issue cadence
    per_step = {r: {m: n / 3.0 for m, n in c.items()} for r, c in roles.items()}
    unpriced = sorted({m for c in roles.values() for m in c if m.startswith("v_")
                       and price_key(m) == DEFAULT_HALF})

    def cls(m):
        if m.startswith("v_"):
            k = price_key(m)
            if k == "v_rcp_f32":
                return "valu_trans"
            if k in ("v_add_f64", "v_cvt_f64_f32"):
                return "valu_f64"
            if k in ("v_add_f32", "v_mul_f32", "v_fma_f32", "v_fmac_f32", "v_add_u32", "v_and_b32",
                     "v_mov_b32", "v_mul_f32_e64 (neg)"):
                return "valu_full"
            if k == "v_pk_add_f32":
                return "valu_pk"
            return "valu_half"
        if m.startswith("ds_read"):
            return "lds_read"
        if m.startswith("ds_"):
            return "lds_write"
        if m.startswith(("buffer_", "global_", "flat_")):
            return "vmem"
        if m == "s_waitcnt":
            return "waitcnt"
        if m == "s_barrier":
            return "barrier"
        if m == "s_nop":
            return "nop"
        if m.startswith(("s_cbranch", "s_branch")):
            return "branch"
        return "salu"

    role_class = {r: defaultdict(float) for r in per_step}
    for r, c in per_step.items():
        for m, n in c.items():
            role_class[r][cls(m)] += n
    # per-wave issue of one step at the single-wave cadence (VALU by its row, LDS by the batched
    # read / write rows, everything else one 4-cycle issue slot, the barrier's own row)
    lds_r, lds_w, bar = wave_cost["ds_read_b32 x8 + lgkmcnt(0) (per read)"], \
        wave_cost["ds_write_b32 x8 + lgkmcnt(0) (per write)"], \
        wave_cost["s_barrier (4-wave block, per barrier)"]

    def wave_issue(c):
        t = 0.0
        for m, n in c.items():
            k = cls(m)
            if m.startswith("v_"):
                t += n * wave_cost[price_key(m)]
            elif k == "lds_read":
                t += n * lds_r
            elif k == "lds_write":
                t += n * lds_w
            elif k == "barrier":
                t += n * bar
            elif k == "waitcnt":
                t += 0.0
            else:
                t += n * 4.0
        return t

    rows = {r["level"]: r for r in csv.DictReader(open(pmc_path)) if r["kernel"] == kernel}
    out = {"kernel": kernel, "isa": str(isa_path), "pmc": str(pmc_path), "rates": str(rates_path),
           "roles_per_step": {r: dict(sorted(c.items())) for r, c in role_class.items()},
           "role_wave_issue_cycles_per_step": {r: round(wave_issue(c), 1) for r, c in per_step.items()},
           "unpriced_valu": unpriced, "levels": {}}
    for lv, (W, H) in levels.items():
        if lv not in rows:
            continue
        p = rows[lv]
        waves = float(p["SQ_WAVES"])
        blocks = int(round(waves / 4))
        n, prod, stage = warp_iter_steps(W, H, blocks)
        # dynamic counts per mnemonic over the launch: 2 producer waves + stage 1 + stage 2 per block
        dyn = defaultdict(float)
        for m, v in per_step["producer"].items():
            dyn[m] += 2 * prod * v
        for m, v in per_step["stage1"].items():
            dyn[m] += stage * v
        for m, v in per_step["stage2"].items():
            dyn[m] += stage * v
        model_valu = sum(v for m, v in dyn.items() if m.startswith("v_"))
        model_trans = sum(v for m, v in dyn.items() if cls(m) == "valu_trans")
        model_f64add = sum(v for m, v in dyn.items() if m.startswith("v_add_f64"))
        model_lds = sum(v for m, v in dyn.items() if m.startswith("ds_"))
        pmc_valu = float(p["SQ_INSTS_VALU"])
        gui = float(p["GRBM_GUI_ACTIVE"]) / 8.0   # kernel cycles (GRBM sums the 8 XCDs)
        dur = float(p["avg_dur_ns"])
        # SIMD issue demand: every wave-instruction at its measured SIMD throughput cost; the
        # model's per-mnemonic mix, scaled to the PMC's VALU count
        scale = pmc_valu / model_valu
        simd_busy = sum(v * simd_cost[price_key(m)] for m, v in dyn.items() if m.startswith("v_")) \
            * scale / 1024.0
        full = sum(v for m, v in dyn.items() if cls(m) == "valu_full") * scale
        lds_cu = (sum(v for m, v in dyn.items() if cls(m) == "lds_read") * simd_cost[
            "ds_read_b32 x8 + lgkmcnt(0) (per read)"] + sum(v for m, v in dyn.items() if cls(m) == "lds_write")
            * simd_cost["ds_write_b32 x8 + lgkmcnt(0) (per write)"]) / 4.0 / 256.0
        wave_life = 4.0 * float(p["SQ_WAVE_CYCLES"]) / waves
        steps_per_block = prod / n
        step = wave_life / steps_per_block   # the pace: cycles per producer step
        prod_issue = wave_issue(per_step["producer"])
        lv_out = {
            "W": W, "H": H, "blocks": n, "kernel_us": round(dur / 1e3, 1),
            "kernel_cycles": round(gui), "clock_ghz": round(gui / dur, 3),
            "valu_per_wave_model": round(model_valu / waves), "valu_per_wave_pmc": round(pmc_valu / waves),
            "valu_model_over_pmc": round(model_valu / pmc_valu, 3),
            "trans_model_over_pmc": round(model_trans / max(1.0, float(p["SQ_INSTS_VALU_TRANS_F32"])), 3),
            "f64add_model_over_pmc": round(model_f64add / max(1.0, float(p["SQ_INSTS_VALU_ADD_F64"])), 3),
            "lds_model_over_pmc": round(model_lds / max(1.0, float(p["SQ_INSTS_LDS"])), 3),
            "simd_valu_busy_cycles": round(simd_busy), "simd_valu_busy_frac": round(simd_busy / gui, 3),
            "simd_valu_frac_at_2_cycles": round(pmc_valu * 2 / 1024.0 / gui, 3),
            "full_rate_share_of_valu": round(full / pmc_valu, 3),
            "lds_pipe_busy_frac": round(lds_cu / gui, 3),
            "wave_life_over_kernel": round(wave_life / gui, 3),
            "wave_split": {k: round(float(p[c]) / float(p["SQ_WAVE_CYCLES"]), 3) for k, c in
                           (("active", "SQ_ACTIVE_INST_ANY"), ("issue_stall", "SQ_WAIT_INST_ANY"),
                            ("waiting", "SQ_WAIT_ANY"))},
            "dual_valu_issue_frac": round(float(p["SQ_ACTIVE_INST_VALU2"]) / float(p["SQ_ACTIVE_INST_VALU"]), 3),
            "step_cycles": round(step), "producer_wave_issue_cycles": round(prod_issue),
            "producer_issue_over_step": round(prod_issue / step, 3),
        }
        # while the launch's waves are resident (life / kernel of the kernel's cycles, the rest
        # is its ramp and tail), the share of SIMD cycles spent issuing VALU; the remainder of
        # the resident time is the named gap: every resident wave of a SIMD waiting at once
        # (the step barrier, LDS and VMEM latency)
        lv_out["simd_valu_busy_while_resident"] = round(lv_out["simd_valu_busy_frac"] /
                                                        lv_out["wave_life_over_kernel"], 3)
        lv_out["launch_ramp_tail_frac"] = round(1 - lv_out["wave_life_over_kernel"], 3)
        lv_out["latency_gap_frac"] = round(lv_out["wave_life_over_kernel"] - lv_out["simd_valu_busy_frac"], 3)
        out["levels"][lv] = lv_out
    if roles_path and Path(roles_path).exists():
        # share of each role's life at the step barrier (r5 tools/wi_probe.hip -DWI_BARRIER)
        txt = Path(roles_path).read_text()
        m = re.findall(r"barrier share of wave life \(waves 0\.\.3, consumers first\):\s+([\d. ]+)", txt)
        if m:
            v = [float(x) for x in m[0].split()]
            out["barrier_share_level0"] = {"stage1": v[0], "stage2": v[1], "producers": (v[2] + v[3]) / 2}
    # explained: SIMD VALU busy + the launch-tail idle of a one-round launch (mean block life /
    # span, r5 probe with the shipped priority: 0.89) -- the rest is SIMD idle at 4 waves/SIMD
    return out


def loop_mix(ins):
    """Mnemonic histogram of one trip of the kernel's main loop: of every loop (back edge) out
    of the entry block whose common path closes, the one that issues the most VALU (k_warp_iter
    and kb_warp_iter: the three role loops, see role_loops)."""
    idx = {a: i for i, (a, _, _, _) in enumerate(ins)}
    best = None
    for i, (a, mn, r, t) in enumerate(ins):
        if t is None or t >= a or not (mn.startswith("s_cbranch") or mn == "s_branch"):
            continue
        h = idx[t]
        if h < 100 or i - h < 50:
            continue
        try:
            path = hot_path(ins, h, i)
        except RuntimeError:   # an outer loop: its trip holds an inner loop
            continue
        if min(path) < h or max(path) > i:
            # not a loop: an out-of-line block (a border form) branching back into the body,
            # whose "trip" runs on through the real loop's back edge and around it (r6:
            # kb_iterate_roll<2, 2> once the sqrt's uniform taut test reshaped the layout)
            continue
        c = defaultdict(int)
        for k in path:
            c[ins[k][1]] += 1
        nv = sum(v for m, v in c.items() if m.startswith("v_"))
        if best is None or nv > best[0]:
            best = (nv, dict(c))
    return best[1]


def class_model(pmc_path, isa_dir, rates_path, kernels=CLASS_KERNELS):
    """The iteration class of one C2 pair alone: per kernel, the SIMD cost of an average VALU
    instruction (its main loop's mix from the ISA, each mnemonic at its measured throughput
    cost), times its PMC VALU count, over its kernel cycles (GRBM_GUI_ACTIVE / 8), summed over
    every dispatch of the class."""
    rates = load_rates(rates_path)
    simd_cost = {k: v[8][1] for k, v in rates.items()}
    rows = list(csv.DictReader(open(pmc_path)))
    out = {"kernels": {}}
    tb = tc = tv = tv2 = 0.0
    for kname, fname in kernels.items():
        if not any(r["kernel"] == kname and r["dispatches"] and int(r["dispatches"]) > 0
                   for r in rows):
            continue   # not dispatched in this run (e.g. the mid-check pass before r6's last engine)
        if kname.startswith(("k_warp_iter", "kb_warp_iter")):
            c = defaultdict(int)
            for r, cc in role_loops(load_isa(Path(isa_dir) / fname)).items():
                for m, v in cc.items():   # a block: 2 producer waves, 1 of each stage
                    c[m] += v * (2 if r == "producer" else 1)
        else:
            c = loop_mix(load_isa(Path(isa_dir) / fname))
        valu = {m: v for m, v in c.items() if m.startswith("v_")}
        n = sum(valu.values())
        cost = sum(v * simd_cost[price_key(m)] for m, v in valu.items()) / n
        kb = kc = kv = 0.0
        for r in rows:
            if r["kernel"] != kname or not r["dispatches"] or int(r["dispatches"]) == 0:
                continue
            d = int(r["dispatches"])
            kv += float(r["SQ_INSTS_VALU"]) * d
            kc += float(r["GRBM_GUI_ACTIVE"]) / 8.0 * d
            kd = float(r["avg_dur_ns"]) * d
            kl = d
            out.setdefault("_dur", 0.0)
            out["_dur"] += kd
            out.setdefault("_launches", 0)
            out["_launches"] += kl
        kb = kv * cost / 1024.0
        # the mix against the counters' own classes: transcendental and f32 add/mul/fma shares
        pt = sum(float(r["SQ_INSTS_VALU_TRANS_F32"]) * int(r["dispatches"]) for r in rows
                 if r["kernel"] == kname and r["dispatches"] and int(r["dispatches"]) > 0)
        pf = sum((float(r["SQ_INSTS_VALU_ADD_F32"]) + float(r["SQ_INSTS_VALU_MUL_F32"]) +
                  float(r["SQ_INSTS_VALU_FMA_F32"])) * int(r["dispatches"]) for r in rows
                 if r["kernel"] == kname and r["dispatches"] and int(r["dispatches"]) > 0)
        it = sum(v for m, v in valu.items() if price_key(m) == "v_rcp_f32")
        if_ = sum(v for m, v in valu.items() if re.match(r"^v_(add|sub|subrev|mul|fma|fmac)_f32", m))
        out["kernels"][kname] = {"valu_simd_cost": round(cost, 3), "valu_frac_at_2_cycles": round(kv * 2 / 1024 / kc, 3),
                                 "simd_valu_busy_frac": round(kb / kc, 3), "kernel_cycles": round(kc),
                                 "trans_share_isa": round(it / n, 4), "trans_share_pmc": round(pt / kv, 4),
                                 "f32_arith_share_isa": round(if_ / n, 4), "f32_arith_share_pmc": round(pf / kv, 4)}
        tb += kb
        tc += kc
        tv += kv * 2 / 1024.0
    out["class_simd_valu_busy_frac"] = round(tb / tc, 4)
    out["class_valu_frac_at_2_cycles"] = round(tv / tc, 4)
    out["class_kernel_cycles"] = round(tc)
    out["class_launches"] = out.pop("_launches")
    out["class_avg_launch_us"] = round(out.pop("_dur") / out["class_launches"] / 1e3, 2)
    out["class_clock_ghz"] = round(tc / (out["class_avg_launch_us"] * 1e3 * out["class_launches"]), 3)
    out["class_busy_cycles_per_launch"] = round(tb / out["class_launches"])
    return out


def report(m):
    L = [f"# Issue model of {m['kernel']} (tools/issue_model.py --model)", "",
         "Per step (one row of a block's band), hot path of each role from the ISA "
         "(instructions per wave):"]
    for r, c in m["roles_per_step"].items():
        L.append(f"  {r:9s} " + ", ".join(f"{k} {v:.1f}" for k, v in c.items()) +
                 f"  | one-wave issue {m['role_wave_issue_cycles_per_step'][r]:.0f} cycles")
    if m["unpriced_valu"]:
        L.append(f"  (priced at half rate by default: {', '.join(m['unpriced_valu'])})")
    L.append("")
    hdr = ("level", "us", "GHz", "VALU/wave model", "pmc", "model/pmc", "trans", "f64", "lds",
           "SIMD busy", "@2cyc", "full-rate", "LDS pipe", "life/kernel", "active", "stall", "wait",
           "VALU2", "step cyc", "prod issue", "issue/step", "busy|resident", "ramp+tail", "latency gap")
    L.append(" | ".join(hdr))
    for lv, d in m["levels"].items():
        ws = d["wave_split"]
        L.append(" | ".join(str(x) for x in (
            lv, d["kernel_us"], d["clock_ghz"], d["valu_per_wave_model"], d["valu_per_wave_pmc"],
            d["valu_model_over_pmc"], d["trans_model_over_pmc"], d["f64add_model_over_pmc"],
            d["lds_model_over_pmc"], d["simd_valu_busy_frac"], d["simd_valu_frac_at_2_cycles"],
            d["full_rate_share_of_valu"], d["lds_pipe_busy_frac"], d["wave_life_over_kernel"],
            ws["active"], ws["issue_stall"], ws["waiting"], d["dual_valu_issue_frac"],
            d["step_cycles"], d["producer_wave_issue_cycles"], d["producer_issue_over_step"],
            d["simd_valu_busy_while_resident"], d["launch_ramp_tail_frac"], d["latency_gap_frac"])))
    if "iteration_class" in m:
        ic = m["iteration_class"]
        L.append("")
        L.append("iteration class of one C2 pair (every dispatch): SIMD VALU busy "
                 f"{ic['class_simd_valu_busy_frac']} of its kernel cycles (priced at 2 cycles per "
                 f"VALU: {ic['class_valu_frac_at_2_cycles']})")
        for k, v in ic["kernels"].items():
            L.append(f"  {k:32s} cost/VALU {v['valu_simd_cost']:.2f}  busy {v['simd_valu_busy_frac']:.3f}"
                     f"  (@2 cycles {v['valu_frac_at_2_cycles']:.3f})  mix ISA/PMC: trans "
                     f"{v['trans_share_isa']:.3f}/{v['trans_share_pmc']:.3f}, f32 add/mul/fma "
                     f"{v['f32_arith_share_isa']:.3f}/{v['f32_arith_share_pmc']:.3f}")
    if "strips_class" in m:
        ic = m["strips_class"]
        L.append("")
        L.append("batched iteration class of one production strip batch (256 x 3072x100): SIMD VALU "
                 f"busy {ic['class_simd_valu_busy_frac']} (priced at 2 cycles: {ic['class_valu_frac_at_2_cycles']})")
        for k, v in ic["kernels"].items():
            L.append(f"  {k:32s} cost/VALU {v['valu_simd_cost']:.2f}  busy {v['simd_valu_busy_frac']:.3f}"
                     f"  (@2 cycles {v['valu_frac_at_2_cycles']:.3f})  mix ISA/PMC: trans "
                     f"{v['trans_share_isa']:.3f}/{v['trans_share_pmc']:.3f}, f32 add/mul/fma "
                     f"{v['f32_arith_share_isa']:.3f}/{v['f32_arith_share_pmc']:.3f}")
    if "barrier_share_level0" in m:
        L.append("")
        L.append("barrier share of wave life at level 0 (r5 probe): " +
                 ", ".join(f"{k} {v:.2f}" for k, v in m["barrier_share_level0"].items()))
    return "\n".join(L) + "\n"


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--collect")
    ap.add_argument("--levels", default="k_warp_iter<:5:30",
                    help="substr:levels:warps of the kernel whose dispatches are tagged by level")
    ap.add_argument("--dump-isa")
    ap.add_argument("--model", action="store_true")
    ap.add_argument("--isa", default=str(ROOT / "profiles/r6/issue/k_warp_iter_6_0_128_1_2.s"))
    ap.add_argument("--pmc", default=str(ROOT / "profiles/r6/issue/pmc_issue_c2.csv"))
    ap.add_argument("--rates", default=str(ROOT / "profiles/r6/issue/issue_rate.txt"))
    ap.add_argument("--roles", default=str(ROOT / "profiles/r5/wi_roles/roles.txt"))
    ap.add_argument("--json")
    a = ap.parse_args()
    if a.collect:
        collect(a.collect, a.levels)
    elif a.dump_isa:
        dump_isa(a.dump_isa)
    elif a.model:
        m = model(a.isa, a.pmc, a.rates, a.roles)
        m["iteration_class"] = class_model(a.pmc, Path(a.isa).parent, a.rates)
        sp = Path(a.pmc).parent / "pmc_issue_strips.csv"
        if sp.exists():   # one production strip batch alone (tools/pmc_issue.sh --strips)
            m["strips_class"] = class_model(sp, Path(a.isa).parent, a.rates, STRIP_CLASS_KERNELS)
        if a.json:
            Path(a.json).write_text(json.dumps(m, indent=1) + "\n")
        sys.stdout.write(report(m))
