#!/usr/bin/env python3
"""Per-level kernel time of TV-L1 solves from a rocprofv3 trace database (rocpd SQLite,
`rocprofv3 --kernel-trace -o NAME` writes NAME_results.db).  The engine's kernels of one
stream are split into levels at each upsample launch (k_upsample / kb_upsample: the flow
moves from level s to s-1) and into solves at each convert (k_convert_u8 / kb_convert);
within a level the time of every engine kernel is summed per kernel family.

    python tools/trace_levels.py gpurun_out/.../run_results.db [--levels 5]

Only meaningful for solves that do not overlap other solves' kernels (one stream, or a
batch alone): concurrent kernels inflate each other's durations."""
import argparse
import collections
import re
import sqlite3


def family(name):
    m = re.match(r"_ZN5tvl1k\d+(\w+?)I", name) or re.match(r"_ZN5tvl1k\d+(\w+?)E", name)
    base = m.group(1) if m else name
    # the streaming passes by their iteration count K: k_iterate_roll<G, K, PX, FM> and
    # kb_iterate_roll<K, PX, FM> (r6: the old test for "Li4E" anywhere in the name also
    # counted k_iterate_roll<G, 2, 4> as a 4-iteration pass)
    k = re.search(r"k_iterate_rollILb[01]ELi(\d)E", name) or re.search(r"kb_iterate_rollILi(\d)E", name)
    if k:
        base += f"<{k.group(1)}>"
    return base


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--levels", type=int, default=5)
    a = ap.parse_args()
    db = sqlite3.connect(a.db)
    names = {r[0]: r[1] for r in db.execute("select id, kernel_name from rocpd_info_kernel_symbol")}
    rows = sorted(db.execute("select start, end, kernel_id, stream_id from rocpd_kernel_dispatch"))
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    solves, level = 0, None
    for s, e, kid, _ in rows:
        n = names[kid]
        if "tvl1k" not in n:
            continue
        f = family(n)
        if "convert" in f:
            solves += 1
            level = a.levels - 1
        elif "upsample" in f and level is not None:
            level -= 1
            continue
        if level is None:
            continue
        per[level][f] += (e - s) / 1e6
    print(f"{solves} solve(s) (batches count once); ms per solve by level, largest families")
    for lv in sorted(per, reverse=True):
        tot = sum(per[lv].values()) / solves
        fams = sorted(per[lv].items(), key=lambda x: -x[1])[:5]
        print(f"  level {lv}: {tot:7.2f} ms  " +
              ", ".join(f"{k} {v / solves:.2f}" for k, v in fams))


if __name__ == "__main__":
    main()
