"""The committed measurement evidence agrees with itself: the bench line's
roofline fraction, which the engine computes from its live per-launch byte accounting and
HIP-event launch times, must match the fraction recomputed by hand from the rocprofv3 kernel
stats and the PMC byte counts of the same tree within 5 %, and the accounted bytes must match
the PMC bytes.  Reads only files under profiles/ (tools/roofline_check.py does the same)."""
import csv
import json
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
PROF = ROOT / "profiles"
ITER = ("k_iterate", "k_warp_iter")


def _bench(name):
    return json.loads(Path(PROF / "r2" / name).read_text().splitlines()[-1])


# (kernel stats of one pair alone, the bench line of the same tree, the PMC traffic record);
# the last triple is the final r2 engine, and profiles/traffic.json (bench.py's `traffic`) is it
@pytest.mark.parametrize("stats,bench,traffic", [
    ("kernel_stats_single_pair_prio.csv", "bench_c2_final.json", "traffic_prio.json"),
    ("latest/kernel_stats_single_pair.csv", "bench_c2_latest.json", "latest/traffic.json")])
def test_roofline_frac_matches_rocprof_and_pmc(stats, bench, traffic):
    traffic = json.loads((PROF / "r2" / traffic).read_text())
    calls = ns = 0.0
    for r in csv.DictReader(open(PROF / "r2" / stats)):
        name = r["Name"].split("(")[0].replace("void ", "").replace("tvl1k::", "")
        if name.startswith(ITER):
            calls += int(r["Calls"])
            ns += float(r["TotalDurationNs"])
    roof = _bench(bench)["roofline"]
    # whole solves of the same schedule in both runs (the traced run solves the isolated pair
    # once more, with events)
    assert calls % roof["launches"] == 0 and traffic["dispatches"] % roof["launches"] == 0
    avg_us = ns / calls / 1e3
    by_hand = traffic["iterate_hbm_bytes_per_launch"] / (avg_us * 1e-6) / 8e12
    assert roof["unit"] == "GB/s" and roof["peak"] == 8000.0
    assert abs(roof["frac"] / by_hand - 1) < 0.05, (roof["frac"], by_hand)
    # the engine's live byte accounting against the PMC bytes of the same launches
    assert abs(roof["bytes_per_launch"] / traffic["iterate_hbm_bytes_per_launch"] - 1) < 0.02
    assert roof["model_bytes_over_peak"] > 1.0 > roof["frac"]   # the SURVEY model is not frac


@pytest.mark.parametrize("bench", ["bench_c2_final.json", "bench_c2_latest.json"])
def test_bench_line_carries_the_contract_fields(bench):
    d = _bench(bench)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
              "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["config"]["workload"].startswith("C2")
    cb = d["cpu_baseline"]
    assert cb["kind"] in ("port", "reference") and cb["cores"] >= 1 and cb["value"] > 0
    modes = d["math_modes"]
    for m in ("fast", "fma"):
        e = modes[m]["epe_vs_headline_px"]
        assert modes[m]["same_iterations"]
        assert e["mean"] <= 1e-3 and e["p99.9"] <= 2e-2 and e["max"] <= 0.5


# ---- rounds 3 and 4: one box, one evidence set each (tools/final_profile.sh ->
# profiles/r3/final/, profiles/r4/final/): the default bench line, one C2 pair alone and one
# production strip batch alone
FINALS = [PROF / "r3" / "final", PROF / "r4" / "final", PROF / "r5" / "final", PROF / "r6" / "final"]


def _class_avg_us(stats_csv, prefixes):
    calls = ns = 0.0
    for r in csv.DictReader(open(stats_csv)):
        name = r["Name"].split("(")[0].replace("void ", "").replace("tvl1k::", "")
        if name.startswith(prefixes):
            calls += int(r["Calls"])
            ns += float(r["TotalDurationNs"])
    return ns / calls / 1e3, calls


@pytest.mark.parametrize("FINAL", FINALS, ids=["r3", "r4", "r5", "r6"])
@pytest.mark.parametrize("which", ["pair", "strips"])
def test_final_roofline_reproduces_by_hand(FINAL, which):
    """The bench line's `roofline.frac` (live byte accounting / HIP-event launch time) by hand
    from the same bytes over the rocprofv3 kernel-trace launch average, within 5 %, and the
    accounted bytes against the PMC FETCH x 2 + WRITE bytes of the same class -- for the C2
    pair and for the production-strip batch."""
    line = json.loads((FINAL / "bench_c2.json").read_text().splitlines()[-1])
    if which == "pair":
        roof = line["roofline"]
        traffic = json.loads((FINAL / "traffic.json").read_text())
        avg_us, calls = _class_avg_us(FINAL / "kernel_stats_single_pair.csv", ITER)
    else:
        roof = line["production_strips"]["roofline"]
        traffic = json.loads((FINAL / "traffic_strips.json").read_text())
        avg_us, calls = _class_avg_us(FINAL / "kernel_stats_strip_batch.csv",
                                      ("kb_iterate", "kb_warp_iter"))
    if roof.get("bound") == "valu":
        # r6: the bound is the VALU issue model's; the same hand check of its timing, then the
        # HBM roofline beside it as in earlier rounds
        v = roof["valu"]
        by_hand = v["busy_cycles_per_launch"] * 1024 / (avg_us * 1e-6) / 1e9 / v["peak"]
        assert abs(v["frac"] / by_hand - 1) < 0.05, (which, v["frac"], by_hand)
        roof = roof["hbm"]
    assert calls > 0 and roof["unit"] == "GB/s" and roof["peak"] == 8000.0
    # the timing: the same bytes over the kernel trace's launch average
    by_hand = roof["bytes_per_launch"] / (avg_us * 1e-6) / 8e12
    assert abs(roof["frac"] / by_hand - 1) < 0.05, (which, roof["frac"], by_hand)
    # the bytes: the engine's accounting against the PMC bytes of the same launch class (the
    # strip batch's tiny levels fetch ~6-7 % beyond the tiling's compulsory bytes, DESIGN 5:
    # since r4 their 64-px bands (256-B rows at 224-B steps) straddle one more 128-B line)
    pmc_frac = traffic["iterate_hbm_bytes_per_launch"] / (avg_us * 1e-6) / 8e12
    assert abs(roof["bytes_per_launch"] / traffic["iterate_hbm_bytes_per_launch"] - 1) < 0.08
    assert abs(roof["frac"] / pmc_frac - 1) < 0.10, (which, roof["frac"], pmc_frac)
    assert 0 < traffic["iterate_valu_frac"] < 1
    assert roof["model_bytes_over_peak"] > 1.0 > roof["frac"]


@pytest.mark.parametrize("FINAL", FINALS, ids=["r3", "r4", "r5", "r6"])
def test_final_bench_line_fields(FINAL):
    d = json.loads((FINAL / "bench_c2.json").read_text().splitlines()[-1])
    assert d["config"]["workload"].startswith("C2") and d["n_gpus"] == 1
    cb = d["cpu_baseline"]
    assert cb["kind"] == "port" and cb["value"] > 0 and "build" in cb
    assert d["production_strips"]["roofline"]["launches"] > 0


def test_bench_reads_the_r6_traffic_record():
    """profiles/traffic*.json (bench.py's `traffic`) are the r6 evidence sets' records: the C2
    class from the last engine (the mid-check pass changed its launch mix), the strips' from
    profiles/r6/final/ (the batched path did not change)."""
    for name, d in (("traffic.json", "final_mid"), ("traffic_strips.json", "final")):
        top = json.loads((PROF / name).read_text())
        r6 = json.loads((PROF / "r6" / d / name).read_text())
        assert top == r6 and f"profiles/r6/{d}/" in top["source"]


def test_r6_bench_line_names_the_valu_bound():
    """The r6 evidence line: `roofline.bound` is `valu` from the committed issue model
    (profiles/r6/issue/model.json), with the HBM roofline beside it, for C2 and the strips."""
    for d in ("final", "final_mid"):
        d = json.loads((PROF / "r6" / d / "bench_c2.json").read_text().splitlines()[-1])
        for r in (d["roofline"], d["production_strips"]["roofline"]):
            assert r["bound"] == "valu" and r["frac"] == r["valu"]["frac"] > r["hbm"]["frac"]
            assert "profiles/r6/issue/model.json" in r["valu"]["source"]
            assert abs(r["valu"]["frac"] / r["valu"]["pmc_frac"] - 1) < 0.10


def test_r5_bench_line_carries_rank_records_and_allotment():
    """VERDICT r4 items 5-6 in the r5 evidence line: one rank record with a PCI id, and the
    CPU baseline's allotment (affinity mask, cgroup quota, OMP_NUM_THREADS) with the oracle
    run on the smallest of them."""
    d = json.loads((PROF / "r5" / "final" / "bench_c2.json").read_text().splitlines()[-1])
    rk = d["ranks"]
    assert len(rk) == 1 and rk[0]["pci"].count(":") == 2 and rk[0]["pairs"] > 0
    a = d["cpu_baseline"]["allotment"]
    assert d["cpu_baseline"]["cores"] == a["threads"]
    assert a["threads"] == min(x for x in (a["affinity_cpus"], a["cgroup_quota_cpus"],
                                           a["omp_num_threads_env"]) if x)


def test_r4_kb_warp_iter_writes_below_fetches():
    """with the warp constants stored on demand, kb_warp_iter's PMC writes
    per dispatch fall below its fetches (r3: 897 MB written against 800 MB fetched)."""
    txt = (PROF / "r4" / "final" / "pmc_summary_strip_batch.txt").read_text()
    per_kernel = json.JSONDecoder().raw_decode(txt[txt.index("\n{") + 1:])[0]
    k = per_kernel["kb_warp_iter<6, 0, 2>"]
    assert k["write_bytes_per_dispatch"] < k["fetch_bytes_per_dispatch_x2"]
