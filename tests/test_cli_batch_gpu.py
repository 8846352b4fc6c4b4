"""Production strip jobs through the batched engine (VERDICT r3 "next" item 6): with the
job-wide top / bottom ROIs of gen_cross_file_list.py (/root/reference/support_scripts/
gen_cross_file_list.py:75-99) the CLI reads only the strips' rows of each slice and solves
each ROI key's strips of a chunk of pairs in one tvl1_calc_batch.  Every output must be
byte-identical to the per-pair path ("strip_batch": 0, one tvl1_calc per strip, r3), which
tests/test_cli_gpu.py holds to the oracle -- and one strip is checked against the oracle
directly here too."""
import ctypes as C
import json
import os
import subprocess

import numpy as np
import pytest
from PIL import Image

from optflow_amd import capi, synth
from oracle import checker

pytestmark = pytest.mark.gpu
OPTFLOW = capi.PKG_ROOT / "bin" / "optflow"
W, H, Z = 400, 300, 7
TOP, BOTTOM = 40, 30


@pytest.fixture(scope="module")
def stack(tmp_path_factory, built):
    d = tmp_path_factory.mktemp("stk")
    sl = synth.gen_stack(W, H, Z, seed=77)
    sl[3][:, :9] = 0                       # the I1 <= 1 mask and an empty-ish mask column
    for z in range(Z):
        Image.fromarray(sl[z]).save(d / f"s{z}.tif")       # uncompressed, one strip
        Image.fromarray(sl[z]).save(d / f"s{z}.png")
    return d, sl


def job(d, ext, otype, out, **kw):
    pairs = [(z, z + 1) for z in range(Z - 1)] + [(0, 4), (2, 6)]
    cfg = {"output_dir": str(out), "scale": 0.5, "output_type": otype, "nscales": 5, "warps": 3,
           "rois": {"top": TOP, "bottom": BOTTOM}, "stats_json": str(out / "stats.json"),
           "images": [{"p": str(d / f"s{a}.{ext}"), "q": str(d / f"s{b}.{ext}"),
                       "pId": f"t{a}", "qId": f"t{b}", "pGroupId": f"{a}.0",
                       "qGroupId": f"{b}.0", "output_name": f"z{a}_{b}"} for a, b in pairs]}
    cfg.update(kw)
    return cfg


def run(cfg, out, env=None):
    out.mkdir(exist_ok=True)
    p = out / "cfg.json"
    p.write_text(json.dumps(cfg))
    r = subprocess.run([str(OPTFLOW), str(p)], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, **(env or {})))
    assert r.returncode == 0, r.stderr
    return r, json.loads((out / "stats.json").read_text())


def outputs(out):
    return {f.name: f.read_bytes() for f in sorted(out.glob("*.tiff"))}


@pytest.mark.parametrize("ext", ["tif", "png"])
@pytest.mark.parametrize("otype", ["flow", "map"])
def test_batched_strips_byte_identical_to_per_pair(stack, tmp_path, ext, otype):
    d, _ = stack
    rb, sb = run(job(d, ext, otype, tmp_path / "b"), tmp_path / "b")
    ru, su = run(job(d, ext, otype, tmp_path / "u", strip_batch=0), tmp_path / "u")
    ob, ou = outputs(tmp_path / "b"), outputs(tmp_path / "u")
    assert len(ob) == 8 * 2 * 2 and ob.keys() == ou.keys()
    for k in ob:
        assert ob[k] == ou[k], k
    for eb, eu in zip(sb, su):
        assert eb["ok"] and eu["ok"]
        assert len(eb["solves"]) == 2
        for a, b in zip(eb["solves"], eu["solves"]):
            assert a["batch"] == 4 and "batch" not in b   # 8 pairs over 2 batch workers
            assert a["roi"] == b["roi"] and a["warp_iterations"] == b["warp_iterations"]
            assert a["read_rows_only"] is (ext == "tif")
    assert sorted(rb.stdout.splitlines()) == sorted(ru.stdout.splitlines())


def test_batched_strip_matches_oracle(stack, tmp_path):
    """The top strip of pair (1, 2): oracle(crop of the 2x2-area pre-scaled slices)."""
    d, _ = stack
    run(job(d, "tif", "flow", tmp_path), tmp_path)
    dec = []
    for z in (1, 2):
        subprocess.run([str(OPTFLOW), "--decode", str(d / f"s{z}.tif"), str(tmp_path / f"d{z}.tif"),
                        "0.5"], check=True)
        dec.append(np.array(Image.open(tmp_path / f"d{z}.tif")))
    h = dec[0].shape[0]
    for suf, sl in (("_top", np.s_[0:TOP]), ("_bottom", np.s_[h - BOTTOM:h])):
        a, b = np.ascontiguousarray(dec[0][sl]), np.ascontiguousarray(dec[1][sl])
        u, v, _, _ = checker.oracle_calc(a, b, capi.make_params(nscales=5, warps=3), warp_iters=False)
        lib = checker.load_oracle()
        lib.orc_postprocess.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t,
                                        C.c_int, C.c_int, C.c_int]
        lib.orc_postprocess(u.ctypes.data, v.ctypes.data, 4 * a.shape[1], b.ctypes.data,
                            a.shape[1], a.shape[1], a.shape[0], 0)
        got = np.array(Image.open(tmp_path / f"z1_2_0.50{suf}_x.tiff"))
        assert np.array_equal(got.view(np.uint32), u.view(np.uint32)), suf


def test_batched_random_points_debug_identical(stack, tmp_path):
    d, _ = stack
    kw = dict(npoints=12, debug=True, inflight=1)
    run(job(d, "tif", "random_points", tmp_path / "b", **kw), tmp_path / "b")
    run(job(d, "tif", "random_points", tmp_path / "u", strip_batch=0, **kw), tmp_path / "u")
    a = (tmp_path / "b" / "point_matches_0.json").read_text()
    assert a == (tmp_path / "u" / "point_matches_0.json").read_text()
    m = json.loads(a)
    assert len(m) == 8 and len(m[0]["matches"]["w"]) == 2 * 12


def test_sampled_random_points(stack, tmp_path):
    """Without debug the points are time-seeded (optflow.cpp:532-535): check the shape and
    that each q - p is the solved flow at p (from a flow run of the same job)."""
    d, _ = stack
    run(job(d, "tif", "random_points", tmp_path / "r", npoints=10), tmp_path / "r")
    run(job(d, "tif", "flow", tmp_path / "f"), tmp_path / "f")
    m = json.loads((tmp_path / "r" / "point_matches_0.json").read_text())
    assert len(m) == 8
    h = int(round(H * 0.5))
    for rec in m:
        mt = rec["matches"]
        assert len(mt["w"]) == 20
        name = f"z{rec['pId'][1:]}_{rec['qId'][1:]}_0.50"
        fx = {s: np.array(Image.open(tmp_path / "f" / f"{name}_{s}_x.tiff")) for s in ("top", "bottom")}
        fy = {s: np.array(Image.open(tmp_path / "f" / f"{name}_{s}_y.tiff")) for s in ("top", "bottom")}
        for k in range(20):
            px, py = mt["p"][0][k] * 0.5, mt["p"][1][k] * 0.5
            s, y0 = ("bottom", h - BOTTOM) if k < 10 else ("top", 0)   # keys in sorted order
            x, y = int(round(px)), int(round(py)) - y0
            assert abs((mt["q"][0][k] - mt["p"][0][k]) * 0.5 - fx[s][y, x]) < 1e-3
            assert abs((mt["q"][1][k] - mt["p"][1][k]) * 0.5 - fy[s][y, x]) < 1e-3


def test_mixed_job_and_fault_recovery(stack, tmp_path):
    """Pairs with their own keys (features off per image, a per-image ROI) and a pair whose
    frames differ in size go the per-pair way; an injected device fault in a strip batch
    is retried on a fresh context.  All outputs equal the all-per-pair run."""
    d, sl = stack
    big = np.zeros((H + 20, W + 30), np.uint8)
    big[:H, :W] = sl[5]
    Image.fromarray(big).save(d / "big.tif")
    cfg = job(d, "tif", "flow", tmp_path / "b")
    cfg["images"][1]["npoints"] = 5                   # an extra key: per pair
    cfg["images"].append({"p": str(d / "s4.tif"), "q": str(d / "big.tif"),
                          "output_name": "odd"})        # sizes differ: aligned per pair
    ref = json.loads(json.dumps(cfg))
    ref["strip_batch"] = 0
    ref["output_dir"] = str(tmp_path / "u")
    ref["stats_json"] = str(tmp_path / "u" / "stats.json")
    rb, sb = run(cfg, tmp_path / "b", env={"OPTFLOW_INJECT_FAULT": "3"})
    assert "retrying on a fresh device context" in rb.stderr
    run(ref, tmp_path / "u")
    ob, ou = outputs(tmp_path / "b"), outputs(tmp_path / "u")
    assert ob.keys() == ou.keys() and len(ob) == 9 * 4
    for k in ob:
        assert ob[k] == ou[k], k
    assert "batch" not in sb[1]["solves"][0] and sb[0]["solves"][0]["batch"] == 4   # 7 = 4 + 3
    assert all(e["ok"] for e in sb)


def test_batched_strips_over_two_device_workers(stack, tmp_path):
    """The CLI's `devices` sharding with batch workers (one per listed device, here the one
    GPU twice, one batch in flight each): every pair once, outputs identical to one worker."""
    d, _ = stack
    r2, s2 = run(job(d, "tif", "flow", tmp_path / "two", devices=[0, 0], inflight=1), tmp_path / "two")
    r1, s1 = run(job(d, "tif", "flow", tmp_path / "one", inflight=1), tmp_path / "one")
    o2, o1 = outputs(tmp_path / "two"), outputs(tmp_path / "one")
    assert o2.keys() == o1.keys() and len(o1) == 8 * 2 * 2
    for k in o1:
        assert o2[k] == o1[k], k
    assert all(e["ok"] for e in s2) and len(s2) == 8
    assert sorted(r2.stdout.splitlines()) == sorted(r1.stdout.splitlines())
    assert {e["solves"][0]["batch"] for e in s2} == {4} and {e["solves"][0]["batch"] for e in s1} == {8}


def test_strip_job_stage_timing(stack, tmp_path):
    """The build-only "timing_json" key: a strip job reports its decode
    pool's band reads and, per batch worker, the seconds of each stage, and the outputs are the
    same as without it."""
    d, _ = stack
    t = tmp_path / "t"
    run(job(d, "tif", "flow", t, timing_json=str(tmp_path / "timing.json")), t)
    run(job(d, "tif", "flow", tmp_path / "u"), tmp_path / "u")
    assert outputs(t) == outputs(tmp_path / "u")
    tm = json.loads((tmp_path / "timing.json").read_text())
    assert tm["pairs"] == Z - 1 + 2 and tm["wall_s"] > 0
    assert tm["decode"]["band_reads"] >= Z and tm["decode"]["band_read_s"] > 0
    ws = tm["batch_workers"]
    assert len(ws) >= 1 and sum(w["pairs"] for w in ws) == tm["pairs"]
    for w in ws:
        if w["pairs"]:
            st = w["stage_s"]
            for k in ("wait_bands", "pack", "upload_gpu", "solve", "read_back", "write_outputs"):
                assert k in st and st[k] >= 0, (k, st)
            assert st["solve"] > 0 and w["worker_s"] >= st["solve"]
