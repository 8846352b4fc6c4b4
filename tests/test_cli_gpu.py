"""End-to-end: the optflow CLI on the GPU vs the oracle (+ the reference's solve_wrapper
post-ops).  Outputs must be bit-identical to oracle(ROI crops) + post-processing."""
import ctypes as C
import json
import subprocess
from pathlib import Path

import numpy as np
import pytest
from PIL import Image

from optflow_amd import capi, synth
from oracle import checker

pytestmark = pytest.mark.gpu
OPTFLOW = capi.PKG_ROOT / "bin" / "optflow"


def run_cli(cfg, tmp_path, name="cfg.json"):
    p = tmp_path / name
    p.write_text(json.dumps(cfg))
    r = subprocess.run([str(OPTFLOW), str(p)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    return r


def oracle_post(I0, I1, params, mode):
    u, v, _, _ = checker.oracle_calc(I0, I1, params, warp_iters=False)
    lib = checker.load_oracle()
    lib.orc_postprocess.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t,
                                    C.c_int, C.c_int, C.c_int]
    H, W = I0.shape
    I1c = np.ascontiguousarray(I1)
    lib.orc_postprocess(u.ctypes.data, v.ctypes.data, 4 * W, I1c.ctypes.data, W, W, H, mode)
    return u, v


@pytest.fixture
def pair(tmp_path, built):
    I0, I1 = synth.gen_pair(150, 110, seed=41)
    I1[:, :6] = 0                       # exercise the I1 <= 1 output mask
    Image.fromarray(I0).save(tmp_path / "p.png")
    Image.fromarray(I1).save(tmp_path / "q.png")
    return I0, I1


def tif(path):
    return np.array(Image.open(path)).astype(np.float32)


def test_flow_output_top_bottom_rois(tmp_path, pair):
    I0, I1 = pair
    cfg = {"output_dir": str(tmp_path), "scale": 1, "output_type": "flow", "nscales": 4,
           "warps": 4, "rois": {"top": 40, "bottom": 50},
           "images": [{"p": str(tmp_path / "p.png"), "q": str(tmp_path / "q.png"),
                       "output_name": "pq"}]}
    r = run_cli(cfg, tmp_path)
    assert f"{tmp_path / 'p.png'} {tmp_path / 'q.png'}" in r.stdout
    params = capi.make_params(nscales=4, warps=4)
    for suf, sl in (("_top", np.s_[0:40]), ("_bottom", np.s_[110 - 50:110])):
        u, v = oracle_post(np.ascontiguousarray(I0[sl]), np.ascontiguousarray(I1[sl]), params, 0)
        assert np.array_equal(tif(tmp_path / f"pq_1.00{suf}_x.tiff"), u)
        assert np.array_equal(tif(tmp_path / f"pq_1.00{suf}_y.tiff"), v)


def test_map_output_default_roi(tmp_path, pair):
    """No ROI -> 'default' full frame -> pre-alignment (optflow.cpp:366-377).  ratio 0
    leaves no match through the ratio test, so find_alignment falls back to the identity
    (features.cpp:157-166) and the features branch gives map = flow + grid (then masked)."""
    I0, I1 = pair
    cfg = {"output_dir": str(tmp_path), "scale": 1, "nscales": 3, "warps": 3, "ratio": 0.0,
           "images": [{"p": str(tmp_path / "p.png"), "q": str(tmp_path / "q.png"),
                       "output_name": "m"}]}
    r = run_cli(cfg, tmp_path)
    assert "Not enough matches. Using no transformation" in r.stdout
    assert "reverting to features" in r.stderr
    u, v = oracle_post(I0, I1, capi.make_params(nscales=3, warps=3), 1)
    assert np.array_equal(tif(tmp_path / "m_1.00_x.tiff"), u)
    assert np.array_equal(tif(tmp_path / "m_1.00_y.tiff"), v)


def test_size_mismatch_is_aligned(tmp_path, built):
    """frame1 = frame0 inside a larger canvas at offset (dx, dy): the CLI aligns frame1 onto
    frame0 (ORB + RANSAC, warpAffine), the flow between the aligned frames is ~0, and the
    features branch maps it back through the affine: map_x(x, y) ~ x + dx, map_y ~ y + dy.
    Approximate by construction (the homography is a fit): median within 0.25 px."""
    h, w, dx, dy = 360, 480, 17, 11
    f0 = np.clip(np.rint(synth.base_texture(w, h, seed=5)), 2, 255).astype(np.uint8)
    f1 = np.zeros((h + 40, w + 40), np.uint8)
    f1[dy:dy + h, dx:dx + w] = f0
    Image.fromarray(f0).save(tmp_path / "a.png")
    Image.fromarray(f1).save(tmp_path / "b.png")
    cfg = {"output_dir": str(tmp_path), "scale": 1, "nscales": 3, "warps": 2, "features": 1,
           "images": [{"p": str(tmp_path / "a.png"), "q": str(tmp_path / "b.png"),
                       "output_name": "al"}]}
    r = run_cli(cfg, tmp_path)
    assert "Not enough matches" not in r.stdout and "twenty percent" not in r.stdout
    mx, my = tif(tmp_path / "al_1.00_x.tiff"), tif(tmp_path / "al_1.00_y.tiff")
    assert mx.shape == (h, w)
    ys, xs = np.mgrid[20:h - 40, 20:w - 40]
    assert abs(np.median(mx[20:h - 40, 20:w - 40] - xs) - dx) < 0.25
    assert abs(np.median(my[20:h - 40, 20:w - 40] - ys) - dy) < 0.25


def test_prescale_half(tmp_path, pair):
    I0, I1 = pair
    cfg = {"output_dir": str(tmp_path), "output_type": "flow", "nscales": 3, "warps": 2,
           "rois": {"custom": [0, 0, 75, 55]},
           "images": [{"p": str(tmp_path / "p.png"), "q": str(tmp_path / "q.png"),
                       "output_name": "h"}]}
    run_cli(cfg, tmp_path)
    dec = []
    for n in ("p", "q"):
        subprocess.run([str(OPTFLOW), "--decode", str(tmp_path / f"{n}.png"),
                        str(tmp_path / f"{n}_s.tif"), "0.5"], check=True)
        dec.append(np.array(Image.open(tmp_path / f"{n}_s.tif")))
    u, v = oracle_post(dec[0], dec[1], capi.make_params(nscales=3, warps=2), 0)
    assert np.array_equal(tif(tmp_path / "h_0.50_x.tiff"), u)


def test_random_points_deterministic_with_debug(tmp_path, pair):
    cfg = {"output_dir": str(tmp_path), "scale": 1, "output_type": "random_points",
           "npoints": 10, "debug": True, "nscales": 3, "warps": 2, "rois": {"top": 30},
           "images": [{"p": str(tmp_path / "p.png"), "q": str(tmp_path / "q.png"),
                       "pId": "a", "qId": "b", "pGroupId": "1.0", "qGroupId": "2.0"}]}
    run_cli(cfg, tmp_path)
    first = (tmp_path / "point_matches_0.json").read_text()
    run_cli(cfg, tmp_path)
    assert (tmp_path / "point_matches_0.json").read_text() == first
    (m,) = json.loads(first)
    assert m["pId"] == "a" and m["qGroupId"] == "2.0"
    pm = m["matches"]
    assert len(pm["w"]) == 10 and len(pm["p"][0]) == 10 and len(pm["q"][1]) == 10
    # q - p is the flow at p (no pre-scale, top ROI at the origin)
    I0, I1 = pair
    u, v = oracle_post(np.ascontiguousarray(I0[:30]), np.ascontiguousarray(I1[:30]),
                       capi.make_params(nscales=3, warps=2), 0)
    for k in range(10):
        x, y = int(pm["p"][0][k]), int(pm["p"][1][k])
        assert abs(pm["q"][0][k] - (x + float(u[y, x]))) < 1e-4
        assert abs(pm["q"][1][k] - (y + float(v[y, x]))) < 1e-4


def test_random_points_sampled_without_debug(tmp_path, pair):
    """Without debug the CLI samples npoints distinct masked px directly and reads back only
    their flow (no full shuffle, no full download).  Each point must be a distinct px with
    q - p = the flow there, and inside the mask (frame0 > 1 or frame1 > 1)."""
    cfg = {"output_dir": str(tmp_path), "scale": 1, "output_type": "random_points",
           "npoints": 40, "nscales": 3, "warps": 2, "rois": {"top": 30},
           "images": [{"p": str(tmp_path / "p.png"), "q": str(tmp_path / "q.png"),
                       "pId": "a", "qId": "b", "pGroupId": "1.0", "qGroupId": "2.0"}]}
    run_cli(cfg, tmp_path)
    (m,) = json.loads((tmp_path / "point_matches_0.json").read_text())
    pm = m["matches"]
    assert len(pm["w"]) == 40 and set(pm["w"]) == {1}
    I0, I1 = pair
    u, v = oracle_post(np.ascontiguousarray(I0[:30]), np.ascontiguousarray(I1[:30]),
                       capi.make_params(nscales=3, warps=2), 0)
    seen = set()
    for k in range(40):
        x, y = int(pm["p"][0][k]), int(pm["p"][1][k])
        assert (x, y) not in seen
        seen.add((x, y))
        assert I0[y, x] > 1 or I1[y, x] > 1
        assert abs(pm["q"][0][k] - (x + float(u[y, x]))) < 1e-4
        assert abs(pm["q"][1][k] - (y + float(v[y, x]))) < 1e-4


def test_two_workers_match_one(tmp_path, built):
    """Pairs sharded over two workers (here both on GPU 0) give byte-identical files."""
    stack = synth.gen_stack(96, 64, 5, seed=77)
    for z in range(5):
        Image.fromarray(stack[z]).save(tmp_path / f"s{z}.png")
    imgs = [{"p": str(tmp_path / f"s{z}.png"), "q": str(tmp_path / f"s{z+1}.png"),
             "output_name": f"z{z}"} for z in range(4)]
    outs = []
    for tag, dev in (("one", [0]), ("two", [0, 0])):
        d = tmp_path / tag
        d.mkdir()
        run_cli({"output_dir": str(d), "scale": 1, "output_type": "flow", "nscales": 3,
                 "warps": 2, "devices": dev, "rois": {"custom": [0, 0, 96, 64]},
                 "images": imgs}, tmp_path, name=f"{tag}.json")
        outs.append({p.name: p.read_bytes() for p in sorted(d.glob("*.tiff"))})
    assert len(outs[0]) == 8 and outs[0] == outs[1]


def test_dualtvl1_profile_via_json(tmp_path, pair):
    """BASELINE configs[0]'s "DualTVL1 CPU" schedule through the CLI's JSON surface
    (build-only keys profile / innerIterations / outerIterations)."""
    I0, I1 = pair
    cfg = {"output_dir": str(tmp_path), "scale": 1, "output_type": "flow", "profile": 1,
           "nscales": 4, "warps": 3, "lambda": 0.15, "medianFiltering": 5,
           "innerIterations": 10, "outerIterations": 3,
           "images": [{"p": str(tmp_path / "p.png"), "q": str(tmp_path / "q.png"),
                       "output_name": "pq", "rois": {"custom": [0, 0, 150, 110]}}]}
    run_cli(cfg, tmp_path)
    params = capi.make_params(profile=1, nscales=4, warps=3, lambda_=0.15, median_filtering=5,
                              inner_iterations=10, outer_iterations=3)
    u, v = oracle_post(I0, I1, params, 0)
    out = sorted(tmp_path.glob("pq*_x.tiff"))
    assert out, list(tmp_path.iterdir())
    assert np.array_equal(tif(out[0]).view(np.uint32), u.view(np.uint32))


@pytest.mark.parametrize("rois", [{"top": 40, "bottom": 50}, None])
def test_device_fault_recovery(tmp_path, built, rois):
    """SURVEY 5 failure handling: a pair whose solve fails on a device error is solved again
    on a rebuilt device context (engine ctx, stream, buffers), and its outputs equal a
    fault-free run's.  OPTFLOW_INJECT_FAULT makes the first attempt of the listed pairs fail
    before any device work; a strip job (ROIs top/bottom, 8 workers) and a full-frame job."""
    import os
    zs = [synth.gen_pair(150, 110, seed=50 + k)[0] for k in range(4)]
    for k, z in enumerate(zs):
        Image.fromarray(z).save(tmp_path / f"s{k}.png")
    images = [{"p": str(tmp_path / f"s{k}.png"), "q": str(tmp_path / f"s{k + 1}.png"),
               "output_name": f"z{k}"} for k in range(3)]
    outs = {}
    for tag, fault in (("clean", None), ("fault", "0,2")):
        d = tmp_path / tag
        d.mkdir()
        cfg = {"output_dir": str(d), "scale": 1, "output_type": "flow", "nscales": 3,
               "warps": 3, "images": images}
        if rois:
            cfg["rois"] = rois
        p = tmp_path / f"{tag}.json"
        p.write_text(json.dumps(cfg))
        env = dict(os.environ)
        if fault:
            env["OPTFLOW_INJECT_FAULT"] = fault
        r = subprocess.run([str(OPTFLOW), str(p)], capture_output=True, text=True, timeout=300,
                           env=env)
        assert r.returncode == 0, r.stderr
        if fault:
            assert r.stderr.count("retrying on a fresh device context") == 2, r.stderr
        outs[tag] = {f.name: tif(f) for f in sorted(d.glob("*.tif*"))}
    assert outs["clean"] and outs["clean"].keys() == outs["fault"].keys()
    for name, a in outs["clean"].items():
        assert np.array_equal(a.view(np.uint32), outs["fault"][name].view(np.uint32)), name


def test_config_error_is_not_a_device_fault(tmp_path, built):
    """A pair whose TV-L1 parameters the engine rejects (TVL1_EINVAL from tvl1_set_params:
    medianFiltering 4) is an input error: reported with "Error:" like the reference's input
    errors, without a device-context rebuild or retry; the other pairs are solved."""
    zs = [synth.gen_pair(120, 90, seed=90 + k)[0] for k in range(3)]
    for k, z in enumerate(zs):
        Image.fromarray(z).save(tmp_path / f"s{k}.png")
    images = [{"p": str(tmp_path / f"s{k}.png"), "q": str(tmp_path / f"s{k + 1}.png"),
               "output_name": f"z{k}"} for k in range(2)]
    images[0]["medianFiltering"] = 4
    cfg = {"output_dir": str(tmp_path), "scale": 1, "output_type": "flow", "nscales": 3,
           "warps": 2, "inflight": 1, "rois": {"custom": [0, 0, 120, 90]}, "images": images}
    p = tmp_path / "bad.json"
    p.write_text(json.dumps(cfg))
    r = subprocess.run([str(OPTFLOW), str(p)], capture_output=True, text=True, timeout=300)
    assert "retrying on a fresh device context" not in r.stderr, r.stderr
    assert "Error: pair 0" in r.stderr and "medianFiltering" in r.stderr, r.stderr
    assert not list(tmp_path.glob("z0_*.tiff"))
    u, v = oracle_post(zs[1], zs[2], capi.make_params(nscales=3, warps=2), 0)
    (fx,) = tmp_path.glob("z1_*_x.tiff")
    assert np.array_equal(tif(fx).view(np.uint32), u.view(np.uint32))


@pytest.mark.parametrize("scale", [0.75, 0.3])
def test_prescale_generic_linear(tmp_path, pair, scale):
    """A pre-scale other than 0.5 (OpenCV's generic INTER_LINEAR, /root/reference/src/
    optflow.cpp:113,125): the solve on the resized frames equals the oracle on the same
    decoded + resized frames, bit for bit."""
    cfg = {"output_dir": str(tmp_path), "output_type": "flow", "nscales": 3, "warps": 2,
           "scale": scale, "images": [{"p": str(tmp_path / "p.png"), "q": str(tmp_path / "q.png"),
                                       "output_name": "g"}]}
    dec = []
    for n in ("p", "q"):
        subprocess.run([str(OPTFLOW), "--decode", str(tmp_path / f"{n}.png"),
                        str(tmp_path / f"{n}_s.tif"), str(scale)], check=True)
        dec.append(np.array(Image.open(tmp_path / f"{n}_s.tif")))
    h, w = dec[0].shape
    cfg["rois"] = {"custom": [0, 0, w, h]}
    run_cli(cfg, tmp_path)
    u, v = oracle_post(dec[0], dec[1], capi.make_params(nscales=3, warps=2), 0)
    (fx,) = tmp_path.glob("g_*_x.tiff")
    (fy,) = tmp_path.glob("g_*_y.tiff")
    assert np.array_equal(tif(fx).view(np.uint32), u.view(np.uint32))
    assert np.array_equal(tif(fy).view(np.uint32), v.view(np.uint32))


@pytest.mark.parametrize("devices", [[0], [0, 0]])
def test_pinned_uploads_match_pageable(tmp_path, built, devices):
    """SURVEY 8(f) N2 pinned uploads: slices decode into page-locked pool buffers (uploaded by
    one DMA each) and flow fields download into them; buffers are recycled across pairs and
    workers.  Outputs are byte-identical to the pageable path (OPTFLOW_PINNED=0), and the
    stats report pinned memory in use (none with OPTFLOW_PINNED=0).  Slices are > 256 KiB so
    the pool pins them; 7 pairs with slice reuse recycle the buffers.  Off by default; on
    with the build-only config key "pinned_host" or OPTFLOW_PINNED=1."""
    import os
    W, H = 640, 480
    stack = synth.gen_stack(W, H, 8, seed=91)
    for z in range(8):
        Image.fromarray(stack[z]).save(tmp_path / f"s{z}.png")
    imgs = [{"p": str(tmp_path / f"s{z}.png"), "q": str(tmp_path / f"s{z + 1}.png"),
             "output_name": f"z{z}"} for z in range(7)]
    outs, pinned = {}, {}
    for tag, env_v in (("pinned", "1"), ("pageable", "0"), ("config", None)):
        d = tmp_path / tag
        d.mkdir()
        cfg = {"output_dir": str(d), "scale": 1, "output_type": "flow", "nscales": 3,
               "warps": 2, "devices": devices, "rois": {"custom": [0, 0, W, H]},
               "stats_json": str(d / "stats.json"), "images": imgs}
        if tag == "config":
            cfg["pinned_host"] = True   # the config key; no env
        p = tmp_path / f"{tag}.json"
        p.write_text(json.dumps(cfg))
        env = dict(os.environ)
        env.pop("OPTFLOW_PINNED", None)
        if env_v is not None:
            env["OPTFLOW_PINNED"] = env_v
        r = subprocess.run([str(OPTFLOW), str(p)], capture_output=True, text=True, timeout=300,
                           env=env)
        assert r.returncode == 0, r.stderr
        st = json.loads((d / "stats.json").read_text())
        assert all(e["ok"] for e in st)
        pinned[tag] = st[0]["host_pinned_bytes"]
        outs[tag] = {f.name: f.read_bytes() for f in sorted(d.glob("*.tiff"))}
    assert len(outs["pinned"]) == 14 and outs["pinned"] == outs["pageable"] == outs["config"]
    # two slices + two flow fields per worker at least, all recycled: bounded by the pool
    assert pinned["pinned"] >= 2 * W * H and pinned["config"] >= 2 * W * H, pinned
    assert pinned["pageable"] == 0, pinned
    assert pinned["pinned"] <= len(devices) * 64 * (1 << 20), pinned
    # the custom ROI reads the whole frame: equal to the oracle on one pair
    u, v = oracle_post(stack[3], stack[4], capi.make_params(nscales=3, warps=2), 0)
    assert np.array_equal(tif(tmp_path / "pinned" / "z3_1.00_x.tiff"), u)
    assert np.array_equal(tif(tmp_path / "pinned" / "z3_1.00_y.tiff"), v)
