"""CPU tests of the optflow CLI surface (reference /root/reference/src/optflow.cpp:29-178,
228-261, 302-392, 500-514): config precedence, ROI geometry,
output naming, gz configs, comments, error reporting and image decoding.
`optflow --plan` resolves everything the pair loop would do without a GPU."""
import gzip
import json
import subprocess
from pathlib import Path

import numpy as np
import pytest
from PIL import Image

from optflow_amd import capi

OPTFLOW = capi.PKG_ROOT / "bin" / "optflow"
REF_EXAMPLE = Path("/root/reference/docs/example.json")


def run(*args, check=True):
    r = subprocess.run([str(OPTFLOW), *map(str, args)], capture_output=True, text=True,
                       timeout=120)
    if check and r.returncode != 0:
        raise AssertionError(f"optflow {args} failed ({r.returncode}): {r.stderr}")
    return r


def plan(cfg_path):
    out = run("--plan", cfg_path).stdout
    return json.loads(out[out.index("\n[") + 1:] if not out.startswith("[") else out)


@pytest.fixture
def slices(tmp_path, built):
    rng = np.random.default_rng(3)
    paths = []
    for z in range(3):
        a = rng.integers(0, 256, (61, 83), dtype=np.uint8)
        p = tmp_path / f"z{z}.png"
        Image.fromarray(a).save(p)
        paths.append(p)
    return paths


def write_cfg(tmp_path, cfg, name="cfg.json", gz=False, text=None):
    p = tmp_path / (name + (".gz" if gz else ""))
    data = (text if text is not None else json.dumps(cfg)).encode()
    if gz:
        with gzip.open(p, "wb") as f:
            f.write(data)
    else:
        p.write_bytes(data)
    return p


def test_help(built):
    r = run("--help")
    assert "Usage" in r.stdout


def test_defaults_and_precedence(tmp_path, slices):
    cfg = {"output_dir": str(tmp_path), "nscales": 5, "tau": 0.3,
           "images": [{"p": str(slices[0]), "q": str(slices[1]), "output_name": "a"},
                      {"p": str(slices[1]), "q": str(slices[2]), "output_name": "b",
                       "scale": 1, "tau": 0.2, "warps": 7, "rois": {"top": 10}}]}
    pl = plan(write_cfg(tmp_path, cfg))
    a, b = pl
    # scale default 0.5 (optflow.cpp:92); output = output_dir/output_name_%0.2f (:155-157)
    assert a["scale"] == 0.5 and a["output"] == f"{tmp_path}/a_0.50"
    assert a["size0"] == [42, 30]          # round-half-even(83*0.5)=42, round(61*0.5)=30
    # TV args: per-image -> global -> default (optflow.cpp:503-512)
    assert a["tv"] == {"tau": 0.3, "lambda": 0.05, "theta": 0.3, "nscales": 5, "warps": 5,
                       "epsilon": 0.01, "iterations": 300, "scaleStep": 0.8, "gamma": 0.0,
                       "medianFiltering": 1, "fastMath": 0, "profile": 0,
                       "innerIterations": 30, "outerIterations": 10}
    assert b["tv"]["tau"] == 0.2 and b["tv"]["warps"] == 7 and b["tv"]["nscales"] == 5
    assert b["output"] == f"{tmp_path}/b_1.00" and b["size0"] == [83, 61]
    # no ROI -> "default" full frame (optflow.cpp:147-154); per-image rois honoured
    assert a["rois"] == {"default": [0, 0, 42, 30]}
    assert b["rois"] == {"top": [0, 0, 83, 10]}
    assert a["output_type"] == "map" and a["features"] is False


def test_roi_geometry_and_sorted_order(tmp_path, slices):
    cfg = {"output_dir": str(tmp_path), "scale": 1.0,
           "rois": {"top": 12, "bottom": 9, "custom": [3, 4, 20, 10]},
           "images": [{"p": str(slices[0]), "q": str(slices[1]), "output_name": "x"}]}
    (pl,) = plan(write_cfg(tmp_path, cfg))
    # get_rois (optflow.cpp:228-261): top=[0,0,cols,top], bottom=[0,rows-b,cols,b]
    assert pl["rois"] == {"bottom": [0, 52, 83, 9], "custom": [3, 4, 20, 10],
                          "top": [0, 0, 83, 12]}
    # keys processed in sorted order; suffix _top/_bottom only (optflow.cpp:343-350)
    base = f"{tmp_path}/x_1.00"
    assert pl["files"] == [base + "_bottom", base, base + "_top"]


def test_custom_diff(tmp_path, slices):
    cfg = {"output_dir": str(tmp_path), "scale": 1,
           "rois": {"custom": {"0": [0, 0, 30, 20], "1": [5, 6, 30, 20]}},
           "images": [{"p": str(slices[0]), "q": str(slices[1]), "output_name": "c"}]}
    (pl,) = plan(write_cfg(tmp_path, cfg))
    assert pl["rois"] == {"custom_diff": {"0": [0, 0, 30, 20], "1": [5, 6, 30, 20]}}


def test_gen_cross_style_gz_shard(tmp_path, slices):
    """The shard format written by support_scripts/gen_cross_file_list.py:75-99."""
    cfg = {"style": 1, "debug": False, "homo": 4, "ratio": 0.7, "ransac": 5,
           "hessianThreshold": 1600, "scale": 0.5, "output_dir": str(tmp_path),
           "rois": {"top": 10, "bottom": 10}, "output_type": "random_points", "npoints": 25,
           "host": "render", "port": "8080", "matchCollection": "m", "owner": "o",
           "images": [{"p": str(slices[0]), "q": str(slices[1]), "pId": "t0", "qId": "t1",
                       "pGroupId": "1.0", "qGroupId": "2.0", "output_name": "t0_t1"}]}
    (pl,) = plan(write_cfg(tmp_path, cfg, name="shard_0.json", gz=True))
    assert pl["output_type"] == "random_points"
    assert pl["rois"] == {"bottom": [0, 20, 42, 10], "top": [0, 0, 42, 10]}
    assert pl["output"] == f"{tmp_path}/t0_t1_0.50"


def test_features_tristate(tmp_path, slices):
    base = {"output_dir": str(tmp_path), "images": [{"p": str(slices[0]), "q": str(slices[1])}]}
    assert plan(write_cfg(tmp_path, {**base, "features": 2}))[0]["features"] is True
    cfg = {**base, "features": 2}
    cfg["images"] = [{"p": str(slices[0]), "q": str(slices[1]), "features": False}]
    assert plan(write_cfg(tmp_path, cfg))[0]["features"] is False


def test_comments_allowed(tmp_path, slices):
    text = ("{ /* block comment */\n \"output_dir\": \"%s\", // line comment\n"
            " \"images\": [{\"p\": \"%s\", \"q\": \"%s\"}]\n}" % (tmp_path, slices[0], slices[1]))
    assert len(plan(write_cfg(tmp_path, None, text=text))) == 1


def test_malformed_json_is_reported(tmp_path, built):
    p = write_cfg(tmp_path, None, text='{\n "a": 1\n "b": 2\n}')
    r = run(p, check=False)
    assert r.returncode == 2 and "line 3" in r.stderr


@pytest.mark.skipif(not REF_EXAMPLE.exists(), reason="reference tree not mounted")
def test_reference_example_json_defects_are_reported(built):
    """docs/example.json is not valid JSON (missing commas after lines
    72 and 81, trailing comma at 67); the reference silently ignores the parse error."""
    r = run(REF_EXAMPLE, check=False)
    assert r.returncode == 2 and "line" in r.stderr


def test_unreadable_image_reported_and_skipped(tmp_path, slices):
    cfg = {"output_dir": str(tmp_path),
           "images": [{"p": str(tmp_path / "missing.png"), "q": str(slices[1])},
                      {"p": str(slices[0]), "q": str(slices[1])}]}
    r = run("--plan", write_cfg(tmp_path, cfg))
    assert f"Error: {tmp_path / 'missing.png'}" in r.stdout
    assert r.stdout.count(str(slices[0])) >= 1


@pytest.mark.parametrize("fmt", ["png", "tif", "tif_lzw", "png16", "pgm"])
def test_decode_formats(tmp_path, built, fmt):
    rng = np.random.default_rng(7)
    a = rng.integers(0, 256, (37, 53), dtype=np.uint8)
    src = tmp_path / f"in.{fmt.split('_')[0].replace('16', '')}"
    if fmt == "tif_lzw":
        Image.fromarray(a).save(src, compression="tiff_lzw")
    elif fmt == "png16":
        Image.fromarray(a.astype(np.uint16) * 257).save(src)
    elif fmt == "pgm":
        src.write_bytes(b"P5\n53 37\n255\n" + a.tobytes())
    else:
        Image.fromarray(a).save(src)
    out = tmp_path / "out.tif"
    run("--decode", src, out)
    assert np.array_equal(np.array(Image.open(out)), a)


def test_prescale_half_is_2x2_mean(tmp_path, built):
    """cv::resize at exactly 0.5 takes OpenCV's INTER_AREA fast path (2x2 mean)."""
    rng = np.random.default_rng(8)
    a = rng.integers(0, 256, (40, 64), dtype=np.uint8)
    src = tmp_path / "a.png"
    Image.fromarray(a).save(src)
    out = tmp_path / "o.tif"
    run("--decode", src, out, 0.5)
    b = np.array(Image.open(out)).astype(int)
    s = a.astype(int)
    ref = (s[0::2, 0::2] + s[1::2, 0::2] + s[0::2, 1::2] + s[1::2, 1::2] + 2) >> 2
    assert b.shape == (20, 32)
    assert np.array_equal(b, ref)   # 32 columns = 4 full 8-wide vector blocks


def _png_bytes(rows, width, height, ctype, depth, filters):
    """A PNG written by hand so every filter type (0-4) is exercised row by row."""
    import struct
    import zlib

    def chunk(t, d):
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)

    bpp = max(1, {0: 1, 2: 3, 4: 2, 6: 4}[ctype] * depth // 8)
    raw = bytearray()
    prev = np.zeros(rows.shape[1], np.int32)
    for y in range(height):
        cur = rows[y].astype(np.int32)
        f = filters[y % len(filters)]
        a = np.concatenate([np.zeros(bpp, np.int32), cur[:-bpp]])
        c = np.concatenate([np.zeros(bpp, np.int32), prev[:-bpp]])
        if f == 0:
            pred = np.zeros_like(cur)
        elif f == 1:
            pred = a
        elif f == 2:
            pred = prev
        elif f == 3:
            pred = (a + prev) // 2
        else:
            p = a + prev - c
            pa, pb, pc = np.abs(p - a), np.abs(p - prev), np.abs(p - c)
            pred = np.where((pa <= pb) & (pa <= pc), a, np.where(pb <= pc, prev, c))
        raw.append(f)
        raw += ((cur - pred) & 0xFF).astype(np.uint8).tobytes()
        prev = cur
    ihdr = struct.pack(">IIBBBBB", width, height, depth, ctype, 0, 0, 0)
    return (b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", ihdr) + chunk(b"IDAT", zlib.compress(bytes(raw), 6))
            + chunk(b"IEND", b""))


@pytest.mark.parametrize("inflate", ["default", "zlib"])
@pytest.mark.parametrize("kind", ["gray8", "gray16", "rgb8", "graya8"])
def test_png_every_filter_type(tmp_path, built, kind, inflate, monkeypatch):
    """PNG unfiltering (None, Sub, Up, Average, Paeth) for 1-, 2-, 3-byte pixels; the
    inflate goes through libdeflate when the image has it, else zlib."""
    rng = np.random.default_rng(11)
    H, W = 23, 41
    a = rng.integers(0, 256, (H, W), dtype=np.uint8)
    if kind == "gray8":
        rows, ctype, depth, want = a, 0, 8, a
    elif kind == "gray16":
        b16 = a.astype(np.uint16) * 257 + rng.integers(0, 2, (H, W)).astype(np.uint16)
        rows = b16.astype(">u2").view(np.uint8).reshape(H, 2 * W)
        ctype, depth, want = 0, 16, (b16 >> 8).astype(np.uint8)
    elif kind == "rgb8":
        rgb = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
        rgb[: H // 2] = a[: H // 2, :, None]          # gray rows take the r == g == b path
        rows, ctype, depth = rgb.reshape(H, 3 * W), 2, 8
        r, g, b = (rgb[..., k].astype(np.int64) for k in range(3))
        want = ((9798 * r + 19235 * g + (32768 - 9798 - 19235) * b + 16384) >> 15).astype(np.uint8)
        want[: H // 2] = a[: H // 2]
    else:
        ga = np.stack([a, rng.integers(0, 256, (H, W), dtype=np.uint8)], -1)
        rows, ctype, depth, want = ga.reshape(H, 2 * W), 4, 8, a
    src = tmp_path / "in.png"
    src.write_bytes(_png_bytes(rows, W, H, ctype, depth, [0, 1, 2, 3, 4, 4, 3, 1]))
    if inflate == "zlib":
        monkeypatch.setenv("OPTFLOW_NO_LIBDEFLATE", "1")
    out = tmp_path / "out.tif"
    run("--decode", src, out)
    assert np.array_equal(np.array(Image.open(out)), want)


@pytest.mark.parametrize("W,H,filters", [(41, 23, [4]), (8, 9, [4]), (7, 13, [4]), (200, 37, [4, 4, 4, 4, 4, 2, 4, 4, 4, 4, 1, 4, 4, 4]),
                                         (64, 4, [4]), (9, 6, [4, 4, 4, 0])])
def test_png_paeth_runs(tmp_path, built, W, H, filters):
    """8-bit gray Paeth rows, which the decoder unfilters 4 rows at a time (imageio.cpp
    paeth4): runs of Paeth rows broken by other filters, heights not a multiple of 4,
    widths at and below the interleaved path's minimum."""
    rng = np.random.default_rng(W * 1000 + H)
    a = rng.integers(0, 256, (H, W), dtype=np.uint8)
    a[: H // 2] = (np.add.outer(np.arange(H // 2), np.arange(W)) * 7 % 256).astype(np.uint8)
    src = tmp_path / "in.png"
    src.write_bytes(_png_bytes(a, W, H, 0, 8, filters))
    out = tmp_path / "out.tif"
    run("--decode", src, out)
    assert np.array_equal(np.array(Image.open(out)), a)


@pytest.mark.parametrize("threads", [1, 3])
def test_decode_ahead_over_many_chunks(tmp_path, built, threads):
    """The decode-ahead pool (build-only "decode_threads") across several chunks of pairs:
    adjacent and strided pairs, repeated slices, different scales and a missing file all come
    out in pair order with each slice's own size, as the serial loop would give."""
    rng = np.random.default_rng(12)
    paths = []
    for z in range(14):
        a = rng.integers(0, 256, (20 + z, 30 + 2 * z), dtype=np.uint8)
        p = tmp_path / f"s{z}.png"
        Image.fromarray(a).save(p)
        paths.append(p)
    imgs = [{"p": str(paths[z]), "q": str(paths[z + 1])} for z in range(13)]
    imgs += [{"p": str(paths[z]), "q": str(paths[z + 4])} for z in range(0, 10, 3)]
    imgs += [{"p": str(paths[2]), "q": str(paths[2]), "scale": 0.5},
             {"p": str(tmp_path / "missing.png"), "q": str(paths[0])},
             {"p": str(paths[5]), "q": str(paths[6])}]
    cfg = {"output_dir": str(tmp_path), "scale": 1, "decode_threads": threads, "images": imgs}
    out = run("--plan", write_cfg(tmp_path, cfg)).stdout
    assert f"Error: {tmp_path / 'missing.png'}" in out
    pl = {p["index"]: p for p in json.loads(out[out.index("\n[") + 1:]) if p}   # null: failed
    assert sorted(pl) == [i for i in range(len(imgs)) if "missing" not in imgs[i]["p"]]
    for i, p in pl.items():
        z = int(Path(imgs[i]["p"]).stem[1:])
        s = imgs[i].get("scale", 1)
        assert p["size0"] == [round((30 + 2 * z) * s), round((20 + z) * s)], (i, p["size0"])


# ---- generic INTER_LINEAR pre-scale (VERDICT r2 "next" item 6): cv::resize(scale) for any
# scale other than 1 and 0.5 (/root/reference/src/optflow.cpp:113,125), restated in
# cli/imageio.cpp as OpenCV's resizeGeneric_ with 11-bit fixed-point coefficients
# (INTER_RESIZE_COEF_BITS): xofs / alpha from float f = (dx + 0.5) / scale - 0.5, clamped at
# both borders, horizontal pass in int, vertical pass (ay0 h0 + ay1 h1 + 2^21) >> 22.
# Parity with OpenCV's own SIMD vertical pass is unpinned (OpenCV is absent here); these
# tests pin the restatement to its published scalar definition.
def linear_coeffs(n_src, n_dst, scale):
    inv = 1.0 / scale
    ofs, a0 = np.zeros(n_dst, int), np.zeros(n_dst, int)
    for d in range(n_dst):
        f = np.float32((d + 0.5) * inv - 0.5)
        s = int(np.floor(f))
        f = np.float32(f - np.float32(s))
        if s < 0:
            f, s = np.float32(0), 0
        if s >= n_src - 1:
            f, s = np.float32(0), n_src - 1
        ofs[d] = s
        a0[d] = int(np.rint((np.float32(1) - f) * np.float32(2048)))
    return ofs, a0, 2048 - a0


def resize_linear_ref(a, scale):
    scale = float(np.float32(scale))   # the reference's `float scale` (optflow.cpp:80,113)
    sh, sw = a.shape
    dw, dh = int(np.rint(sw * scale)), int(np.rint(sh * scale))
    xo, ax0, ax1 = linear_coeffs(sw, dw, scale)
    yo, ay0, ay1 = linear_coeffs(sh, dh, scale)
    s = a.astype(np.int64)
    xo1 = np.minimum(xo + 1, sw - 1)
    h = np.where(xo + 1 < sw, s[:, xo] * ax0 + s[:, xo1] * ax1, s[:, xo] * 2048)   # (sh, dw)
    h0, h1 = h[yo], h[np.minimum(yo + 1, sh - 1)]
    out = (ay0[:, None] * h0 + ay1[:, None] * h1 + (1 << 21)) >> 22
    return np.clip(out, 0, 255).astype(np.uint8)


def decode_scaled(tmp_path, a, scale):
    src = tmp_path / "a.png"
    Image.fromarray(a).save(src)
    out = tmp_path / "o.tif"
    run("--decode", src, out, scale)
    return np.array(Image.open(out))


@pytest.mark.parametrize("scale", [0.75, 0.3, 1.5])
@pytest.mark.parametrize("W,H", [(53, 37), (101, 67)])
def test_prescale_generic_constant_stays_constant(tmp_path, built, scale, W, H):
    a = np.full((H, W), 173, np.uint8)
    b = decode_scaled(tmp_path, a, scale)
    f = float(np.float32(scale))
    assert b.shape == (int(np.rint(H * f)), int(np.rint(W * f)))
    assert np.all(b == 173)


@pytest.mark.parametrize("scale", [0.75, 0.3, 1.5])
def test_prescale_generic_ramp_known_answers(tmp_path, built, scale):
    """A horizontal ramp 3x + 7 (rows equal, so the vertical pass multiplies by 2048):
    out = S[sx] + ((3 * alpha1 + 1024) >> 11) in the interior, S[W-1] where the source
    column clamps at the right border, S[0] where it clamps at the left (upscale)."""
    W, H = 77, 9
    a = np.tile((3 * np.arange(W) + 7).astype(np.uint8), (H, 1))
    b = decode_scaled(tmp_path, a, scale)
    scale = float(np.float32(scale))
    dw = int(np.rint(W * scale))
    inv = 1.0 / scale
    for dx in range(dw):
        f = np.float32((dx + 0.5) * inv - 0.5)
        sx = int(np.floor(f))
        if sx < 0:                          # left clamp (upscale): alpha = (2048, 0)
            want = 7
        elif sx >= W - 1:                   # right clamp
            want = 3 * (W - 1) + 7
        else:
            frac = np.float32(f - np.float32(sx))
            a1 = 2048 - int(np.rint((np.float32(1) - frac) * np.float32(2048)))
            want = 3 * sx + 7 + ((3 * a1 + 1024) >> 11)
        assert np.all(b[:, dx] == want), (dx, b[0, dx], want)
    if scale > 1:
        assert b[0, 0] == 7 and b[0, -1] == 3 * (W - 1) + 7


@pytest.mark.parametrize("scale", [0.75, 0.3, 1.5, 0.8])
@pytest.mark.parametrize("W,H", [(53, 37), (128, 95)])
def test_prescale_generic_matches_restatement(tmp_path, built, scale, W, H):
    rng = np.random.default_rng(W * 7 + H)
    a = rng.integers(0, 256, (H, W), dtype=np.uint8)
    assert np.array_equal(decode_scaled(tmp_path, a, scale), resize_linear_ref(a, scale))


def test_plan_reports_strip_batching(tmp_path, slices):
    """Strip jobs of the production shape (gen_cross_file_list.py: global top / bottom ROIs,
    per-image keys only p, q, the ids and output_name) go to the batched path; a pair with its
    own keys, features, or a job with other ROIs / strip_batch 0 does not."""
    base = {"output_dir": str(tmp_path), "scale": 1, "rois": {"top": 10, "bottom": 12},
            "output_type": "random_points",
            "images": [{"p": str(slices[0]), "q": str(slices[1]), "pId": "a", "qId": "b",
                        "pGroupId": "1.0", "qGroupId": "2.0", "output_name": "ab"},
                       {"p": str(slices[1]), "q": str(slices[2]), "npoints": 4},
                       {"p": str(slices[1]), "q": str(slices[2]), "features": 1}]}
    pl = plan(write_cfg(tmp_path, base))
    assert [e["strip_batch"] for e in pl] == [True, False, False]
    for extra in ({"strip_batch": 0}, {"rois": {"custom": [0, 0, 20, 20]}}, {"features": 1}):
        cfg = dict(base, **extra)
        assert not any(e["strip_batch"] for e in plan(write_cfg(tmp_path, cfg, name="c2.json")))
