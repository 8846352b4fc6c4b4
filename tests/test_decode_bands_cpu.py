"""ROI-limited slice reads for strip jobs (VERDICT r3 "next" item 6): `optflow --decode-bands`
reads only the rows the top / bottom ROIs of the pre-scaled slice need (strip-organised
TIFF: pread of the rows or of the strips that hold them) and must give exactly the rows of
the whole decode + cv::resize restatement (`optflow --decode`, /root/reference/src/
optflow.cpp:104-131) -- at scale 1, at the production scale 0.5 (INTER_AREA 2x2) and at
generic scales (fixed-point bilinear), for uncompressed, LZW and deflate TIFFs with several
strip sizes, WhiteIsZero, and PNG (decoded whole)."""
import subprocess

import numpy as np
import pytest
from PIL import Image

from optflow_amd import capi

OPTFLOW = capi.PKG_ROOT / "bin" / "optflow"


def run(*a):
    r = subprocess.run([str(OPTFLOW), *map(str, a)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    return r.stdout


def whole(src, out, scale):
    run("--decode", src, out, scale)
    return np.array(Image.open(out))


def write_tiff(path, a, compression=None, rps=None, photometric=None):
    im = Image.fromarray(a)
    kw = {}
    if compression:
        kw["compression"] = compression
    if rps:
        kw["tiffinfo"] = {278: rps}
    if photometric is not None:   # WhiteIsZero: stored values are inverted
        from PIL import TiffImagePlugin
        info = TiffImagePlugin.ImageFileDirectory_v2()
        info[262] = photometric
        if rps:
            info[278] = rps
        kw["tiffinfo"] = info
        im = Image.fromarray(255 - a)
    im.save(path, **kw)


CASES = [("raw", None, None), ("raw_rps7", None, 7), ("raw_rps1", None, 1),
         ("lzw_rps16", "tiff_lzw", 16), ("deflate_rps5", "tiff_adobe_deflate", 5)]


@pytest.mark.parametrize("name,comp,rps", CASES, ids=[c[0] for c in CASES])
@pytest.mark.parametrize("scale", [1.0, 0.5, 0.75, 0.3])
def test_bands_equal_whole_decode(tmp_path, built, name, comp, rps, scale):
    rng = np.random.default_rng(5)
    a = rng.integers(0, 256, (157, 203), dtype=np.uint8)
    src = tmp_path / f"{name}.tif"
    write_tiff(src, a, comp, rps)
    full = whole(src, tmp_path / "w.tif", scale)
    H = full.shape[0]
    top, bottom = 13, 17
    out = run("--decode-bands", src, tmp_path / "b.tif", scale, top, bottom)
    W_, H_ = (int(t) for t in out.split()[0].split("x"))
    assert (H_, W_) == full.shape
    assert out.split()[1] == "partial"
    got = np.array(Image.open(tmp_path / "b.tif"))
    np.testing.assert_array_equal(got, np.concatenate([full[:top], full[H - bottom:]]))


def test_white_is_zero_and_png(tmp_path, built):
    rng = np.random.default_rng(6)
    a = rng.integers(0, 256, (90, 64), dtype=np.uint8)
    write_tiff(tmp_path / "wz.tif", a, None, 8, photometric=0)
    Image.fromarray(a).save(tmp_path / "a.png")
    for src, kind in ((tmp_path / "wz.tif", "partial"), (tmp_path / "a.png", "whole")):
        full = whole(src, tmp_path / "w.tif", 0.5)
        out = run("--decode-bands", src, tmp_path / "b.tif", 0.5, 10, 9)
        assert out.split()[1] == kind
        got = np.array(Image.open(tmp_path / "b.tif"))
        np.testing.assert_array_equal(got, np.concatenate([full[:10], full[-9:]]))


def test_band_outside_image_is_an_error(tmp_path, built):
    a = np.zeros((40, 30), np.uint8)
    Image.fromarray(a).save(tmp_path / "a.tif")
    r = subprocess.run([str(OPTFLOW), "--decode-bands", str(tmp_path / "a.tif"),
                        str(tmp_path / "b.tif"), "0.5", "30", "5"], capture_output=True, text=True)
    assert r.returncode == 1 and "outside" in r.stderr


def raw_tiff(path, a, rps, predictor=1, bad_strip=None):
    """A hand-written little-endian 8-bit gray uncompressed TIFF (PIL cannot write the
    predictor without compression).  predictor 2 stores each row's horizontal differences;
    bad_strip points that strip's offset past the end of the file."""
    import struct
    H, W = a.shape
    data = a.astype(np.int16)
    if predictor == 2:
        data = np.concatenate([data[:, :1], np.diff(data, axis=1)], axis=1) % 256
    data = data.astype(np.uint8)
    strips = [data[y:y + rps].tobytes() for y in range(0, H, rps)]
    body = b"".join(strips)
    offs, o = [], 8
    for s in strips:
        offs.append(o)
        o += len(s)
    if bad_strip is not None:
        offs[bad_strip] = 8 + len(body) + 4096
    n = len(strips)
    ifd_at = 8 + len(body) + 2 * 4 * n
    arrays = struct.pack(f"<{n}I", *offs) + struct.pack(f"<{n}I", *map(len, strips))
    ents = [(256, 4, 1, W), (257, 4, 1, H), (258, 3, 1, 8), (259, 3, 1, 1), (262, 3, 1, 1),
            (273, 4, n, 8 + len(body) if n > 1 else offs[0]), (277, 3, 1, 1), (278, 4, 1, rps),
            (279, 4, n, 8 + len(body) + 4 * n if n > 1 else len(strips[0])), (317, 3, 1, predictor)]
    ifd = struct.pack("<H", len(ents)) + b"".join(
        struct.pack("<HHII", t, ty, c, v) if ty == 4 or c > 1 else struct.pack("<HHIHH", t, ty, c, v, 0)
        for t, ty, c, v in ents) + struct.pack("<I", 0)
    path.write_bytes(b"II*\0" + struct.pack("<I", ifd_at) + body + arrays + ifd)


@pytest.mark.parametrize("scale", [1.0, 0.5])
def test_uncompressed_predictor2_bands_equal_whole_decode(tmp_path, built, scale):
    """the ROI read applies Predictor=2 to uncompressed strips as the whole decode
    does, so batched and per-pair strip jobs see the same bytes."""
    rng = np.random.default_rng(8)
    a = rng.integers(0, 256, (61, 47), dtype=np.uint8)
    src = tmp_path / "pred2.tif"
    raw_tiff(src, a, rps=6, predictor=2)
    full = whole(src, tmp_path / "w.tif", scale)
    if scale == 1.0:
        np.testing.assert_array_equal(full, a)   # the hand-written file decodes to a
    out = run("--decode-bands", src, tmp_path / "b.tif", scale, 7, 5)
    assert out.split()[1] == "partial"
    got = np.array(Image.open(tmp_path / "b.tif"))
    np.testing.assert_array_equal(got, np.concatenate([full[:7], full[-5:]]))


def test_out_of_range_strip_elsewhere_is_an_error(tmp_path, built):
    """a strip outside the file that the bands do not need still fails the read,
    as the whole decode (and the per-pair path) fails it."""
    a = np.random.default_rng(9).integers(0, 256, (60, 40), dtype=np.uint8)
    src = tmp_path / "bad.tif"
    raw_tiff(src, a, rps=10, bad_strip=3)   # rows 30-39: inside neither band
    for args in (("--decode", src, tmp_path / "w.tif", 1.0),
                 ("--decode-bands", src, tmp_path / "b.tif", 1.0, 10, 10)):
        r = subprocess.run([str(OPTFLOW), *map(str, args)], capture_output=True, text=True)
        assert r.returncode != 0 and "out of range" in r.stderr, (args[0], r.stderr)
