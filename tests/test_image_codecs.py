"""Host image codecs (cnn-super-resolution_amd/host/src/Image.cpp, Jpeg.cpp)
through bin/image_tool; no device needed.

The reference decodes every image with its vendored stb_image v2.06
(src/opencl/UtilsOpenCL.cpp:88-95) and its data flow is JPEG end to end
(generate_training_samples.py:36-41 writes *_large.jpg / *_small.jpg,
src/Main_cl.cpp:267-301 reads them).  The JPEG decoder is pinned by:
- the reference's own fixture test/data/color_grid2.jpg (a progressive
  JPEG, copied as tests/golden/color_grid2.jpg) run through the
  SwapLumaTest pipeline (test/specs/SwapLumaTest.cpp:39-90) against the
  reference's expected output color_grid2_luma_swapped.png
  (tests/golden/swap_luma.json): within the 2-LSB decoder budget;
- PIL's libjpeg on baseline / progressive / subsampled / restart-marker /
  grayscale / odd-sized files: bit-exact (both implement the published IJG
  "islow" integer inverse DCT, fancy upsampling and 16-bit JFIF color
  conversion; stb_image's own fixed-point variants sit within 2 LSB of them,
  which is the budget against the reference fixture).
"""
import json
import os
import subprocess

import numpy as np
import pytest

import srcnn_oracle as orc
from conftest import GOLDEN, ROOT

TOOL = os.path.join(ROOT, "cnn-super-resolution_amd", "bin", "image_tool")
Image = pytest.importorskip("PIL.Image")


def decode(path, tmp_path, ext=".ppm"):
    out = str(tmp_path / ("decoded" + ext))
    p = subprocess.run([TOOL, str(path), out], capture_output=True, text=True, timeout=60)
    assert p.returncode == 0, p.stdout
    return np.asarray(Image.open(out)).astype(np.int16)


def test_reference_fixture_swap_luma(tmp_path):
    """SwapLumaTest on our decode of the reference's JPEG fixture."""
    d = json.load(open(os.path.join(GOLDEN, "swap_luma.json")))
    w, h, pad = d["w"], d["h"], d["padding"]
    rgb = decode(os.path.join(GOLDEN, "color_grid2.jpg"), tmp_path)
    assert rgb.shape == (h, w, 3)
    rgba = np.concatenate([rgb, np.full((h, w, 1), 255, np.int16)], axis=2).astype(np.uint8).ravel()
    lw, lh = w - 2 * pad, h - 2 * pad
    n = lw * lw                                              # SwapLumaTest.cpp:48
    new_luma = (np.arange(n, dtype=np.float32) * np.float32(1.0)) / np.float32(n)
    out = orc.swap_luma(rgba, new_luma, w, h, lw, lh).astype(int)
    exp = np.array(d["expected_rgba"], np.uint8).reshape(-1, 4)[:, :3].reshape(-1).astype(int)
    diff = np.abs(out - exp)
    assert diff.max() <= 2, diff.max()
    assert np.count_nonzero(diff) <= 0.025 * diff.size, np.count_nonzero(diff)
    # and the decode itself against the fixture's PIL decode in the golden file
    pil = np.array(d["rgba"], np.int16).reshape(h, w, 4)[:, :, :3]
    assert np.abs(rgb - pil).max() <= 2


def _smooth(rng, w, h):
    g = rng.random((h // 8 + 2, w // 8 + 2, 3))
    im = Image.fromarray((g * 255).astype(np.uint8)).resize((max(w, 8), max(h, 8)), Image.BICUBIC)
    a = np.asarray(im).astype(np.int16) + rng.integers(-20, 20, (max(h, 8), max(w, 8), 3))
    return Image.fromarray(np.clip(a, 0, 255).astype(np.uint8)).resize((w, h))


CASES = {
    "baseline444": dict(quality=90, subsampling=0),
    "baseline420": dict(quality=90, subsampling=2),
    "baseline422": dict(quality=75, subsampling=1),
    "progressive420": dict(quality=85, subsampling=2, progressive=True),
    "progressive444": dict(quality=95, subsampling=0, progressive=True),
    "low_quality": dict(quality=30, subsampling=2),
    "restart_blocks": dict(quality=80, subsampling=2, restart_marker_blocks=3),
    "progressive_restart": dict(quality=80, subsampling=2, progressive=True, restart_marker_rows=1),
}


@pytest.mark.parametrize("size", [(37, 23), (64, 48), (17, 9), (1, 1)], ids=str)
@pytest.mark.parametrize("case", sorted(CASES))
def test_jpeg_decode_matches_libjpeg(tmp_path, case, size):
    rng = np.random.default_rng(sum(size) + len(case))
    p = tmp_path / "in.jpg"
    _smooth(rng, *size).save(p, "JPEG", **CASES[case])
    got = decode(p, tmp_path)
    ref = np.asarray(Image.open(p).convert("RGB")).astype(np.int16)
    assert got.shape == ref.shape
    assert np.array_equal(got, ref), np.abs(got - ref).max()


def test_jpeg_grayscale(tmp_path):
    rng = np.random.default_rng(3)
    p = tmp_path / "g.jpg"
    _smooth(rng, 40, 30).convert("L").save(p, quality=85)
    got = decode(p, tmp_path, ".pgm")
    ref = np.asarray(Image.open(p)).astype(np.int16)
    assert got.shape == ref.shape == (30, 40)
    assert np.array_equal(got, ref)


def test_jpeg_errors(tmp_path):
    rng = np.random.default_rng(4)
    p = tmp_path / "t.jpg"
    _smooth(rng, 32, 32).save(p, quality=80)
    raw = open(p, "rb").read()
    bad = tmp_path / "trunc.jpg"
    bad.write_bytes(raw[:40])
    r = subprocess.run([TOOL, str(bad), str(tmp_path / "o.ppm")], capture_output=True, text=True)
    assert r.returncode == 1 and "JPEG" in r.stdout
    cmyk = tmp_path / "cmyk.jpg"
    Image.new("CMYK", (16, 16), (10, 20, 30, 40)).save(cmyk)
    r = subprocess.run([TOOL, str(cmyk), str(tmp_path / "o.ppm")], capture_output=True, text=True)
    assert r.returncode == 1 and "JPEG" in r.stdout


def test_png_and_pnm_round_trip(tmp_path):
    rng = np.random.default_rng(5)
    a = rng.integers(0, 256, (13, 21, 3), dtype=np.uint8)
    Image.fromarray(a).save(tmp_path / "a.png")
    assert np.array_equal(decode(tmp_path / "a.png", tmp_path), a)
    Image.fromarray(a).save(tmp_path / "a.ppm")
    assert np.array_equal(decode(tmp_path / "a.ppm", tmp_path, ".png"), a)
