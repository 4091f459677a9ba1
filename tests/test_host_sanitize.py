"""Host file parsers under AddressSanitizer + UndefinedBehaviorSanitizer (CPU).

`cnn train -i DIR` and `cnn dry -i IMAGE` decode user files (the reference
decodes with its vendored stb_image, src/opencl/UtilsOpenCL.cpp:88-95) and
read user config.json / parameters.json.  tools/sanitize_host.sh builds the
JPEG / PNG / PNM decoders and the JSON reader with -fsanitize=address,undefined
and runs host/test/codec_fuzz.cpp, a deterministic mutation fuzzer, over seed
files: baseline 4:2:0 / 4:2:2 / 4:4:4, progressive, grayscale and
restart-interval JPEGs, PNG (RGB, RGBA, gray, gray+alpha, palette), PNM, the
reference's own JPEG fixture and config.json.  Every mutation must decode or
raise; a crash or a sanitizer report fails the test.  (The first run of this
fuzzer found an over-subscribed Huffman table overrunning the decoder's
lookup table; the decoder now rejects it before writing.)
"""
import os
import shutil
import subprocess

import numpy as np
import pytest

from conftest import ROOT

PIL = pytest.importorskip("PIL.Image")


def _seeds(d):
    rng = np.random.default_rng(3)
    a = (rng.random((37, 53, 3)) * 255).astype(np.uint8)
    a[:, :20] = 128  # flat area: runs of zero AC coefficients / EOB runs
    im = PIL.fromarray(a)
    out = []

    def save(name, img, **kw):
        p = os.path.join(d, name)
        img.save(p, **kw)
        out.append(p)
    save("base420.jpg", im, quality=85, subsampling=2)
    save("base422.jpg", im, quality=75, subsampling=1)
    save("base444.jpg", im, quality=90, subsampling=0)
    save("prog.jpg", im, quality=85, progressive=True)
    save("gray.jpg", im.convert("L"), quality=80)
    save("grayprog.jpg", im.convert("L"), quality=80, progressive=True)
    try:
        save("rst.jpg", im, quality=80, restart_marker_blocks=2)
    except TypeError:  # older Pillow without restart markers
        pass
    # an Adobe APP14 marker (transform byte = 1, YCbCr) right after SOI: its
    # truncations exercise the segment-length checks of read_adobe
    base = open(out[0], "rb").read()
    app14 = b"\xff\xee\x00\x0eAdobe\x00\x64\x00\x00\x00\x00\x01"
    p = os.path.join(d, "adobe.jpg")
    with open(p, "wb") as fh:
        fh.write(base[:2] + app14 + base[2:])
    out.append(p)
    save("rgb.png", im)
    save("rgba.png", im.convert("RGBA"))
    save("gray.png", im.convert("L"))
    save("la.png", im.convert("LA"))
    save("pal.png", im.convert("P"))
    save("img.ppm", im)
    save("img.pgm", im.convert("L"))
    out.append(os.path.join(ROOT, "tests", "golden", "color_grid2.jpg"))
    out.append(os.path.join(ROOT, "tests", "golden", "config", "config.json"))
    return out


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_codecs_under_asan_ubsan(tmp_path):
    seeds = _seeds(str(tmp_path))
    env = dict(os.environ, SANITIZE_OUT=str(tmp_path / "build"))
    r = subprocess.run([os.path.join(ROOT, "tools", "sanitize_host.sh"), "--iters", "1200"] + seeds,
                       env=env, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    lines = [l for l in r.stdout.splitlines() if "mutations=" in l]
    assert len(lines) == len(seeds)
    # the mutations exercise both outcomes: many decode, many are rejected
    dec = sum(int(l.split("decoded=")[1].split()[0]) for l in lines)
    rej = sum(int(l.split("rejected=")[1].split()[0]) for l in lines)
    assert dec > 1000 and rej > 1000, lines
