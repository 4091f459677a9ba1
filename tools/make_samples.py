#!/usr/bin/env python3
"""Training-sample generator for `cnn train` (the reference's
generate_training_samples.py, re-done): from every image of --in-dir, crop a
random --out-size square (the ground truth, <name>_large.png) and degrade it
by downscaling with --degrade-factor and upscaling back with Lanczos
resampling (the network input, <name>_small.png).  PNG by default
(lossless); --format jpg writes the reference's JPEG pairs, which the C++
side decodes too (host/src/Jpeg.cpp).

  python tools/make_samples.py -i raw_dir -o samples_dir -s 33 -d 2 [--per-image N] [--seed S]
  python tools/make_samples.py --synthetic 64 -o samples_dir -s 33      # no input images needed
"""
import argparse
import os
import random

import numpy as np
from PIL import Image


def degrade(large, factor):
    w, h = large.size
    small = large.resize((max(1, int(w / factor)), max(1, int(h / factor))), Image.LANCZOS)
    return small.resize((w, h), Image.LANCZOS)


def synthetic_image(rng, size):
    """Smooth colour field with a few hard edges (luma structure to learn)."""
    g = rng.random((size // 8 + 2, size // 8 + 2, 3))
    img = Image.fromarray((g * 255).astype(np.uint8)).resize((size, size), Image.BICUBIC)
    a = np.asarray(img).astype(np.float32)
    yy, xx = np.mgrid[0:size, 0:size]
    for _ in range(3):
        cx, cy, r = rng.integers(0, size, 2).tolist() + [int(rng.integers(size // 8, size // 3))]
        a[(xx - cx) ** 2 + (yy - cy) ** 2 < r * r] *= 0.5
    return Image.fromarray(np.clip(a, 0, 255).astype(np.uint8))


def main():
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--in-dir", "-i")
    ap.add_argument("--out-dir", "-o", required=True)
    ap.add_argument("--out-size", "-s", type=int, required=True)
    ap.add_argument("--degrade-factor", "-d", type=float, default=2.0)
    ap.add_argument("--per-image", type=int, default=1, help="crops per input image")
    ap.add_argument("--synthetic", type=int, default=0, help="generate N synthetic source images")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--format", choices=["png", "jpg"], default="png",
                    help="jpg writes <name>_large.jpg / _small.jpg like the reference's "
                         "generate_training_samples.py:36-41 (PIL default quality)")
    a = ap.parse_args()
    rnd = random.Random(a.seed)
    rng = np.random.default_rng(a.seed)
    sources = []
    if a.synthetic:
        sources = [("synthetic%d" % i, synthetic_image(rng, max(64, 2 * a.out_size)))
                   for i in range(a.synthetic)]
    elif a.in_dir:
        for f in sorted(os.listdir(a.in_dir)):
            p = os.path.join(a.in_dir, f)
            if os.path.isfile(p):
                try:
                    sources.append((os.path.splitext(f)[0], Image.open(p).convert("RGB")))
                except OSError:
                    print("cannot read '%s', skipped" % f)
    else:
        ap.error("either --in-dir or --synthetic")
    os.makedirs(a.out_dir, exist_ok=True)
    n = 0
    for name, im in sources:
        if im.width < a.out_size or im.height < a.out_size:
            print("'%s' is smaller than --out-size, skipped" % name)
            continue
        for k in range(a.per_image):
            x = rnd.randint(0, im.width - a.out_size)
            y = rnd.randint(0, im.height - a.out_size)
            large = im.crop((x, y, x + a.out_size, y + a.out_size))
            base = os.path.join(a.out_dir, "sample_%d" % n)
            large.save(base + "_large." + a.format)
            degrade(large, a.degrade_factor).save(base + "_small." + a.format)
            n += 1
    print("created %d sample pairs" % n if n else "No files were created")


if __name__ == "__main__":
    main()
