"""Inference sharding by row bands (srcnn_amd/parallel.frame_band; SURVEY.md
8(e): "inference shards by spatial tile with a halo and needs no collective").

CPU: the bands of every rank cover the output rows exactly once, their input
slices stay inside the frame, and the oracle forward of the bands, stitched
together, is bit-identical to the oracle forward of the whole frame (every
output pixel is the same loop nest over the same inputs).
"""
import numpy as np
import pytest

from conftest import ROOT  # noqa: F401  (sys.path set-up)
from srcnn_amd import parallel

NETS = [(64, 32, 9, 1, 5), (32, 16, 9, 1, 3), (16, 8, 5, 3, 3)]


@pytest.mark.parametrize("h", [13, 14, 40, 97])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_bands_partition_output_rows(h, world):
    w = 30
    ctx = 12
    covered = []
    for r in range(world):
        i0, ni, o0, no = parallel.frame_band(w, h, (9, 1, 5), r, world)
        assert i0 == o0 and 0 <= i0 and i0 + ni <= h
        if no:
            assert ni == no + ctx
            covered.extend(range(o0, o0 + no))
        else:
            assert ni == 0
    assert covered == list(range(h - ctx))


def test_band_rejects_small_frames():
    with pytest.raises(ValueError):
        parallel.frame_band(12, 40, (9, 1, 5), 0, 2)
    with pytest.raises(ValueError):
        parallel.shard(10, 2, 2)


@pytest.mark.parametrize("net_t", NETS, ids=["default", "f3_3", "spatial"])
@pytest.mark.parametrize("world", [2, 3, 5])
def test_stitched_bands_equal_whole_frame(net_t, world):
    import srcnn_oracle as orc
    from hip_util import make_params
    rng = np.random.default_rng(31)
    w, h = 41, 37
    X = (rng.random(w * h, dtype=np.float32) - 0.5)
    p = make_params(rng, net_t, sd=0.05)
    ctx = net_t[2] + net_t[3] + net_t[4] - 3
    ow = w - ctx
    whole = orc.forward(net_t, X, w, h, 1, p)
    stitched = np.full_like(whole, np.nan)
    for r in range(world):
        i0, ni, o0, no = parallel.frame_band(w, h, net_t[2:], r, world)
        if no:
            band = orc.forward(net_t, X[i0 * w:(i0 + ni) * w], w, ni, 1, p)
            stitched[o0 * ow:(o0 + no) * ow] = band
    assert np.array_equal(stitched, whole)
