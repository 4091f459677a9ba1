"""The `cnn` command line (cnn-super-resolution_amd/host/tools/cnn.cpp), the
reference's src/Main_cl.cpp, and the sample generator tools/make_samples.py."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT

CNN = os.path.join(ROOT, "cnn-super-resolution_amd", "bin", "cnn")
MAKE_SAMPLES = os.path.join(ROOT, "tools", "make_samples.py")


def cnn(*args, timeout=600):
    return subprocess.run([CNN, *args], capture_output=True, text=True, timeout=timeout)


def write_config(path, params_file=""):
    cfg = {"n1": 64, "n2": 32, "f1": 9, "f2": 1, "f3": 5, "momentum": 0.9,
           "weight_decay_parameter": 0.001, "learning_rates": [0.001, 0.001, 0.0001],
           "parameters_file": params_file}
    for i in (1, 2, 3):
        cfg["parameters_distribution_%d" % i] = {"mean_w": 0.0, "mean_b": 0.0,
                                                 "std_deviation_w": 0.01, "std_deviation_b": 0.0}
    with open(path, "w") as fh:
        json.dump(cfg, fh)


def test_cli_help_and_argument_errors():
    p = cnn("-h")
    assert p.returncode == 0 and "usage: cnn" in p.stdout
    p = cnn("-c", "x.json")
    assert p.returncode == 1 and "--config and --in are required" in p.stdout
    p = cnn("-c", "x.json", "-i", "y.png")
    assert p.returncode == 1 and "Either provide out path or do the dry run" in p.stdout
    p = cnn("--bogus")
    assert p.returncode == 1 and "unknown argument" in p.stdout


def test_cli_config_errors_are_reported(tmp_path):
    p = cnn("dry", "-c", str(tmp_path / "missing.json"), "-i", "x.png")
    assert p.returncode == 1 and "[ERROR]" in p.stdout


def test_make_samples(tmp_path):
    subprocess.check_call([sys.executable, MAKE_SAMPLES, "--synthetic", "2", "--per-image", "3",
                           "-o", str(tmp_path), "-s", "33", "--seed", "1"])
    files = sorted(os.listdir(tmp_path))
    assert len(files) == 12
    from PIL import Image
    a = Image.open(tmp_path / "sample_0_large.png")
    b = Image.open(tmp_path / "sample_0_small.png")
    assert a.size == b.size == (33, 33)
    assert np.abs(np.asarray(a, np.int16) - np.asarray(b, np.int16)).max() > 0  # degraded


@pytest.mark.gpu
def test_cli_train_then_forward(tmp_path):
    samples = tmp_path / "samples"
    subprocess.check_call([sys.executable, MAKE_SAMPLES, "--synthetic", "6", "--per-image", "4",
                           "-o", str(samples), "-s", "33", "--seed", "2"])
    cfg = tmp_path / "config.json"
    write_config(cfg)
    params = tmp_path / "parameters.json"
    p = cnn("train", "-c", str(cfg), "-i", str(samples), "-o", str(params), "-e", "30",
            "--seed", "7")
    print(p.stdout[-3000:])
    assert p.returncode == 0, p.stdout
    assert "DONE" in p.stdout and "mean validation error" in p.stdout
    d = json.load(open(params))
    assert d["epochs"] == 30
    assert len(d["layer1"]["weights"]) == 9 * 9 * 64 and len(d["layer3"]["bias"]) == 1
    assert all(np.isfinite(d["layer2"]["weights"]))
    # forward with the trained parameters
    cfg2 = tmp_path / "config2.json"
    write_config(cfg2, str(params))
    from PIL import Image
    img = Image.open(samples / "sample_0_small.png").resize((64, 48))
    src = tmp_path / "in.png"
    img.save(src)
    out = tmp_path / "out.png"
    p = cnn("-c", str(cfg2), "-i", str(src), "-o", str(out))
    print(p.stdout[-2000:])
    assert p.returncode == 0, p.stdout
    res = Image.open(out)
    assert res.size == (64, 48) and res.mode == "RGB"


# the reference's profile.py regex (profile.py:9), verbatim as data
PROFILE_REGEX = r"Kernel '.*/(.*?]).*?([\-e.\d]+)ns.*?([\-e.\d]+)s"


def _train_args(tmp_path, samples, out, *extra):
    cfg = tmp_path / "config.json"
    if not cfg.exists():
        write_config(cfg)
    return ("train", "-c", str(cfg), "-i", str(samples), "-o", str(out), "-e", "5", "--seed", "3",
            *extra)


@pytest.mark.gpu
def test_cli_devices_one_rank_matches_single_device(tmp_path):
    """`train --devices 1` runs the data-parallel driver (thread per device,
    ncclCommInitAll, RCCL all-reduce of the flat gradients, sharded
    validation + scalar all-reduce) on one rank: it must produce exactly the
    parameters of the plain single-device run."""
    samples = tmp_path / "samples"
    subprocess.check_call([sys.executable, MAKE_SAMPLES, "--synthetic", "5", "--per-image", "4",
                           "-o", str(samples), "-s", "33", "--seed", "4"])
    a, b = tmp_path / "single.json", tmp_path / "dp.json"
    p = cnn(*_train_args(tmp_path, samples, a))
    assert p.returncode == 0, p.stdout
    p = cnn(*_train_args(tmp_path, samples, b, "--devices", "1"))
    print(p.stdout[-2000:])
    assert p.returncode == 0, p.stdout
    assert "Data-parallel training on 1 devices" in p.stdout and "DONE" in p.stdout
    assert json.load(open(a)) == json.load(open(b))


@pytest.mark.gpu
def test_cli_profile_output_parses_with_reference_regex(tmp_path):
    """`cnn profile` prints one line per kernel in the reference's format
    "Kernel '<dir>/<file>'[<defines>] total execution time: Nns = Ss"
    (src/opencl/Kernel.cpp:32-36, src/opencl/Context.cpp:88-96), which the
    reference's profile.py parses (profile.py:9-18)."""
    import re
    samples = tmp_path / "samples"
    subprocess.check_call([sys.executable, MAKE_SAMPLES, "--synthetic", "3", "--per-image", "4",
                           "-o", str(samples), "-s", "33", "--seed", "5"])
    p = cnn("profile", *_train_args(tmp_path, samples, tmp_path / "p.json"))
    assert p.returncode == 0, p.stdout
    found = re.findall(PROFILE_REGEX, p.stdout)
    names = {x[0] for x in found}
    print(sorted(names))
    assert "srcnn_train_fwd_bwd'[-D N1=64 -D N2=32 -D F1=9 -D F2=1 -D F3=5]" in names
    assert "srcnn_update_all'[-D N1=64 -D N2=32 -D F1=9 -D F2=1 -D F3=5]" in names
    assert "extract_luma'[-D NORMALIZE]" in names
    for name, ns, s in found:
        assert int(ns) >= 0 and abs(float(s) - int(ns) / 1e9) <= 1e-6 + 1e-3 * float(s)
    train = [x for x in found if x[0].startswith("srcnn_train_fwd_bwd")][0]
    assert int(train[1]) > 0  # device time was recorded


@pytest.mark.gpu
def test_cli_trains_on_reference_jpeg_samples(tmp_path):
    """The reference's sample layout: <name>_large.jpg / <name>_small.jpg
    pairs (generate_training_samples.py:36-41, src/Main_cl.cpp:267-301),
    decoded by host/src/Jpeg.cpp; then a JPEG photo through forward."""
    samples = tmp_path / "samples"
    subprocess.check_call([sys.executable, MAKE_SAMPLES, "--synthetic", "4", "--per-image", "4",
                           "-o", str(samples), "-s", "33", "--seed", "6", "--format", "jpg"])
    assert any(f.endswith("_large.jpg") for f in os.listdir(samples))
    params = tmp_path / "p.json"
    p = cnn(*_train_args(tmp_path, samples, params))
    print(p.stdout[-2000:])
    assert p.returncode == 0 and "DONE" in p.stdout, p.stdout
    assert "Skipping sample" not in p.stdout
    cfg2 = tmp_path / "config2.json"
    write_config(cfg2, str(params))
    from PIL import Image
    src = tmp_path / "photo.jpg"
    Image.open(samples / "sample_0_small.jpg").resize((72, 56)).save(src, quality=90, subsampling=2)
    out = tmp_path / "out.png"
    p = cnn("-c", str(cfg2), "-i", str(src), "-o", str(out))
    assert p.returncode == 0, p.stdout
    assert Image.open(out).size == (72, 56)


def _flat_params(path):
    d = json.load(open(path))
    return np.concatenate([np.asarray(d["layer%d" % i][k], np.float64) for i in (1, 2, 3)
                           for k in ("weights", "bias")])


@pytest.mark.gpu
@pytest.mark.parametrize("ranks", [2, 3])
def test_cli_data_parallel_ranks_match_single_device(tmp_path, ranks):
    """`train --devices N` with N > 1 on one GPU: N host threads on device 0
    (--same-device), the gradients summed by the host-sum exchange (the test
    seam of cnn.cpp; RCCL takes one rank per device).  This runs the driver's
    training-set sharding (some ranks get fewer samples), the per-rank
    validation sums and the exchange + identical update on every rank; the
    parameters must equal the single-device run on the union of the shards up
    to the fp32 order of the gradient sums (rank partial sums added in rank
    order instead of one sequential sum)."""
    samples = tmp_path / "samples"
    subprocess.check_call([sys.executable, MAKE_SAMPLES, "--synthetic", "5", "--per-image", "4",
                           "-o", str(samples), "-s", "33", "--seed", "4"])
    a, b, c = tmp_path / "single.json", tmp_path / "dp.json", tmp_path / "dp1.json"
    p = cnn(*_train_args(tmp_path, samples, a))
    assert p.returncode == 0, p.stdout
    single_err = [l for l in p.stdout.splitlines() if "mean validation error" in l]
    p = cnn(*_train_args(tmp_path, samples, b, "--devices", str(ranks), "--same-device", "--exchange", "host"))
    print(p.stdout[-2000:])
    assert p.returncode == 0, p.stdout
    assert "Data-parallel training on %d devices (0..0), host-sum" % ranks in p.stdout
    dp_err = [l for l in p.stdout.splitlines() if "mean validation error" in l]
    assert len(dp_err) == len(single_err) > 0
    for x, y in zip(single_err, dp_err):  # "[epoch] mean validation error: v (...)"
        vx, vy = float(x.split(":")[1].split()[0]), float(y.split(":")[1].split()[0])
        assert vy == pytest.approx(vx, rel=1e-4)
    ps, pd = _flat_params(a), _flat_params(b)
    scale = np.abs(ps).max()
    assert np.abs(pd - ps).max() <= 1e-5 * scale, np.abs(pd - ps).max() / scale
    # one rank through the same exchange reproduces the single device exactly
    p = cnn(*_train_args(tmp_path, samples, c, "--devices", "1", "--exchange", "host"))
    assert p.returncode == 0, p.stdout
    assert json.load(open(a)) == json.load(open(c))


def test_cli_same_device_needs_host_exchange(tmp_path):
    p = cnn("train", "-c", "x.json", "-i", str(tmp_path), "--devices", "2", "--same-device")
    assert p.returncode == 1 and "--same-device needs --exchange host" in p.stdout


@pytest.mark.gpu
def test_cli_save_momentum_resumes_training(tmp_path):
    """`train --save-momentum` (opt-in extension): the
    parameters file also holds each layer's momentum, and training resumed from
    it continues the momentum SGD (update_parameters.cl:1-33) where it stopped.
    4 epochs straight vs 2 + 2 resumed: equal up to the fp32 order of the
    per-sample gradient sums (the resumed run draws its own epoch shuffles;
    --validation-percent 0, so the shuffles only reorder those sums).  Resuming
    from the same file without the momentum keys -- the reference's behaviour,
    ConfigBasedDataPipeline.cpp:419-465 -- lands measurably further away.  The
    reference's loader skips the extra keys, so the file stays readable by it."""
    samples = tmp_path / "samples"
    subprocess.check_call([sys.executable, MAKE_SAMPLES, "--synthetic", "4", "--per-image", "4",
                           "-o", str(samples), "-s", "33", "--seed", "8"])
    cfg = tmp_path / "config.json"
    write_config(cfg)
    common = ("-i", str(samples), "--seed", "3", "--validation-percent", "0")
    straight, half = tmp_path / "straight.json", tmp_path / "half.json"
    p = cnn("train", "-c", str(cfg), "-o", str(straight), "-e", "4", *common)
    assert p.returncode == 0, p.stdout
    p = cnn("train", "-c", str(cfg), "-o", str(half), "-e", "2", "--save-momentum", *common)
    assert p.returncode == 0, p.stdout
    d = json.load(open(half))
    for i, (nw, nb) in zip((1, 2, 3), ((81 * 64, 64), (64 * 32, 32), (25 * 32, 1))):
        assert len(d["layer%d" % i]["momentum_weights"]) == nw
        assert len(d["layer%d" % i]["momentum_bias"]) == nb
    assert np.abs(d["layer1"]["momentum_weights"]).max() > 0
    # the same file without momentum: a reference-format parameters file
    bare = tmp_path / "bare.json"
    json.dump({k: ({kk: vv for kk, vv in v.items() if not kk.startswith("momentum")} if isinstance(v, dict) else v)
               for k, v in d.items()}, open(bare, "w"))
    outs = {}
    for name, src in (("resumed", half), ("bare", bare)):
        c = tmp_path / ("config_%s.json" % name)
        write_config(c, str(src))
        outs[name] = tmp_path / ("%s.json" % name)
        p = cnn("train", "-c", str(c), "-o", str(outs[name]), "-e", "2", *common)
        assert p.returncode == 0, p.stdout
        assert "momentum_weights" not in json.load(open(outs[name]))["layer1"]  # not asked to save it
    ref = _flat_params(straight)
    scale = np.abs(ref).max()
    err_resumed = np.abs(_flat_params(outs["resumed"]) - ref).max() / scale
    err_bare = np.abs(_flat_params(outs["bare"]) - ref).max() / scale
    print("resumed", err_resumed, "bare", err_bare)
    assert err_resumed <= 1e-5
    assert err_bare > 20 * max(err_resumed, 1e-7)


def test_cli_usage_lists_save_momentum():
    p = cnn("-h")
    assert p.returncode == 0 and "--save-momentum" in p.stdout
