"""bench.py's launcher (CPU): `--gpus N` must measure N ranks.

Without a torch.distributed.run environment, `bench.py --gpus N > 1` starts
the N rank processes itself (torch.distributed.run as a child, before any GPU
call); under a launcher, WORLD_SIZE must equal --gpus or the run exits
non-zero before touching the GPU.  The per-rank loop is the reference's
training loop (src/Main_cl.cpp:161-195) sharded over GPUs.
"""
import os
import subprocess
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402  (module import touches no GPU)


def test_launch_plan_single_gpu():
    assert bench.launch_plan(1, {}) == ("run", 1)


def test_launch_plan_spawns_without_launcher():
    assert bench.launch_plan(8, {}) == ("spawn", 8)
    assert bench.launch_plan(2, {"WORLD_SIZE": ""}) == ("spawn", 2)


def test_launch_plan_under_launcher():
    assert bench.launch_plan(4, {"WORLD_SIZE": "4", "RANK": "3"}) == ("run", 4)


@pytest.mark.parametrize("gpus,ws", [(2, "3"), (1, "8"), (8, "1")])
def test_launch_plan_mismatch_is_an_error(gpus, ws):
    with pytest.raises(SystemExit) as e:
        bench.launch_plan(gpus, {"WORLD_SIZE": ws})
    assert "WORLD_SIZE" in str(e.value)


def test_launch_plan_rejects_bad_values():
    with pytest.raises(SystemExit):
        bench.launch_plan(0, {})
    with pytest.raises(SystemExit):
        bench.launch_plan(2, {"WORLD_SIZE": "two"})


def test_spawn_command_forwards_arguments():
    argv = ["--gpus", "2", "--steps", "3", "--all-ranks-on-device", "0", "--comm", "torch"]
    cmd = bench.spawn_command(2, argv, 29512)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=2" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29512" in cmd
    i = cmd.index(os.path.join(ROOT, "bench.py"))
    assert cmd[i + 1:] == argv


def _run_bench(args, env_extra, timeout=240):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "TORCHELASTIC_RUN_ID"):
        env.pop(k, None)
    env.update(env_extra)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, cwd=ROOT,
                          capture_output=True, text=True, timeout=timeout)


def test_mismatch_exits_nonzero_before_any_gpu_call():
    r = _run_bench(["--gpus", "2", "--steps", "1"], {"WORLD_SIZE": "3"})
    assert r.returncode != 0
    assert "WORLD_SIZE=3 but --gpus 2" in r.stderr
    assert r.stdout.strip() == ""  # no JSON line


def test_gpus_2_launches_two_ranks():
    """No GPU here: the two spawned ranks fail at their first device call, and
    that failure must come back as the parent's exit status (never a silent
    1-rank line)."""
    import torch
    if torch.cuda.device_count() > 0:
        pytest.skip("a GPU is present: this checks the launcher without one")
    r = _run_bench(["--gpus", "2", "--steps", "1", "--warmup", "0", "--no-wide", "--no-forward",
                    "--no-cpu-baseline"], {})
    assert "[bench] launching 2 ranks" in r.stderr
    assert "--nproc-per-node=2" in r.stderr
    assert r.returncode != 0
    # a rank reported its own failure (bench.main's rank-tagged exit record,
    # whatever the device error's wording), and torch.distributed.run's
    # failure report names both ranks: the first to fail, and the other one,
    # failed or stopped by the launcher (no rank is left running)
    assert "[bench rank 0/2] failed" in r.stderr or "[bench rank 1/2] failed" in r.stderr
    import re
    assert set(re.findall(r"rank\s*:\s*(\d) \(local_rank", r.stderr)) == {"0", "1"}
    assert '"n_gpus": 1' not in r.stdout
