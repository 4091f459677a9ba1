"""The C++ cnn_sr:: host API (cnn-super-resolution_amd/host) through its spec
runner, which mirrors the reference's test/specs/*.cpp on the golden vectors.

CPU: the specs that need no device (Config / JSON / parameters I/O / image
codec).  GPU: every spec, through DataPipeline / ConfigBasedDataPipeline on
libsrcnn_hip.so (including fused-vs-op-level training agreement).
"""
import os
import subprocess

import pytest

from conftest import GOLDEN, ROOT

BIN = os.path.join(ROOT, "cnn-super-resolution_amd", "bin", "pipeline_specs")


def run_specs(*args, timeout=600):
    assert os.path.exists(BIN), "build with `make -C cnn-super-resolution_amd` first"
    p = subprocess.run([BIN, "--golden", GOLDEN, *args], capture_output=True, text=True,
                       timeout=timeout)
    print(p.stdout[-6000:], p.stderr[-2000:])
    return p


def test_host_specs_cpu():
    p = run_specs("--cpu-only")
    assert p.returncode == 0, p.stdout
    assert "7 of 7 specs passed" in p.stdout


def test_host_library_links_only_the_c_abi():
    """libcnn_sr.so reaches the GPU only through libsrcnn_hip.so's C ABI."""
    lib = os.path.join(ROOT, "cnn-super-resolution_amd", "lib", "libcnn_sr.so")
    out = subprocess.run(["nm", "-D", "--undefined-only", lib], capture_output=True, text=True).stdout
    hip = [l.split()[-1] for l in out.splitlines() if l.split()[-1].startswith("hip")]
    assert not hip, hip
    assert "srcnn_train_fwd_bwd" in out and "srcnn_conv_fwd" in out


@pytest.mark.gpu
def test_host_specs_gpu():
    p = run_specs(timeout=900)
    assert p.returncode == 0, p.stdout
    assert "FAIL" not in p.stdout
