"""Builds and runs the C++ go/fec mirror test (tests/cpp/test_fec_api.cpp) against librqhip.so."""
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
PKG = ROOT / "rl-quic-raptor_amd"


@pytest.fixture(scope="module")
def cpp_bin(tmp_path_factory):
    out = tmp_path_factory.mktemp("cpp") / "test_fec_api"
    subprocess.run(["g++", "-O1", "-std=c++17", "-I", str(PKG / "csrc"), str(ROOT / "tests/cpp/test_fec_api.cpp"),
                    "-L", str(PKG / "build"), "-lrqhip", "-Wl,-rpath," + str(PKG / "build"), "-o", str(out)],
                   check=True)
    return out


def test_cpp_mirror_cpu(cpp_bin):
    r = subprocess.run([str(cpp_bin), "cpu"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "cpu ok" in r.stdout


@pytest.mark.gpu
def test_cpp_mirror_gpu(cpp_bin):
    r = subprocess.run([str(cpp_bin), "gpu"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "gpu ok" in r.stdout
