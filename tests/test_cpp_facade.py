"""The C++ facade (include/orbfe.hpp) as a reference-side adapter would use it: two extractor
instances on two threads (Frame.cc:113-116), pyramid level views, ComputeStereoMatches over the
two extractors, DescriptorDistance -- checked
against the oracle's C API inside the C++ program (tests/cpp/extract_parity.cpp)."""
import os
import subprocess

import pytest

from conftest import gpu_available

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CPP = os.path.join(ROOT, "tests", "cpp")


def _build():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    subprocess.run(["make", "-s", "-C", CPP], check=True)
    return os.path.join(CPP, "build", "extract_parity")


@pytest.mark.skipif(gpu_available(), reason="checks the no-device path")
def test_cpp_facade_builds_and_fails_loudly_without_gpu():
    exe = _build()
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert out.returncode == 77, out.stdout + out.stderr
    assert "no HIP device" in out.stdout


@pytest.mark.gpu
def test_cpp_facade_parity(require_gpu):
    exe = _build()
    out = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    lines = out.stdout.strip().splitlines()
    assert lines[-1].startswith("OK"), out.stdout
    assert any(l.startswith("stereo: ") for l in lines), out.stdout
