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


# The drop-in adapters themselves (adapter/ORBextractor_gpu.cc + adapter/Frame_gpu.cc) compiled over
# the test-only OpenCV / reference declarations of tests/cpp/cvstub and run as the reference's
# stereo Frame constructor runs them (Frame.cc:113-125), frame after frame: operator()'s keypoints
# and descriptors, both extractors' mvImagePyramid (ORBextractor.h:100) held at once, the CPU
# ComputeStereoMatches over those levels and Frame_gpu.cc's GPU ComputeStereoMatches, all against
# the oracle (tests/cpp/adapter_e2e.cpp). Two builds: host pyramid (default) and
# ORBFE_ADAPTER_GPU_STEREO=1 (mvImagePyramid left empty, no pyramid copy).
E2E = ("adapter_e2e", "adapter_e2e_gpustereo")


@pytest.mark.skipif(gpu_available(), reason="checks the no-device path")
def test_adapter_e2e_builds_and_fails_loudly_without_gpu():
    _build()
    for name in E2E:
        out = subprocess.run([os.path.join(CPP, "build", name)], capture_output=True, text=True, timeout=120)
        assert out.returncode == 77, out.stdout + out.stderr
        assert "no HIP device" in out.stdout


def run_adapter_e2e(name: str, iters: int = 50) -> dict:
    import json
    out = subprocess.run([os.path.join(CPP, "build", name), str(iters)], capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    lines = out.stdout.strip().splitlines()
    assert lines[-1].startswith("OK"), out.stdout
    rec = [l for l in lines if l.startswith("ADAPTER ")]
    assert rec, out.stdout
    return json.loads(rec[-1][len("ADAPTER "):])


@pytest.mark.gpu
@pytest.mark.parametrize("name", E2E)
def test_adapter_e2e_parity(require_gpu, name):
    _build()
    r = run_adapter_e2e(name, iters=10)
    assert r["gpu_stereo_build"] == (1 if name.endswith("gpustereo") else 0)
    assert r["stereo_matched_3_frames"] > 0
    print(name, r)
