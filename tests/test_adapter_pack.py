"""The reference-side adapter (adapter/): every ORBmatcher method template of orbfe_adapter.hpp
instantiated on ORB-SLAM2-shaped test structs with a recording matcher -- each SoA field the GPU
would receive against the objects, and the reference's application of the results (ascending
order, the rotation filter's undo codes, Fuse's replace / add, vbPrevMatched in place). Built with
ASan + UBSan; CPU only (tests/cpp/adapter_pack_test.cpp)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CPP = os.path.join(ROOT, "tests", "cpp")


def test_adapter_packers_and_appliers():
    subprocess.run(["make", "-s", "-C", CPP, "build/adapter_pack_test"], check=True)
    out = subprocess.run([os.path.join(CPP, "build", "adapter_pack_test")], capture_output=True, text=True,
                         timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.strip().endswith("OK adapter packers and appliers"), out.stdout


def test_adapter_sources_are_guarded():
    """The OpenCV-typed adapter files compile only inside the reference's tree: each is guarded by
    __has_include(<opencv2/core.hpp>) and the reference header it implements, so here (no OpenCV)
    they preprocess to nothing and still compile."""
    for name, hdr in (("ORBextractor_gpu.cc", "ORBextractor.h"), ("ORBmatcher_gpu.cc", "ORBmatcher.h"),
                      ("Frame_gpu.cc", "Frame.h")):
        path = os.path.join(ROOT, "adapter", name)
        text = open(path).read()
        assert f'#if __has_include(<opencv2/core.hpp>) && __has_include("{hdr}")' in text, name
        subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-I", os.path.join(ROOT, "include"),
                        "-I", os.path.join(ROOT, "adapter"), path], check=True)
