"""liborbfe.so without a GPU: it loads, exports every symbol include/*.h declares, its host-only
helpers work, and compute entry points fail loudly (no CPU fallback) when no device is present."""
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import gpu_available

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = ["orbfe.h", "orbfe_match_batch.h", "orbfe_debug.h", "orbfe_synth.h", "orbfe_vocab.h", "orbfe_frustum.h",
           "orbfe_stereo.h", "orbfe_keyframe.h", "orbfe_pack.h"]


def declared_functions():
    names = set()
    for h in HEADERS:
        src = open(os.path.join(ROOT, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names |= set(re.findall(r"\b(orbfe_\w+)\s*\(", src))
    return names


def test_library_exports_every_declared_symbol():
    from orb_slam2_2021_amd import _lib as L
    lib = L.lib()
    out = subprocess.run(["nm", "-D", "--defined-only", L.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\bT (orbfe_\w+)", out))
    missing = declared_functions() - exported
    assert not missing, f"declared but not exported: {sorted(missing)}"
    for name in declared_functions():
        getattr(lib, name)
    assert set(L.EXPORTED) <= exported


def test_library_carries_gfx950_code():
    from orb_slam2_2021_amd import _lib as L
    blob = open(L.LIB_PATH, "rb").read()
    assert b"gfx950" in blob
    assert b"k_octree" in blob and b"k_sft_nodes" in blob


def test_synthetic_frames_are_deterministic():
    from orb_slam2_2021_amd import synth_frame
    a, ar = synth_frame(7, 376, 1241, right=True)
    b = synth_frame(7, 376, 1241)
    assert np.array_equal(a, b)
    assert not np.array_equal(a, ar)
    assert not np.array_equal(a, synth_frame(8, 376, 1241))
    assert 100 < a.mean() < 140 and a.std() > 40


def test_host_descriptor_distance():
    from orb_slam2_2021_amd import ORBmatcher
    from oracle import orbref
    rng = np.random.default_rng(4)
    for _ in range(50):
        a, b = rng.integers(0, 256, (2, 32), dtype=np.uint8)
        assert ORBmatcher.DescriptorDistance(a, b) == orbref.descriptor_distance(a, b)


@pytest.mark.skipif(gpu_available(), reason="checks the no-device error path")
def test_compute_without_device_fails_loudly():
    from orb_slam2_2021_amd import ORBextractor, ORBmatcher, OrbfeError
    with pytest.raises(OrbfeError):
        ORBextractor(2000, 1.2, 8, 20, 7)
    with pytest.raises(OrbfeError):
        ORBmatcher(0.6, True)


def test_missing_library_raises(tmp_path):
    code = ("import os, sys; os.environ['ORBFE_LIB'] = %r; sys.path.insert(0, %r)\n"
            "from orb_slam2_2021_amd import _lib\n"
            "try:\n    _lib.lib()\nexcept _lib.LibraryMissing:\n    print('raised')\n"
            % (str(tmp_path / "nope.so"), ROOT))
    out = subprocess.run(["python", "-c", code], capture_output=True, text=True, timeout=120)
    assert "raised" in out.stdout


def test_bad_arguments_rejected_without_device():
    from orb_slam2_2021_amd import _lib as L
    from ctypes import byref, c_void_p
    lib = L.lib()
    h = c_void_p()
    assert lib.orbfe_extractor_create(0, 1.2, 8, 20, 7, 0, byref(h)) == L.ORBFE_ERR_ARG
    assert lib.orbfe_extractor_create(2000, 1.0, 8, 20, 7, 0, byref(h)) == L.ORBFE_ERR_ARG
    assert lib.orbfe_extract(None, None, 10, 10, 10, None, 0, None, None) == L.ORBFE_ERR_ARG
    assert lib.orbfe_descriptor_distance(None, None) == L.ORBFE_ERR_ARG
    # k_pack sums counts in 32-bit halves: n_images * cap >= 2^31 is refused before any launch
    from ctypes import c_size_t, c_void_p
    one = c_void_p(16)
    assert lib.orbfe_pack_keypoints_device(1 << 16, one, one, one, 1 << 15, one, c_size_t(1 << 62), one,
                                           None) == L.ORBFE_ERR_ARG
    assert b"2^31" in lib.orbfe_last_error()
    # the one-call C3 plan (orbfe_c3.h) checks its configuration before touching a device
    cfg = L.c3_config(n_images=64, rows=376, cols=1241, cap=2048, n_vocab=32, levelsup=4, n_stereo=32)
    assert lib.orbfe_c3_create(byref(cfg), None, 0, None, 0, None, None, None, 0, byref(h)) == L.ORBFE_ERR_ARG
    assert lib.orbfe_c3_run(None, 0, 0, one, None, 0) == L.ORBFE_ERR_ARG
    assert lib.orbfe_c3_finish(None, 0, None) == L.ORBFE_ERR_ARG
    assert lib.orbfe_c3_destroy(None) == L.ORBFE_OK


def test_product_never_imports_the_oracle():
    """The oracle is test infrastructure: the package must not import or load it."""
    pkg = os.path.join(ROOT, "orb_slam2_2021_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith(".py"):
                src = open(os.path.join(dirpath, f)).read()
                assert "import oracle" not in src and "from oracle" not in src, f
                assert "orbref" not in src, f
    code = ("import sys; sys.path.insert(0, %r)\n"
            "import orb_slam2_2021_amd, orb_slam2_2021_amd.parallel, orb_slam2_2021_amd.synthetic\n"
            "print(sorted(m for m in sys.modules if m.startswith('oracle')))" % ROOT)
    out = subprocess.run(["python", "-c", code], capture_output=True, text=True, timeout=120)
    assert out.stdout.strip() == "[]", out.stdout + out.stderr
