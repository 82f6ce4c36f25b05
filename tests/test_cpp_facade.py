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


# The matcher half of the drop-in (adapter/ORBmatcher_gpu.cc) compiled over the cvstub Frame /
# KeyFrame / MapPoint / ORBmatcher declarations and run as Tracking, LocalMapping and LoopClosing
# call it (tests/cpp/matcher_e2e.cpp): the motion model's SearchByProjection(F, LastFrame) with th 7
# and the 2*th retry (taken and not taken) and th 15 mono, SearchLocalPoints' SearchByProjection(F,
# vpLocalMapPoints) at th 1 / 5, SearchForTriangulation against the previous and the next KeyFrame
# (bOnlyStereo off / on), relocalisation's SearchByBoW(KF, F) + SearchByProjection(F, KF, sFound,
# 10, 100), and ComputeSim3's SearchByProjection(KF, Scw, ...); every applied mvpMapPoints /
# vpMapPointMatches / vpMatched / vMatchedPairs entry against the oracle.
def _matcher_e2e(*args, timeout=300):
    _build()
    return subprocess.run([os.path.join(CPP, "build", "matcher_e2e"), *args], capture_output=True, text=True,
                          timeout=timeout)


def _matcher_record(out) -> dict:
    import json
    lines = out.stdout.strip().splitlines()
    assert lines[-1] == "OK", out.stdout + out.stderr
    rec = [l for l in lines if l.startswith("MATCHER ")]
    assert rec, out.stdout
    return json.loads(rec[-1][len("MATCHER "):])


def _check_scenarios(r: dict):
    assert r["motion_stereo_retry"]["retried"] and not r["motion_stereo_th7"]["retried"]
    for k in ("motion_stereo_th7", "motion_mono_th15", "local_th1", "local_th5", "triangulation_kf0",
              "triangulation_kf2", "triangulation_kf2_only_stereo", "bow", "reloc_projection", "sim3_projection"):
        assert (r[k].get("nmatches") or r[k].get("pairs")) > 0, (k, r[k])


def test_matcher_e2e_scene_on_cpu():
    """--dry: the scene and the oracle side only (no device): every scenario is non-trivial and the
    retry case takes Tracking's 2*th retry."""
    out = _matcher_e2e("--dry")
    assert out.returncode == 0, out.stdout + out.stderr
    _check_scenarios(_matcher_record(out))


@pytest.mark.skipif(gpu_available(), reason="checks the no-device path")
def test_matcher_e2e_fails_loudly_without_gpu():
    out = _matcher_e2e()
    assert out.returncode == 77, out.stdout + out.stderr
    assert "no HIP device" in out.stdout


@pytest.mark.gpu
def test_matcher_adapter_e2e_parity(require_gpu):
    out = _matcher_e2e()
    assert out.returncode == 0, out.stdout + out.stderr
    r = _matcher_record(out)
    _check_scenarios(r)
    print(r)


# adapter/ORBmatcher_gpu.cc's packers under ThreadSanitizer (tests/cpp/matcher_tsan.cpp, CPU): the
# keyframe searches that read mfMinDistance / mfMaxDistance on Tracking / LoopClosing / LocalMapping
# threads while a writer runs UpdateNormalAndDepth + SetWorldPos on the same MapPoints (the writes
# MapPoint.cc:396-398 makes under mMutexPos). Clean as shipped; the --control run adds an unlocked
# reader of the same members, which the sanitizer must report.
def _tsan(*args):
    _build()
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=0 exitcode=66")
    return subprocess.run([os.path.join(CPP, "build", "matcher_tsan"), *args], capture_output=True, text=True,
                          timeout=300, env=env)


def test_matcher_adapter_packers_race_free_under_tsan():
    out = _tsan()
    assert out.returncode == 0 and "ThreadSanitizer" not in out.stderr, out.stdout + out.stderr
    assert out.stdout.startswith("OK"), out.stdout


def test_matcher_tsan_control_reports_unlocked_reader():
    out = _tsan("--control")
    assert out.returncode == 66, out.stdout + out.stderr
    assert "WARNING: ThreadSanitizer: data race" in out.stderr and "unlocked_min" in out.stderr
