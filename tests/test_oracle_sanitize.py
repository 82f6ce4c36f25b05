"""The oracle under AddressSanitizer + UndefinedBehaviorSanitizer: `make -C oracle
sanitize` builds oracle/sanitize_main.cpp with every oracle source and the synthetic-frame
generator (-fsanitize=address,undefined, no recovery) and the driver walks extraction (4 shapes x
2 resize modes, flat and small images), ComputeStereoMatches, the vocabulary transform,
SearchForTriangulation and SearchByProjection. Any report aborts the driver. CPU only."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_oracle_clean_under_asan_ubsan():
    b = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "sanitize"], capture_output=True,
                       text=True, timeout=600)
    if b.returncode != 0 and "asan" in (b.stderr + b.stdout).lower():
        pytest.skip("compiler without the sanitizer runtimes")
    assert b.returncode == 0, b.stderr
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([os.path.join(ROOT, "oracle", "build", "orbref_sanitize")], capture_output=True,
                       text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert r.stdout.strip().endswith("OK")
