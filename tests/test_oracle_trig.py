"""The descriptor steering's cos / sin (ORBextractor.cc:109-110) against glibc, on the CPU.

ORBextractor.cc:66 `using namespace std;` makes `cos(angle)` with a float angle std::cos(float),
i.e. glibc cosf / sinf, which are not correctly rounded. The oracle calls them directly; the GPU
runs a port of glibc's algorithm (steer_cos_sin in orbfe_extract.hip). Here the oracle's own
restatement of that algorithm (oracle/trig_check.cpp) is checked against glibc on EVERY float
degree value in [0, 360) -- a superset of fastAtan2's outputs, ~1.1e9 values; the GPU port gets
the same exhaustive check in test_gpu_trig.py.
"""
import os

from oracle import orbref


def test_glibc_sincosf_restatement_exhaustive():
    bad, first = orbref.trig_mismatch(threads=min(8, os.cpu_count() or 1))
    assert bad == 0, f"{bad} steering angles differ from glibc cosf/sinf; first degree bits {first:#010x}"
