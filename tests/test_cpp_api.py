"""The C++ API harness (tests/cpp/test_api.cpp): the reference's gtest suites restated against the
drop-in C++ headers, run as a child process (ordered before anything initialises the GPU here)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CPP = os.path.join(ROOT, "tests", "cpp")
BIN = os.path.join(CPP, "build", "test_api")


def _build():
    subprocess.run(["make", "-C", CPP, "-j4"], check=True, capture_output=True, text=True)
    return BIN


def test_cpp_harness_builds():
    """CPU-side: the C++ API compiles with g++ alone against include/ and links the libraries."""
    assert os.path.exists(_build())


@pytest.mark.gpu
@pytest.mark.subprocess
def test_cpp_api_suite():
    exe = _build()
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600)
    print(r.stdout[-4000:])
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert " 0 failed" in r.stdout


def test_cpu_simulator_suite():
    """CPU-only: the product qsim::CPUSimulator (libqsim.so) against the test oracle, thread
    invariance, sampling, errors and the cuda_config alias (tests/cpp/test_cpu_api.cpp)."""
    _build()
    exe = os.path.join(CPP, "build", "test_cpu_api")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert " 0 failed" in r.stdout
