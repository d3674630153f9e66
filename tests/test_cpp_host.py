"""The C++ host mirror (include/hbrbc.hpp, include/hbrbc_broadcast.hpp): the
reference's Rust API restated in C++ over the C ABI, exercised by
tests/cpp/test_host.cpp the way the reference's own tests exercise it
(merkle.rs test_merkle, the broadcast doc-test, test_broadcast_different_sizes
schedules, rse error outcomes, the golden N=4 "Foo" root)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "test_host")


def _binary():
    if not os.path.exists(BIN):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "tests", "cpp")])
    return BIN


def test_cpp_host_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    r = subprocess.run([_binary()], capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "HbrbcUnavailable" in r.stderr   # no CPU fallback


@pytest.mark.gpu
def test_cpp_host_mirror_on_gpu():
    r = subprocess.run([_binary()], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "all passed" in r.stdout
