"""Runs the C++ host-mirror behaviour tests (stl.fusion_amd/host/test_fusion.cpp) on the GPU.

The binary links the in-tree engine (stl.fusion_amd/lib/libfgi.so) through the host mirror
(host/build/libfusion.so); both are built by __graft_entry__.build() / `make -C stl.fusion_amd/host`.
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST = os.path.join(ROOT, "stl.fusion_amd", "host")
BIN = os.path.join(HOST, "build", "test_fusion")


def test_host_mirror_builds_and_links():
    """CPU: the mirror compiles against include/fgi.h and links libfgi.so (no GPU call)."""
    subprocess.run(["make", "-s", "-C", HOST], check=True, timeout=300)
    assert os.path.exists(BIN)
    out = subprocess.run(["ldd", BIN], capture_output=True, text=True, check=True).stdout
    assert "libfgi.so" in out and "libfusion.so" in out and "not found" not in out


@pytest.mark.gpu
def test_host_mirror_scenarios(gpu_available):
    subprocess.run(["make", "-s", "-C", HOST], check=True, timeout=300)
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "checks passed" in r.stdout
