"""A plain C client of include/gossip.h (tests/c/abi_test.c, gcc -std=c99):
the header compiles as C, the library links, and the error paths hold.  On
the GPU the same program runs a broadcast end to end (one device, and one and
two shards through gs_create_multi)."""
from __future__ import annotations

import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "gossip_simulator_amd")


def build(tmp_path):
    exe = str(tmp_path / "abi_test")
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-O1", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "c", "abi_test.c"), "-o", exe, "-L", PKG, "-lgossip_hip",
                    f"-Wl,-rpath,{PKG}", "-Wl,-rpath,/opt/rocm/lib"], check=True)
    return exe


def test_c_client_builds_and_error_paths(tmp_path):
    exe = build(tmp_path)
    env = dict(os.environ, HIP_VISIBLE_DEVICES="-1") if not os.path.exists("/dev/kfd") else dict(os.environ)
    if os.path.exists("/dev/kfd"):
        pytest.skip("a GPU is visible: the gpu variant covers this host")
    r = subprocess.run([exe, "cpu"], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0, r.stderr


@pytest.mark.gpu
def test_c_client_end_to_end_on_gpu(tmp_path):
    exe = build(tmp_path)
    r = subprocess.run([exe, "gpu"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "abi_test gpu: ok" in r.stdout
