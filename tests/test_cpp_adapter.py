"""The C++ host adapter (zkevm-prover_amd/host/zkgpu_goldilocks.hpp) used the
way src/starkpil calls the Goldilocks library, checked against the oracle."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "build", "adapter_check")


def build_adapter_check():
    os.makedirs(os.path.join(ROOT, "build"), exist_ok=True)
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    subprocess.check_call([
        "g++", "-O2", "-std=c++17", "-o", BIN, os.path.join(ROOT, "tests/cpp/adapter_check.cpp"),
        "-L" + os.path.join(ROOT, "zkevm-prover_amd/lib"), "-lzkgpu",
        "-L" + os.path.join(ROOT, "oracle/build"), "-loracle",
        "-Wl,-rpath,$ORIGIN/../zkevm-prover_amd/lib", "-Wl,-rpath,$ORIGIN/../oracle/build"])
    return BIN


def test_adapter_compiles():
    import zkgpu
    if not os.path.exists(zkgpu.LIB_PATH):
        zkgpu.build()
    assert os.path.exists(build_adapter_check())


@pytest.mark.gpu
def test_adapter_runs_bit_exact():
    if not os.path.exists(BIN):
        build_adapter_check()
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=300)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ALL OK" in r.stdout
