"""The C++ drop-in surface (vdb::IVFFlatIndex, vdb::TransferManager) driven by test
programs that mirror the reference's own tests (tests/cpp/simple_test.cpp <-
test/simple_test.cpp, tests/cpp/gpu_vs_cpu_test.cpp <- test/gpu_vs_cpu_test.cpp with
its ctest arguments 10000 100 64 32), each cross-checked bit for bit with the oracle."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
CPP = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cpp")


@pytest.fixture(scope="module")
def binaries():
    subprocess.check_call(["make", "-s", "-C", CPP])
    return os.path.join(CPP, "bin")


def test_simple_test_program(binaries):
    p = subprocess.run([os.path.join(binaries, "simple_test")], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "bit-identical to CPU path: yes" in p.stdout


def test_gpu_vs_cpu_program_ctest_args(binaries):
    p = subprocess.run([os.path.join(binaries, "gpu_vs_cpu_test"), "10000", "100", "64", "32"], capture_output=True,
                       text=True, timeout=600)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "results differing from the CPU path: 0" in p.stdout


def test_gpu_vs_cpu_program_on_a_group_handle(binaries):
    # the same program with Config::devices = {0, 0}: one index sharded over two members
    # (here sharing the one GPU), results still bit-identical to the CPU path
    env = dict(os.environ, VDB_TEST_DEVICES="0,0")
    p = subprocess.run([os.path.join(binaries, "gpu_vs_cpu_test"), "10000", "100", "64", "32"], capture_output=True,
                       text=True, timeout=600, env=env)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "sharded over 2 device(s)" in p.stdout
    assert "results differing from the CPU path: 0" in p.stdout
