"""CPU unit test of the run-time floor under the screened scan (csrc/floor.hpp): the host
logic that reads each screened batch's report from page-locked memory and decides which
batches run the exact scan. Compiled with g++ (no GPU, no HIP headers) and run on
synthetic reports: trip rule, backoff, probe batch, out-of-order completion, torn and
overwritten reports, a probe whose report never arrives (tests/cpp/floor_test.cpp)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_floor_logic(tmp_path):
    exe = tmp_path / "floor_test"
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-Wall", "-Werror", "-o", str(exe),
                           os.path.join(ROOT, "tests", "cpp", "floor_test.cpp")])
    r = subprocess.run([str(exe)], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=60)
    print(r.stdout)
    assert r.returncode == 0, r.stdout
    assert "all checks passed" in r.stdout
