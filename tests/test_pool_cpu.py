"""The context allocator's splitting pool (combblas_amd/csrc/pool.h) under random traffic, on
the CPU: tests/native/pool_check.cpp builds with g++ and checks after every step that the blocks
tile each segment, free neighbours are merged (never across adjacent segments), no two live
blocks overlap, and returning everything leaves each segment one free block."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def pool_check(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("pool") / "pool_check")
    subprocess.run(["g++", "-O1", "-std=c++17", "-g", "-fsanitize=address,undefined", "-o", exe,
                    os.path.join(ROOT, "tests", "native", "pool_check.cpp")], check=True)
    return exe


@pytest.mark.parametrize("seed", [1, 2, 3, 7])
def test_pool_random_traffic(pool_check, seed):
    r = subprocess.run([pool_check, str(seed), "20000"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ok" in r.stdout and "served from the pool" in r.stdout, r.stdout
