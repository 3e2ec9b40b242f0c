"""The C++ drop-in layer (include/clrrt_adapter.hpp) linked against libclrrt without Python: the native
program tests/native/capi_exact.cpp (built by cl-rrt_amd/csrc/Makefile) grows the 200-obstacle tree
through Engine::expandTree / expandBudget (expandTree rrtplanner.cpp:123-174) and must reproduce the
oracle's tree, counters and checkObsDistance values in tests/golden/capi_exact_obb200_s3.bin."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "native", "capi_exact")
FIX = os.path.join(ROOT, "tests", "golden", "capi_exact_obb200_s3.bin")


def test_native_adapter_compiles_against_the_header():
    """CPU: the adapter and the test program compile (host C++ only; no GPU call)."""
    subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-Wall", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "native", "capi_exact.cpp")], check=True)


@pytest.mark.gpu
def test_native_capi_exact_matches_oracle():
    assert os.path.exists(EXE), "tests/native/capi_exact not built (make -C cl-rrt_amd/csrc)"
    out = subprocess.run([EXE, FIX], capture_output=True, text=True, timeout=120)
    print(out.stdout)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "failures 0" in out.stdout
