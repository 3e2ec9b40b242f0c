"""The std::sort replay used by EXACT mode (cl-rrt_amd/csrc/clrrt_stdsort.hpp) against the real
libstdc++ std::sort / heap algorithms on tie-heavy (id, key) sequences.  CPU only."""
import os
import subprocess
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))


def test_stdsort_replay_matches_libstdcxx():
    with tempfile.TemporaryDirectory() as td:
        exe = os.path.join(td, "stdsort_check")
        subprocess.run(["g++", "-O2", "-std=c++17", "-o", exe, os.path.join(HERE, "native", "stdsort_check.cpp")],
                       check=True)
        out = subprocess.run([exe], capture_output=True, text=True)
        assert out.returncode == 0, out.stdout + out.stderr
        assert "mismatching 0" in out.stdout


def test_wave_partition_argument_matches_replay():
    """wave_std_sort's parallel partition (both scans' stops paired, swaps after the crossing) gives the
    sequential replay's permutation (tests/native/wave_sort_check.cpp)."""
    with tempfile.TemporaryDirectory() as td:
        exe = os.path.join(td, "wave_sort_check")
        subprocess.run(["g++", "-O2", "-std=c++17", "-o", exe, os.path.join(HERE, "native", "wave_sort_check.cpp")],
                       check=True)
        out = subprocess.run([exe], capture_output=True, text=True)
        assert out.returncode == 0, out.stdout + out.stderr
        assert "mismatches 0" in out.stdout
