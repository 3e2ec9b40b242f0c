"""The restatement of glibc's double sin/cos/tan used by the HIP rollouts
(cl-rrt_amd/csrc/clrrt_glibc.hpp) against the host libm, bit for bit.  CPU only."""
import os
import subprocess
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))


def test_glibc_sin_cos_tan_bit_exact():
    with tempfile.TemporaryDirectory() as td:
        exe = os.path.join(td, "glibc_check")
        subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-o", exe,
                        os.path.join(HERE, "native", "glibc_check.cpp")], check=True)
        out = subprocess.run([exe, "1000000"], capture_output=True, text=True)
        assert out.returncode == 0, out.stdout + out.stderr
        assert "sin mismatches 0, cos mismatches 0" in out.stdout and "mismatches 0" in out.stdout


def test_glibc_data_header_is_current():
    """tools/gen_glibc_libm.py validates the libm image (hash) and regenerates the same header."""
    root = os.path.dirname(HERE)
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "h.hpp")
        subprocess.run(["python3", os.path.join(root, "tools", "gen_glibc_libm.py"), "--out", out], check=True,
                       capture_output=True)
        assert open(out).read() == open(os.path.join(root, "cl-rrt_amd", "csrc", "clrrt_glibc_data.hpp")).read()
