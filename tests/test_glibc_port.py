"""The restatements of glibc's double sin/cos/tan/atan2 and float trig used by the HIP kernels
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


def test_glibc_sincosf_bit_exact():
    """clrrt::glibc::sincosf / sinf (OBB::setVertices and dubinsDistance's float cos/sin) against the host
    libm's sincosf, sinf and cosf on every 7th float bit pattern (pass 1 for all 2^32: 0 mismatches)."""
    with tempfile.TemporaryDirectory() as td:
        exe = os.path.join(td, "sincosf_check")
        subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fopenmp", "-o", exe,
                        os.path.join(HERE, "native", "sincosf_check.cpp")], check=True)
        out = subprocess.run([exe, "7"], capture_output=True, text=True)
        assert out.returncode == 0, out.stdout + out.stderr
        assert "mismatches 0" in out.stdout


def test_glibc_float_inverse_trig_bit_exact():
    """clrrt::glibcf::atanf / acosf / asinf / atan2f (dubinsDistance's float libm calls) against the host
    libm on every 7th float and 2*10^6 random/edge pairs (pass 1 and 10^8 pairs: 0 mismatches)."""
    with tempfile.TemporaryDirectory() as td:
        exe = os.path.join(td, "glibcf_check")
        subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fopenmp", "-o", exe,
                        os.path.join(HERE, "native", "glibcf_check.cpp")], check=True)
        out = subprocess.run([exe, "7", "2000000"], capture_output=True, text=True)
        assert out.returncode == 0, out.stdout + out.stderr
        assert "atanf mismatches 0, acosf mismatches 0, asinf mismatches 0" in out.stdout
        assert "atan2f mismatches 0" in out.stdout


def test_glibc_atan2_bit_exact():
    """clrrt::glibc::atan2 (feasibleNode's angles, feasibleGoalBias' angleRef, the node records' angPar)
    against the host libm's atan2 (FMA variant) on special values and 4*10^6 random pairs over 600 decades
    of magnitude, incl. angles within 1e-12 of pi/4 (4*10^7 pairs: 0 mismatches)."""
    with tempfile.TemporaryDirectory() as td:
        exe = os.path.join(td, "atan2_check")
        subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-o", exe,
                        os.path.join(HERE, "native", "atan2_check.cpp")], check=True)
        out = subprocess.run([exe, "4000000"], capture_output=True, text=True)
        assert out.returncode == 0, out.stdout + out.stderr
        assert "mismatches 0" in out.stdout


def test_glibc_exp_bit_exact():
    """clrrt::glibc::exp (the W2 obstacle-cost term Wcost[2] exp(-Wcost[3] Dobs), simulation.cpp:91) against
    the host libm's exp (its FMA variant) on special values and 4*10^6 arguments incl. the subnormal range
    (4*10^7: 0 mismatches)."""
    with tempfile.TemporaryDirectory() as td:
        exe = os.path.join(td, "exp_check")
        subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-o", exe,
                        os.path.join(HERE, "native", "exp_check.cpp")], check=True)
        out = subprocess.run([exe, "4000000"], capture_output=True, text=True)
        assert out.returncode == 0, out.stdout + out.stderr
        assert "exp mismatches 0" in out.stdout
