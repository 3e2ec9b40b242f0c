"""CPU check of the nearest-node prefilter's Dubins lower bound (cl-rrt_amd/csrc/clrrt_dubins_lb.hpp):
never above the float Dubins key (dubinsDistance, rrtplanner.cpp:371-406, restated with glibc's float
functions) on random node-frame points, including points at the turning-circle boundary."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_dubins_lower_bound_is_valid(tmp_path):
    exe = tmp_path / "dlb"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-o", str(exe),
                    os.path.join(ROOT, "tests", "native", "dubins_lb_check.cpp")], check=True)
    r = subprocess.run([str(exe), "1000000"], capture_output=True, text=True)
    print(r.stdout)
    assert r.returncode == 0, r.stdout
