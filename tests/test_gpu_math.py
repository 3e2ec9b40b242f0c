"""Elementary functions as the HIP kernels evaluate them vs the host glibc (the oracle's libm).

sin/cos/tan are restated from glibc (clrrt_glibc.hpp) and IEEE basic operations are correctly
rounded on both sides: those must agree bit for bit.  The remaining libm calls on the path go to
the GPU math library; their disagreement rates with glibc are measured and printed (they only feed
boolean gates or float keys) and bounded here.
"""
import ctypes as C
import math

import numpy as np
import pytest

import clrrt

pytestmark = pytest.mark.gpu

_libm = C.CDLL("libm.so.6")
for _n in ("cosf", "sinf", "acosf", "asinf", "sqrtf"):
    getattr(_libm, _n).restype = C.c_float
    getattr(_libm, _n).argtypes = [C.c_float]
_libm.sincos.restype = None
_libm.sincos.argtypes = [C.c_double, C.POINTER(C.c_double), C.POINTER(C.c_double)]


def _sincos(a, k):
    s, c = C.c_double(), C.c_double()
    _libm.sincos(a, C.byref(s), C.byref(c))
    return (s.value, c.value)[k]


_libm.round.restype = C.c_double
_libm.round.argtypes = [C.c_double]
_libm.atan2f.restype = C.c_float
_libm.atan2f.argtypes = [C.c_float, C.c_float]


def _f32(x):
    return float(np.float32(x))


HOST = {
    0: lambda a, b: math.sin(a), 1: lambda a, b: math.cos(a), 2: lambda a, b: math.tan(a),
    3: lambda a, b: math.sqrt(a), 4: lambda a, b: math.fmod(a, b), 5: lambda a, b: math.atan2(a, b),
    6: lambda a, b: math.exp(a), 7: lambda a, b: a / b,
    8: lambda a, b: float(_libm.cosf(_f32(a))), 9: lambda a, b: float(_libm.sinf(_f32(a))),
    10: lambda a, b: float(_libm.atan2f(_f32(a), _f32(b))), 11: lambda a, b: float(_libm.acosf(_f32(a))),
    12: lambda a, b: float(_libm.asinf(_f32(a))), 13: lambda a, b: float(_libm.sqrtf(_f32(a))),
    14: lambda a, b: float(np.float32(_f32(a)) / np.float32(_f32(b))), 15: lambda a, b: float(_libm.round(a)),
    16: lambda a, b: _sincos(a, 0), 17: lambda a, b: _sincos(a, 1),
    # the rollout step's case-selected forms (glibc::sincos_sel, glibc::sin_cos_fma_sel)
    20: lambda a, b: _sincos(a, 0), 21: lambda a, b: _sincos(a, 1),
    22: lambda a, b: math.sin(a), 23: lambda a, b: math.cos(a),
    # the rollout step's branch-free block (glibc::step_trig: x2 = a, x3 = b)
    24: lambda a, b: _sincos(a, 0), 25: lambda a, b: _sincos(a, 1), 26: lambda a, b: math.sin(a),
    27: lambda a, b: math.cos(a), 28: lambda a, b: math.tan(b),
}
NAMES = ["sin", "cos", "tan", "sqrt", "fmod", "atan2", "exp", "div", "cosf", "sinf", "atan2f", "acosf",
         "asinf", "sqrtf", "fdiv", "round", "sincos.sin", "sincos.cos", None, None, "sincos_sel.sin",
         "sincos_sel.cos", "sin_cos_fma_sel.sin", "sin_cos_fma_sel.cos", "step_trig.s2", "step_trig.c2",
         "step_trig.swp", "step_trig.cwp", "step_trig.t3"]
FNS = [f for f in range(29) if f not in (18, 19)]  # 18, 19: latency diagnostics
EXACT = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 20, 21, 22, 23, 24, 25, 26, 27, 28}


def _inputs(fn, n, rng):
    if fn in (0, 1, 8, 9, 16, 17, 20, 21, 22, 23, 24, 25, 26, 27, 28):
        a = rng.uniform(-7, 7, n)
        a[: n // 8] = rng.uniform(-1e-8, 1e-8, n // 8)  # the tiny-argument cases
        a[n // 8: n // 4] = rng.uniform(-3e4, 3e4, n // 8)
    elif fn == 2:
        a = rng.uniform(-0.52, 0.52, n)
    elif fn in (3, 13):
        a = rng.uniform(0, 5000, n)
    elif fn == 6:
        a = rng.uniform(-750, 10, n)
        a[: n // 4] = rng.uniform(-260, 0, n // 4)  # -W3 Dobs
    elif fn in (11, 12):
        a = rng.uniform(-1, 1, n)
    elif fn == 15:
        a = rng.uniform(-500, 500, n)
    else:
        a = rng.uniform(-60, 60, n)
    b = rng.uniform(-60, 60, n)
    if fn >= 24:  # x3: steering angles (|x3| <= 0.52), tiny ones, tan's polynomial range, up to its table's end
        b = rng.uniform(-0.6, 0.6, n)
        b[: n // 8] = rng.uniform(-1e-9, 1e-9, n // 8)
        b[n // 8: n // 4] = rng.uniform(-0.07, 0.07, n // 8)
        b[n // 4: n // 4 + n // 16] = rng.uniform(-0.787, 0.787, n // 16)
    if fn == 4:
        b = np.full(n, 2 * math.pi)
    return a, b


def test_device_math_vs_glibc():
    pl = clrrt.Planner(clrrt.default_params(), max_nodes=4, max_rows=4, max_batch=1)
    rng = np.random.default_rng(5)
    n = 20000
    report = {}
    for fn in FNS:
        a, b = _inputs(fn, n, rng)
        g = pl.selftest_math(fn, a, b)
        h = np.array([HOST[fn](x, y) for x, y in zip(a, b)])
        mism = int(np.sum(g.view(np.uint64) != h.view(np.uint64)))
        report[NAMES[fn]] = mism / n
    print("device-vs-glibc mismatch rate:", {k: f"{v:.4%}" for k, v in report.items()})
    for fn in EXACT:
        assert report[NAMES[fn]] == 0.0, NAMES[fn]
    for k, v in report.items():
        assert v < 0.5, k
