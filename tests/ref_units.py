"""Hot-path unit cases pinned to the reference's OWN code — TEST INFRASTRUCTURE.

Three evaluators share one case format per unit (include/clrrt.h, CLRRT_UNIT_*):
  * `reference`: oracle/_ref/libref_units_O2.so (and _O0), compiled by `make -C oracle ref` from
    verbatim line ranges of /root/reference (only where /root/reference exists);
  * `oracle`: oracle/liboracle.so's unit hooks, i.e. the very functions the oracle's expandTree runs;
  * `device`: clrrt_selftest_units, i.e. the very device functions the rollout kernels run.
tests/golden/make_ref_units.py draws the cases, checks reference == oracle on 10^5 of each and writes
a subset with the reference's outputs to tests/golden/ref_units.npz; tests/test_ref_units.py checks
the oracle (CPU) and the device (GPU) against that fixture bit for bit.

Units and the reference code behind each (paths relative to /root/reference/rrt):
  obb      old_collisioncheck.cpp:34,36 (vehicle box) + :14-16 (obstacle at t) -> getOBBdist :98-148,
           OBB ctor/setVertices/setNorms/findMaxMin collision.h:17-35, old_collisioncheck.cpp:56-95
  geom     OBB(pos, w, h, o) vertices and normals (old_collisioncheck.cpp:56-76)
  ode      VehicleODE + IntegrateEuler simulation.cpp:7-34 (Prius, vehicle.h:39-60; dt 0.04)
  lateral  transformToVehicle + interpolate controller.cpp:115-148
  profile  getReference's body reference.cpp:13-18 (LinearSpacedVector functions.h:11-21) +
           generateVelocityProfile reference.cpp:73-170
  angle    angleDiff / wrapToPi functions.h:43-57
"""
import ctypes as C
import math
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_DIR = os.path.join(ROOT, "oracle", "_ref")
FIXTURE = os.path.join(ROOT, "tests", "golden", "ref_units.npz")
NMAX = 1024  # CLRRT_UNIT_PROFILE_NMAX

UNITS = ("obb", "ode", "lateral", "profile", "angle")
IN_W = {"obb": 11, "ode": 9, "lateral": 9, "profile": 12, "angle": 2, "geom": 5}
DEVICE_UNIT = {"obb": 0, "ode": 1, "lateral": 2, "profile": 3, "angle": 4}

# parameters.launch values used by the oracle (tests/oracle_binding / clrrt.abi.default_params)
MINDLA, TLA, DLAVMIN, DT, RES = 3.2, 1.4, 3.0, 0.04, 0.2


# ------------------------------------------------------------------------------------------ cases
def cases(unit, n, seed):
    """n cases of a unit, drawn to exercise its branches (touching boxes, saturations, degenerate
    Lagrange nodes, all three profile shapes, angle wrap boundaries)."""
    r = np.random.default_rng(seed)
    if unit == "obb":
        x = r.uniform(0, 60, n); y = r.uniform(-20, 20, n)
        th = np.where(r.random(n) < 0.9, r.uniform(-7, 7, n), r.uniform(-60, 60, n))
        t = np.where(r.random(n) < 0.3, 0.0, r.uniform(0, 20, n))
        # obstacle centre near the vehicle box so about half the pairs overlap
        cx = x + 1.424 * np.cos(th) + r.uniform(-7, 7, n)
        cy = y + 1.424 * np.sin(th) + r.uniform(-7, 7, n)
        oth = np.where(r.random(n) < 0.9, r.uniform(-3.2, 3.2, n), r.uniform(-40, 40, n))
        sx = r.uniform(2, 6, n); sy = r.uniform(4, 10, n)
        mv = r.random(n) < 0.5
        vx = np.where(mv, r.uniform(-2, 2, n), 0.0); vy = np.where(mv, r.uniform(-2, 2, n), 0.0)
        # moving obstacles: shift back so they are near the vehicle at time t
        cx = cx - vx * t; cy = cy - vy * t
        return np.stack([x, y, th, t, cx, cy, oth, sx, sy, vx, vy], 1)
    if unit == "geom":
        return np.stack([r.uniform(-50, 50, n), r.uniform(-50, 50, n), r.uniform(0.5, 5, n),
                         r.uniform(1, 10, n), r.uniform(-7, 7, n)], 1)
    if unit == "ode":
        x4 = np.where(r.random(n) < 0.05, 0.0, r.uniform(-1, 12, n))
        return np.stack([r.uniform(-50, 50, n), r.uniform(-50, 50, n), r.uniform(-10, 10, n),
                         r.uniform(-0.7, 0.7, n), x4, r.uniform(-8, 4, n), r.uniform(0, 20, n),
                         r.uniform(-0.7, 0.7, n), r.uniform(-8, 3, n)], 1)
    if unit == "lateral":
        # three consecutive reference points built by accumulation (val += h), a preview point near
        # them; 3% with a duplicated junction point (the goal reference's degenerate case)
        x0 = r.uniform(-10, 60, n); y0 = r.uniform(-20, 20, n)
        ang = r.uniform(-math.pi, math.pi, n); h = r.uniform(0.02, 0.3, n)
        hx = h * np.cos(ang); hy = h * np.sin(ang)
        xv = np.stack([x0, x0 + hx, x0 + hx + hx], 1); yv = np.stack([y0, y0 + hy, y0 + hy + hy], 1)
        dup = r.random(n) < 0.03
        xv[dup, 2] = xv[dup, 1]; yv[dup, 2] = yv[dup, 1]
        bend = r.random(n) < 0.2  # a corner at the middle point
        a2 = ang + r.uniform(-1.2, 1.2, n)
        xv[bend, 2] = xv[bend, 1] + (h * np.cos(a2))[bend]; yv[bend, 2] = yv[bend, 1] + (h * np.sin(a2))[bend]
        d = r.uniform(-0.5, 0.5, n); lat = r.uniform(-3, 3, n)
        Px = xv[:, 1] + d * np.cos(ang) - lat * np.sin(ang); Py = yv[:, 1] + d * np.sin(ang) + lat * np.cos(ang)
        hd = ang + r.uniform(-1, 1, n)
        return np.concatenate([xv, yv, np.stack([Px, Py, hd], 1)], 1)
    if unit == "profile":
        ax = r.uniform(-5, 60, n); ay = r.uniform(-20, 20, n)
        L = np.where(r.random(n) < 0.3, r.uniform(0.5, 5, n), r.uniform(0.5, 70, n))
        a = r.uniform(-math.pi, math.pi, n)
        res = np.where(r.random(n) < 0.7, RES, r.uniform(0.2, 0.3, n))
        v0 = np.where(r.random(n) < 0.1, 0.0, r.uniform(0, 6, n))
        vmax = np.where(r.random(n) < 0.6, 5.0, r.uniform(1, 9, n))
        gv = np.where(r.random(n) < 0.7, 0.0, r.uniform(0, 5, n))
        gb = (r.random(n) < 0.3).astype(np.float64)
        return np.stack([ax, ay, ax + L * np.cos(a), ay + L * np.sin(a), res, v0, vmax,
                         r.uniform(0, 60, n), r.uniform(-10, 10, n), r.uniform(-math.pi, math.pi, n), gv, gb], 1)
    if unit == "angle":
        a = r.uniform(-20, 20, n); b = r.uniform(-20, 20, n)
        k = r.random(n) < 0.05  # exact multiples of pi (wrap boundaries)
        a[k] = np.round(a[k] / math.pi) * math.pi
        return np.stack([a, b], 1)
    raise ValueError(unit)


# ------------------------------------------------------------------------------------------ evaluators
def _dp(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def reference_lib(opt="O2"):
    """oracle/_ref/libref_units_<opt>.so, or None when it has not been built (no /root/reference)."""
    path = os.path.join(REF_DIR, f"libref_units_{opt}.so")
    if not os.path.exists(path):
        return None
    L = C.CDLL(path)
    L.ref_set_globals.argtypes = [C.c_double] * 5
    L.ref_set_globals(MINDLA, TLA, DLAVMIN, DT, RES)
    return L


def run_reference(L, unit, x, obb_mode=0):
    x = np.ascontiguousarray(x, dtype=np.float64)
    n = x.shape[0]
    if unit == "obb":
        out = np.zeros(n); L.ref_obb(C.c_int(n), _dp(x), C.c_int(obb_mode), _dp(out)); return out[:, None]
    if unit == "geom":
        out = np.zeros((n, 16), np.float32)
        L.ref_obb_geom(C.c_int(n), _dp(x), out.ctypes.data_as(C.POINTER(C.c_float))); return out
    if unit == "ode":
        out = np.zeros((n, 11)); L.ref_ode(C.c_int(n), _dp(x), _dp(out))
        return out[:, [0, 1, 2, 3, 4, 5, 6, 10]], out[:, 7:10]
    if unit == "lateral":
        out = np.zeros(n); L.ref_lateral(C.c_int(n), _dp(x), _dp(out)); return out[:, None]
    if unit == "profile":
        out = np.zeros((n, 1 + NMAX)); L.ref_profile(C.c_int(n), _dp(x), C.c_int(NMAX), _dp(out))
        xs = np.zeros((n, NMAX)); ys = np.zeros((n, NMAX))
        N = out[:, 0].astype(np.int64)
        for k in range(n):  # the line itself (LinearSpacedVector) from the same getReference body
            m = min(N[k], NMAX)
            lx = np.zeros(N[k]); ly = np.zeros(N[k])
            L.ref_linspace(C.c_double(x[k, 0]), C.c_double(x[k, 2]), C.c_long(N[k]), _dp(lx))
            L.ref_linspace(C.c_double(x[k, 1]), C.c_double(x[k, 3]), C.c_long(N[k]), _dp(ly))
            xs[k, :m] = lx[:m]; ys[k, :m] = ly[:m]
        return np.concatenate([out, xs, ys], 1)
    if unit == "angle":
        out = np.zeros((n, 2)); L.ref_angle(C.c_int(n), _dp(x), _dp(out)); return out
    raise ValueError(unit)


def reference_prius(L):
    out = np.zeros(14)
    L.ref_prius(_dp(out))
    return out


_orc = None


def oracle_lib():
    global _orc
    if _orc is None:
        from oracle_binding import lib
        L = lib()
        vp, P = C.c_void_p, C.POINTER
        for name, args in {"orc_unit_obb": [C.c_int, P(C.c_double), P(C.c_double)],
                           "orc_unit_obb_geom": [C.c_int, P(C.c_double), P(C.c_float)],
                           "orc_unit_ode": [vp, C.c_int, P(C.c_double), P(C.c_double)],
                           "orc_unit_lateral": [C.c_int, P(C.c_double), P(C.c_double)],
                           "orc_unit_linspace": [C.c_double, C.c_double, C.c_long, P(C.c_double)],
                           "orc_unit_profile": [vp, C.c_int, P(C.c_double), C.c_int, P(C.c_double)],
                           "orc_unit_angle": [C.c_int, P(C.c_double), P(C.c_double)]}.items():
            getattr(L, name).argtypes = args
            getattr(L, name).restype = None
        _orc = L
    return _orc


def run_oracle(unit, x):
    from oracle_binding import Oracle
    from clrrt import abi
    L = oracle_lib()
    x = np.ascontiguousarray(x, dtype=np.float64)
    n = x.shape[0]
    if unit == "obb":
        out = np.zeros(n); L.orc_unit_obb(n, _dp(x), _dp(out)); return out[:, None]
    if unit == "geom":
        out = np.zeros((n, 16), np.float32)
        L.orc_unit_obb_geom(n, _dp(x), out.ctypes.data_as(C.POINTER(C.c_float))); return out
    if unit in ("ode", "profile"):
        o = Oracle(abi.default_params(), None)
        if unit == "ode":
            out = np.zeros((n, 8)); L.orc_unit_ode(o.h, n, _dp(x), _dp(out)); return out
        out = np.zeros((n, 1 + NMAX)); L.orc_unit_profile(o.h, n, _dp(x), NMAX, _dp(out))
        xs = np.zeros((n, NMAX)); ys = np.zeros((n, NMAX))
        N = out[:, 0].astype(np.int64)
        for k in range(n):
            m = min(N[k], NMAX)
            lx = np.zeros(N[k]); ly = np.zeros(N[k])
            L.orc_unit_linspace(x[k, 0], x[k, 2], int(N[k]), _dp(lx))
            L.orc_unit_linspace(x[k, 1], x[k, 3], int(N[k]), _dp(ly))
            xs[k, :m] = lx[:m]; ys[k, :m] = ly[:m]
        return np.concatenate([out, xs, ys], 1)
    if unit == "lateral":
        out = np.zeros(n); L.orc_unit_lateral(n, _dp(x), _dp(out)); return out[:, None]
    if unit == "angle":
        out = np.zeros((n, 2)); L.orc_unit_angle(n, _dp(x), _dp(out)); return out
    raise ValueError(unit)


def run_device(planner, unit, x):
    return planner.selftest_units(DEVICE_UNIT[unit], x)


# ------------------------------------------------------------------------------------------ comparison
def mismatches(a, b):
    """Rows where a and b differ in any bit (any NaN equals any NaN: payloads are not specified)."""
    a = np.asarray(a); b = np.asarray(b)
    if a.dtype == np.float32:
        ai, bi = a.view(np.uint32), b.view(np.uint32)
    else:
        a = a.astype(np.float64); b = b.astype(np.float64)
        ai, bi = a.view(np.uint64), b.view(np.uint64)
    diff = (ai != bi) & ~(np.isnan(a) & np.isnan(b))
    return np.nonzero(diff.reshape(diff.shape[0], -1).any(1))[0]
