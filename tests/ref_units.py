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
  dubins   dubinsDistance rrtplanner.cpp:371-406 (explore key; optimize key = costE + key, :254)
  feasible feasibleNode rrtplanner.cpp:271-289 (device: brute-force decider, walk decider, prefilter)
  goalbias feasibleGoalBias rrtplanner.cpp:292-315
  goalref  getGoalReference reference.cpp:25-70 + generateVelocityProfile(GB) :72-170
  ctrl     Controller controller.cpp:23-113 over a state sequence, in the Simulation constructor's order
           (simulation.cpp:39-43): ctor, profile, then getControls per state
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
NEW_UNITS = ("dubins", "feasible", "goalbias", "goalref", "ctrl")
CTRL_K = 24  # CLRRT_UNIT_CTRL_K
IN_W = {"obb": 11, "ode": 9, "lateral": 9, "profile": 12, "angle": 2, "geom": 5, "dubins": 6, "feasible": 7,
        "goalbias": 8, "goalref": 8, "ctrl": 12 + 6 * CTRL_K}
DEVICE_UNIT = {"obb": 0, "ode": 1, "lateral": 2, "profile": 3, "angle": 4, "dubins": 5, "feasible": 6,
               "goalbias": 7, "goalref": 8, "ctrl": 9}
RHO = 4.77

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
    if unit == "dubins":
        return _dubins_cases(r, n)
    if unit == "feasible":
        return _feasible_cases(r, n)
    if unit == "goalbias":
        return _goalbias_cases(r, n)
    if unit == "goalref":
        return _goalref_cases(r, n)
    if unit == "ctrl":
        return _ctrl_cases(r, n)
    raise ValueError(unit)


def _rot(th, x, y):
    return x * np.cos(th) - y * np.sin(th), x * np.sin(th) + y * np.cos(th)


def _dubins_cases(r, n):
    """Sample/node pairs: random offsets, offsets on the turning circles' boundaries (the inside
    branch switch, rrtplanner.cpp:395), near thetac = 0 (the while loop :386), zero and far offsets;
    headings beyond +-pi; costE with exact repeats (ties of the optimize key)."""
    nx = r.uniform(-5, 60, n); ny = r.uniform(-20, 20, n)
    th = np.where(r.random(n) < 0.9, r.uniform(-math.pi, math.pi, n), r.uniform(-20, 20, n))
    kind = r.choice(5, n, p=[0.55, 0.2, 0.1, 0.05, 0.1])
    rad = r.exponential(8.0, n); ang = r.uniform(-math.pi, math.pi, n)
    lx, ly = rad * np.cos(ang), rad * np.sin(ang)  # the rotated offset (qx, qy) the key forms
    # on a circle of radius rho centred at (0, +-rho): qx^2 + (|qy| -+ rho)^2 = rho^2 (1 + eps)
    eps = r.choice([0.0, 1e-7, -1e-7, 1e-5, -1e-5, 1e-3, -1e-3], n)
    phi = r.uniform(-math.pi, math.pi, n); sgn = np.where(r.random(n) < 0.5, 1.0, -1.0)
    bx = RHO * np.sqrt(1 + eps) * np.cos(phi); by = sgn * (RHO + RHO * np.sqrt(1 + eps) * np.sin(phi))
    lx = np.where(kind == 1, bx, lx); ly = np.where(kind == 1, by, ly)
    tiny = r.choice([0.0, 1e-7, -1e-7, 1e-4, -1e-4], n)
    lx = np.where(kind == 2, tiny, lx); ly = np.where(kind == 2, r.uniform(-12, 12, n), ly)
    lx = np.where(kind == 3, 0.0, lx); ly = np.where(kind == 3, 0.0, ly)
    far = r.uniform(100, 1000, n)
    lx = np.where(kind == 4, far * np.cos(ang), lx); ly = np.where(kind == 4, far * np.sin(ang), ly)
    # the key rotates the world offset by -heading: world offset = R(heading) (qx, qy)
    wx, wy = _rot(th, lx, ly)
    sx = nx + wx; sy = ny + wy
    sx = np.where(kind == 3, nx, sx); sy = np.where(kind == 3, ny, sy)
    ce = np.where(r.random(n) < 0.4, 0.0, r.uniform(0, 100, n))
    rep = r.random(n) < 0.2
    ce[rep] = np.round(ce[rep], 1)
    return np.stack([sx, sy, nx, ny, th, ce], 1)


def _feasible_cases(r, n):
    """feasibleNode at and near both limits: angle pi/4 +- {0, 1e-12, 1e-9, 1e-6, 1e-4} from angPar and
    length 2.1 ref_res (1 +- {0, 1e-12, 1e-9, 1e-6}); zero-length parent references (angPar = atan2(0, 0))."""
    bx = r.uniform(-5, 60, n); by = r.uniform(-20, 20, n)
    a = r.uniform(-math.pi, math.pi, n)
    L0 = np.where(r.random(n) < 0.1, 0.0, r.uniform(0.2, 30, n))
    fx = bx - L0 * np.cos(a); fy = by - L0 * np.sin(a)
    res = np.where(r.random(n) < 0.7, 0.2, r.uniform(0.2, 0.3, n))
    near_a = r.random(n) < 0.45
    delta = r.choice([0.0, 1e-12, -1e-12, 1e-9, -1e-9, 1e-6, -1e-6, 1e-4, -1e-4], n)
    phi = np.where(near_a, np.where(r.random(n) < 0.5, 1.0, -1.0) * (math.pi / 4) + delta,
                   r.uniform(-math.pi, math.pi, n))
    near_l = r.random(n) < 0.35
    dl = r.choice([0.0, 1e-12, -1e-12, 1e-9, -1e-9, 1e-6, -1e-6], n)
    d = np.where(near_l, 2.1 * res * (1 + dl), np.where(r.random(n) < 0.5, r.uniform(0, 2, n), r.uniform(0, 30, n)))
    ang = np.where(L0 == 0, phi, a + phi)  # angPar = 0 for a zero-length reference
    sx = bx + d * np.cos(ang); sy = by + d * np.sin(ang)
    return np.stack([sx, sy, fx, fy, bx, by, res], 1)


def _goal(r, n):
    g0 = r.uniform(10, 60, n); g1 = r.uniform(-15, 15, n); g2 = r.uniform(-math.pi, math.pi, n)
    g3 = np.where(r.random(n) < 0.6, 0.0, r.uniform(0, 5, n))
    return g0, g1, g2, g3


def _goalbias_cases(r, n):
    """feasibleGoalBias near its circle limits (R1 - 0.3 around the reference's centres, whose y uses
    cos, rrtplanner.cpp:297-299) and near its angle limit pi/8 (:312)."""
    g0, g1, g2, g3 = _goal(r, n)
    R1 = 4.77; R2 = R1 - 0.3
    x = g0 + r.uniform(-15, 15, n); y = g1 + r.uniform(-15, 15, n)
    circ = r.random(n) < 0.3
    side = np.where(r.random(n) < 0.5, -math.pi / 2, math.pi / 2)
    cx = g0 + R1 * np.cos(g2 + side); cy = g1 + R1 * np.cos(g2 + side)
    dd = R2 * (1 + r.choice([0.0, 1e-12, -1e-12, 1e-9, -1e-9, 1e-5, -1e-5], n)); pa = r.uniform(-math.pi, math.pi, n)
    x = np.where(circ, cx + dd * np.cos(pa), x); y = np.where(circ, cy + dd * np.sin(pa), y)
    ang = r.random(n) < 0.4
    dl = r.choice([0.0, 1e-12, -1e-12, 1e-9, -1e-9, 1e-5, -1e-5, 0.3, -0.3], n)
    aref = g2 + np.where(r.random(n) < 0.5, 1.0, -1.0) * (math.pi / 8 + dl) + np.where(r.random(n) < 0.5, 0.0, math.pi)
    dist = r.uniform(2, 30, n)
    bx = np.where(ang, g0 - dist * np.cos(aref), x + r.uniform(-3, 3, n))
    by = np.where(ang, g1 - dist * np.sin(aref), y + r.uniform(-3, 3, n))
    return np.stack([g0, g1, g2, g3, x, y, bx, by], 1)


def _goalref_cases(r, n):
    """getGoalReference from parent reference ends around the goal, including ends within half a
    resolution of the alignment points (a one-point first segment)."""
    g0, g1, g2, g3 = _goal(r, n)
    bx = g0 + r.uniform(-40, 10, n); by = g1 + r.uniform(-20, 20, n)
    near = r.random(n) < 0.1
    s = np.where(r.random(n) < 0.5, 1.0, -1.0)
    bx = np.where(near, g0 + s * np.cos(g2) + r.uniform(-0.05, 0.05, n), bx)
    by = np.where(near, g1 + s * np.sin(g2) + r.uniform(-0.05, 0.05, n), by)
    v0 = np.where(r.random(n) < 0.1, 0.0, r.uniform(0, 6, n))
    res = np.where(r.random(n) < 0.7, RES, r.uniform(0.2, 0.3, n))
    return np.stack([g0, g1, g2, g3, bx, by, v0, res], 1)


def _ctrl_cases(r, n):
    """Controllers on straight references (lengths down to 3 points) and two-segment goal references,
    driven through CTRL_K states that progress along the reference past its end (IDwp reaches N-3 and
    N-1), with lateral/heading noise, standstill, jumps and a few far-off states."""
    K = CTRL_K
    out = np.zeros((n, 12 + 6 * K))
    for i in range(n):
        gb = r.random() < 0.3
        g0, g1, g2, g3 = (v[0] for v in _goal(r, 1))
        res = RES if r.random() < 0.7 else r.uniform(0.2, 0.3)
        if gb:
            ax, ay = g0 + r.uniform(-30, 5), g1 + r.uniform(-15, 15)
            pc = np.array([g0, g1]) - np.array([math.cos(g2), math.sin(g2)])
            pf = pc + 5.2 * np.array([math.cos(g2), math.sin(g2)])
            poly = [np.array([ax, ay]), pc, pf]
            sx = sy = 0.0
        else:
            ax, ay = r.uniform(-5, 40), r.uniform(-15, 15)
            L = r.uniform(0.42, 1.2) if r.random() < 0.15 else r.uniform(1, 40)
            a = r.uniform(-math.pi, math.pi)
            sx, sy = ax + L * math.cos(a), ay + L * math.sin(a)
            poly = [np.array([ax, ay]), np.array([sx, sy])]
        seg = [np.linalg.norm(poly[k + 1] - poly[k]) for k in range(len(poly) - 1)]
        tot = max(sum(seg), 1e-9)
        vstart = 0.0 if r.random() < 0.1 else r.uniform(0, 6)
        vmax = 5.0 if r.random() < 0.6 else r.uniform(1, 9)
        out[i, :12] = [1.0 if gb else 0.0, ax, ay, sx, sy, g0, g1, g2, g3, vstart, vmax, res]
        span = r.uniform(0.3, 1.6)
        fr = np.sort(r.uniform(0, span, K)) if r.random() < 0.8 else np.linspace(0, span, K)
        fr[0] = 0.0
        for j in range(K):
            d = fr[j] * tot
            k = 0
            while k < len(seg) - 1 and d > seg[k]:
                d -= seg[k]; k += 1
            t = poly[k + 1] - poly[k]
            h = math.atan2(t[1], t[0]) if np.linalg.norm(t) > 0 else 0.0
            p = poly[k] + (d / max(seg[k], 1e-9)) * t
            lat = r.normal(0, 0.4)
            p = p + lat * np.array([-math.sin(h), math.cos(h)])
            hd = h + r.normal(0, 0.25)
            if r.random() < 0.03:
                p = p + r.uniform(-20, 20, 2)
                hd = r.uniform(-math.pi, math.pi)
            v = 0.0 if r.random() < 0.05 else r.uniform(0, 8)
            out[i, 12 + 6 * j: 18 + 6 * j] = [p[0], p[1], hd, r.uniform(-0.5, 0.5), v, r.uniform(-3, 2)]
    return out


# ------------------------------------------------------------------------------------------ evaluators
def _dp(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def config_vector(params, coll=None):
    """ref_config's 26 doubles from an abi.Params (oracle/ref_units.cpp)."""
    p = params
    c = [p.sim_dt, p.ctrl_tla, p.ctrl_mindla, p.ctrl_dlavmin, p.ctrl_Kp, p.ctrl_Ki, p.ref_res, p.ref_int,
         p.ref_mindist, p.vmax, *p.Wcost[:], *p.goal[:], float(p.collision_mode if coll is None else coll),
         float(p.obs_use_pred), float(p.bend), p.lane_shift0, *p.Cxy[:]]
    return np.array(c, dtype=np.float64)


_REF_LIBS = {}


def reference_lib(opt="O2"):
    """oracle/_ref/libref_units_<opt>.so, or None when it has not been built (no /root/reference).
    Loaded on first use (only CPU tests call this)."""
    if opt in _REF_LIBS:
        return _REF_LIBS[opt]
    path = os.path.join(REF_DIR, f"libref_units_{opt}.so")
    if not os.path.exists(path):
        return None
    L = C.CDLL(path)
    L.ref_set_globals.argtypes = [C.c_double] * 5
    L.ref_set_globals(MINDLA, TLA, DLAVMIN, DT, RES)
    L.ref_config.argtypes = [C.POINTER(C.c_double)]
    from clrrt import abi  # noqa: F401  (params layout)
    import clrrt
    L.ref_config(_dp(config_vector(clrrt.default_params())))
    _REF_LIBS[opt] = L
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
    if unit == "dubins":  # the explore key; the optimize key is costE + key in float (rrtplanner.cpp:254)
        k = np.zeros(n, np.float32)
        L.ref_dubins(C.c_int(n), _dp(x), k.ctypes.data_as(C.POINTER(C.c_float)))
        return np.stack([k.astype(np.float64), (x[:, 5].astype(np.float32) + k).astype(np.float64)], 1)
    if unit == "feasible":
        out = np.zeros(n); L.ref_feasible(C.c_int(n), _dp(x), _dp(out)); return out[:, None]
    if unit == "goalbias":
        out = np.zeros(n); L.ref_goal_bias(C.c_int(n), _dp(x), _dp(out)); return out[:, None]
    if unit == "goalref":
        out = np.zeros((n, 1 + 3 * NMAX)); L.ref_goal_ref(C.c_int(n), _dp(x), C.c_int(NMAX), _dp(out)); return out
    if unit == "ctrl":
        out = np.zeros((n, 4 + 8 * CTRL_K)); L.ref_controller(C.c_int(n), _dp(x), C.c_int(CTRL_K), _dp(out))
        return out
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
                           "orc_unit_angle": [C.c_int, P(C.c_double), P(C.c_double)],
                           "orc_unit_dubins": [C.c_int, P(C.c_double), P(C.c_double)],
                           "orc_unit_feasible": [vp, C.c_int, P(C.c_double), P(C.c_double)],
                           "orc_unit_goal_bias": [vp, C.c_int, P(C.c_double), P(C.c_double)],
                           "orc_unit_goal_ref": [vp, C.c_int, P(C.c_double), C.c_int, P(C.c_double)],
                           "orc_unit_ctrl": [vp, C.c_int, P(C.c_double), C.c_int, P(C.c_double)]}.items():
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
    if unit == "dubins":
        out = np.zeros((n, 2)); L.orc_unit_dubins(n, _dp(x), _dp(out)); return out
    o = Oracle(abi.default_params(), None)
    if unit == "feasible":
        out = np.zeros(n); L.orc_unit_feasible(o.h, n, _dp(x), _dp(out)); return out[:, None]
    if unit == "goalbias":
        out = np.zeros(n); L.orc_unit_goal_bias(o.h, n, _dp(x), _dp(out)); return out[:, None]
    if unit == "goalref":
        out = np.zeros((n, 1 + 3 * NMAX)); L.orc_unit_goal_ref(o.h, n, _dp(x), NMAX, _dp(out)); return out
    if unit == "ctrl":
        out = np.zeros((n, 4 + 8 * CTRL_K)); L.orc_unit_ctrl(o.h, n, _dp(x), CTRL_K, _dp(out)); return out
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
