"""ctypes mirrors of the records declared in include/clrrt.h (the libclrrt C-ABI).

Field order and types follow the header exactly; `_check_sizes()` asserts the sizes the
header documents so a drift between the two fails at import time.
"""
import ctypes as C

CLRRT_ABI_VERSION = 11  # include/clrrt.h
UNIT_OBB, UNIT_ODE, UNIT_LATERAL, UNIT_PROFILE, UNIT_ANGLE = 0, 1, 2, 3, 4  # CLRRT_UNIT_*
UNIT_DUBINS, UNIT_FEASIBLE, UNIT_GOALBIAS, UNIT_GOALREF, UNIT_CTRL = 5, 6, 7, 8, 9
UNIT_PROFILE_NMAX = 1024
UNIT_CTRL_K = 24
CLRRT_MODE_EXACT = 0
CLRRT_PARENT_PREV = -2  # goal-biased record: parent = the record before it (include/clrrt.h)
CLRRT_MODE_BATCH = 1
CLRRT_COLLISION_STUB = 0
CLRRT_COLLISION_OBB = 1

ROLL_ITERLIMIT, ROLL_END, ROLL_GOAL, ROLL_COLLISION, ROLL_ACCLIMIT = range(5)
ROLL_NAMES = {ROLL_ITERLIMIT: "iterlimit", ROLL_END: "end", ROLL_GOAL: "goal",
              ROLL_COLLISION: "collision", ROLL_ACCLIMIT: "acclimit"}
REINIT_EMPTY, REINIT_ALL_ERASED, REINIT_COLLISION, REINIT_KEPT = range(4)  # CLRRT_REINIT_*
CLRRT_WORLD_TO_CAR, CLRRT_CAR_TO_WORLD = 0, 1


class Vehicle(C.Structure):
    _fields_ = [(n, C.c_double) for n in ("dmax", "ddmax", "Td", "Ta", "amin", "amax", "L", "Vch", "Kus")]


class Params(C.Structure):
    _fields_ = [
        ("veh", Vehicle),
        ("sim_dt", C.c_double), ("ctrl_tla", C.c_double), ("ctrl_mindla", C.c_double),
        ("ctrl_dlavmin", C.c_double), ("ctrl_Kp", C.c_double), ("ctrl_Ki", C.c_double),
        ("ref_int", C.c_double), ("ref_mindist", C.c_double), ("ref_res", C.c_double),
        ("vmax", C.c_double), ("ay_road_max", C.c_double),
        ("goal", C.c_double * 4), ("Wcost", C.c_double * 5),
        ("lane_shift0", C.c_double), ("Cxy", C.c_double * 3),
        ("bend", C.c_int32), ("obs_use_pred", C.c_int32), ("sort_limit", C.c_int32),
        ("collision_mode", C.c_int32),
    ]


class Obstacle(C.Structure):
    _fields_ = [(n, C.c_double) for n in ("cx", "cy", "theta", "size_x", "size_y", "vx", "vy")]


class Node(C.Structure):
    _fields_ = [
        ("state", C.c_double * 10), ("ref_front", C.c_double * 2), ("ref_back", C.c_double * 2),
        ("ref_vback", C.c_double), ("ang_par", C.c_double), ("parent", C.c_int32),
        ("costE", C.c_float), ("costS", C.c_float), ("goal", C.c_int32), ("nrows", C.c_int32),
        ("owner", C.c_int32), ("row_offset", C.c_int64),
    ]


class Rng(C.Structure):
    _fields_ = [("r", C.c_int32 * 34), ("pos", C.c_int32)]


class Sample(C.Structure):
    _fields_ = [("x", C.c_double), ("y", C.c_double), ("explore", C.c_int32), ("pad", C.c_int32)]


class Counters(C.Structure):
    _fields_ = [(n, C.c_int64) for n in ("sim_count", "fail_collision", "fail_acclimit",
                                          "fail_iterlimit", "rollouts")]


class Stats(C.Structure):
    _fields_ = [("iterations", C.c_int64), ("nodes_added", C.c_int64), ("goal_nodes_added", C.c_int64),
                ("rounds", C.c_int64), ("speculated", C.c_int64), ("elapsed_ms", C.c_double),
                ("capacity_stop", C.c_int64), ("deferred", C.c_int64)]


class Iteration(C.Structure):  # clrrt_iteration
    _fields_ = [("nodes", C.c_int32), ("sim_count", C.c_int32), ("fail_collision", C.c_int32),
                ("fail_acclimit", C.c_int32), ("fail_iterlimit", C.c_int32), ("rollouts", C.c_int32)]


class Capacity(C.Structure):
    _fields_ = [("max_nodes", C.c_int64), ("max_rows", C.c_int64), ("max_batch", C.c_int32),
                ("max_obstacles", C.c_int32)]


class SimCase(C.Structure):
    _fields_ = [("state", C.c_double * 10), ("ax", C.c_double), ("ay", C.c_double), ("hx", C.c_double),
                ("hy", C.c_double), ("vstart", C.c_double), ("ref_n", C.c_int32), ("goal_biased", C.c_int32)]


class RolloutJob(C.Structure):
    _fields_ = [("parent", C.c_int32), ("gb", C.c_int32), ("sample", C.c_double * 2)]


class RolloutResult(C.Structure):
    _fields_ = [("outcome", C.c_int32), ("nrows", C.c_int32), ("costE", C.c_double),
                ("costS", C.c_double), ("final_state", C.c_double * 10), ("ref_back", C.c_double * 2),
                ("ref_vback", C.c_double), ("ref_n", C.c_int32), ("pad", C.c_int32)]


class ExchangeIO(C.Structure):  # clrrt_exchange_io (the sharded expansion's exchange hook)
    _fields_ = [("n_local", C.c_int32), ("flags", C.c_int32), ("elapsed_ms", C.c_double), ("aux_local", C.c_int64),
                ("bbox_local", C.c_double * 4), ("stream", C.c_void_p),
                ("dev_all", C.c_void_p), ("n_all", C.c_int32), ("pad", C.c_int32), ("max_elapsed_ms", C.c_double),
                ("aux_sum", C.c_int64), ("bbox_all", C.c_double * 4)]


def _check_sizes():
    assert C.sizeof(Node) == 160, C.sizeof(Node)
    assert C.sizeof(Obstacle) == 56
    assert C.sizeof(Rng) == 140
    assert C.sizeof(Sample) == 24
    assert C.sizeof(RolloutResult) == 136, C.sizeof(RolloutResult)
    assert C.sizeof(ExchangeIO) == 128, C.sizeof(ExchangeIO)


_check_sizes()


def default_params(v0=0.0, goal=(40.0, 0.0, 0.0, 0.0), vmax=5.0, collision_mode=CLRRT_COLLISION_STUB):
    """Pure-Python twin of clrrt_params_default (used where the C library is not loaded, e.g. by
    the oracle tests).  Values: rrt/launch/parameters.launch:3-20, Vehicle::setPrius
    (rrt/include/rrt/vehicle.h:39-60), rrt_node.cpp:10-18, rrtplanner.cpp:13."""
    p = Params()
    lf, lr, Cf, Cr, m, L = 1.0868, 1.6132, 22201.0, 22201.0, 950.0 + 640.0, 2.7
    p.veh.dmax, p.veh.ddmax, p.veh.Td, p.veh.Ta = 0.52, 0.3294, 0.3, 0.3
    p.veh.amin, p.veh.amax, p.veh.L, p.veh.Vch = -6.0, 2.0, L, 20.0
    p.veh.Kus = (m / L) * (lr / Cf - lf / Cr)
    p.sim_dt, p.ctrl_tla, p.ctrl_mindla, p.ctrl_dlavmin = 0.04, 1.4, 3.2, 3.0
    p.ctrl_Kp, p.ctrl_Ki, p.ref_int, p.ref_mindist = 8.0, 0.05, 0.02, 0.2
    p.ref_res = max(abs(v0) * p.ref_int, p.ref_mindist)
    p.vmax, p.ay_road_max = vmax, 0.0
    for i in range(4):
        p.goal[i] = goal[i]
    for i, w in enumerate((10.0, 5.0, 0.0, 4.0, 1.0)):
        p.Wcost[i] = w
    p.lane_shift0 = 0.0
    p.bend, p.obs_use_pred, p.sort_limit, p.collision_mode = 0, 1, 10, collision_mode
    return p
