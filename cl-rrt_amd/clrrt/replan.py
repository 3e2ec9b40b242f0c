"""Config 5 replanning loop (BASELINE.json configs[4]; SURVEY.md §8(d) "Cfg 5"): 5 Hz planMotion
queries with the tree re-initialised from the previous best path (commit_path = 1).

One query follows MotionPlanner::planMotion (rrt/src/motionplanner.cpp:8-77):
    carPose = transformStateToLocal(worldState)                      :14-15  (x, y, heading -> 0)
    transformNodesWorldToCar(bestNodes, worldState)                   :22
    initializeTree(RRT, veh, bestNodes, carPose)                      :32
    for (Timer timer(200); timer.Get(); ) expandTree(...)             :39-43
    bestNodes = extractBestPath(RRT.tree)                             :51
    transformNodesCarToworld(bestNodes, worldState)                   :54
The scenario around it is this benchmark's, not the reference's (the reference takes its state,
goal and obstacles from ROS topics): a fixed world goal and obstacle set, moving obstacles advanced
at their velocity, both handed to each query in the car frame, and the ego moved 0.2 s along the
committed path between queries.  Backends: the HIP planner (`PlannerBackend`) and, in the tests,
the CPU oracle through the same five calls.
"""
import math

import numpy as np

from . import abi

QUERY_PERIOD = 0.2  # 5 Hz


def world_to_car_pose(x, y, pose):
    """transformPointWorldToCar (transformations.cpp:6-11), vectorised."""
    c, s = math.cos(pose[2]), math.sin(pose[2])
    return (x * c - pose[0] * c - pose[1] * s + y * s, y * c - pose[1] * c + pose[0] * s - x * s)


def obstacles_in_car_frame(obs_world, t, pose):
    """World obstacles (cx, cy, theta, size_x, size_y, vx, vy) at time t, in the car frame of `pose`
    (centre transformed, heading and velocity rotated -- rotateVelocityVector, transformations.cpp:318)."""
    o = np.array(obs_world, dtype=np.float64).reshape(-1, 7)
    cx, cy = o[:, 0] + o[:, 5] * t, o[:, 1] + o[:, 6] * t
    o[:, 0], o[:, 1] = world_to_car_pose(cx, cy, pose)
    o[:, 2] = o[:, 2] - pose[2]
    c, s = math.cos(pose[2]), math.sin(pose[2])
    vx, vy = o[:, 5].copy(), o[:, 6].copy()
    o[:, 5], o[:, 6] = c * vx + s * vy, -s * vx + c * vy
    return o


def goal_in_car_frame(goal_world, pose):
    gx, gy = world_to_car_pose(np.array([goal_world[0]]), np.array([goal_world[1]]), pose)
    return (float(gx[0]), float(gy[0]), float(goal_world[2] - pose[2]), float(goal_world[3]))


def advance_pose(pose, path_rows, dt=QUERY_PERIOD):
    """The ego after `dt` s along the committed path (rows in world x, y; row headings stay in the
    car frame of the query that grew them, as transformNodesCarToworld leaves them).  No path: keep
    going straight at the current speed."""
    if path_rows is None or len(path_rows) == 0:
        v = pose[4]
        return np.array([pose[0] + v * dt * math.cos(pose[2]), pose[1] + v * dt * math.sin(pose[2]), pose[2],
                         pose[3], v, pose[5]])
    t0 = path_rows[0, 6]
    k = int(np.searchsorted(path_rows[:, 6] - t0, dt - 1e-9))
    k = min(k, len(path_rows) - 1)
    r = path_rows[k]
    return np.array([r[0], r[1], pose[2] + r[2], r[3], r[4], r[5]])


class PlannerBackend:
    """The five planMotion steps on the HIP planner (clrrt.Planner)."""

    def __init__(self, planner, make_params):
        self.pl = planner
        self.make_params = make_params

    def begin_query(self, pose, goal_car, obs_car):
        self.pl.set_params(self.make_params(pose[4], goal_car))
        self.pl.set_obstacles(obs_car)
        self.pl.path_transform(False, pose)
        return self.pl.tree_init_from_path([0.0, 0.0, 0.0, pose[3], pose[4], pose[5]])

    def end_query(self, pose):
        ids, _, _ = self.pl.extract_best_path()
        self.pl.path_commit(ids)
        self.pl.path_transform(True, pose)
        _, rows = self.pl.path_download()
        return ids, rows


def run_queries(backend, expand, n_queries, obs_world, goal_world=(40.0, 0.0, 0.0, 0.0), v0=0.0,
                on_query=None):
    """Run n_queries replanning queries; `expand(q)` grows the tree of query q.  Returns the list of
    per-query (pose, outcome, path ids)."""
    pose = np.array([0.0, 0.0, 0.0, 0.0, v0, 0.0])
    log = []
    for q in range(n_queries):
        t = q * QUERY_PERIOD
        oc = backend.begin_query(pose, goal_in_car_frame(goal_world, pose), obstacles_in_car_frame(obs_world, t, pose))
        expand(q)
        ids, rows = backend.end_query(pose)
        log.append((pose.copy(), oc, list(ids)))
        if on_query is not None:
            on_query(q, pose, oc, ids)
        pose = advance_pose(pose, rows)
    return log


def default_make_params(collision_mode, vmax=5.0):
    def make(v0, goal_car):
        return abi.default_params(v0=v0, goal=goal_car, vmax=vmax, collision_mode=collision_mode)
    return make
