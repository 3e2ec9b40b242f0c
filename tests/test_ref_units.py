"""Hot-path units pinned to the REFERENCE'S OWN CODE (tests/ref_units.py, tests/golden/ref_units.npz).

The fixture holds cases with the outputs of the reference's own functions compiled from verbatim line
ranges of /root/reference (oracle/Makefile `ref`, CMake Release flags).  Bar: bit for bit (any NaN
equals any NaN).
  * CPU: the oracle's unit hooks (the functions its expandTree runs) against the fixture; when the
    reference build is present (development container), 10^5 fresh cases per unit live, and the
    collision decision under every choice of the reference's unset normsY[3].
  * GPU: clrrt_selftest_units (the device functions the rollout and nearest-node kernels run) against
    the fixture.
Units: the OBB test, the ODE step, the lateral error, getReference + the velocity profile, the angle
helpers (round 2), and dubinsDistance, feasibleNode (every device decider), feasibleGoalBias,
getGoalReference + the goal-biased profile, and the Controller over state sequences (round 3).
The tree-level pins (candidate lists, whole Simulations, expandTree, re-initialisation) are in
tests/test_ref_tree.py.
"""
import os

import numpy as np
import pytest

import ref_units as R

FIX = np.load(R.FIXTURE, allow_pickle=False)
UNITS = ("obb", "geom", "ode", "lateral", "profile", "angle", "dubins", "feasible", "goalbias", "goalref", "ctrl")
DEVICE_UNITS = ("obb", "ode", "lateral", "profile", "angle", "dubins", "feasible", "goalbias", "goalref", "ctrl")


def _fixture_out(unit):
    y = FIX[f"{unit}_out"]
    if unit not in ("profile", "goalref"):
        return y
    # trimmed columns (N, v[:m], x[:m], y[:m]) -> the full NMAX layout
    m = (y.shape[1] - 1) // 3
    full = np.zeros((y.shape[0], 1 + 3 * R.NMAX))
    full[:, :1 + m] = y[:, :1 + m]
    full[:, 1 + R.NMAX:1 + R.NMAX + m] = y[:, 1 + m:1 + 2 * m]
    full[:, 1 + 2 * R.NMAX:1 + 2 * R.NMAX + m] = y[:, 1 + 2 * m:]
    return full


def _compare(unit, got, want):
    if unit == "geom":
        cols = list(range(11)) + [12, 13, 14]
        bad = R.mismatches(got[:, cols], want[:, cols])
        # the oracle's canonical axis-3 y-normal is what the reference writes into normsX[3]
        bad3 = R.mismatches(got[:, 15:16], want[:, 15:16])
        return np.union1d(bad, bad3)
    return R.mismatches(got, want)


@pytest.mark.parametrize("unit", UNITS)
def test_oracle_matches_reference_fixture(unit):
    x = FIX[f"{unit}_in"]
    got = R.run_oracle(unit, x)
    bad = _compare(unit, got, _fixture_out(unit))
    assert len(bad) == 0, f"{unit}: {len(bad)} of {len(x)} cases differ from the reference, first {bad[:5]}"


def test_fixture_exercises_branches():
    obb = FIX["obb_out"][:, 0]
    assert 0.1 < np.mean(obb == 0) < 0.5  # overlaps and separations
    assert np.any(FIX["obb_in"][:, 9] != 0) and np.any(FIX["obb_in"][:, 9] == 0)  # moving and static
    ode_in = FIX["ode_in"]
    assert np.any(np.abs(ode_in[:, 3]) > 0.52) and np.any(ode_in[:, 8] < -6)  # saturations
    lat = FIX["lateral_out"][:, 0]
    assert np.any(~np.isfinite(lat))  # the duplicated-junction (0/0) case
    prof_in = FIX["profile_in"]
    assert np.any(prof_in[:, 11] == 1) and np.any(prof_in[:, 11] == 0)  # goal-biased and not
    # dubins: both key branches (inside a turning circle, rrtplanner.cpp:395) and ties of the optimize key
    d_in = FIX["dubins_in"]
    q = d_in[:, :2] - d_in[:, 2:4]
    c, s_ = np.cos(-d_in[:, 4]), np.sin(-d_in[:, 4])
    qx, qy = c * q[:, 0] - s_ * q[:, 1], np.abs(s_ * q[:, 0] + c * q[:, 1])
    inside = (qx ** 2 + (qy - R.RHO) ** 2 <= R.RHO ** 2)
    assert 0.05 < inside.mean() < 0.6
    assert len(np.unique(FIX["dubins_out"][:, 1])) < len(d_in)
    # feasibleNode: both outcomes, cases within 1e-9 rad of pi/4 and within 1e-9 relative of 2.1 ref_res
    f_in, f_out = FIX["feasible_in"], FIX["feasible_out"][:, 0]
    assert 0.1 < f_out.mean() < 0.6
    v = f_in[:, :2] - f_in[:, 4:6]
    ap = np.arctan2(f_in[:, 5] - f_in[:, 3], f_in[:, 4] - f_in[:, 2])
    dang = np.abs(np.abs(np.angle(np.exp(1j * (np.arctan2(v[:, 1], v[:, 0]) - ap)))) - np.pi / 4)
    assert np.sum(dang < 1e-8) > 50 and np.sum(dang < 1e-11) > 20
    dl = np.abs(np.hypot(v[:, 0], v[:, 1]) / (2.1 * f_in[:, 6]) - 1)
    assert np.sum(dl < 1e-8) > 50
    # feasibleGoalBias: both outcomes
    assert 0.05 < FIX["goalbias_out"].mean() < 0.6
    # controller: IDwp reaches N - 3 and N - 1 (endreached), ym of every sign
    ctrl = FIX["ctrl_out"][:, 4:].reshape(len(FIX["ctrl_out"]), -1, 8)
    assert 0.2 < ctrl[:, :, 1].mean() < 0.8
    assert np.any(ctrl[:, :, 4] > 0) and np.any(ctrl[:, :, 4] < 0)


def test_prius_matches_reference():
    from clrrt import abi
    p = abi.default_params()
    ref = FIX["prius"]  # Vehicle::setPrius vehicle.h:39-60
    got = [p.veh.dmax, p.veh.ddmax, p.veh.Td, p.veh.Ta, p.veh.amin, p.veh.amax, p.veh.L]
    assert np.array_equal(np.array(got), ref[:7])
    assert p.veh.Vch == ref[11] and p.veh.Kus == ref[13]


# the reference build is loaded lazily, by the CPU tests that use it (no -m gpu test does)
live = pytest.mark.skipif(not os.path.exists(os.path.join(R.REF_DIR, "libref_units_O3.so")),
                          reason="reference build absent (no /root/reference: `make -C oracle ref`)")


@live
@pytest.mark.parametrize("unit", UNITS)
def test_oracle_matches_reference_live(unit):
    n = {"profile": 20000, "goalref": 20000, "ctrl": 5000}.get(unit, 100000)
    x = R.cases(unit, n, 11)
    want = R.run_reference(R.reference_lib("O3"), unit, x)
    if unit == "ode":
        want, keep = want
        # IntegrateEuler's i <= x.size() loop leaves x[7..9] untouched (zero-filled dx[7..10])
        assert np.all(keep == np.array([7.0, 8.0, 9.0]))
    bad = _compare(unit, R.run_oracle(unit, x), want)
    assert len(bad) == 0, f"{unit}: {len(bad)} of {n} cases differ, first {bad[:5]}"


@live
def test_unset_axis3_never_changes_a_collision_decision():
    """setNorms leaves normsY[3] unset (old_collisioncheck.cpp:74-75); whatever it holds (0, any
    value, NaN), the reference's overlap decision equals the canonical axis's on 10^5 pairs."""
    L = R.reference_lib("O3")
    x = R.cases("obb", 100000, 12)
    dec = R.run_reference(L, "obb", x, 0)[:, 0] == 0
    assert 0.1 < dec.mean() < 0.5
    for mode in (1, 2, 3):
        assert np.array_equal(R.run_reference(L, "obb", x, mode)[:, 0] == 0, dec), mode


@pytest.mark.gpu
@pytest.mark.parametrize("unit", DEVICE_UNITS)
def test_device_matches_reference_fixture(unit):
    import clrrt
    pl = clrrt.Planner(clrrt.default_params(), device=0, max_nodes=1 << 10, max_rows=1 << 12, max_batch=16)
    try:
        x = FIX[f"{unit}_in"]
        got = R.run_device(pl, unit, x)
        if unit == "feasible":
            # the exact decider and the searches' decider equal the reference; the brute-force prefilter
            # lets every feasible node through
            want = _fixture_out(unit)[:, 0]
            for col in (0, 1):
                bad = np.nonzero(got[:, col] != want)[0]
                assert len(bad) == 0, (f"feasible decider {col}: {len(bad)} of {len(x)} differ, first {bad[:5]}: "
                                       f"{x[bad[:3]]}")
            assert np.all(got[want == 1, 2] == 1), "the prefilter rejects a feasible node"
            return
        bad = R.mismatches(got, _fixture_out(unit))
        assert len(bad) == 0, (f"{unit}: {len(bad)} of {len(x)} device results differ from the reference, "
                               f"first {bad[:5]}: {got[bad[:3]][:, :4]} vs {_fixture_out(unit)[bad[:3]][:, :4]}")
    finally:
        pl.close()
