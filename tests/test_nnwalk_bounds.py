"""CPU checks of the lower bounds the walk search (cl-rrt_amd/csrc/clrrt_nnwalk.hip) prunes with.

The search skips a node, tile or super-tile only when a lower bound on the float Dubins key
(dubinsDistance, rrt/src/rrtplanner.cpp:371-406) exceeds the sample's current 11th key.  These tests
restate the key in float32 numpy on many random node-frame points and check the bounds the kernel
relies on, with the margins it uses:
  * key >= rho * beta - 5e-3  (beta = angle between the node heading and the sample direction);
  * key >= |q| - 1e-4 - 1e-5 |q|;
  * acos_apx (Abramowitz & Stegun 4.4.45) within 1e-4 rad of acos on [-1, 1].
"""
import numpy as np

RHO = np.float32(4.77)


def dubins_key_f32(tx, ty):
    """dubinsDistance after the rotation into the node frame (ty folded to >= 0), float32 like the
    reference's float locals."""
    tx = tx.astype(np.float32)
    ty = np.abs(ty).astype(np.float32)
    rho = RHO
    dc = np.sqrt(tx * tx + (ty - rho) * (ty - rho))
    thc = np.arctan2(tx, rho - ty).astype(np.float32)
    thc = np.where(thc < 0, (thc.astype(np.float64) + 2 * np.pi).astype(np.float32), thc)
    df = np.sqrt(tx * tx + (ty + rho) * (ty + rho))
    inside = (tx * tx + (ty + rho) * (ty + rho) <= rho * rho) | (tx * tx + (ty - rho) * (ty - rho) <= rho * rho)
    with np.errstate(all="ignore"):
        out = np.sqrt(dc * dc - rho * rho) + rho * (thc - np.arccos(rho / dc))
        al = (2 * np.pi - np.arccos((5 * rho * rho - df * df) / (4 * rho * rho)).astype(np.float64)).astype(np.float32)
        inn = rho * (al + np.arcsin(tx / df) - np.arcsin(rho * np.sin(al) / df))
    return np.where(inside, inn, out).astype(np.float64)


def _points(rng, n, scale):
    return rng.uniform(-1, 1, n) * scale, np.abs(rng.uniform(-1, 1, n) * scale)


def test_turning_bound():
    rng = np.random.default_rng(7)
    for scale in (0.05, 0.5, 2.0, 5.0, 12.0, 40.0):
        tx, ty = _points(rng, 400_000, scale)
        key = dubins_key_f32(tx, ty)
        ok = np.isfinite(key)
        beta = np.arctan2(ty, tx)
        gap = key[ok] - float(RHO) * beta[ok]
        assert gap.min() >= -5e-3, (scale, gap.min())


def test_euclidean_bound():
    rng = np.random.default_rng(8)
    for scale in (0.05, 0.5, 5.0, 40.0):
        tx, ty = _points(rng, 400_000, scale)
        key = dubins_key_f32(tx, ty)
        q = np.hypot(tx, ty)
        ok = np.isfinite(key)
        assert (key[ok] - (q[ok] * (1 - 1e-5) - 1e-4)).min() >= 0, scale


def test_acos_approximation():
    x = np.linspace(-1, 1, 2_000_001).astype(np.float32)
    ax = np.abs(x)
    p = np.float32(1.5707288) + ax * (np.float32(-0.2121144) + ax * (np.float32(0.0742610) + ax * np.float32(-0.0187293)))
    r = np.sqrt(np.float32(1) - ax) * p
    r = np.where(x < 0, np.float32(np.pi) - r, r)
    assert np.abs(r.astype(np.float64) - np.arccos(x.astype(np.float64))).max() < 1e-4
