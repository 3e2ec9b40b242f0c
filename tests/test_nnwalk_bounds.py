"""CPU checks of the lower bounds the walk search (cl-rrt_amd/csrc/clrrt_nnwalk.hip) prunes with.

The search skips a node, tile or super-tile only when a lower bound on the float Dubins key
(dubinsDistance, rrt/src/rrtplanner.cpp:371-406) exceeds the sample's current 11th key.  These tests
restate the key in float32 numpy on many random node-frame points and check the bounds the kernel
relies on, with the margins it uses:
  * key >= rho * beta - 5e-3  (beta = angle between the node heading and the sample direction);
  * key >= |q| - 1e-4 - 1e-5 |q|;
  * acos_apx (Abramowitz & Stegun 4.4.45) within 1e-4 rad of acos on [-1, 1];
  * atan2_apx (A&S 4.4.49) within 1e-6 rad of atan2, and walk_key_range (the stage-1 key bounds of
    the walk's drains) below / above the key of every offset within pos_err of its own.
"""
import numpy as np
import pytest

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


F = np.float32


def atan2_apx(y, x):
    """atan2_apx of clrrt_nnwalk.hip in float32."""
    y, x = y.astype(F), x.astype(F)
    ax, ay = np.abs(x), np.abs(y)
    z = (np.minimum(ax, ay) / np.maximum(ax, ay)).astype(F)
    z2 = z * z
    p = F(0.0028662257)
    for c in (-0.0161657367, 0.0429096138, -0.0752896400, 0.1065626393, -0.1420889944, 0.1999355085,
              -0.3333314528):
        p = p * z2 + F(c)
    a = z + z * z2 * p
    a = np.where(ay > ax, F(1.57079633) - a, a)
    a = np.where(x < 0, F(3.14159265) - a, a)
    return np.where(y < 0, -a, a).astype(F)


def walk_key_range(tx, ty, pos_err, inside_bracket=False):
    """walk_key_range of clrrt_nnwalk.hip in float32 (inside the turning circle: the rho pi floor, or with
    inside_bracket -- walk_key_range<true>, the large-tree walk -- a bracket of the inside branch)."""
    tx, ty = tx.astype(F), ty.astype(F)
    rho = RHO
    t2 = tx * tx + ty * (ty - F(2) * rho)
    out = t2 >= F(0.01)
    near = (t2 > F(-0.01)) & ~out
    t = np.sqrt(np.maximum(t2, F(0)))
    th = atan2_apx(tx, rho - ty)
    th = np.where(th < 0, th + F(6.28318531), th)
    L = t + rho * (th - atan2_apx(t, rho))
    m = F(2) * pos_err + F(2e-4) + F(2e-5) * L
    lo = np.where(out, L - m, np.where(near, np.minimum(L - m - F(1e-4), F(14.9)), F(14.9)))
    hi = np.where(out, L + m, np.inf)
    # surely inside: the inside branch restated with atan2 (clrrt_nnwalk.hip walk_key_range<true>)
    ins = t2 <= F(-0.01)
    df2 = tx * tx + (ty + rho) * (ty + rho)
    cA = np.clip((F(5) * rho * rho - df2) * (F(1) / (F(4) * rho * rho)), F(-1), F(1))
    sA = np.sqrt(np.maximum((F(1) - cA) * (F(1) + cA), F(0)))
    u = rho * sA
    w = np.sqrt(np.maximum(df2 - u * u, F(0)))
    cw = w / np.sqrt(df2)
    use = ins & (sA >= F(0.05)) & (cw >= F(0.05)) & inside_bracket
    with np.errstate(all="ignore"):
        Li = rho * ((F(6.28318531) - atan2_apx(sA, cA)) + atan2_apx(tx, ty + rho) + atan2_apx(u, w))
        mi = F(2e-3) + F(1e-4) * Li + pos_err * (F(8) + F(8) / sA + F(8) / cw)
    lo = np.where(use, np.maximum(Li - mi, F(14.9)), lo)
    hi = np.where(use, Li + mi, hi)
    return lo.astype(np.float64), hi.astype(np.float64)


def test_atan2_approximation():
    rng = np.random.default_rng(11)
    for scale in (1e-3, 1.0, 50.0, 1e4):
        y = (rng.uniform(-1, 1, 1_000_000) * scale).astype(F)
        x = (rng.uniform(-1, 1, 1_000_000) * scale).astype(F)
        err = np.abs(atan2_apx(y, x).astype(np.float64) - np.arctan2(y.astype(np.float64), x.astype(np.float64)))
        err = np.minimum(err, 2 * np.pi - err)  # +-pi
        assert err.max() < 1e-6, (scale, err.max())


def test_stage1_key_bound():
    """walk_key_range at an offset jittered by up to pos_err brackets the float key at the true one."""
    rng = np.random.default_rng(12)
    pos = 4 * 2e-5  # 4 * delta of a 300 m frame (delta = 2^-24 * coordinate bound) -- generous
    tight = []
    for scale in (2.0, 6.0, 12.0, 40.0, 150.0):
        tx, ty = _points(rng, 400_000, scale)
        tx, ty = tx.astype(F), ty.astype(F)
        key = dubins_key_f32(tx, ty)
        ang = rng.uniform(0, 2 * np.pi, tx.size)
        r = pos * np.sqrt(rng.uniform(0, 1, tx.size))
        jx = (tx + r * np.cos(ang)).astype(F)
        jy = np.abs(ty + r * np.sin(ang)).astype(F)
        pe = F(pos) + F(1e-6) * (np.abs(jx) + jy)
        lb, ub = walk_key_range(jx, jy, pe)
        ok = np.isfinite(key)
        assert (key[ok] - lb[ok]).min() >= 0, (scale, (key[ok] - lb[ok]).min())
        okh = ok & np.isfinite(ub)
        assert (ub[okh] - key[okh]).min() >= 0, (scale, (ub[okh] - key[okh]).min())
        tight.append(np.median(key[okh] - lb[okh]))
    assert max(tight) < 0.02, tight  # and it is tight: the stage-1 filter rejects what the key would


def test_stage1_bound_near_turning_circle():
    """Offsets within 0.3 of the turning circle (both sides), jittered: the near-circle branch (the
    outside key or rho pi) and the inside branch stay below the float key."""
    rng = np.random.default_rng(13)
    rho = float(RHO)
    for band in (0.02, 0.1, 0.3):
        n = 1_000_000
        r = rho + rng.uniform(-band, band, n)
        a = rng.uniform(0, 2 * np.pi, n)
        tx = (r * np.cos(a)).astype(F)
        ty = np.abs(rho + r * np.sin(a)).astype(F)
        key = dubins_key_f32(tx, ty)
        pos = 8e-5
        ang = rng.uniform(0, 2 * np.pi, n)
        rr = pos * np.sqrt(rng.uniform(0, 1, n))
        jx = (tx + rr * np.cos(ang)).astype(F)
        jy = np.abs(ty + rr * np.sin(ang)).astype(F)
        lb, ub = walk_key_range(jx, jy, F(pos) + F(1e-6) * (np.abs(jx) + jy))
        ok = np.isfinite(key)
        assert (key[ok] - lb[ok]).min() >= 0, (band, (key[ok] - lb[ok]).min())
        okh = ok & np.isfinite(ub)
        assert (ub[okh] - key[okh]).min() >= 0, band


@pytest.mark.parametrize("bracket", [False, True])
def test_stage1_bound_inside_turning_circle(bracket):
    """Offsets uniformly inside the turning circle, jittered by up to 6e-4 (beyond the frame error of
    any bench tree): the walk's bounds (the rho pi floor there, or the large-tree walk's bracket of the
    inside branch) bracket the float key."""
    rng = np.random.default_rng(14)
    rho = float(RHO)
    n = 2_000_000
    r = np.sqrt(rng.uniform(0, 1, n)) * rho
    a = rng.uniform(0, 2 * np.pi, n)
    tx = (r * np.cos(a)).astype(F)
    ty = np.abs(rho + r * np.sin(a)).astype(F)
    key = dubins_key_f32(tx, ty)
    for pos in (8e-5, 6e-4):
        ang = rng.uniform(0, 2 * np.pi, n)
        rr = pos * np.sqrt(rng.uniform(0, 1, n))
        jx = (tx + rr * np.cos(ang)).astype(F)
        jy = np.abs(ty + rr * np.sin(ang)).astype(F)
        lb, ub = walk_key_range(jx, jy, F(pos) + F(1e-6) * (np.abs(jx) + jy), inside_bracket=bracket)
        ok = np.isfinite(key)
        assert (key[ok] - lb[ok]).min() >= 0, (pos, (key[ok] - lb[ok]).min())
        okh = ok & np.isfinite(ub)
        assert not okh.any() or (ub[okh] - key[okh]).min() >= 0, pos
        if bracket:  # and it is a bracket: most inside offsets get a finite upper bound
            assert okh.mean() > 0.5, okh.mean()
