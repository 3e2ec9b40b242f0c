"""EXACT candidate lists with std::sort ties, against the oracle's std::sort replay (rrtplanner.cpp:227-268).

Round 5 changed how far `k_nn_exact_fused` replays std::sort for a tied sample: only up to the largest key that a tie
of the list involves, the list's entries above it following in key order (round 4: up to the sort_limit-th key, or the
whole array when fewer than sort_limit entries are feasible).  These trees put many exact copies of the root and
clusters of copied nodes (equal keys for every sample) next to few feasible entries, so the new short replays run for
ties inside the list, at its boundary and in lists of fewer than sort_limit entries.  Checker: the oracle's
`orc_sort_nodes` (libstdc++ introsort restated, pinned to the reference's own lists by test_ref_tree.py).
"""
import numpy as np
import pytest

import oracle_binding as ob
import ref_tree as T

CASES = [  # (seed, nodes, root copies, samples): small trees give lists of fewer than sort_limit entries with ties
    (14, 40, 6, 256),
    (16, 30, 4, 256),
    (11, 200, 120, 512),
    (12, 1500, 600, 512),
    (13, 8000, 2000, 256),
]


def _samples(rng, H, n):
    S = T.sort_samples(rng, H, n)
    # a quarter just ahead of the root (every root copy feasible and tied) at distances where few others are
    q = n // 4
    r = rng.uniform(2.5, 12.0, q)
    a = rng.uniform(-0.7, 0.7, q)
    S[:q, 0] = 0.9 + r * np.cos(a)
    S[:q, 1] = r * np.sin(a)
    return S


@pytest.mark.gpu
@pytest.mark.parametrize("seed,n,copies,ns", CASES)
def test_exact_lists_with_ties_match_oracle(seed, n, copies, ns):
    import clrrt
    from clrrt import abi
    rng = np.random.default_rng(seed)
    H = T.sort_tree(rng, n, copies)
    S = _samples(rng, H, ns)
    arr = T.node_array(H)
    pl = clrrt.Planner(T.params(0), device=0, max_nodes=max(1 << 14, 2 * n), max_rows=1 << 20, max_batch=1024)
    try:
        pl.tree_load(arr)
        smp = (abi.Sample * ns)()
        for j in range(ns):
            smp[j].x, smp[j].y, smp[j].explore = S[j, 0], S[j, 1], int(S[j, 2])
        ids, keys = pl.sort_nodes_batch(smp, exact=True)
    finally:
        pl.close()
    o = ob.Oracle(T.params(0))
    o.L.orc_load_tree(o.h, arr, len(H))
    short_tied = tied = 0
    for j in range(ns):
        oi, ok = o.sort_nodes(S[j, 0], S[j, 1], int(S[j, 2]), stable=False)
        m = min(10, len(oi))
        assert list(ids[j, :m]) == list(oi[:m]), (j, list(ids[j]), oi[:m])
        assert m == 10 or ids[j, m] < 0, (j, list(ids[j]))
        assert np.array_equal(keys[j, :m].astype(np.float32), np.asarray(ok[:m], np.float32)), j
        t = any(ok[i] == ok[i + 1] for i in range(len(ok) - 1) if i < 10)
        tied += t
        short_tied += t and m < 10
    # the cases the round-5 replay change touches do occur here
    assert tied > ns // 10, tied
    assert short_tied > 0 or n > 100, short_tied
