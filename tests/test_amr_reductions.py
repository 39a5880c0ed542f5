"""Host topology (afh.amr: af_adjust_refinement restated) and the tree
reductions (afh_tree_sum_cc, afh_tree_reduce_loc).

Known answer: afivo's own test_reduction (afivo/tests/test_reduction.f90,
answer file afivo/tests/answers/test_reduction_3d): a periodic 2*pi cube with
one 8^3 coarse box, refined 16 times where all(r_min < 0.4) up to level 10,
derefined elsewhere; after each af_adjust_refinement every box holds
sum(box%ix), and af_tree_max_cc / af_tree_min_cc (with location) are
printed. The highest_id sequence and the max/min values below are the
answer file's numbers (data, not source). The topology must match it id for
id (the highest_id after each call), the device and oracle reductions its
values, and the located cell must hold the value.
"""
import math

import numpy as np
import pytest

from afh import capi
from afh.amr import DO_REF, RM_REF, AfTree
from afh.model import Tree

# afivo/tests/answers/test_reduction_3d: highest_id printed before call i,
# max after call i (the min is 3 throughout)
KAT_HIGHEST_ID = [1, 9, 17, 49, 105, 273, 713, 2033, 8545] + [49921] * 7
KAT_MAX = [6, 6, 8, 12, 20, 40, 76, 148, 292] + [292] * 7
KAT_MIN = 3.0


def kat_run(lib, device, n_iter):
    t = AfTree(8, [2 * math.acos(-1.0)] * 3, [8] * 3, periodic=(True,) * 3)

    def ref_func(ids):  # test_reduction.f90 ref_func, buffer 0
        f = [DO_REF if (np.all(t.r_min[b] < 0.4) and t.lvl[b] < 10) else RM_REF
             for b in ids]
        return np.array(f), np.zeros(len(ids), np.uint32)

    for i in range(n_iter):
        assert t.highest_id == KAT_HIGHEST_ID[i], i
        t.adjust_refinement(ref_func)
        topo = t.topology()
        tree = Tree(lib, topo, 1, 0, device=device)
        v = np.zeros(tree.cc_shape)
        s = topo["meta_ix"].sum(axis=1)  # set_values: sum(box%ix) on interiors
        v[:, 1:-1, 1:-1, 1:-1] = s[:, None, None, None]
        tree.put_cc(1, v)
        mx, lmax = tree.reduce_loc(1, capi.RED_MAX)
        mn, lmin = tree.reduce_loc(1, capi.RED_MIN)
        assert mx == KAT_MAX[i] and mn == KAT_MIN, (i, mx, mn)
        # "4 - max/min": the value at the located cell
        for val, (bid, ii, jj, kk) in ((mx, lmax), (mn, lmin)):
            assert v[bid - 1, kk, jj, ii] == val
            assert t.in_use[bid] and not t.has_children(bid)
        # the reference's loop order keeps the first box holding the value
        leaves = t.leaves()
        assert lmax[0] == next(b for b in leaves if s[b - 1] == mx)
        tree.close()
    return t


def test_reduction_kat_topology_oracle():
    """The whole KAT (16 calls, 49921 boxes) on the C oracle."""
    kat_run(capi.oracle_library(), -1, 16)


@pytest.mark.gpu
def test_reduction_kat_hip():
    kat_run(capi.hip_library(), 0, 16)


def sum_ref(topo, v, power):
    """af_tree_sum_cc restated with numpy: levels, then leaves."""
    s = 0.0
    for l in range(1, int(topo["highest_lvl"]) + 1):
        leaves = topo["lvl_leaves_%d" % l]
        if not len(leaves):
            continue
        dr = topo["meta_dr"][leaves[0] - 1]
        fac = dr[0] * dr[1] * dr[2]
        for b in leaves:
            s = s + fac * np.sum(v[b - 1, 1:-1, 1:-1, 1:-1] ** power)
    return s


def random_tree(lib, device, seed=1):
    from afh.tree import build_tree
    topo = build_tree(8, (16, 16, 16), (2e-3,) * 3, 2,
                      refine=lambda lvl, r0, r1: lvl < 4 and np.all(r0 < 1.1e-3))
    rng = np.random.default_rng(seed)
    tree = Tree(lib, topo, 2, 0, device=device)
    v = rng.standard_normal(tree.cc_shape) * 1e18
    tree.put_cc(2, v)
    return topo, tree, v


def check_sums_and_locs(lib, device):
    topo, tree, v = random_tree(lib, device)
    for p in (1, 2, 3):
        ref = sum_ref(topo, v, p)
        got = tree.sum_cc(2, p)
        assert abs(got - ref) <= 1e-12 * abs(ref) + 1e-300, (p, got, ref)
    leaves = [b for l in range(1, int(topo["highest_lvl"]) + 1)
              for b in topo["lvl_leaves_%d" % l]]
    for op, fn in ((capi.RED_MAX, np.argmax), (capi.RED_MIN, np.argmin),
                   (capi.RED_MAXABS, lambda a: np.argmax(np.abs(a)))):
        val, (bid, i, j, k) = tree.reduce_loc(2, op)
        # the first leaf (loop order) holding the extremum, first cell i fastest
        best = None
        for b in leaves:
            a = v[b - 1, 1:-1, 1:-1, 1:-1].ravel()  # k, j, i order = i fastest
            q = fn(a)
            x = abs(a[q]) if op == capi.RED_MAXABS else a[q]
            if best is None or (x < best[0] if op == capi.RED_MIN else x > best[0]):
                best = (x, b, q)
        x, b, q = best
        assert val == x and bid == b
        assert (i - 1) + 8 * (j - 1) + 64 * (k - 1) == q
    return tree


def test_sum_and_loc_oracle():
    check_sums_and_locs(capi.oracle_library(), -1)


@pytest.mark.gpu
def test_sum_and_loc_hip():
    check_sums_and_locs(capi.hip_library(), 0)


def test_retired_tree_after_in_place_regrid():
    """An in-place regrid hands the pools to the new tree: the old handle and
    a fluid bound to it fail with AFH_ERR_STATE (the oracle keeps the
    device library's contract)."""
    lib = capi.oracle_library()
    t = AfTree(8, [2e-3] * 3, [8] * 3)
    t.refine_up_to_lvl(2)
    old = Tree(lib, t.topology(), 2, 0, box_capacity=200)
    old.set_cc_methods(1, [(capi.BC_NEUMANN, 0.0)] * 6)
    old.set_cc_prolong(1, capi.PROLONG_LINEAR)
    t.refine_up_to_lvl(3)
    new = old.regrid(t.topology())
    with pytest.raises(capi.AfhError, match="retired"):
        old.get_cc(1)
    with pytest.raises(capi.AfhError, match="retired"):
        old.sum_cc(1)
    assert new.get_cc(1).shape[0] == t.highest_id
