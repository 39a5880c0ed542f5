"""The weighted Morton split of a partition frontier (afh.dist.Partition,
afh_dist_core.h partition(); SURVEY.md 8(e): "a level-by-level Morton sort,
weighted by cells"; the reference spreads every level's boxes over its
workers, afivo/src/m_af_multigrid.f90:666-687).

On the AMR trees of BASELINE configs 4 and 5 (the reference's
set_initial_conditions, rebuilt on the C oracle) the leaf boxes per rank at
N = 8 stay within 1.15 of the mean (round 3's partition, whole subtrees of
the first level with a box per rank: S5 2.90, S4 1.75). The native partition
and every exchange plan equal the Python statement on those trees, with
frontiers that span several levels.
"""
import numpy as np
import pytest

import golden
from afh import capi
from afh.dist import NativeShard, Partition

_TREES = {}


def tree(cfg):
    """The topology after set_initial_conditions (cached per session)."""
    if cfg not in _TREES:
        from afh.driver import Simulation
        from afh.users import USERS
        sim = Simulation(capi.oracle_library(), golden.load("case_" + cfg),
                         user=USERS.get(cfg))
        sim.set_initial_conditions()
        _TREES[cfg] = sim.af.topology()
        sim.tree.close()
    return _TREES[cfg]


def leaf_loads(topo, owner, n):
    leaves = np.concatenate([topo["lvl_leaves_%d" % l]
                             for l in range(1, int(topo["highest_lvl"]) + 1)]).astype(np.int64)
    o = np.asarray(owner)[leaves - 1]
    return np.bincount(o[o >= 0], minlength=n)


@pytest.mark.parametrize("cfg", ["s4", "s5"])
@pytest.mark.parametrize("n", [2, 4, 8])
def test_leaf_balance(cfg, n):
    topo = tree(cfg)
    part = Partition(topo, n)
    loads = leaf_loads(topo, part.owner, n)
    assert loads.min() > 0
    assert loads.max() / loads.mean() <= 1.15, (cfg, n, loads.tolist())
    # descendants follow their frontier box; replicated boxes are ancestors
    # of frontier boxes (or level 1), never leaves below level 1
    lvl, par = np.asarray(topo["meta_lvl"]), np.asarray(topo["meta_parent"])
    for b in range(1, int(topo["n_boxes"]) + 1):
        if lvl[b - 1] < 1:
            continue
        o = part.owner[b - 1]
        if lvl[b - 1] >= 2 and part.owner[par[b - 1] - 1] >= 0:
            assert o == part.owner[par[b - 1] - 1]
        if o < 0 and lvl[b - 1] >= 2:
            assert topo["meta_children"][b - 1][0] > 0


def test_uniform_tree_split_unchanged():
    """On a uniform tree the first frontier is balanced: whole level-2
    subtrees in Morton chunks, nothing replicated below level 2 (8 coarse
    boxes, 64 on level 2: 8 level-2 subtrees per rank)."""
    from afh.tree import uniform_tree
    topo = uniform_tree(8, (16, 16, 16), (2e-3, 2e-3, 2e-3), 4)
    part = Partition(topo, 8)
    lvl = np.asarray(topo["meta_lvl"])
    assert part.lp == 2
    assert np.all(part.owner[lvl == 1] < 0) and np.all(part.owner[lvl >= 2] >= 0)
    assert np.bincount(part.owner[lvl == 2], minlength=8).tolist() == [8] * 8


@pytest.mark.parametrize("cfg,n", [("s5", 8), ("s4", 8), ("s5", 3)])
def test_native_partition_equals_python(cfg, n):
    topo = tree(cfg)
    part = Partition(topo, n)
    sh = NativeShard(capi.oracle_library(), topo, n, 0, transport=capi.DIST_LOCAL,
                     group=type("G", (), {"h": None})())
    np.testing.assert_array_equal(sh.owner, part.owner)
    assert sh.lp == part.lp


def test_native_plans_equal_python_mixed_frontier():
    """Every plan of S5 over 3 ranks (HALO / RIMS on every level, CFLUX,
    RESTRICT on every level with owned boxes under replicated parents)."""
    from test_dist_native import KINDS, _python_regions
    topo = tree("s5")
    n = 3
    part = Partition(topo, n)
    assert len(part.restrict_levels()) >= 1
    sh = NativeShard(capi.oracle_library(), topo, n, 0, transport=capi.DIST_LOCAL,
                     group=type("G", (), {"h": None})())
    n_regions = 0
    for kind in KINDS:
        levels = [0] if kind == capi.HOOK_CFLUX else range(1, part.nlvl + 1)
        for level in levels:
            for recv in range(n):
                for send in range(n):
                    if recv == send:
                        continue
                    got = sh.plan(kind, level, recv, send)
                    want = _python_regions(part, kind, level, recv, send)
                    np.testing.assert_array_equal(got, want,
                                                  err_msg=str((kind, level, recv, send)))
                    n_regions += len(got)
    assert n_regions > 0


def test_compact_topology_ids():
    """dist.compact_topology (the rank-local regrid's small trees): boxes of
    a shared id space keep their positions, references to boxes outside the
    set point to the one unused id, physical / refinement boundaries (<= 0)
    stay, and the oracle builds a tree from it."""
    from afh.dist import compact_topology
    from afh.model import Tree
    topo = tree("s5")
    nb = int(topo["n_boxes"])
    lvl = np.asarray(topo["meta_lvl"])
    used = np.nonzero(lvl > 0)[0] + 1
    rng = np.random.default_rng(3)
    present = np.sort(rng.choice(used, size=len(used) // 3, replace=False))
    extra = np.setdiff1d(used, present)[:25]
    space = np.union1d(present, extra)
    c = compact_topology(topo, present, space)
    n = len(space)
    assert int(c["n_boxes"]) == n + 1
    pos = {int(b): k for k, b in enumerate(space)}
    inset = set(int(b) for b in present)
    nbr, cnb = np.asarray(topo["meta_neighbors"]), np.asarray(c["meta_neighbors"])
    for b in present:
        k = pos[int(b)]
        assert c["meta_lvl"][k] == lvl[b - 1]
        for q in range(6):
            g = nbr[b - 1][q]
            want = g if g <= 0 else (pos[g] + 1 if g in inset else n + 1)
            assert cnb[k][q] == want
    for b in extra:  # in the id space, not present: holes
        assert c["meta_lvl"][pos[int(b)]] == 0
    for l in range(1, int(topo["highest_lvl"]) + 1):
        ids = np.asarray(topo["lvl_ids_%d" % l])
        want = [pos[int(b)] + 1 for b in ids if int(b) in inset]
        assert list(c["lvl_ids_%d" % l]) == want
    t = Tree(capi.oracle_library(), c, 3, 1)
    assert t.n_boxes == n + 1
    t.close()
    assert nb > n


@pytest.mark.parametrize("cfg,n,cells", [("s5", 8, 64 * 512), ("s5", 3, 100 * 512),
                                         ("s4", 8, 150 * 512), ("s5", 8, 10 ** 9)])
def test_native_partition_levels_equals_python(cfg, n, cells):
    """The size floor (round 6): the frontier starts at the first level of at
    least `cells` cells; everything below it is replicated, leaves included;
    no such level: the whole tree replicated (lp None)."""
    topo = tree(cfg)
    part = Partition(topo, n, min_level_cells=cells)
    sh = NativeShard(capi.oracle_library(), topo, n, 0, transport=capi.DIST_LOCAL,
                     group=type("G", (), {"h": None})(), min_level_cells=cells)
    np.testing.assert_array_equal(sh.owner, part.owner)
    assert sh.lp == part.lp
    lvl = np.asarray(topo["meta_lvl"])
    nc3 = int(topo["nc"]) ** 3
    big = [l for l in range(2, int(topo["highest_lvl"]) + 1)
           if np.sum(lvl == l) * nc3 >= cells and np.sum(lvl == l) >= n]
    if not big:
        assert part.lp is None and np.all(part.owner < 0)
        return
    assert part.lp >= big[0]
    assert np.all(part.owner[(lvl >= 1) & (lvl < big[0])] < 0)
    loads = leaf_loads(topo, part.owner, n)
    assert loads.min() > 0


def test_uniform_tree_levels_floor():
    """A uniform tree of 8^3 boxes (8, 64, 512, 4096 per level) with a floor
    above level 2's cells: levels 1-2 replicated, the frontier on level 3
    (512 boxes, 64 per rank)."""
    from afh.tree import uniform_tree
    topo = uniform_tree(8, (16, 16, 16), (2e-3, 2e-3, 2e-3), 4)
    part = Partition(topo, 8, min_level_cells=65 * 512)
    lvl = np.asarray(topo["meta_lvl"])
    assert part.lp == 3
    assert np.all(part.owner[lvl <= 2] < 0) and np.all(part.owner[lvl >= 3] >= 0)
    assert np.bincount(part.owner[lvl == 3], minlength=8).tolist() == [64] * 8
