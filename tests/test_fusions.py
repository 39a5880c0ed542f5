"""Round-3 launch fusions, each bitwise its unfused form (run-time switches
read at tree / multigrid / fluid creation):

* AFH_PAIR_PUSH: the small-box fused red-black pair writes the level's face
  ghosts itself (k_gsrb_pair_box PUSH) vs the pair + a level fill;
* AFH_CS_DIRECT_SMALL: the exact level-1 solve of a grid up to 1024 cells
  in one workgroup (k_cs_direct_small) vs gather + six transforms + scatter
  (on an 8^3 level-1 grid, streamer_3d.cfg's; S1's 16^3 runs the launches);
* AFH_UPD_NET: the compiled reaction network (afh_networks.h, k_update's
  unrolled reaction loop) vs the generic loop -- on the S3 tree with
  air_chemistry_v2 (9 species, 25 reactions) and on S1's old-style model;
* AFH_ALL_LVL: the small-box flux, the density update and the residual of
  every level in one launch (the box's grid spacing / coefficients from its
  level) vs one launch per level -- on the S3 tree (8 leaf levels).

Round 4:

* AFH_PROLONG_PUSH: the small-box correction (k_prolong_box) fills the
  level's faces itself vs k_prolong + a level fill;
* AFH_RSTR_PUSH: the small-box restriction pushes the coarse level's faces
  (k_rstr_box) and the parents' edges, corners and rhs come in one launch
  (k_parent_rhs_box) vs k_rstr_fas_col + a level fill + k_parent_rhs --
  on S1, on a tree of 8^3 boxes and on the S3 and S5 AMR trees (refinement
  boundaries on every level, physical faces);
* AFH2_GC_BOX: a 2-D level fill with corners in one workgroup per box
  (k2_gc_box) vs k2_gc + k2_corners;
* AFH2_ALL_LVL: the 2-D residual and gradient of every level in one launch
  vs one launch per level;
* AFH2_GRAPHS: 2-D V-cycles replayed from captured graphs vs eager;
* AFH2_CORNER_FOLD: the 2-D up leg's corners folded into the next correction;
* AFH2_GC_TREE_ONE: a 2-D tree fill without refinement boundaries in one launch.

The fused forms are also what every other GPU test runs (they are the
defaults); these tests pin them to the unfused forms on full workloads.
(Round 5 removed the switches of forms measured slower or neutral, with
their tests: the x ghost cells in the 64^3 pair, the pair and fill
geometry experiments, and the 2-D packing / fitted workgroups / shuffled
flux / any-count update; the kept forms are the defaults these tests ran
against.)
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _s1(monkeypatch, env, config="s1", phi_faces=False):
    import bench
    from afh import capi
    from afh.streamer import IV
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    c = bench.build_case(capi.hip_library(), config, 0, 0)
    c.fuse_rhs(True, ghosts=False)
    if phi_faces:
        c.faces_from_phi(True)
    out = {"res0": c.field_compute(0, n_vcycles=2)}
    for k in range(4):
        out["step%d" % k] = bench.unit_step(c, 1e-13, k)
    for v in ("e", "pos", "neg", "phi", "efld", "rhs", "tmp"):
        out[v] = c.tree.get_cc(IV[v])
    c.tree.close()
    return out


def _same(a, b):
    for k in a:
        if isinstance(a[k], np.ndarray):
            assert np.array_equal(a[k], b[k]), (k, np.nanmax(np.abs(a[k] - b[k])))
        else:
            assert a[k] == b[k], (k, a[k], b[k])


@pytest.mark.parametrize("switch", ["AFH_PAIR_PUSH", "AFH_CS_DIRECT_SMALL",
                                    "AFH_UPD_NET", "AFH_ALL_LVL", "AFH_PROLONG_PUSH",
                                    "AFH_RSTR_PUSH"])
def test_s1_fusion_bitwise(switch, monkeypatch):
    """Config 2 (S1: 512 leaf boxes of 16^3, 4 levels): field solve and four
    unit steps with the fusion on and off."""
    # AFH_UPD_NET=2: the compiled network must match (S1's old-style model)
    a = _s1(monkeypatch, {switch: "2" if switch == "AFH_UPD_NET" else "1"})
    b = _s1(monkeypatch, {switch: "0"})
    _same(a, b)


@pytest.mark.parametrize("k", ["2", "8"])
def test_s1_restriction_columns_bitwise(k, monkeypatch):
    """k_rstr_fas_col with columns of 2 and 8 coarse cells (S1's 16^3 boxes:
    one column per (i, j) at 8) against the default 4 and the one-cell form
    (AFH_RSTR_COL=0): the same operand order, so bitwise."""
    a = _s1(monkeypatch, {"AFH_RSTR_K": k})
    b = _s1(monkeypatch, {"AFH_RSTR_K": "4"})
    _same(a, b)
    c = _s1(monkeypatch, {"AFH_RSTR_COL": "0"})
    _same(a, c)


@pytest.mark.parametrize("k", ["2", "8"])
def test_s1_residual_columns_bitwise(k, monkeypatch):
    """k_residual with columns of 2 and 8 cells against 4 (S1's 16^3 boxes):
    the residuals and their maximum are per-cell values, so bitwise."""
    _same(_s1(monkeypatch, {"AFH_RES_K": k}), _s1(monkeypatch, {"AFH_RES_K": "4"}))


@pytest.mark.parametrize("k", ["2", "8"])
def test_s1_prolong_columns_bitwise(k, monkeypatch):
    """k_prolong with columns of 2 and 8 cells (AFH_PROLONG_K, read when the
    multigrid is created) against 4."""
    _same(_s1(monkeypatch, {"AFH_PROLONG_K": k}), _s1(monkeypatch, {"AFH_PROLONG_K": "4"}))


def test_direct_small_bitwise_8cubed(monkeypatch):
    """k_cs_direct_small on an 8^3 level-1 grid (one box, 3 levels of 8^3
    boxes): field solve and four unit steps, one workgroup vs the launches."""
    import bench
    monkeypatch.setitem(bench.CONFIGS, "c8", (8, (8, 8, 8), 3, (8e-3, 8e-3, 8e-3)))
    a = _s1(monkeypatch, {"AFH_CS_DIRECT_SMALL": "1"}, "c8")
    b = _s1(monkeypatch, {"AFH_CS_DIRECT_SMALL": "0"}, "c8")
    _same(a, b)


@pytest.mark.parametrize("config", ["c16x8"])
def test_direct_small_bitwise_lines(config, monkeypatch):
    """k_cs_direct_small, one thread per grid line (the line in registers,
    the matrix entries wave-uniform), on a 16 x 8 x 8 level-1 grid of two
    boxes (lines of different lengths per dimension): bitwise the gather +
    six transforms + scatter."""
    import bench
    monkeypatch.setitem(bench.CONFIGS, "c16x8", (8, (16, 8, 8), 3, (16e-3, 8e-3, 8e-3)))
    a = _s1(monkeypatch, {"AFH_CS_DIRECT_SMALL": "1"}, config)
    b = _s1(monkeypatch, {"AFH_CS_DIRECT_SMALL": "0"}, config)
    _same(a, b)


def test_s3_all_level_launches_bitwise(monkeypatch):
    """Config 3: two unit steps (field solve with its residuals, flux,
    update with the chemistry limit) with every leaf level in one launch and
    with one launch per level."""
    import bench
    from afh import capi
    outs = []
    for v in ("1", "0"):
        monkeypatch.setenv("AFH_ALL_LVL", v)
        case = bench.DriverCase(bench.build_driver_case(capi.hip_library(), 0, "s3"))
        case.fuse_rhs(True, ghosts=False)
        res = [bench.unit_step(case, 1e-13, k) for k in range(2)]
        sim = case.sim
        outs.append((res, [sim.tree.get_cc(iv) for iv in range(1, sim.n_var_cell + 1)]))
    assert outs[0][0] == outs[1][0]
    for x, y in zip(outs[0][1], outs[1][1]):
        assert np.array_equal(x, y, equal_nan=True)


def _case2d(monkeypatch, env, config):
    import bench
    from afh import capi
    from afh.streamer import IV
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    c = bench.build_case(capi.hip_library_2d(), config, 0, 0)
    out = {"res0": c.field_compute(0, n_vcycles=2)}
    for k in range(4):
        out["step%d" % k] = bench.unit_step(c, 1e-13, k)
    for v in ("e", "pos", "neg", "phi", "efld", "rhs", "tmp"):
        out[v] = c.tree.get_cc(IV[v])
    c.tree.close()
    return out


@pytest.mark.parametrize("config", ["2d-uniform", "c2d16"])
def test_2d_pair_bitwise(config, monkeypatch):
    """The 2-D fused pair with its pushed fills (k2_pair_box, AFH_PAIR2D)
    against the split half-sweeps + level fills: BASELINE config 1's bench
    tree (8 levels of 8^2 boxes) and a 16^2-box tree; field solves and four
    unit steps, every variable bitwise."""
    import bench
    monkeypatch.setitem(bench.CONFIGS, "c2d16", (16, (16, 16), 4, (16e-3, 16e-3)))
    _same(_case2d(monkeypatch, {"AFH_PAIR2D": "1"}, config),
          _case2d(monkeypatch, {"AFH_PAIR2D": "0"}, config))


@pytest.mark.parametrize("config", ["2d-uniform", "c2d16"])
def test_2d_gc_box_bitwise(config, monkeypatch):
    """2-D level fills with corners in one launch (k2_gc_box, AFH2_GC_BOX,
    several small boxes per workgroup) against k2_gc + k2_corners: field
    solves and four unit steps."""
    import bench
    monkeypatch.setitem(bench.CONFIGS, "c2d16", (16, (16, 16), 4, (16e-3, 16e-3)))
    packed = _case2d(monkeypatch, {"AFH2_GC_BOX": "1"}, config)
    _same(packed, _case2d(monkeypatch, {"AFH2_GC_BOX": "0"}, config))


@pytest.mark.parametrize("config", ["2d-uniform", "c2d16"])
def test_2d_all_level_launches_bitwise(config, monkeypatch):
    """2-D residual and gradient of every level in one launch (the box's
    level coefficients / spacing from its meta; AFH2_ALL_LVL) against one
    launch per level: field solves and four unit steps."""
    import bench
    monkeypatch.setitem(bench.CONFIGS, "c2d16", (16, (16, 16), 4, (16e-3, 16e-3)))
    _same(_case2d(monkeypatch, {"AFH2_ALL_LVL": "1"}, config),
          _case2d(monkeypatch, {"AFH2_ALL_LVL": "0"}, config))


@pytest.mark.parametrize("config", ["2d-uniform", "c2d16"])
def test_2d_vcycle_graphs_bitwise(config, monkeypatch):
    """2-D V-cycles replayed from captured hipGraphs (AFH2_GRAPHS) against
    eager launches: field solves (the first V-cycle of a variant eager, the
    next captured) and four unit steps, every variable bitwise."""
    import bench
    monkeypatch.setitem(bench.CONFIGS, "c2d16", (16, (16, 16), 4, (16e-3, 16e-3)))
    _same(_case2d(monkeypatch, {"AFH2_GRAPHS": "1"}, config),
          _case2d(monkeypatch, {"AFH2_GRAPHS": "0"}, config))


@pytest.mark.parametrize("config", ["2d-uniform", "c2d16"])
def test_2d_corner_fold_bitwise(config, monkeypatch):
    """The up leg's corner pass after the 2-D pair folded into the next
    level's correction (k2_block_corners, AFH2_CORNER_FOLD, the default)
    against k2_corners: field solves and four unit steps, every variable
    (ghost cells included) bitwise."""
    import bench
    monkeypatch.setitem(bench.CONFIGS, "c2d16", (16, (16, 16), 4, (16e-3, 16e-3)))
    _same(_case2d(monkeypatch, {"AFH2_CORNER_FOLD": "1"}, config),
          _case2d(monkeypatch, {"AFH2_CORNER_FOLD": "0"}, config))


@pytest.mark.parametrize("config", ["2d-uniform", "c2d16"])
def test_2d_gc_tree_one_launch_bitwise(config, monkeypatch):
    """afh_gc_tree of a tree without refinement boundaries as one launch over
    every level (AFH2_GC_TREE_ONE, the default) against level by level: field
    solves and four unit steps, every variable bitwise."""
    import bench
    monkeypatch.setitem(bench.CONFIGS, "c2d16", (16, (16, 16), 4, (16e-3, 16e-3)))
    _same(_case2d(monkeypatch, {"AFH2_GC_TREE_ONE": "1"}, config),
          _case2d(monkeypatch, {"AFH2_GC_TREE_ONE": "0"}, config))


@pytest.mark.parametrize("switch", ["AFH_PROLONG_PUSH", "AFH_RSTR_PUSH"])
def test_push_bitwise_8cubed(switch, monkeypatch):
    import bench
    monkeypatch.setitem(bench.CONFIGS, "c8", (8, (8, 8, 8), 3, (8e-3, 8e-3, 8e-3)))
    _same(_s1(monkeypatch, {switch: "1"}, "c8"), _s1(monkeypatch, {switch: "0"}, "c8"))


@pytest.mark.parametrize("config", ["s3", "s5"])
def test_push_bitwise_amr(config, monkeypatch):
    """Configs 3 and 5: four unit steps (field solves, flux, update) with
    the pushing correction and restriction on and both off."""
    import bench
    from afh import capi
    outs = []
    for v in ("1", "0"):
        monkeypatch.setenv("AFH_PROLONG_PUSH", v)
        monkeypatch.setenv("AFH_RSTR_PUSH", v)
        case = bench.DriverCase(bench.build_driver_case(capi.hip_library(), 0, config))
        case.fuse_rhs(True, ghosts=False)
        res = [bench.unit_step(case, 1e-13, k) for k in range(4)]
        sim = case.sim
        outs.append((res, [sim.tree.get_cc(iv) for iv in range(1, sim.n_var_cell + 1)]))
    assert outs[0][0] == outs[1][0]
    for x, y in zip(outs[0][1], outs[1][1]):
        assert np.array_equal(x, y, equal_nan=True)


def test_s3_compiled_network_bitwise(monkeypatch):
    """Config 3's chemistry: the species step on the S3 tree with the
    compiled air_chemistry_v2 network, bitwise the generic reaction loop
    (both Heun stages, the chemistry time-step limit)."""
    import golden
    from afh import capi
    from afh.driver import Simulation
    outs = []
    for net in ("2", "0"):  # 2: the compiled network must match
        monkeypatch.setenv("AFH_UPD_NET", net)
        sim = Simulation(capi.hip_library(), golden.load("case_s3"), device=0)
        sim.set_initial_conditions()
        lims = [list(sim.fluid.forward_euler(1e-12, 0, [0], [1.0], 1, False)),
                list(sim.fluid.forward_euler(5e-13, 1, [0, 1], [0.5, 0.5], 0, True))]
        states = [sim.tree.get_cc(iv + s) for iv in sim.densities for s in (0, 1)]
        outs.append((lims, states))
    assert outs[0][0] == outs[1][0]
    for x, y in zip(outs[0][1], outs[1][1]):
        assert np.array_equal(x, y)


@pytest.mark.parametrize("config", ["s1", "c32"])
def test_gradient_folded_into_residual_bitwise(config, monkeypatch):
    """afh_mg_set_gradient_output: |E| from the V-cycle's final residual pass
    (one read of phi for both) against field_from_potential's own gradient
    pass -- the field solve and four unit steps (16^3 and 32^3 boxes: residual
    columns of 4 and 8), every variable bitwise."""
    import bench
    from afh import capi
    from afh.streamer import IV
    monkeypatch.setitem(bench.CONFIGS, "c32", (32, (32, 32, 32), 3, (8e-3, 8e-3, 8e-3)))
    outs = []
    for fold in (True, False):
        c = bench.build_case(capi.hip_library(), config, 0, 0)
        c.fuse_rhs(True, ghosts=False)
        c.faces_from_phi(True)
        if not fold:
            c.mg.set_gradient_output(0)
        out = {"res0": c.field_compute(0, n_vcycles=2)}
        for k in range(4):
            out["step%d" % k] = bench.unit_step(c, 1e-13, k)
        for v in ("e", "pos", "neg", "phi", "efld", "rhs", "tmp"):
            out[v] = c.tree.get_cc(IV[v])
        c.tree.close()
        outs.append(out)
    _same(outs[0], outs[1])

@pytest.mark.parametrize("config,cgs,dom", [
    ("c64", (64, 64, 64), (8e-3, 8e-3, 8e-3)),
    ("c64y", (64, 128, 64), (8e-3, 16e-3, 8e-3))])
def test_dpair_bitwise_64cubed(config, cgs, dom, monkeypatch):
    """Two red-black iterations in one pass (k_gsrb_dpair, AFH_GSRB_DPAIR) vs
    two fused pairs with the level fill between: 64^3 boxes, three levels,
    the dpair on the top level of 64 (128) boxes (AFH_GSRB_DPAIR_MIN=64);
    halos from face, edge and corner neighbours and the physical faces'
    ghosts formed in the kernel (Dirichlet z, Neumann x / y). Field solve
    and four unit steps bitwise."""
    import bench
    monkeypatch.setitem(bench.CONFIGS, config, (64, cgs, 3, dom))
    monkeypatch.setenv("AFH_GSRB_DPAIR_MIN", "64")
    a = _s1(monkeypatch, {"AFH_GSRB_DPAIR": "1"}, config)
    b = _s1(monkeypatch, {"AFH_GSRB_DPAIR": "0"}, config)
    _same(a, b)


def test_dpair_bitwise_s1_64(monkeypatch):
    """The same on the headline tree (S1-64: the 512 leaf boxes of 64^3, the
    default dpair level)."""
    a = _s1(monkeypatch, {"AFH_GSRB_DPAIR": "1"}, "s1-64")
    b = _s1(monkeypatch, {"AFH_GSRB_DPAIR": "0"}, "s1-64")
    _same(a, b)


@pytest.mark.parametrize("config", ["s1-64", "s1"])
def test_fused_species_step_bitwise(config, monkeypatch):
    """The fused forward-Euler species step (k_fe_lds: flux + update in one
    plane march; AFH_FE_FUSED=2: every eligible step, both Heun stages; the
    default runs it for the first) as the bench runs it -- face fields from
    phi, rhs folded into the update, the compiled 3-species network -- against
    k_flux_lds + k_update: field solve and four unit steps (both Heun stages,
    the chemistry limit on the second), every variable and every returned
    limit bitwise. S1 (16^3 boxes) exercises the 16^3 tiles of the kernel."""
    a = _s1(monkeypatch, {"AFH_FE_FUSED": "2"}, config, phi_faces=True)
    b = _s1(monkeypatch, {"AFH_FE_FUSED": "0"}, config, phi_faces=True)
    _same(a, b)


def _s5_steps(monkeypatch, conc, steps=12):
    import bench
    from afh import capi
    monkeypatch.setenv("AFH_HELMH_CONC", conc)
    sim = bench.build_driver_case(capi.hip_library(), 0, "s5", "pfmg")
    case = bench.DriverCase(sim)
    case.fuse_rhs(True, ghosts=False)
    case.field_compute(0)
    res = [bench.unit_step(case, 1e-13, k) for k in range(steps)]
    sim.photoi_set_src()
    out = {"res": str(res), "n_var_tree": sim.n_var_tree}
    for iv in range(1, sim.n_var_cell + 1):
        if iv not in (sim.i_rhs, sim.i_tmp):  # (scratch of the last solve)
            out["cc%d" % iv] = sim.tree.get_cc(iv)
    sim.tree.close()
    return out


def test_helmholtz_modes_concurrent_bitwise(monkeypatch):
    """S5's Bourdon-3 Helmholtz modes solved concurrently (one side stream
    each, their own rhs / tmp / spare image: AFH_HELMH_CONC, the default) vs
    one after another on the shared variables: every variable of the
    reference's list bitwise after twelve unit steps (photoionization every
    photoi%per_steps steps) and one more photoi_set_src."""
    a = _s5_steps(monkeypatch, "1")
    b = _s5_steps(monkeypatch, "0")
    assert a["n_var_tree"] == b["n_var_tree"] + 4
    a.pop("n_var_tree"), b.pop("n_var_tree")
    _same(a, b)
