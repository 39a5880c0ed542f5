"""Host electrode operators (afh.electrode) against the reference's own: the
rod8 fixture holds, for the rod electrode of oracle/harness/golden_gen.f90
(r0 = (0.5, 0.5, 1) L, r1 = (0.5, 0.5, 0.6) L, radius 0.1 L), the lsf cell
values set_lsf_box wrote and the stencils afivo's mg_set_operators_tree
stored (mg_box_lsf_stencil, bc_correction, the distance stencil), dumped by
the compiled reference (oracle/make_golden.py read_lsf)."""
import numpy as np

import golden
from afh import electrode


def _rod8():
    g = golden.load("rod8")
    L = np.asarray(g["domain"], float)
    f = electrode.RodLSF(np.array([0.5, 0.5, 1.0]) * L, np.array([0.5, 0.5, 0.6]) * L,
                         0.1 * L[2])
    return g, f


def test_lsf_cell_values_match_reference():
    g, f = _rod8()
    nc = int(g["nc"])
    ref = g["init__lsf"]
    for b in range(int(g["n_boxes"])):
        r = electrode.cell_centers(g["meta_r_min"][b], g["meta_dr"][b], nc, 0, nc + 1)
        assert np.array_equal(f(r), ref[b]), b


def test_box_operators_match_reference():
    g, f = _rod8()
    nc = int(g["nc"])
    v_ids = [int(x) for x in g["lsf_v_ids"]]
    d_ids = [int(x) for x in g["lsf_d_ids"]]
    ref_st, ref_d = golden.electrode_stencils(g)
    v0 = float(g["current_voltage"])
    found = []
    for b in range(int(g["n_boxes"])):
        lsf = g["init__lsf"][b][1:-1, 1:-1, 1:-1]
        op = electrode.box_operators(f, lsf, g["meta_r_min"][b], g["meta_dr"][b], nc, v0)
        if op is None:
            assert b + 1 not in v_ids
            continue
        found.append(b + 1)
        v, fb, ix, dd = op
        rv, rbcc = ref_st[b + 1]
        assert np.array_equal(v, rv), b + 1
        assert np.array_equal(fb, rbcc if rbcc is not None else np.zeros_like(fb)), b + 1
        rix, rdd, rbv = ref_d[b + 1]
        assert np.array_equal(ix, rix) and np.array_equal(dd, rdd), b + 1
        assert np.all(rbv == v0)
    assert found == v_ids == d_ids
