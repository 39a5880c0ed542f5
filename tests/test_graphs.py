"""V-cycles replayed as captured hipGraphs (launch amortisation in
afh_mg_fas_vcycle*): bitwise the eager launches, across regrids (new trees,
new graphs) and boundary-condition changes (afh_set_cc_methods and
afh_set_bc drop the captured graph)."""
import os

import numpy as np
import pytest

import golden
from afh import capi
from afh.driver import Simulation


def _run(graphs, steps=6):
    old = os.environ.get("AFH_GRAPHS")
    os.environ["AFH_GRAPHS"] = "1" if graphs else "0"
    try:
        sim = Simulation(capi.hip_library(), golden.load("rtest_test_3d"), device=0)
        sim.start()
        for _ in range(steps):
            sim.step()
        # a new applied voltage: the captured V-cycle must not replay the old
        # boundary values
        sim.voltage *= 1.25
        sim.tree.set_cc_methods(sim.i_phi, sim.phi_bc(), capi.RB_MG_SIDES)
        res = sim.field_compute(0, True)
        res += sim.field_compute(0, True)
        # the same through afh_set_bc (field_set_voltage's route,
        # INTEGRATION.md): a value change, then a type change (the coarse
        # solve's tables follow the types) and back
        sim.voltage *= 0.5
        sim.tree.set_bc(sim.i_phi, 6, capi.BC_DIRICHLET, sim.voltage)
        res += sim.field_compute(0, True)
        res += sim.field_compute(0, True)
        sim.tree.set_bc(sim.i_phi, 1, capi.BC_DIRICHLET, 0.0)
        res += sim.field_compute(0, True)
        res += sim.field_compute(0, True)
        sim.tree.set_bc(sim.i_phi, 1, capi.BC_NEUMANN, 0.0)
        res += sim.field_compute(0, True)
        res += sim.field_compute(0, True)
    finally:
        if old is None:
            os.environ.pop("AFH_GRAPHS")
        else:
            os.environ["AFH_GRAPHS"] = old
    return sim, np.array(sim.log), res


@pytest.mark.gpu
def test_graph_vcycles_bitwise_eager():
    a, la, ra = _run(True)
    b, lb, rb = _run(False)
    assert np.array_equal(la, lb)
    assert ra == rb
    for iv in (a.i_phi, a.i_efld, a.i_electron):
        assert np.array_equal(a.tree.get_cc(iv), b.tree.get_cc(iv))
