"""The streamer time step over the C ABI (src/streamer.f90 + m_fluid + m_field).

``StreamerCase`` registers variables in the order the streamer does
(species with num_steps+1 copies, phi with 2, electric_fld, rhs, tmp;
src/m_chemistry.f90:262-270, src/m_streamer.f90:237-302), sets the
ghost-cell methods of streamer.f90:81-84 / m_field.f90:349-350, and exposes
field_compute (m_field.f90:405-485), forward_euler (m_fluid.f90:21-99) and a
Heun step (af_advance, afivo/src/m_af_advance.f90:160-164).
"""
import math
import os

import numpy as np

from . import capi
from .model import Fluid, Multigrid, Tree

# cc / fc variable indices (1-based, as af_add_cc_variable assigns them)
IV = {"e": 1, "pos": 4, "neg": 7, "phi": 10, "phi_2": 11, "efld": 12,
      "rhs": 13, "tmp": 14}
N_VAR_CELL = 14
FV = {"flux": 1, "field": 2}
N_VAR_FACE = 2

UC_EPS0 = 8.8541878176e-12
UC_ELEM_CHARGE = 1.6022e-19
UC_BOLTZMANN = 1.3806503e-23


def standard_reactions():
    """Old-style transport data model, src/m_chemistry.f90:205-239."""
    return [
        {"rate_type": capi.RATE_TABULATED_FIELD, "table_col": 1,
         "rate_factor": 1.0, "ix_in": [1], "ix_out": [1, 2],
         "mult_out": [2, 1]},  # e + M -> e + e + M+
        {"rate_type": capi.RATE_TABULATED_FIELD, "table_col": 2,
         "rate_factor": 1.0, "ix_in": [1], "ix_out": [3],
         "mult_out": [1]},  # e + M -> M-
    ]


def gas_number_density(pressure_bar=1.0, temperature=300.0):
    """Ideal gas law, src/m_gas.f90:174-176."""
    return 1e5 * pressure_bar / (UC_BOLTZMANN * temperature)


def tables_from(golden):
    td = {"rows_cols": golden["td_rows_cols"], "x_min": golden["td_xmin"],
          "inv_fac": golden["td_inv_fac"]}
    chem = {"rows_cols": golden["chem_rows_cols"], "x_min": golden["chem_xmin"],
            "inv_fac": golden["chem_inv_fac"]}
    return td, chem


class StreamerCase:
    """One streamer simulation state on a tree, driven through `lib`."""

    def __init__(self, lib, topo, td, chem, voltage, n_gas=None,
                 coarse_cycles=20, device=-1, shard=None, n_var_cell=N_VAR_CELL,
                 box_capacity=0, coarse_mode=None, coarse_tol=0.0):
        """shard: an afh.dist.Shard or NativeShard -- this rank's part of a sharded tree
        (the tree is created from the rank's level lists and the exchange
        hooks are attached); None for a single-rank tree."""
        self.lib = lib
        self.topo = topo
        self.shard = shard
        if shard:
            self.tree = shard.make_tree(lib, topo, n_var_cell, N_VAR_FACE, device=device,
                                        box_capacity=box_capacity)
        else:
            self.tree = Tree(lib, topo, n_var_cell, N_VAR_FACE, device=device,
                             box_capacity=box_capacity)
        t = self.tree
        self.ndim = t.ndim
        neumann0 = [(capi.BC_NEUMANN, 0.0)] * (2 * self.ndim)
        for sp in ("e", "pos", "neg"):
            for s in range(3):
                # the default prolong_limiter (streamer.f90:81-84 passes
                # none): MC in 2-D, gminmod43 in 3-D
                t.set_cc_methods(IV[sp] + s, neumann0, capi.RB_GC_INTERP_LIM)
        t.set_cc_methods(IV["efld"], neumann0, capi.RB_GC_INTERP)
        self.voltage = voltage
        for s in (0, 1):
            t.set_cc_methods(IV["phi"] + s, self.phi_bc(voltage, self.ndim), capi.RB_MG_SIDES)
        self.coarse_cycles = coarse_cycles
        # coarse_mode=capi.COARSE_PFMG: the reference's HYPRE PFMG restated
        # (coarse_cycles iterations at most, to coarse_tol)
        self.coarse_mode, self.coarse_tol = coarse_mode, coarse_tol
        self.i_lsf = 0  # level-set variable of an electrode (set_electrode)
        # keep the face fluxes of the species step in FV["flux"] (the fused
        # device step otherwise leaves them on chip)
        self.store_flux = False
        self._fused_rhs = False  # afh_fluid_set_rhs_output active
        self._faces_from_phi = False  # afh_fluid_set_field_source active
        # field_compute(defer=True): the residual list the next species_step
        # fills (AFH_DEFER=0 turns deferral off, for A/B runs)
        self._deferred_res = None
        # (the 2-D library has them since round 4, afivo_hip_2d.h)
        self._defer_ok = (os.environ.get("AFH_DEFER", "1") != "0" and
                          (self.ndim == 3 or lib.has("fluid_fetch_step")))
        self.mg = Multigrid(t, IV["phi"], IV["rhs"], IV["tmp"],
                            coarse_cycles=coarse_cycles, coarse_mode=coarse_mode,
                            coarse_tol=coarse_tol)
        self._mg_helm = {}
        self.n_gas = gas_number_density() if n_gas is None else n_gas
        self.fluid = Fluid(t, [IV["e"], IV["pos"], IV["neg"]], [-1, 1, -1],
                           IV["e"], IV["efld"], FV["flux"], FV["field"],
                           self.n_gas, td, chem, standard_reactions())
        self.domain = np.asarray(topo["domain"], float)
        if shard:
            shard.attach(self.tree)

    @staticmethod
    def phi_bc(voltage, ndim=3):
        """field_bc_homogeneous, src/m_field.f90:547-567: Dirichlet 0 / V on
        the faces of the last dimension, Neumann 0 elsewhere."""
        return [(capi.BC_NEUMANN, 0.0)] * (2 * ndim - 2) + [(capi.BC_DIRICHLET, 0.0),
                                                              (capi.BC_DIRICHLET, voltage)]

    def helmholtz_mg(self, lambda2):
        """mg_t of a photoionization Helmholtz mode on phi / rhs / tmp
        (m_photoi_helmh.f90:149-158): helmholtz_lambda = lambda^2, same
        coarse solver as the field; created once per lambda^2."""
        if lambda2 not in self._mg_helm:
            self._mg_helm[lambda2] = Multigrid(
                self.tree, IV["phi"], IV["rhs"], IV["tmp"],
                helmholtz_lambda=lambda2, coarse_cycles=self.coarse_cycles,
                coarse_mode=self.coarse_mode, coarse_tol=self.coarse_tol)
        return self._mg_helm[lambda2]

    def set_electrode(self, i_lsf, stencils, lsf_faces):
        """Electrode operators (m_field.f90:255-346): the stencils afivo's
        mg_set_operators_tree stored on the boxes the electrode crosses,
        handed to the field multigrid. stencils: {box id: (v, bc_correction)};
        lsf_faces: {box id: (ix, dd, bval)} (global ids; a sharded tree takes
        those of the boxes it stores)."""
        self.i_lsf = i_lsf
        for bid, (v, bcc) in stencils.items():
            lid = self.tree.local_id(bid)
            if lid:
                self.mg.set_box_stencil(lid, v, bcc)
        for bid, (ix, dd, bv) in lsf_faces.items():
            lid = self.tree.local_id(bid)
            if lid:
                self.mg.set_box_lsf(lid, ix, dd, bv, i_lsf)

    def fuse_rhs(self, on=True, ghosts=True):
        """Fold field_set_rhs of the new state into every density update
        (afh_fluid_set_rhs_output): the field_compute that follows reuses it."""
        self.fluid.set_rhs_output(IV["rhs"] if on else 0, ghosts)
        self._fused_rhs = on

    def faces_from_phi(self, on=True):
        """The flux evaluates the face field from phi (afh_fluid_set_field_source)
        and field_from_potential stores |E| only (not with an electrode)."""
        self.fluid.set_field_source(IV["phi"] if on else 0, -1.0)
        if self.lib.has("mg_set_gradient_output"):
            # |E| from the V-cycle's residual pass (field_from_potential's
            # gradient then has nothing left to do)
            self.mg.set_gradient_output(IV["efld"] if on else 0, -1.0)
        self._faces_from_phi = on

    def set_voltage(self, voltage):
        self.voltage = voltage
        self.tree.set_bc(IV["phi"], 2 * self.ndim, capi.BC_DIRICHLET, voltage)

    def min_dr(self):
        return float(np.min(self.topo["meta_dr"]))

    def field_from_potential(self):
        """m_field.f90:488-505."""
        self.mg.compute_phi_gradient(0 if self._faces_from_phi else FV["field"], -1.0,
                                     IV["efld"])
        self.tree.gc_tree(IV["efld"])

    def field_compute(self, s_in, n_vcycles=2, max_rel_residual=1e-4,
                      check_residual=True, defer=False):
        """m_field.f90:405-485 with have_guess = .true.; returns residuals.

        defer (one V-cycle, whose convergence test decides nothing): the
        residual stays folded on the device and the returned list is filled
        by the next species_step, which reads it with the step's limits in one
        transfer; nothing here waits for the device."""
        residuals = []
        threshold = None
        # the library knows whether the last update's rhs of s_in is current
        fused = self._fused_rhs and self.fluid.rhs_valid(s_in)
        if defer and n_vcycles == 1 and check_residual and self._defer_ok:
            if not fused:
                self.fluid.field_set_rhs(IV["rhs"], s_in)
            self.mg.fas_vcycle_fold()
            self.field_from_potential()
            self._deferred_res = residuals
            return residuals
        if check_residual:
            if fused:
                max_rhs = self.fluid.rhs_maxabs(s_in)
            else:
                max_rhs = self.fluid.field_set_rhs_maxabs(IV["rhs"], s_in)
            threshold = max(1e-6, max_rhs * max_rel_residual,
                            1e-10 * abs(self.voltage) /
                            (self.domain[-1] * self.min_dr()))
        elif not fused:
            self.fluid.field_set_rhs(IV["rhs"], s_in)
        for _ in range(n_vcycles):
            if check_residual:
                residuals.append(self.mg.fas_vcycle_maxres())
                if residuals[-1] < threshold:
                    break
            else:
                self.mg.fas_vcycle(True)
        self.field_from_potential()
        return residuals

    def forward_euler(self, dt, s_deriv, s_prev, w_prev, s_out, i_step,
                      n_steps, **field_kw):
        """m_fluid.f90:21-99 (without the CFL/ dt_max combination)."""
        if i_step > 1:
            self.field_compute(s_deriv, **field_kw)
        return list(self.species_step(dt, s_deriv, s_prev, w_prev, s_out,
                                      i_step == n_steps))

    def species_step(self, dt, s_deriv, s_prev, w_prev, s_out, last_step, fetch=True):
        """forward_euler's species part (m_fluid.f90:56-70): flux_upwind_tree +
        flux_update_densities; returns dt_limits(1:4).

        fetch=False: the limits stay folded on the device and nothing is
        returned (None). af_advance overwrites dt_lim in every sub-step
        (m_af_advance.f90:160-164, m_fluid.f90:97-98), so the limits of a
        Heun step's first sub-step are never read; a deferred V-cycle
        residual stays pending too (it is overwritten by the next one)."""
        if not fetch and not self.lib.has("fluid_forward_euler_fold"):
            self.fluid.forward_euler(dt, s_deriv, s_prev, w_prev, s_out, last_step,
                                     self.store_flux)
            return None
        if not fetch:
            self.fluid.forward_euler_fold(dt, s_deriv, s_prev, w_prev, s_out,
                                          last_step, self.store_flux)
            return None
        if self._deferred_res is not None:
            res, self._deferred_res = self._deferred_res, None
            self.fluid.forward_euler_fold(dt, s_deriv, s_prev, w_prev, s_out,
                                          last_step, self.store_flux)
            lim, (max_res,) = self.fluid.fetch_step(last_step, capi.SLOT_MAXRES)
            res.append(max_res)
            return lim
        return self.fluid.forward_euler(dt, s_deriv, s_prev, w_prev, s_out,
                                        last_step, self.store_flux)

    def heun_step(self, dt, **field_kw):
        """af_advance with af_heuns_method (m_af_advance.f90:160-164)."""
        l1 = self.forward_euler(dt, 0, [0], [1.0], 1, 1, 2, **field_kw)
        l2 = self.forward_euler(0.5 * dt, 1, [0, 1], [0.5, 0.5], 0, 2, 2,
                                **field_kw)
        return [min(a, b) for a, b in zip(l1, l2)]


def gaussian_seed(topo, r0, width, n0=5e18, bg=1e15):
    """Initial densities on every box incl. ghost cells (the golden harness'
    set_init), returned as (n_e, n_pos, n_neg, phi-guess factory input)."""
    nc = int(topo["nc"])
    idx = np.arange(nc + 2) - 0.5
    r_min, dr = topo["meta_r_min"], topo["meta_dr"]
    x = r_min[:, 0, None] + idx[None, :] * dr[:, 0, None]
    y = r_min[:, 1, None] + idx[None, :] * dr[:, 1, None]
    z = r_min[:, 2, None] + idx[None, :] * dr[:, 2, None]
    d2 = ((x - r0[0]) ** 2)[:, None, None, :] + ((y - r0[1]) ** 2)[:, None, :, None] \
        + ((z - r0[2]) ** 2)[:, :, None, None]
    ne = bg + n0 * np.exp(-d2 / width ** 2)
    return ne, x, y, z


def seed_state(case, r0=None, width=None):
    """S1-style seed: n_e = n_+ = 1e15 + 5e18 exp(-|r-r0|^2/w^2), n_- = 1e14,
    phi = linear background."""
    if case.ndim == 2:
        return _seed_state_2d(case, r0, width)
    topo = case.topo
    dom = np.asarray(topo["domain"], float)
    r0 = 0.5 * dom if r0 is None else np.asarray(r0)
    width = 0.025 * dom[2] if width is None else width
    ne, x, y, z = gaussian_seed(topo, r0, width)
    t = case.tree
    t.put_cc(IV["e"], ne)
    t.put_cc(IV["pos"], ne)
    t.put_cc(IV["neg"], np.full(ne.shape, 1e14))
    phi = np.broadcast_to(case.voltage * (z / dom[2])[:, :, None, None], ne.shape)
    t.put_cc(IV["phi"], np.ascontiguousarray(phi))
    t.gc_tree(IV["phi"])
    return ne


def cells(topo):
    return sum(len(topo["lvl_leaves_%d" % l]) for l in
               range(1, int(topo["highest_lvl"]) + 1)) * int(topo["nc"]) ** int(topo.get("ndim", 3))


def _seed_state_2d(case, r0=None, width=None):
    """seed_state on a 2-D tree (the same seed, the field along y)."""
    topo = case.topo
    dom = np.asarray(topo["domain"], float)
    r0 = 0.5 * dom if r0 is None else np.asarray(r0)
    width = 0.025 * dom[-1] if width is None else width
    nc = int(topo["nc"])
    idx = np.arange(nc + 2) - 0.5
    r_min, dr = topo["meta_r_min"], topo["meta_dr"]
    x = r_min[:, 0, None] + idx[None, :] * dr[:, 0, None]
    y = r_min[:, 1, None] + idx[None, :] * dr[:, 1, None]
    d2 = ((x - r0[0]) ** 2)[:, None, :] + ((y - r0[1]) ** 2)[:, :, None]
    ne = 1e15 + 5e18 * np.exp(-d2 / width ** 2)
    t = case.tree
    t.put_cc(IV["e"], ne)
    t.put_cc(IV["pos"], ne)
    t.put_cc(IV["neg"], np.full(ne.shape, 1e14))
    phi = np.broadcast_to(case.voltage * (y / dom[1])[:, :, None], ne.shape)
    t.put_cc(IV["phi"], np.ascontiguousarray(phi))
    t.gc_tree(IV["phi"])
    return ne
