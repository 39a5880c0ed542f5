"""The streamer time loop over the device path (src/streamer.f90 restated).

``Simulation`` is what the reference's main program does around the hot
path, with every per-cell operation a call into the C ABI (the HIP library,
or the C oracle for the CPU twin) and the mesh topology on the host
(afh.amr.AfTree, af_adjust_refinement restated):

* set-up: the variable registry, tables and reactions as the reference's
  initializers left them (a case exported by oracle/_ref/export_case from a
  .cfg, tests/golden/rtest_*.npz), af_init + set_initial_conditions
  (streamer.f90:460-519: af_refine_up_to_lvl to refine_max_dx,
  init_cond_set_box, then field_compute without a guess + refinement until
  no box is added);
* the time loop (streamer.f90:177-415): output times, step retry with
  copy_current_state / restore_previous_state (639-668), af_advance with
  Heun's method (m_af_advance.f90:160-164) around forward_euler
  (m_fluid.f90:21-99), field_compute after the step, the dt update,
  photoi_set_src every photoi_per_steps, and a regrid every refine_per_steps
  (restrict + ghost cells of the densities, default_refinement on the device,
  af_adjust_refinement on the host, afh_tree_regrid on the device);
* output_regression_log (src/m_output.f90:783-837) from device reductions.

Parameters the reference reads from its .cfg come from the exported case;
routines it takes as callbacks are the library's (field_bc_homogeneous,
af_bc_neumann_zero, photoi_helmh_bc, default_refinement).
"""
import math
import os

import numpy as np

from . import capi, electrode
from .amr import AfTree
from .model import Fluid, Multigrid, Tree, photoi_helmh_compute

UC_EPS0 = 8.8541878176e-12
UC_ELEM_CHARGE = 1.6022e-19

# Bourdon-3 Helmholtz photoionization modes, src/m_photoi_helmh.f90:106-118
# (SI values; lambdas * frac_O2 * p, coeffs * (frac_O2 * p)^2)
BOURDON3_LAMBDAS = (4147.85, 10950.93, 66755.67)
BOURDON3_COEFFS = (1117314.935, 28692377.5, 2748842283.0)


class Case:
    """Accessors for an exported case (oracle/make_cases.py arrays)."""

    def __init__(self, d):
        self.d = dict(d)

    def r(self, k):
        return float(self.d[k][0])

    def ra(self, k):
        return np.asarray(self.d[k], float)

    def i(self, k):
        return int(self.d[k][0])

    def ia(self, k):
        return [int(x) for x in self.d[k]]

    def s(self, k):
        return str(self.d[k][0])

    def sa(self, k):
        return [str(x) for x in self.d[k]]

    def lt(self, name):
        n_points, n_cols = self.ia(name + "_shape")
        rc = self.ra(name + "_rows_cols").reshape(n_cols, n_points).T
        return {"rows_cols": rc, "x_min": self.r(name + "_xmin"),
                "inv_fac": self.r(name + "_inv_fac")}


def _norm2(v):
    """NORM2 as the reference's Fortran runtime computes it (afh.electrode.norm2)."""
    return float(electrode.norm2(np.asarray(v, float)[None])[0])


def _dist_vec_line(r, r0, r1):
    """GM_dist_vec_line (src/m_geometry.f90:23-43) for an array of points r
    (n, 3): distance vectors and fractions."""
    d = r1 - r0
    line_len2 = np.sum(d * d)
    frac = np.sum((r - r0) * d, axis=1)
    dv = np.empty_like(r)
    lo, hi = frac <= 0.0, frac >= line_len2
    mid = ~(lo | hi)
    dv[lo] = r[lo] - r0
    dv[hi] = r[hi] - r1
    f = frac[mid] / line_len2
    dv[mid] = r[mid] - (r0 + (frac[mid, None] / line_len2) * d)
    out = np.zeros(len(r))
    out[hi] = 1.0
    out[mid] = f
    return dv, out


def density_line(r, r0, r1, n0, n1, width, falloff):
    """GM_density_line (src/m_geometry.f90:53-113) at points r (n, 3)."""
    dv, frac = _dist_vec_line(r, r0, r1)
    dist = electrode.norm2(dv)
    if falloff == "smoothstep":
        t = dist / width - 1
        val = np.where(dist < width, 1.0,
                       np.where(dist < 2 * width, 1 - (3 * (t * t) - 2 * (t * t * t)), 0.0))
    elif falloff == "gaussian":
        val = np.exp(-(dist / width) ** 2)
    elif falloff == "step":
        val = np.where(dist < width, 1.0, 0.0)
    elif falloff == "sigmoid":
        tmp = dist / width
        val = np.where(tmp > math.log(0.5 * np.finfo(float).max), 0.0,
                       2 / (1 + np.exp(np.minimum(tmp, 700.0))))
    else:
        raise ValueError("seed_falloff %s not supported" % falloff)
    return val * (frac * n0 + (1 - frac) * n1)


class Simulation:
    """One streamer simulation (src/streamer.f90) over a C-ABI library."""

    def __init__(self, lib, case, device=-1, coarse_cycles=0, capacity_factor=2.0,
                 fuse_rhs=True, user=None, coarse_tol=0.0, coarse_mode=None):
        """user: the program's m_user hooks (afh.users), e.g. the gas density
        function and initial conditions of programs/3d_sprite.
        coarse_cycles / coarse_tol: the level-1 solve (0: exact; else at most
        coarse_cycles MG cycles, stopped at |r| < coarse_tol |b| when
        coarse_tol > 0 -- HYPRE PFMG's rule). coarse_mode=capi.COARSE_PFMG:
        the reference's solver itself, HYPRE StructPFMG restated
        (csrc/afh_pfmg.h), at most coarse_cycles iterations to coarse_tol
        (the reference: 50, 1e-6)."""
        c = case if isinstance(case, Case) else Case(case)
        self.c, self.lib, self.device = c, lib, device
        self.user = user
        self.coarse_cycles = coarse_cycles
        self.coarse_tol = coarse_tol
        self.coarse_mode = coarse_mode
        self.capacity_factor = capacity_factor
        # NDIM: the exported coarse grid has one entry per dimension (2: the
        # reference's 2-D build, programs/standard_2d, on libafivo_hip_2d.so)
        self.ndim = len(c.ia("coarse_grid_size_value"))
        # the rhs folded into the density update and the face field formed
        # from phi are entry points of the 3-D library only
        self.fused_rhs = fuse_rhs and lib.has("fluid_set_rhs_output")
        # field_compute reads max|rhs| with the first residual (AFH_DEFER=0:
        # before the V-cycle, as the reference orders it; for A/B runs)
        self._defer_ok = os.environ.get("AFH_DEFER", "1") != "0"
        # the flux takes the face field from phi (afh_fluid_set_field_source):
        # the gradient then writes |E| only; not with an electrode (its
        # boxes' gradient is mg_box_lpllsf_gradient). AFH_FACES_FROM_PHI=0
        # stores and reads the face field, as the reference does (A/B runs)
        self._faces_from_phi_ok = (os.environ.get("AFH_FACES_FROM_PHI", "1") != "0" and
                                   lib.has("fluid_set_field_source"))
        self.faces_from_phi = False
        if c.s("time_integrator") != "heuns_method":
            raise NotImplementedError("time integrator %s" % c.s("time_integrator"))
        self.n_states = 2  # af_advance_num_steps(af_heuns_method)
        if c.i("use_dielectric") or c.i("cylindrical"):
            raise NotImplementedError("dielectric / cylindrical cases")
        # electrode (m_field.f90:196-346): a rod or sphere as level-set
        # function; its operators are computed on the host per box
        # (afh.electrode, mg_set_operators_tree) and handed to the library
        self.lsf = None
        if c.i("use_electrode"):
            kind = c.s("field_electrode_type")
            L0, o0 = c.ra("domain_len"), c.ra("domain_origin")
            r0 = o0 + c.ra("field_rod_r0") * L0
            r1 = o0 + c.ra("field_rod_r1") * L0
            if kind == "rod":
                self.lsf = electrode.RodLSF(r0, r1, c.r("field_rod_radius"))
            elif kind == "sphere":
                self.lsf = electrode.SphereLSF(r0, c.r("field_rod_radius"))
            else:
                raise NotImplementedError("electrode type %s" % kind)
            if c.i("photoi%enabled"):
                raise NotImplementedError("Helmholtz photoionization with an electrode")
            self.electrode_grounded = bool(c.i("field_electrode_grounded"))
            self._ops = {}  # box geometry -> box_operators (tags persist)
        # registry (af_add_cc_variable order of the reference's modules)
        self.cc_names = c.sa("cc_names")
        # gas density given by a function (streamer.f90:86-95 with
        # user_gas_density, m_gas.f90:146-148): the cc variable "M", set on
        # every cell of a box (ghosts included) when the box is created
        # (set_gas_density_from_user_function, streamer.f90:672-681)
        self.i_gas_dens = 0
        if not c.i("gas_constant_density"):
            if user is None or not hasattr(user, "gas_density"):
                raise NotImplementedError("a variable gas density needs the user's gas_density")
            self.i_gas_dens = list(self.cc_names).index("M") + 1
            self.gas_fractions = list(c.ra("gas_fractions"))
        self.n_var_cell, self.n_var_face = len(self.cc_names), len(c.sa("fc_names"))
        self.n_scratch = 0  # (set with photoionization below)
        (self.i_phi, self.i_electron, self.i_1pos_ion, self.i_efld, self.i_rhs,
         self.i_tmp, self.i_photo, self.f_flux, self.f_field, self.i_lsf) = c.ia("ivars")
        n_species, self.n_gas, n_reac = c.ia("n_species")
        self.species_list = c.sa("species_list")
        self.species_charge = c.ia("species_charge")
        self.species_itree = c.ia("species_itree")
        self.densities = c.ia("all_densities")
        self.plasma = [n for n in range(n_species) if self.species_itree[n] > 0]
        # mobile ions (input_data%mobile_ions): flux species 2.. after the
        # electrons (m_streamer.f90:253-282), as (plasma species index
        # (1-based), flux face variable, scaled mobility) for the fluid
        self.ions = []
        n_ions = c.i("n_mobile_ions") if "n_mobile_ions" in c.d else 0
        if n_ions:
            fs, fv = c.ia("flux_species"), c.ia("flux_variables")
            mob = c.ra("ion_mobilities")
            if len(fs) != 1 + n_ions or fs[0] != self.i_electron:
                raise NotImplementedError("electron energy equation")
            plasma_iv = [self.species_itree[n] for n in self.plasma]
            for q in range(n_ions):
                self.ions.append((plasma_iv.index(fs[1 + q]) + 1, fv[1 + q], float(mob[q])))
        self.N = c.r("gas_number_density")
        self.L = c.ra("domain_len")
        self.origin = c.ra("domain_origin")
        # field_given_by (m_field.f90:132-170): the exported voltage at t = 0
        if c.r("current_voltage") != 0 and "table" in c.s("field_given_by"):
            raise NotImplementedError("tabulated voltages")
        self.voltage = c.r("current_voltage")
        # dt parameters (m_dt.f90)
        self.dt_max, self.dt_min = c.r("dt_max"), c.r("dt_min")
        self.dt_safety = c.r("dt_safety_factor")
        self.cfl = c.r("dt_cfl_number_value")
        self.dt_growth = c.r("dt_max_growth_factor")
        self.num_vcycles = c.i("multigrid_num_vcycles")
        self.max_rel_res = c.r("multigrid_max_rel_residual")
        # photoionization (m_photoi.f90, m_photoi_helmh.f90)
        self.photoi = bool(c.i("photoi%enabled"))
        if self.photoi:
            if c.s("photoi%method") != "helmholtz" or c.s("photoi%source_type") != "Zheleznyak":
                raise NotImplementedError("photoionization other than Helmholtz/Zheleznyak")
            if c.s("photoi_helmh%author") != "Bourdon-3":
                raise NotImplementedError("Helmholtz modes other than Bourdon-3")
            comps = c.sa("gas_components")
            frac_o2 = c.ra("gas_fractions")[comps.index("O2")] if "O2" in comps else 0.0
            p = c.r("gas_pressure_value")
            self.helm_lambdas = [lam * frac_o2 * p for lam in BOURDON3_LAMBDAS]
            self.helm_coeffs = [cf * (frac_o2 * p) ** 2 for cf in BOURDON3_COEFFS]
            self.helm_iv = [self.cc_names.index("helmh_%d" % (n + 1)) + 1 for n in range(3)]
            qp = c.r("photoi%quenching_pressure")
            self.photoi_coeff = c.r("photoi%eta") * (qp / (c.r("gas_pressure_value") + qp))
            self.photo_species = c.i("photoi_species_index") - self.n_gas
        # the Helmholtz modes 1 .. n-1 get an rhs and a tmp variable of their
        # own (after the reference's variables): afh_photoi_helmh_compute then
        # solves the modes concurrently, bitwise the one-after-another solve
        # (AFH_HELMH_CONC=0: the shared variables, modes in turn)
        self.n_scratch = 0
        if self.photoi and os.environ.get("AFH_HELMH_CONC", "1") != "0":
            self.n_scratch = 2 * (len(BOURDON3_LAMBDAS) - 1)
        self.td = c.lt("td")
        self.chem = c.lt("chem")
        self.reactions = []
        for n in range(1, n_reac + 1):
            rt, _, n_coeff, lti, _ = c.ia("reaction_%d" % n)
            if n_coeff > 4:
                raise NotImplementedError("rate with %d coefficients" % n_coeff)
            # constant N: the gas species are folded into the rate factors
            # (m_chemistry.f90:1086-1099) and leave the index space; variable
            # N: they stay first, the library gives them gas_fractions * N
            shift = ((lambda ix: [x - self.n_gas for x in ix]) if not self.i_gas_dens
                     else (lambda ix: list(ix)))
            self.reactions.append({
                "rate_type": rt, "table_col": lti,
                "rate_factor": c.r("reaction_%d_factor" % n),
                "c": list(c.ra("reaction_%d_data" % n)),
                "ix_in": shift(c.ia("reaction_%d_in" % n)),
                "ix_out": shift(c.ia("reaction_%d_out" % n)),
                "mult_out": c.ia("reaction_%d_mult" % n)})
        # init conditions (m_init_cond.f90:38-144)
        self.background = c.r("background_density")
        self.seeds = []
        nd = self.ndim
        for n in range(len(c.ra("seed_density"))):
            self.seeds.append({
                "r0": c.ra("seed_rel_r0")[nd * n:nd * n + nd] * self.L + self.origin,
                "r1": c.ra("seed_rel_r1")[nd * n:nd * n + nd] * self.L + self.origin,
                "n0": c.ra("seed_density")[n], "n1": c.ra("seed_density2")[n],
                "type": c.ia("seed_charge_type")[n], "width": c.ra("seed_width")[n],
                "falloff": c.sa("seed_falloff")[n]})
        # state (streamer.f90:107-114, initialize_modules: global_dt = dt_min)
        self.it = 0
        self.time = self.global_time = self.photoi_prev_time = 0.0
        self.global_dt = self.dt = self.dt_min
        self.n_steps_rejected = 0
        self.frac_rejected = 0.0
        self.output_cnt = 0
        self.log = []
        # mesh: af_init (streamer.f90:151-153)
        nc = c.i("box_size")
        self.af = AfTree(nc, self.origin + self.L, c.ia("coarse_grid_size_value"),
                         r_min=self.origin)
        self.tree = self.fluid = self.mg = None
        self.helm = []
        self.shard = None  # shard_over
        # V-cycles replayed from hipGraphs (of them segmented, sharded), over
        # every multigrid this run has bound (afh_mg_graph_stats)
        self.graph_replays = [0, 0]

    # ------------------------------------------------------------- device
    @property
    def n_var_tree(self):
        """cc variables of the device tree: the reference's, then the
        concurrent Helmholtz modes' scratch (rhs, tmp per mode but the last)."""
        return self.n_var_cell + self.n_scratch

    def _capacity(self):
        return max(64, int(self.capacity_factor * self.af.highest_id))

    def graph_stats(self):
        """(V-cycles replayed from hipGraphs, of them segmented) over this
        run's multigrids, the bound ones included."""
        tot = list(self.graph_replays)
        for m in [self.mg] + self.helm:
            if m is not None and m.lib.has("mg_graph_stats"):
                tot = [a + b for a, b in zip(tot, m.graph_stats())]
        return tuple(tot)

    def _bind(self, tree):
        """Multigrid and fluid state bound to a (new) device tree."""
        for m in [self.mg] + self.helm:
            if m is not None:
                if m.lib.has("mg_graph_stats"):
                    self.graph_replays = [a + b for a, b in
                                          zip(self.graph_replays, m.graph_stats())]
                m.close()
        if self.fluid is not None:
            self.fluid.close()
        self.tree = tree
        self.mg = Multigrid(tree, self.i_phi, self.i_rhs, self.i_tmp,
                            coarse_cycles=self.coarse_cycles, coarse_tol=self.coarse_tol,
                            coarse_mode=self.coarse_mode)
        self.helm = []
        if self.photoi:
            for k, (iv, lam) in enumerate(zip(self.helm_iv, self.helm_lambdas)):
                own = self.n_scratch and k + 1 < len(self.helm_iv)
                i_rhs = self.n_var_cell + 1 + 2 * k if own else self.i_rhs
                i_tmp = self.n_var_cell + 2 + 2 * k if own else self.i_tmp
                self.helm.append(Multigrid(tree, iv, i_rhs, i_tmp,
                                           helmholtz_lambda=lam * lam,
                                           coarse_cycles=self.coarse_cycles,
                                           coarse_tol=self.coarse_tol,
                                           coarse_mode=self.coarse_mode))
        c = self.c
        td_cols = c.ia("td_cols")
        self.fluid = Fluid(
            tree, [self.species_itree[n] for n in self.plasma],
            [self.species_charge[n] for n in self.plasma], self.i_electron,
            self.i_efld, self.f_flux, self.f_field, self.N, self.td, self.chem,
            self.reactions, dt_chemistry_nmin=c.r("dt_chemistry_nmin"),
            gas_temperature=c.r("gas_temperature_value"),
            td_energy_col=max(0, td_cols[4]),
            i_photo=self.i_photo if self.photoi else 0,
            photo_species=self.photo_species if self.photoi else 0,
            i_gas_dens=self.i_gas_dens,
            gas_fractions=self.gas_fractions if self.i_gas_dens else (),
            ions=self.ions)
        # secondary emission from ions at the walls (input_data%ion_se_yield,
        # handle_ion_se_flux in forward_euler, m_fluid.f90:63-67)
        if self.ions and "ion_se_yield" in c.d and c.r("ion_se_yield") > 0:
            if not self.lib.has("fluid_set_ion_se_yield"):
                raise NotImplementedError(
                    "ion secondary emission (ion_se_yield > 0) is not built in this "
                    "library (the 2-D build: include/afivo_hip_2d.h)")
            self.fluid.set_ion_se_yield(c.r("ion_se_yield"))
        if self.fused_rhs:
            self.fluid.set_rhs_output(self.i_rhs, True)
        self.faces_from_phi = self._faces_from_phi_ok and self.lsf is None
        if self.faces_from_phi:
            self.fluid.set_field_source(self.i_phi, -1.0)
            self.mg.set_gradient_output(self.i_efld, -1.0)
        if self.lsf is not None:
            # forward_euler's flux_update_densities with set_box_mask
            # (m_fluid.f90:73, 469-483): no update inside the electrode
            self.fluid.set_update_mask(self.i_lsf)
            self._set_electrode()

    def lsf_boundary_value(self):
        """mg%lsf_boundary_value (m_field.f90:439-443)."""
        return 0.0 if self.electrode_grounded else self.voltage

    def _set_electrode(self):
        """set_lsf_box on every box (cells 0..nc+1, m_field.f90:608-619) and
        the operators of mg_set_operators_tree (m_af_multigrid.f90:
        1133-1205): box tags and stencils, computed once per box (afivo
        keeps them with the box), bc_correction with the current electrode
        potential; the electrode boxes for refine_electrode_dx and
        electrode_species_bc."""
        nc, ng = self.af.nc, self.af.nc + 2
        n_glob = self._n_global()
        lsf = np.zeros((n_glob, ng, ng, ng))
        bv = self.lsf_boundary_value()
        self.electrode_ids = []
        self.electrode_box = np.zeros(n_glob, np.uint8)
        used = [b for b in range(1, self.af.highest_id + 1) if self.af.in_use[b]]
        r = np.stack([electrode.cell_centers(self.af.r_min[b], self.af.dr[b], nc, 0, nc + 1)
                      for b in used])
        lsf[np.asarray(used) - 1] = self.lsf(r)
        key = {b: (tuple(self.af.r_min[b]), tuple(self.af.dr[b])) for b in used}
        new = [b for b in used if key[b] not in self._ops]
        ops = electrode.boxes_operators(
            self.lsf, [(lsf[b - 1][1:-1, 1:-1, 1:-1], self.af.r_min[b], self.af.dr[b])
                       for b in new], nc, 1.0)
        for b, op in zip(new, ops):
            self._ops[key[b]] = op
        for b in used:
            op = self._ops[key[b]]
            if op is None:
                continue
            v, fb, ix, dd = op  # fb: f times 1
            self.electrode_box[b - 1] = 1
            # a sharded tree: the boxes it stores, by their library ids;
            # electrode_species_bc on the boxes it computes
            lid = self.tree.local_id(b)
            if not lid:
                continue
            if self.shard is None or self._computes(b):
                self.electrode_ids.append(lid)
            self.mg.set_box_stencil(lid, v, fb * bv)
            self.mg.set_box_lsf(lid, ix, dd, np.full((nc, nc, nc), bv), self.i_lsf)
        self.tree.put_cc(self.i_lsf, lsf)

    def _create_tree(self):
        t = Tree(self.lib, self.af.topology(), self.n_var_tree, self.n_var_face,
                 device=self.device, box_capacity=self._capacity())
        return self._set_methods(t)

    def _n_global(self):
        """Boxes of the whole tree (a sharded tree stores only some)."""
        t = self.tree
        return t.n_global if t.global_ids is not None else t.n_boxes

    def _computes(self, b):
        """This rank computes box b (owns it, or it is on a replicated level)."""
        sh = self.shard
        owner = sh.owner if hasattr(sh, "owner") else sh.part.owner
        o = int(owner[b - 1])
        return o < 0 or o == sh.rank

    def shard_over(self, shard):
        """Continue the run sharded over ranks (afh.dist.NativeShard, or the
        Python Shard): this rank's part of the current tree -- the boxes it
        owns, the replicated levels and the replicas its exchanges refresh --
        is created from the current topology and filled with the current
        data of every variable, the multigrids and the fluid are bound to it
        and the shard's exchange hook is attached. Every rank must hold the
        same state before (e.g. the same deterministic set-up). A refinement
        of the sharded run (adjust_refinement) needs the library's own
        sharding (afh.dist.NativeShard); with the Python Shard it raises."""
        topo = self.af.topology()
        full = self.tree
        t = self._set_methods(shard.make_tree(self.lib, topo, self.n_var_tree,
                                              self.n_var_face, device=self.device))
        for iv in range(1, self.n_var_cell + 1):
            t.put_cc(iv, full.get_cc(iv))
        for iv in range(1, self.n_var_face + 1):
            t.put_fc(iv, full.get_fc(iv))
        self.shard = shard
        self._bind(t)
        shard.attach(t)
        full.close()
        return t

    def _gather_full(self):
        """The whole tree on this rank: every rank's computed boxes (owned,
        and the replicated ones from rank 0) with every cell and face
        variable, in one numeric all-gather (NativeShard.allgather_rows), in
        a new single-rank tree."""
        sh = self.shard
        owner = np.asarray(sh.owner)
        t = self._create_tree()
        mine = np.nonzero((owner == sh.rank) | ((owner < 0) & (sh.rank == 0)))[0]
        cc = [self.tree.get_cc(iv) for iv in range(1, self.n_var_cell + 1)]
        fc = [self.tree.get_fc(iv) for iv in range(1, self.n_var_face + 1)]
        rows = np.concatenate([a[mine].reshape(len(mine), -1) for a in cc + fc], axis=1)
        for ids, vals in sh.allgather_rows(mine, rows):
            off = 0
            for a in cc + fc:
                w = int(np.prod(a.shape[1:]))
                a[ids] = vals[:, off:off + w].reshape((len(ids),) + a.shape[1:])
                off += w
        for iv, a in enumerate(cc, 1):
            t.put_cc(iv, a)
        for iv, a in enumerate(fc, 1):
            t.put_fc(iv, a)
        return t

    def _adjust_refinement_sharded(self):
        """af_adjust_refinement of a sharded run. The refinement flags of
        the computed boxes are all-gathered and every rank decides the same
        new topology on a copy of the host tree; the new tree is sharded with
        a fresh partition (the load balance follows the refinement), and
        each rank builds its part of it from the boxes it needs
        (_regrid_rank_local: only boxes whose data live on another rank
        travel, point to point). AFH_REGRID_GATHER=1: the round-3 form, the
        whole tree gathered on every rank and regridded as a single rank
        does. Both are bitwise the single-rank run."""
        import copy
        sh = self.shard
        if not hasattr(sh, "renew"):
            raise NotImplementedError("refinement of a run sharded by the Python Shard "
                                      "(afh.dist.Shard); use afh.dist.NativeShard")
        # the refinement flags of the computed boxes decide first, on a copy
        # of the host topology: most calls change nothing and move no data
        t = self.tree
        eb = (None if self.lsf is None else
              np.append(self.electrode_box[t.global_ids - 1], 0).astype(np.uint8))
        flags, masks = self.fluid.refine_flags(self.refine_desc(), eb)
        owner = np.asarray(sh.owner)
        mine = np.nonzero((owner == sh.rank) | ((owner < 0) & (sh.rank == 0)))[0]
        lid = np.searchsorted(t.global_ids, mine + 1)
        gf = np.zeros(len(owner), np.int32)
        gm = np.zeros(len(owner), np.uint32)
        # (flags and masks as exact float64 rows of a numeric all-gather)
        fm = np.stack([flags[lid], masks[lid]], axis=1).astype(np.float64)
        for ids, v in sh.allgather_rows(mine, fm):
            gf[ids], gm[ids] = v[:, 0].astype(np.int32), v[:, 1].astype(np.uint32)
        probe = copy.deepcopy(self.af)
        info = probe.adjust_refinement(
            lambda ids: (gf[np.asarray(ids, np.int64) - 1], gm[np.asarray(ids, np.int64) - 1]))
        if not (info.n_add or info.n_rm):
            return info
        if os.environ.get("AFH_REGRID_GATHER", "0") != "1":
            return self._regrid_rank_local(probe, info)
        full = self._gather_full()
        old = self.tree
        sh.detach()
        self.shard = None
        self._bind(full)
        old.close()
        info = self.adjust_refinement()
        self.shard_over(sh.renew(self.af.topology()))
        return info

    def _regrid_sources(self, old, new, owner_new, sh_new, rank):
        """The boxes rank's regrid reads: W, the new tree's boxes it stores
        closed over what afh_tree_regrid reads to create them (a new box's
        parent, its same-level neighbours for the ghost fill, the parent's
        neighbours for refinement-boundary faces, recursively through new
        boxes), and the old boxes behind W (W's persisting boxes, and the
        removed children of those that lose them, for auto_restrict)."""
        nb_old, nb_new = int(old["n_boxes"]), int(new["n_boxes"])
        lo, ln = np.asarray(old["meta_lvl"]), np.asarray(new["meta_lvl"])
        xo, xn = np.asarray(old["meta_ix"]), np.asarray(new["meta_ix"])
        par = np.asarray(new["meta_parent"])
        nmat = np.asarray(new["meta_neighbor_mat"])
        cho, chn = np.asarray(old["meta_children"]), np.asarray(new["meta_children"])

        def kept(b):
            return (b <= nb_old and lo[b - 1] > 0 and lo[b - 1] == ln[b - 1] and
                    np.array_equal(xo[b - 1], xn[b - 1]))

        W = set(int(b) for b in sh_new.local_ids(rank))
        stack = [b for b in W if not kept(b)]
        while stack:
            b = stack.pop()
            p = int(par[b - 1])
            cand = [p] + [int(c) for c in nmat[b - 1]]
            if p > 0:
                cand += [int(c) for c in nmat[p - 1]]
            for c in cand:
                if 0 < c <= nb_new and ln[c - 1] > 0 and c not in W:
                    W.add(c)
                    if not kept(c):
                        stack.append(c)
        W_old = set()
        for b in W:
            if kept(b):
                W_old.add(b)
                if cho[b - 1][0] > 0 and chn[b - 1][0] == 0:
                    W_old.update(int(c) for c in cho[b - 1])
        return sorted(W), sorted(W_old)

    def _regrid_rank_local(self, probe, info):
        """This rank's part of the refined tree without a whole-tree gather:
        (1) every rank computes, for every rank, the new boxes it stores and
        the old boxes behind them (_regrid_sources); (2) the old owner of
        each such box sends it (every cell and face variable, ghost cells
        included) to the ranks that need it, point to point
        (NativeShard.exchange_rows; replicated boxes and a rank's own are
        local); (3) the old boxes go into a small tree of the old topology,
        afh_tree_regrid moves them onto the new topology -- auto_restrict,
        the persisting boxes, the new boxes prolonged and their ghost cells
        filled level by level, exactly the single-rank data movement -- and
        (4) this rank's boxes of the new partition are copied from it into
        the new sharded tree. Both small trees number their boxes by one id
        space (dist.compact_topology), so a persisting box keeps its id."""
        from .dist import compact_topology
        sh = self.shard
        old_topo, new_topo = self.af.topology(), probe.topology()
        sh2 = sh.renew(new_topo)
        owner_old = np.asarray(sh.owner)
        me, n = sh.rank, sh.n
        src = [self._regrid_sources(old_topo, new_topo, sh2.owner, sh2, q) for q in range(n)]
        # (2) the rows this rank sends: its owned boxes other ranks read --
        # on the device, the boxes packed into device tensors and sent as
        # they are (Tree.pack_boxes, NativeShard.exchange_rows_dev); on the
        # host (the oracle), whole-tree arrays
        t_old = self.tree
        nvc, nvf = self.n_var_cell, self.n_var_face
        new_rows = self._row_buffers(sh)
        tdev = new_rows
        if new_rows is not None:
            cc = fc = None
            w_row = t_old.row_width(nvc, nvf)

            def rows_of(gids):
                lid = [t_old.local_id(b) for b in gids]
                buf = new_rows(len(lid), w_row)
                t_old.pack_boxes(lid, nvc, nvf, buf)
                return buf
        else:
            cc = [t_old.get_cc_local(iv) for iv in range(1, nvc + 1)]
            fc = [t_old.get_fc_local(iv) for iv in range(1, nvf + 1)]

            def rows_of(gids):
                lid = np.array([t_old.local_id(b) for b in gids], np.int64) - 1
                return np.concatenate([a[lid].reshape(len(lid), -1) for a in cc + fc], axis=1)

        sends = {}
        for q in range(n):
            if q == me:
                continue
            ids = [b for b in src[q][1] if owner_old[b - 1] == me]
            if ids:
                sends[q] = (np.asarray(ids, np.int64), rows_of(ids))
        got = (sh.exchange_rows_dev(sends, self._torch_dev) if tdev is not None
               else sh.exchange_rows(sends))
        self.regrid_rows_received = sum(len(v[0]) for v in got.values())
        self.regrid_device_rows = tdev is not None
        # (3) the old boxes behind this rank's part, in a tree of their own
        W, W_old = src[me]
        space = sorted(set(W) | set(W_old))
        pos = {b: k for k, b in enumerate(space)}
        t_ow = self._set_methods(Tree(self.lib, compact_topology(old_topo, W_old, space),
                                      self.n_var_tree, self.n_var_face, device=self.device))
        local = [b for b in W_old if owner_old[b - 1] == me or owner_old[b - 1] < 0]
        if tdev is not None:
            # device to device: the local boxes and the received rows into the
            # small tree (its boxes nobody fills are read by nothing)
            if local:
                t_ow.unpack_boxes([pos[b] + 1 for b in local], nvc, nvf, rows_of(local))
            for ids, rows in got.values():
                t_ow.unpack_boxes([pos[int(b)] + 1 for b in ids], nvc, nvf, rows)
            del got, sends
            t_nw = t_ow.regrid(compact_topology(new_topo, W, space))
            sh.detach()
            self.shard = None
            self.af = probe
            t = self._set_methods(sh2.make_tree(self.lib, new_topo, self.n_var_tree,
                                                self.n_var_face, device=self.device))
            k = [pos[int(b)] + 1 for b in t.global_ids]
            buf = new_rows(len(k), w_row)
            t_nw.pack_boxes(k, nvc, nvf, buf)
            t.unpack_boxes(np.arange(1, len(k) + 1), nvc, nvf, buf)
            del buf
            return self._regrid_finish(info, sh2, t, t_nw, t_ow, t_old)
        data = [np.full((len(space) + 1,) + a.shape[1:], np.nan) for a in cc + fc]
        if local:
            rl = rows_of(local)
            k = np.array([pos[b] for b in local])
            off = 0
            for d in data:
                w = int(np.prod(d.shape[1:]))
                d[k] = rl[:, off:off + w].reshape((len(k),) + d.shape[1:])
                off += w
        for ids, rows in got.values():
            k = np.array([pos[int(b)] for b in ids])
            off = 0
            for d in data:
                w = int(np.prod(d.shape[1:]))
                d[k] = rows[:, off:off + w].reshape((len(k),) + d.shape[1:])
                off += w
        del cc, fc
        for iv in range(1, self.n_var_cell + 1):
            t_ow.put_cc(iv, data[iv - 1])
        for iv in range(1, self.n_var_face + 1):
            t_ow.put_fc(iv, data[self.n_var_cell + iv - 1])
        del data
        t_nw = t_ow.regrid(compact_topology(new_topo, W, space))
        # (4) the new sharded tree from it
        sh.detach()
        self.shard = None
        self.af = probe
        t = self._set_methods(sh2.make_tree(self.lib, new_topo, self.n_var_tree,
                                            self.n_var_face, device=self.device))
        k = np.array([pos[int(b)] for b in t.global_ids])
        for iv in range(1, self.n_var_cell + 1):
            a = t_nw.get_cc(iv)
            out = np.full((t.n_boxes,) + a.shape[1:], np.nan)
            out[:-1] = a[k]
            t.put_cc(iv, out)
        for iv in range(1, self.n_var_face + 1):
            a = t_nw.get_fc(iv)
            out = np.full((t.n_boxes,) + a.shape[1:], np.nan)
            out[:-1] = a[k]
            t.put_fc(iv, out)
        return self._regrid_finish(info, sh2, t, t_nw, t_ow, t_old)

    def _regrid_finish(self, info, sh2, t, t_nw, t_ow, t_old):
        t_nw.close()
        t_ow.close()
        self.shard = sh2
        self._bind(t)
        sh2.attach(t)
        t_old.close()
        if self.i_gas_dens and info.n_add:  # m_af_core.f90:866-869
            self._set_gas([b for l in sorted(info.add) for b in info.add[l]])
        return info

    def _row_buffers(self, sh):
        """How the rank-local regrid allocates its box rows when the boxes can
        move device to device (the HIP library on a GPU), else None: torch
        device tensors under the RCCL transport (its send / receive take
        them), library device buffers (model.DeviceRows) for thread ranks."""
        from .model import DeviceRows
        self._torch_dev = None
        if self.device < 0 or not self.lib.has("tree_pack_boxes"):
            return None
        if sh.transport == capi.DIST_LOCAL:
            # a receiver's unpack reads the sender's buffer directly, so the
            # rows stay on the device only when every thread rank of the
            # group runs on the same GPU (no peer access is enabled); a group
            # spread over several GPUs moves them through host arrays
            devices = sh.allgather(self.device)
            if len(set(devices)) != 1:
                return None
            lib, dev = self.lib, self.device
            return lambda n, w: DeviceRows(lib, dev, n, w)
        import torch
        self._torch_dev = torch.device("cuda", self.device)
        return lambda n, w: torch.empty((n, w), dtype=torch.float64, device=self._torch_dev)

    def _set_methods(self, t):
        neumann0 = [(capi.BC_NEUMANN, 0.0)] * 6
        # z faces Dirichlet 0, other faces Neumann 0 (photoi_helmh_bc)
        helm_bc = [(capi.BC_NEUMANN, 0.0)] * 4 + [(capi.BC_DIRICHLET, 0.0)] * 2
        if self.photoi:  # photoi_initialize (m_photoi.f90:105-106): first auto var
            t.set_cc_methods(self.i_photo, helm_bc, capi.RB_GC_INTERP)
            t.set_cc_prolong(self.i_photo, capi.PROLONG_LINEAR)
            for iv in self.helm_iv:  # mg_helm(n)%sides_bc, mg_sides_rb
                t.set_cc_methods(iv, helm_bc, capi.RB_MG_SIDES)
                # mg_init (m_af_multigrid.f90:102-105) sets the methods without
                # a prolongation argument: af_prolong_linear, and the mode's
                # phi becomes an auto variable (prolonged into new boxes,
                # m_af_core.f90:387-391, 420-425, 842-881)
                t.set_cc_prolong(iv, capi.PROLONG_LINEAR)
        # field_initialize (m_field.f90:349-350)
        t.set_cc_methods(self.i_efld, neumann0, capi.RB_GC_INTERP)
        t.set_cc_prolong(self.i_efld, capi.PROLONG_LINEAR)
        # streamer.f90:81-84: densities and their copies, af_gc_interp_lim,
        # af_prolong_limit (prolong_density = limit), gminmod43
        for iv in self.densities:
            for s in range(self.n_states + 1):
                t.set_cc_methods(iv + s, neumann0, capi.RB_GC_INTERP_LIM)
            t.set_cc_prolong(iv, capi.PROLONG_LIMIT)
        # phi and its copy: field_bc_homogeneous, mg_sides_rb; mg_init
        # (m_af_multigrid.f90:102-105) makes phi (not its copy) an auto
        # variable with af_prolong_linear: new boxes get phi prolonged from
        # their parent and their ghost cells filled (auto_prolong,
        # m_af_core.f90:842-881), the guess of the field solve after a regrid
        for s in (0, 1):
            t.set_cc_methods(self.i_phi + s, self.phi_bc(), capi.RB_MG_SIDES)
        t.set_cc_prolong(self.i_phi, capi.PROLONG_LINEAR)
        # streamer.f90:98-104: rhs gets neumann_zero, af_gc_interp, limit
        t.set_cc_methods(self.i_rhs, neumann0, capi.RB_GC_INTERP)
        t.set_cc_prolong(self.i_rhs, capi.PROLONG_LIMIT)
        return t

    def phi_bc(self):
        """field_bc_homogeneous (src/m_field.f90:547-567): Dirichlet 0 and
        the voltage on the faces normal to the last dimension."""
        return [(capi.BC_NEUMANN, 0.0)] * (2 * self.ndim - 2) + [
            (capi.BC_DIRICHLET, 0.0), (capi.BC_DIRICHLET, self.voltage)]

    # --------------------------------------------------------- physics
    def field_from_potential(self):
        """m_field.f90:488-505 (with faces_from_phi the face field is not
        stored: the flux evaluates it from phi)."""
        self.mg.compute_phi_gradient(0 if self.faces_from_phi else self.f_field, -1.0,
                                     self.i_efld)
        self.tree.gc_tree(self.i_efld)

    def field_compute(self, s_in, have_guess=True):
        """field_compute (src/m_field.f90:405-485); returns the residuals.

        With the rhs folded into the last update (fused_rhs) and a guess, the
        first V-cycle runs before max|rhs| is read, and both maxima come back
        in one transfer (the threshold is first used after that V-cycle)."""
        vres = []
        if self.fused_rhs and self.fluid.rhs_valid(s_in):
            if have_guess and self.num_vcycles >= 1 and self._defer_ok:
                self.mg.fas_vcycle_fold()
                r0, max_rhs = self.tree.fetch_reduced(capi.SLOT_MAXRES, capi.SLOT_RHS)
                vres.append(r0)
            else:
                max_rhs = self.fluid.rhs_maxabs(s_in)
        else:
            max_rhs = self.fluid.field_set_rhs_maxabs(self.i_rhs, s_in)
        # with an electrode the initial convergence test is less strict
        conv_fac = 1e-8 if self.lsf is not None else 1e-10
        threshold = max(1e-6, max_rhs * self.max_rel_res,
                        conv_fac * abs(self.voltage) / (self.L[-1] * self.af.min_dr()))
        res = []
        if not have_guess:
            for i in range(1, 101):
                self.mg.fas_fmg(True, have_guess=True)
                res.append(self.tree.maxabs_cc(self.i_tmp))
                if res[-1] < threshold:
                    break
                if i > 2:
                    ratio = min(res[-3:]) / max(res[-3:])
                    if 0.5 < ratio < 2.0 and res[-1] < 1e8:
                        break
            else:
                raise RuntimeError("No convergence in initial field computation")
        while len(vres) < self.num_vcycles and not (vres and vres[-1] < threshold):
            vres.append(self.mg.fas_vcycle_maxres())
        self.field_from_potential()
        return res + vres

    def forward_euler(self, dt, s_deriv, s_prev, w_prev, s_out, i_step, n_steps):
        """forward_euler (src/m_fluid.f90:21-99): returns dt_lim."""
        if i_step > 1:
            self.field_compute(s_deriv, True)
        lim = self.fluid.forward_euler(dt, s_deriv, s_prev, w_prev, s_out,
                                       i_step == n_steps)
        limits = [lim[0] * self.cfl, lim[1], lim[2], lim[3]]
        return min(self.dt_max, min(limits))

    def advance(self, dt):
        """af_advance with af_heuns_method (m_af_advance.f90:121-214): dt_lim
        of the last sub-step."""
        self.forward_euler(dt, 0, [0], [1.0], 1, 1, 2)
        dt_lim = self.forward_euler(0.5 * dt, 1, [0, 1], [0.5, 0.5], 0, 2, 2)
        self.time = self.time + dt
        return dt_lim

    def copy_current_state(self):
        """streamer.f90:639-651."""
        for iv in self.densities:
            self.tree.copy_cc(iv, iv + self.n_states)
        self.tree.copy_cc(self.i_phi, self.i_phi + 1)

    def restore_previous_state(self):
        """streamer.f90:654-668."""
        for iv in self.densities:
            self.tree.copy_cc(iv + self.n_states, iv)
        self.tree.copy_cc(self.i_phi + 1, self.i_phi)
        self.field_from_potential()

    def photoi_set_src(self):
        """photoi_set_src (src/m_photoi.f90:140-186), Zheleznyak + Helmholtz."""
        self.fluid.photoi_set_src(self.i_rhs, self.photoi_coeff, alpha_col=3)
        return photoi_helmh_compute(self.helm, self.helm_coeffs, self.i_photo,
                                    self.c.r("photoi_helmh%max_rel_residual"), 10)

    # ------------------------------------------------------- refinement
    def refine_desc(self):
        """default_refinement's parameters (src/m_refine.f90:198-298) as of
        global_time."""
        c = self.c
        d = capi.RefineDesc()
        d.i_electron, d.i_efld = self.i_electron, self.i_efld
        d.td_alpha_col, d.td_eta_col = 3, 4
        d.use_alpha_effective = c.i("refine_use_alpha_effective")
        d.buffer_width = c.i("refine_buffer_width")
        d.adx_fac, d.adx = c.r("refine_adx_fac"), c.r("refine_adx")
        d.min_dens, d.derefine_dx = c.r("refine_min_dens"), c.r("derefine_dx")
        d.max_dx, d.min_dx = c.r("refine_max_dx"), c.r("refine_min_dx")
        d.electrode_dx = c.r("refine_electrode_dx")
        d.init_fac = c.r("refine_init_fac")
        nd = self.ndim

        def v3(a, n):  # entry n of a list of nd-vectors, as the 3-slot field
            return [float(x) for x in a[nd * n:nd * n + nd]] + [0.0] * (3 - nd)

        d.n_seeds = 0
        if self.global_time < c.r("refine_init_time"):
            d.n_seeds = len(self.seeds)
            for n, sd in enumerate(self.seeds):
                d.seed_r0[n][:] = v3(sd["r0"], 0)
                d.seed_r1[n][:] = v3(sd["r1"], 0)
                d.seed_width[n] = sd["width"]
        rdr, rts = c.ra("refine_regions_dr"), c.ra("refine_regions_tstop")
        rmin, rmax = c.ra("refine_regions_rmin"), c.ra("refine_regions_rmax")
        k = 0
        for n in range(len(rdr)):
            if self.global_time <= rts[n]:
                d.region_dr[k] = rdr[n]
                d.region_rmin[k][:] = v3(rmin, n)
                d.region_rmax[k][:] = v3(rmax, n)
                k += 1
        d.n_regions = k
        ldr = c.ra("refine_limits_dr")
        lmin, lmax = c.ra("refine_limits_rmin"), c.ra("refine_limits_rmax")
        d.n_limits = len(ldr)
        for n in range(len(ldr)):
            d.limit_dr[n] = ldr[n]
            d.limit_rmin[n][:] = v3(lmin, n)
            d.limit_rmax[n][:] = v3(lmax, n)
        return d

    def adjust_refinement(self):
        """af_adjust_refinement with default_refinement: the criterion on the
        device, the topology on the host, the data moved by the device."""
        if self.shard is not None:
            return self._adjust_refinement_sharded()
        flags, masks = self.fluid.refine_flags(
            self.refine_desc(), self.electrode_box if self.lsf is not None else None)

        def fn(ids):
            ix = np.asarray(ids, np.int64) - 1
            return flags[ix], masks[ix]

        info = self.af.adjust_refinement(fn)
        if info.n_add or info.n_rm:
            new = self.tree.regrid(self.af.topology())
            old = self.tree
            self._bind(new)
            old.close()
            if self.i_gas_dens and info.n_add:  # m_af_core.f90:866-869
                self._set_gas([b for l in sorted(info.add) for b in info.add[l]])
        return info

    # -------------------------------------------------- initial state
    def init_cond_set_box(self, ids, arrays):
        """init_cond_set_box (src/m_init_cond.f90:217-291) on boxes `ids`
        (cells 0..nc+1), into host arrays {iv: (n_boxes, ng, ng, ng)}."""
        ng = self.af.nc + 2
        shape = (ng,) * self.ndim
        ne, ni = arrays[self.i_electron], arrays[self.i_1pos_ion]
        for b in ids:
            r = self.box_cells(b)
            e = np.full(len(r), self.background)
            p = np.full(len(r), self.background)
            for sd in self.seeds:
                dens = density_line(r, sd["r0"], sd["r1"], sd["n0"], sd["n1"],
                                    sd["width"], sd["falloff"])
                if sd["type"] == -1:
                    e = e + dens
                elif sd["type"] == 0:
                    p = p + dens
                    e = e + dens
                elif sd["type"] == 1:
                    p = p + dens
                else:
                    raise ValueError("Invalid seed_charge_type")
            if self.lsf is not None:
                # every density zero inside the electrode (m_init_cond.f90:
                # 284-288; lsf as set_lsf_box gives it, _set_electrode)
                nc = self.af.nc
                inside = self.lsf(electrode.cell_centers(
                    self.af.r_min[b], self.af.dr[b], nc, 0, nc + 1)[None])[0] <= 0
                e = np.where(inside.ravel(), 0.0, e)
                p = np.where(inside.ravel(), 0.0, p)
            ne[b - 1] = e.reshape(shape)
            ni[b - 1] = p.reshape(shape)

    def box_cells(self, b):
        """af_r_cc (r_min + (i - 0.5) dr) of every cell 0..nc+1 of box b,
        (ng^NDIM, NDIM), i fastest."""
        ng = self.af.nc + 2
        idx = np.arange(ng) - 0.5
        rmin, dr = self.af.r_min[b], self.af.dr[b]
        axes = [rmin[d] + idx * dr[d] for d in reversed(range(self.ndim))]
        g = np.meshgrid(*axes, indexing="ij")
        return np.stack([a.ravel() for a in reversed(g)], axis=1)

    def _set_gas(self, ids):
        """set_gas_density_from_user_function (streamer.f90:672-681) on boxes ids."""
        ng = self.af.nc + 2
        a = self.tree.get_cc(self.i_gas_dens)
        for b in ids:
            a[b - 1] = self.user.gas_density(self.box_cells(b)).reshape((ng,) * self.ndim)
        self.tree.put_cc(self.i_gas_dens, a)

    def _set_init(self, ids):
        arrays = {iv: self.tree.get_cc(iv) for iv in (self.i_electron, self.i_1pos_ion)}
        self.init_cond_set_box(ids, arrays)
        if self.user is not None and hasattr(self.user, "initial_conditions"):
            # user_initial_conditions after init_cond_set_box (streamer.f90:472-475)
            shape = (self.af.nc + 2,) * self.ndim
            for b in ids:
                ne, ni = self.user.initial_conditions(self, self.box_cells(b))
                arrays[self.i_electron][b - 1] = ne.reshape(shape)
                arrays[self.i_1pos_ion][b - 1] = ni.reshape(shape)
        for iv, a in arrays.items():
            self.tree.put_cc(iv, a)

    def set_initial_conditions(self):
        """streamer.f90:460-519."""
        c = self.c
        max_dx = c.r("refine_max_dx")
        lvl = 1
        while lvl < 29 and not np.all(self.af.lvl_dr(lvl) <= max_dx):
            lvl += 1
        self.af.refine_up_to_lvl(lvl)
        self._bind(self._create_tree())
        all_ids = [b for l in range(1, self.af.highest_lvl + 1)
                   for b in self.af.lvls[l]["ids"]]
        if self.i_gas_dens:
            self._set_gas(all_ids)
        self._set_init(all_ids)
        for _ in range(100):
            self.field_compute(0, have_guess=False)
            info = self.adjust_refinement()
            added = [b for l in sorted(info.add) for b in info.add[l]]
            if added:
                self._set_init(added)
            if info.n_add == 0:
                break

    # ------------------------------------------------------------- output
    def regression_row(self):
        """output_regression_log (src/m_output.f90:783-837): it, time, dt,
        then per species sum(n)/vol, sum(n^2)/vol, max(n)."""
        vol = self.af.total_volume()
        ns = len(self.species_list)
        sums, sq, mx = np.zeros(ns), np.zeros(ns), np.zeros(ns)
        for n in range(ns):
            iv = self.species_itree[n]
            if iv > 0:
                sums[n] = self.tree.sum_cc(iv, 1)
                sq[n] = self.tree.sum_cc(iv, 2)
                mx[n] = self.tree.max_cc(iv)
        return np.concatenate([[self.output_cnt, self.global_time, self.global_dt],
                               sums / vol, sq / vol, mx])

    def output_write(self):
        self.log.append(self.regression_row())

    # --------------------------------------------------------------- run
    def step(self):
        """One iteration of the main loop (streamer.f90:177-415); False at
        the end time."""
        c = self.c
        self.it += 1
        if self.time >= c.r("end_time"):
            return False
        output_dt = c.r("output%dt")
        write_out = self.time + self.dt >= self.time_last_output + output_dt
        if write_out:
            self.dt = max(0.0, self.time_last_output + output_dt - self.time)
        # (no pulses: field_pulse_period = huge, start_of_new_pulse is false)
        if self.photoi and self.it % c.i("photoi%per_steps") == 0:
            self.photoi_set_src()
            self.photoi_prev_time = self.time
        if self.lsf is not None:  # set_electrode_densities (streamer.f90:244-246)
            self.fluid.electrode_species_bc(
                self.i_lsf, self.i_1pos_ion, self.electrode_ids,
                c.s("species_boundary_condition") == "neumann_zero")
        dt_lim = 1e100
        for n in range(1, 11):
            self.copy_current_state()
            dt_lim_step = self.advance(self.dt)
            dt_lim = min(dt_lim, dt_lim_step)
            if self.dt <= dt_lim_step:
                break
            self.n_steps_rejected += 1
            self.dt = self.dt_safety * dt_lim_step
            self.time = self.global_time
            write_out = False
            self.restore_previous_state()
        else:
            raise RuntimeError("All time steps were rejected")
        self.frac_rejected = 0.99 * self.frac_rejected + (0.01 if n > 1 else 0.0)
        self.field_compute(0, True)
        tmp = self.dt_growth if self.frac_rejected <= 0.1 else 1.0
        self.dt = min(tmp * self.global_dt, self.dt_safety * min(dt_lim, self.dt_max))
        self.global_dt = self.dt
        self.global_time = self.time
        # dt below dt_min: the reference writes the output (its regression
        # row included) and then stops (streamer.f90:357-378)
        if self.global_dt < self.dt_min:
            write_out = True
        if write_out:
            self.output_cnt += 1
            self.time_last_output = self.global_time
            self.output_write()
        if self.global_dt < self.dt_min:
            raise RuntimeError("dt too small")
        if self.it % c.i("refine_per_steps") == 0:
            for iv in self.densities:
                self.tree.restrict_tree(iv)
                self.tree.gc_tree(iv)
            info = self.adjust_refinement()
            if info.n_add > 0 or info.n_rm > 0:
                self.field_compute(0, True)
                if self.photoi:
                    self.photoi_set_src()
                    self.photoi_prev_time = self.time
        return True

    def clone(self, lib, device=-1):
        """The same simulation state on another library (e.g. the C oracle
        for a CPU baseline): topology, every cell and face variable, time."""
        import copy
        other = Simulation(lib, self.c, device=device, coarse_cycles=self.coarse_cycles,
                           coarse_tol=self.coarse_tol, coarse_mode=self.coarse_mode,
                           capacity_factor=self.capacity_factor, fuse_rhs=self.fused_rhs,
                           user=self.user)
        other.af = copy.deepcopy(self.af)
        for k in ("it", "time", "global_time", "photoi_prev_time", "global_dt", "dt",
                  "output_cnt", "time_last_output"):
            if hasattr(self, k):
                setattr(other, k, getattr(self, k))
        other._bind(other._create_tree())
        for iv in range(1, self.n_var_cell + 1):
            other.tree.put_cc(iv, self.tree.get_cc(iv))
        for iv in range(1, self.n_var_face + 1):
            other.tree.put_fc(iv, self.tree.get_fc(iv))
        return other

    # ------------------------------------------------------- .dat files
    def write_dat(self, name):
        """af_write_tree(tree, name, write_sim_data) as the streamer's output
        does (m_af_output.f90:41-194, streamer.f90:521-536): the topology of
        the host tree, every cell and face variable from the device, the
        simulation record appended; writes name + ".dat". The global
        reaction rates and J.E integrals (ST_global_rates / JdotE, outputs of
        the reference's analysis module, not computed here) are written as
        zeros."""
        from .datfile import DatTree, sim_data_bytes
        if self.faces_from_phi:
            # the face field the reference stores: mg_box_lpl_gradient of the
            # potential the last field_from_potential used (phi unchanged since)
            self.mg.compute_phi_gradient(self.f_field, -1.0, 0)
        t = DatTree.from_aftree(self.af, self.cc_names, self.c.sa("fc_names"))
        used = [b for b in range(1, self.af.highest_id + 1) if self.af.in_use[b]]
        for iv in range(1, self.n_var_cell + 1):
            a = self.tree.get_cc(iv)
            for b in used:
                t.boxes[b].cc[iv] = a[b - 1]
        for iv in range(1, self.n_var_face + 1):
            a = self.tree.get_fc(iv)
            for b in used:
                t.boxes[b].fc[iv] = a[b - 1]
        t.other = sim_data_bytes(self.it, self.output_cnt, self.time, self.global_time,
                                 self.photoi_prev_time, self.global_dt,
                                 np.zeros(len(self.reactions)), 0.0, self.frac_rejected)
        t.write(name + ".dat")
        return t

    def restart(self, path):
        """restart_from_file (streamer.f90:117-138): af_read_tree with
        read_sim_data, the consistency checks, then the device tree built
        from the file's topology and data (box ids as stored)."""
        from .datfile import DatTree, parse_sim_data
        t = DatTree.read(path)
        if t.n_cell != self.af.nc:
            raise ValueError("restart_from_file: incompatible box size")
        if t.n_var_cell != self.n_var_cell:
            raise ValueError("restart_from_file: incompatible variable list")
        if t.other is None:
            raise ValueError("af_read_tree: other data is not present")
        d = parse_sim_data(t.other, len(self.reactions))
        self.af = t.aftree()
        self._bind(self._create_tree())
        nb = self.tree.n_boxes
        for iv in range(1, self.n_var_cell + 1):
            a = np.zeros(self.tree.cc_shape)
            if t.cc_write_binary[iv - 1]:
                for b, box in t.boxes.items():
                    a[b - 1] = box.cc[iv]
            self.tree.put_cc(iv, a[:nb])
        for iv in range(1, self.n_var_face + 1):
            a = np.zeros(self.tree.fc_shape)
            if t.fc_write_binary[iv - 1]:
                for b, box in t.boxes.items():
                    a[b - 1] = box.fc[iv]
            self.tree.put_fc(iv, a[:nb])
        self.it, self.output_cnt = d["it"], d["output_cnt"]
        self.time, self.global_time = d["time"], d["global_time"]
        self.photoi_prev_time, self.global_dt = d["photoi_prev_time"], d["global_dt"]
        self.frac_rejected = d["fraction_steps_rejected"]
        self.dt = self.global_dt
        self.time_last_output = self.time  # streamer.f90:172
        return t

    def start(self):
        self.set_initial_conditions()
        self.output_cnt = 0
        self.output_write()
        self.time_last_output = self.time

    def run(self, max_steps=None):
        self.start()
        n = 0
        while self.step():
            n += 1
            if max_steps is not None and n >= max_steps:
                break
        return np.array(self.log)
