"""ctypes mirror of include/afivo_hip.h.

The same structures and signatures serve two shared libraries:
  * the product, libafivo_hip.so (prefix ``afh_``), built from csrc/;
  * the test oracle, oracle/lib/libafo.so (prefix ``afo_``) -- loaded only by
    tests/, __graft_entry__.smoke() and bench.py's cpu_baseline.
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
REPO = os.path.dirname(PKG)
# AFH_HIP_LIB: an alternative build of the same library (A/B timing of
# kernel variants on one box, scripts/ab.sh)
HIP_LIB = os.environ.get("AFH_HIP_LIB") or os.path.join(PKG, "csrc", "libafivo_hip.so")
ORACLE_LIB = os.path.join(REPO, "oracle", "lib", "libafo.so")
# the NDIM = 2 build (BASELINE config 1; include/afivo_hip_2d.h)
HIP_LIB_2D = os.path.join(PKG, "csrc", "libafivo_hip_2d.so")

AFH_OK = 0
BC_DIRICHLET, BC_NEUMANN, BC_CONTINUOUS, BC_DIRICHLET_COPY = -10, -11, -12, -13
RB_GC_INTERP, RB_GC_INTERP_LIM, RB_MG_SIDES = 1, 2, 3
LIM_NONE, LIM_VANLEER, LIM_KOREN, LIM_MINMOD, LIM_MC, LIM_GMINMOD43, LIM_ZERO = range(1, 8)
RATE_TABULATED_FIELD, RATE_CONSTANT, RATE_LINEAR, RATE_EXP_V1, RATE_EXP_V2 = range(1, 6)
RATE_K1, RATE_K3 = 6, 8
(RATE_K4, RATE_K5, RATE_K6, RATE_K7, RATE_K8, RATE_K9, RATE_K10, RATE_K11,
 RATE_K12, RATE_K13, RATE_K14, RATE_K15) = range(9, 21)
COARSE_CYCLES, COARSE_DIRECT, COARSE_PFMG = 1, 2, 3
MAX_SPECIES = 32
MAX_IONS = 8
MAX_REACTIONS = 128

i32 = C.c_int32
f64 = C.c_double
P_i32 = C.POINTER(i32)
P_f64 = C.POINTER(f64)


class BoxMeta(C.Structure):
    _fields_ = [("lvl", i32), ("ix", i32 * 3), ("parent", i32),
                ("children", i32 * 8), ("neighbors", i32 * 6),
                ("neighbor_mat", i32 * 27), ("r_min", f64 * 3), ("dr", f64 * 3)]


BOX_META_DTYPE = np.dtype([("lvl", "<i4"), ("ix", "<i4", 3), ("parent", "<i4"),
                           ("children", "<i4", 8), ("neighbors", "<i4", 6),
                           ("neighbor_mat", "<i4", 27),
                           ("r_min", "<f8", 3), ("dr", "<f8", 3)])


class TreeDesc(C.Structure):
    _fields_ = [("n_cell", i32), ("n_boxes", i32), ("highest_lvl", i32),
                ("n_var_cell", i32), ("n_var_face", i32),
                ("coarse_grid_size", i32 * 3), ("periodic", i32 * 3),
                ("r_base", f64 * 3), ("dr_base", f64 * 3),
                ("boxes", C.c_void_p),
                ("lvl_ids", P_i32), ("lvl_ids_off", P_i32),
                ("lvl_leaves", P_i32), ("lvl_leaves_off", P_i32),
                ("lvl_parents", P_i32), ("lvl_parents_off", P_i32),
                ("box_capacity", i32)]


class BC(C.Structure):
    _fields_ = [("type", i32), ("value", f64)]


class LT(C.Structure):
    _fields_ = [("n_points", i32), ("n_cols", i32), ("x_min", f64),
                ("inv_fac", f64), ("rows_cols", P_f64)]


class Reaction(C.Structure):
    _fields_ = [("rate_type", i32), ("table_col", i32), ("rate_factor", f64),
                ("c", f64 * 4), ("n_in", i32), ("ix_in", i32 * 4),
                ("n_out", i32), ("ix_out", i32 * 4), ("mult_out", i32 * 4)]


class FluidDesc(C.Structure):
    _fields_ = [("n_species", i32), ("species_iv", i32 * MAX_SPECIES),
                ("species_charge", i32 * MAX_SPECIES), ("i_electron", i32),
                ("i_efld", i32), ("f_flux", i32), ("f_field", i32),
                ("limiter", i32), ("gas_number_density", f64), ("td", LT),
                ("chem", LT), ("n_reactions", i32),
                ("reactions", C.POINTER(Reaction)), ("dt_chemistry_nmin", f64),
                ("gas_temperature", f64), ("td_energy_col", i32),
                ("i_gas_dens", i32), ("n_gas_species", i32),
                ("gas_fractions", f64 * 8), ("i_photo", i32),
                ("photo_species", i32), ("n_ions", i32),
                ("ion_species", i32 * MAX_IONS), ("f_ion_flux", i32 * MAX_IONS),
                ("ion_mobility", f64 * MAX_IONS)]


class MgDesc(C.Structure):
    _fields_ = [("i_phi", i32), ("i_rhs", i32), ("i_tmp", i32),
                ("n_cycle_down", i32), ("n_cycle_up", i32),
                ("helmholtz_lambda", f64), ("coarse_mode", i32),
                ("coarse_cycles", i32), ("coarse_tol", f64)]


MAX_REFINE_REGIONS = 8
RM_REF, KEEP_REF, DO_REF = -1, 0, 1
_R = MAX_REFINE_REGIONS


class RefineDesc(C.Structure):
    """afh_refine_desc: default_refinement's parameters (src/m_refine.f90)."""
    _fields_ = [("i_electron", i32), ("i_efld", i32), ("td_alpha_col", i32),
                ("td_eta_col", i32), ("use_alpha_effective", i32),
                ("buffer_width", i32), ("adx_fac", f64), ("adx", f64),
                ("min_dens", f64), ("derefine_dx", f64), ("max_dx", f64),
                ("min_dx", f64), ("electrode_dx", f64), ("n_seeds", i32),
                ("init_fac", f64), ("seed_r0", (f64 * 3) * _R),
                ("seed_r1", (f64 * 3) * _R), ("seed_width", f64 * _R),
                ("n_regions", i32), ("region_dr", f64 * _R),
                ("region_rmin", (f64 * 3) * _R), ("region_rmax", (f64 * 3) * _R),
                ("n_limits", i32), ("limit_dr", f64 * _R),
                ("limit_rmin", (f64 * 3) * _R), ("limit_rmax", (f64 * 3) * _R)]


assert C.sizeof(BoxMeta) == BOX_META_DTYPE.itemsize, (C.sizeof(BoxMeta),
                                                      BOX_META_DTYPE.itemsize)

# name -> (restype, argtypes); names without prefix
_VP = C.c_void_p
_PVP = C.POINTER(C.c_void_p)
SIGNATURES = {
    "last_error": (C.c_char_p, []),
    "tree_create": (i32, [C.POINTER(TreeDesc), i32, _PVP]),
    "set_cc_prolong": (i32, [_VP, i32, i32, i32]),
    "refine_cell_flags": (i32, [i32, C.c_uint32, i32, i32, P_i32]),
    "refine_flags": (i32, [_VP, C.POINTER(RefineDesc), C.POINTER(C.c_uint8),
                           P_i32, C.POINTER(C.c_uint32)]),
    "tree_regrid": (i32, [_VP, C.POINTER(TreeDesc), _PVP]),
    "tree_destroy": (i32, [_VP]),
    "tree_sync": (i32, [_VP]),
    "set_cc_methods": (i32, [_VP, i32, C.POINTER(BC), i32, i32]),
    "set_bc": (i32, [_VP, i32, i32, i32, f64]),
    "cc_put": (i32, [_VP, i32, P_f64]),
    "cc_get": (i32, [_VP, i32, P_f64]),
    "fc_put": (i32, [_VP, i32, P_f64]),
    "fc_get": (i32, [_VP, i32, P_f64]),
    "tree_pack_boxes": (i32, [_VP, P_i32, i32, i32, i32, P_f64]),
    "tree_unpack_boxes": (i32, [_VP, P_i32, i32, i32, i32, P_f64]),
    "device_alloc": (i32, [i32, C.c_int64, C.POINTER(_VP)]),
    "device_free": (i32, [_VP]),
    "gc_lvl": (i32, [_VP, i32, i32, i32]),
    "gc_tree": (i32, [_VP, i32, i32]),
    "restrict_tree": (i32, [_VP, i32]),
    "tree_copy_cc": (i32, [_VP, i32, i32]),
    "tree_maxabs_cc": (i32, [_VP, i32, P_f64]),
    "tree_sum_cc": (i32, [_VP, i32, i32, P_f64]),
    "tree_reduce_loc": (i32, [_VP, i32, i32, P_f64, P_i32]),
    "mg_create": (i32, [_VP, C.POINTER(MgDesc), _PVP]),
    "mg_destroy": (i32, [_VP]),
    "mg_fas_vcycle": (i32, [_VP, i32, i32]),
    "mg_fas_vcycle_maxres": (i32, [_VP, i32, P_f64]),
    "mg_fas_vcycle_fold": (i32, [_VP, i32]),
    "tree_fetch_reduced": (i32, [_VP, i32, P_i32, P_f64]),
    "mg_fas_fmg": (i32, [_VP, i32, i32]),
    "mg_coarse_iterations": (i32, [_VP, P_i32]),
    "mg_graph_stats": (i32, [_VP, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
    "mg_set_gradient_output": (i32, [_VP, i32, f64]),
    "mg_compute_phi_gradient": (i32, [_VP, i32, f64, i32]),
    "mg_set_box_stencil": (i32, [_VP, i32, P_f64, P_f64]),
    "mg_set_box_lsf": (i32, [_VP, i32, i32, P_i32, P_f64, P_f64, i32]),
    "fluid_create": (i32, [_VP, C.POINTER(FluidDesc), _PVP]),
    "fluid_destroy": (i32, [_VP]),
    "electrode_species_bc": (i32, [_VP, i32, i32, i32, i32, P_i32]),
    "fluid_set_update_mask": (i32, [_VP, i32]),
    "fluid_set_rhs_output": (i32, [_VP, i32, i32]),
    "fluid_set_field_source": (i32, [_VP, i32, f64]),
    "fluid_set_ion_se_yield": (i32, [_VP, f64]),
    "fluid_ion_se_flux": (i32, [_VP]),
    "fluid_rhs_maxabs": (i32, [_VP, i32, P_f64]),
    "fluid_rhs_valid": (i32, [_VP, i32, P_i32]),
    "photoi_set_src": (i32, [_VP, i32, i32, f64]),
    "photoi_helmh_compute": (i32, [C.POINTER(_VP), i32, P_f64, i32, f64, i32, P_i32]),
    "field_set_rhs": (i32, [_VP, i32, i32]),
    "field_set_rhs_maxabs": (i32, [_VP, i32, i32, P_f64]),
    "flux_upwind_tree": (i32, [_VP, i32, P_f64]),
    "flux_update_densities": (i32, [_VP, f64, i32, i32, P_i32, P_f64, i32,
                                    i32, P_f64]),
    "fluid_forward_euler": (i32, [_VP, f64, i32, i32, P_i32, P_f64, i32, i32,
                                  i32, P_f64]),
    "fluid_forward_euler_fold": (i32, [_VP, f64, i32, i32, P_i32, P_f64, i32, i32, i32]),
    "fluid_fetch_step": (i32, [_VP, i32, i32, P_i32, P_f64, P_f64]),
    "profile_enable": (i32, [_VP, i32]),
    "profile_read": (i32, [_VP, P_f64, C.POINTER(C.c_int64), P_f64]),
    "tree_set_hook": (i32, [_VP, C.c_void_p, _VP]),
    "tree_set_stream": (i32, [_VP, _VP]),
    "plan_create": (i32, [_VP, P_i32, i32, P_i32, C.POINTER(C.c_int64)]),
    "plan_create_fc": (i32, [_VP, P_i32, i32, P_i32, C.POINTER(C.c_int64)]),
    "plan_pack": (i32, [_VP, i32, i32, _VP]),
    "plan_unpack": (i32, [_VP, i32, i32, _VP]),
    # native box sharding
    "dist_partition": (i32, [C.POINTER(TreeDesc), i32, P_i32, P_i32]),
    "dist_partition_levels": (i32, [C.POINTER(TreeDesc), i32, C.c_int64, P_i32, P_i32]),
    "dist_plan": (i32, [C.POINTER(TreeDesc), P_i32, i32, i32, i32, i32, P_i32, i32, P_i32]),
    "dist_local_ids": (i32, [C.POINTER(TreeDesc), P_i32, i32, P_i32, i32, P_i32]),
    "tree_create_sharded": (i32, [C.POINTER(TreeDesc), P_i32, i32, i32, _PVP]),
    "dist_group_create": (i32, [i32, _PVP]),
    "dist_group_destroy": (i32, [_VP]),
    "dist_rccl_unique_id": (i32, [_VP]),
    "dist_rccl_comm": (i32, [_VP, i32, i32, i32, _PVP]),
    "dist_rccl_comm_destroy": (i32, [_VP]),
    "dist_create": (i32, [_VP, C.POINTER(TreeDesc), P_i32, i32, i32, i32, _VP, _PVP]),
    "dist_destroy": (i32, [_VP]),
    "dist_stats": (i32, [_VP, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
    "dist_peer_bytes": (i32, [_VP, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
}
DIST_LOCAL, DIST_RCCL = 1, 2
HOOK_HALO, HOOK_RIMS, HOOK_RESTRICT, HOOK_MAX, HOOK_MIN, HOOK_CFLUX = 1, 2, 3, 4, 5, 6
HOOK_SUM = 7
RED_MAX, RED_MIN, RED_MAXABS = 1, 2, 3
# deferred reduction slots (afh_tree_fetch_reduced, afh_fluid_fetch_step)
SLOT_MAXRES, SLOT_RHS = 3, 4
# int32_t (*)(void *ctx, int32_t kind, int32_t level, int32_t iv, double *vals,
#             int32_t n)
HOOK_FN = C.CFUNCTYPE(i32, C.c_void_p, i32, i32, i32, P_f64, i32)
PROF_GSRB, PROF_GHOST, PROF_FLUX, PROF_UPDATE, PROF_GSRB_PAIR, PROF_GSRB_PAIR_TILED = 1, 2, 3, 4, 5, 6
PROF_FE = 7
PROF_CS = 8
PROLONG_NONE, PROLONG_LINEAR, PROLONG_LIMIT = 0, 1, 2
ORACLE_EXTRA = {
    "mg_gsrb_boxes": (i32, [_VP, i32, i32]),
    "mg_update_coarse": (i32, [_VP, i32]),
    "mg_solve_coarse": (i32, [_VP]),
    "mg_correct_children": (i32, [_VP, i32]),
}


class AfhError(RuntimeError):
    pass


class Library:
    """A loaded C-ABI library; call functions without their prefix."""

    def __init__(self, path, prefix, extra=None, only=None):
        """only: the entry points the library implements (a subset of
        SIGNATURES; the 2-D build's, include/afivo_hip_2d.h)."""
        if not os.path.exists(path):
            raise AfhError("shared library not built: %s" % path)
        self.path = path
        self.prefix = prefix
        self.lib = C.CDLL(path)
        sigs = dict(SIGNATURES)
        if extra:
            sigs.update(extra)
        if only is not None:
            sigs = {n: sigs[n] for n in only}
        self.fn = {}
        for name, (res, args) in sigs.items():
            f = getattr(self.lib, prefix + name)
            f.restype = res
            f.argtypes = args
            self.fn[name] = f

    def call(self, name, *args):
        rc = self.fn[name](*args)
        if rc != AFH_OK:
            msg = self.fn["last_error"]().decode()
            raise AfhError("%s%s failed (%d): %s" % (self.prefix, name, rc, msg))
        return rc

    def symbols(self):
        return [self.prefix + n for n in self.fn]

    def has(self, name):
        """Whether the library implements entry point `name` (the 2-D build
        exports a subset, include/afivo_hip_2d.h)."""
        return name in self.fn


_loaded = {}


def hip_library():
    """The product library. Raises if it was not built -- no CPU fallback."""
    if "hip" not in _loaded:
        _loaded["hip"] = Library(HIP_LIB, "afh_")
    return _loaded["hip"]


def hip_library_2d():
    """The NDIM = 2 product library (the entry points of afivo_hip_2d.h).
    Raises if it was not built -- no CPU fallback."""
    if "hip2d" not in _loaded:
        only = [n[len("afh_"):] for n in header_symbols("afivo_hip_2d.h")]
        _loaded["hip2d"] = Library(HIP_LIB_2D, "afh_", only=only)
    return _loaded["hip2d"]


def oracle_library():
    """The test oracle (oracle/lib/libafo.so)."""
    if "oracle" not in _loaded:
        _loaded["oracle"] = Library(ORACLE_LIB, "afo_", ORACLE_EXTRA)
    return _loaded["oracle"]


def header_symbols(header="afivo_hip.h"):
    """Every afh_* function declared in include/<header>."""
    import re
    src = open(os.path.join(REPO, "include", header)).read()
    return sorted(set(re.findall(r"\b(afh_[a-z_0-9]+)\s*\(", src)))
