"""Host-side mirror of the reference's operator surface over the C ABI.

Names follow the Fortran routines they stand for: ``Tree`` is af_t with its
box pool on the device, ``Multigrid`` is mg_t (mg_fas_vcycle,
mg_compute_phi_gradient), ``Fluid`` is the m_fluid / m_field module state
(field_set_rhs, flux_upwind_tree, flux_update_densities). Every method calls
straight through to the shared library it was created with; there is no
Python compute path.
"""
import ctypes as C

import numpy as np

from . import capi


def _i32(a):
    return np.ascontiguousarray(a, dtype=np.int32)


def _lists(topo, kind):
    h = int(topo["highest_lvl"])
    arrs = [np.asarray(topo["lvl_%s_%d" % (kind, l)], np.int32) for l in range(1, h + 1)]
    off = np.zeros(h + 1, np.int32)
    off[1:] = np.cumsum([len(a) for a in arrs])
    flat = np.concatenate(arrs) if arrs else np.zeros(0, np.int32)
    return _i32(flat), off


def tree_desc(topo, n_var_cell, n_var_face, box_capacity=0):
    """afh_tree_desc of a topology dict; returns (desc, arrays it points to).
    A 2-D topology (topo["ndim"] == 2: ix / r_min / dr of 2, children and
    neighbors of 4, a 3 x 3 neighbor_mat) fills the leading entries of the
    3-D-sized fields (include/afivo_hip_2d.h)."""
    nb = int(topo["n_boxes"])
    meta = np.zeros(nb, capi.BOX_META_DTYPE)
    for k in ("lvl", "ix", "parent", "children", "neighbors", "neighbor_mat", "r_min", "dr"):
        v = np.asarray(topo["meta_" + k])
        if v.ndim == 2 and v.shape[1] < meta[k].shape[1]:
            meta[k][:, :v.shape[1]] = v
        else:
            meta[k] = v
    lists = {k: _lists(topo, k) for k in ("ids", "leaves", "parents")}
    pad = lambda a, fill: [x for x in a] + [fill] * (3 - len(a))  # noqa: E731
    d = capi.TreeDesc()
    d.n_cell, d.n_boxes, d.highest_lvl = int(topo["nc"]), nb, int(topo["highest_lvl"])
    d.n_var_cell, d.n_var_face = n_var_cell, n_var_face
    d.coarse_grid_size[:] = pad([int(x) for x in topo["coarse_grid_size"]], 1)
    d.periodic[:] = [0, 0, 0]
    d.r_base[:] = pad([float(x) for x in topo["r_base"]], 0.0)
    d.dr_base[:] = pad([float(x) for x in topo["dr_base"]], 0.0)
    d.boxes = meta.ctypes.data
    d.box_capacity = int(box_capacity)
    for k in ("ids", "leaves", "parents"):
        flat, off = lists[k]
        setattr(d, "lvl_%s" % k, flat.ctypes.data_as(capi.P_i32))
        setattr(d, "lvl_%s_off" % k, off.ctypes.data_as(capi.P_i32))
    return d, (meta, lists)


class DeviceRows:
    """An (n, w) float64 array in device memory owned by the library
    (afh_device_alloc): the row buffer of Tree.pack_boxes / unpack_boxes when
    no torch device tensor is used (the thread ranks of one process)."""

    def __init__(self, lib, device, n, w):
        self.lib, self.shape = lib, (int(n), int(w))
        p = C.c_void_p()
        lib.call("device_alloc", int(device), 8 * self.shape[0] * self.shape[1], C.byref(p))
        self._p = p

    def data_ptr(self):
        return self._p.value or 0

    def is_contiguous(self):
        return True

    def close(self):
        if self._p:
            self.lib.call("device_free", self._p)
            self._p = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Tree:
    """af_t: topology + device box pool of n_var_cell / n_var_face variables."""

    def __init__(self, lib, topo, n_var_cell, n_var_face, device=-1, _regrid_of=None,
                 box_capacity=0, shard_of=None):
        """box_capacity: boxes the device pools hold (afivo's box_limit; 0 =
        the topology's box count); a regrid that fits them works in place.
        shard_of: (full topology, owner, rank) -- the library builds this
        rank's part of a sharded tree (afh_tree_create_sharded); `topo` is
        then that rank's view (afh.dist.local_topology)."""
        self.lib = lib
        self.topo = topo
        # multigrid / fluid objects bound to this tree: closed before it, so
        # that no library object outlives the tree it points to. Strong
        # references: the garbage collector clears weak references before it
        # finalizes a cycle, in any order.
        self._deps = []
        self.nc = int(topo["nc"])
        self.ndim = int(topo.get("ndim", 3))
        self.n_boxes = int(topo["n_boxes"])
        self.highest_lvl = int(topo["highest_lvl"])
        self.n_var_cell = n_var_cell
        self.n_var_face = n_var_face
        self.box_capacity = int(box_capacity)
        d, self._keep = tree_desc(topo, n_var_cell, n_var_face, self.box_capacity)
        h = C.c_void_p()
        # sharded: the global id of every stored box, in local-id order (the
        # library stores only the boxes the rank reads, plus one unused id)
        self.global_ids = None
        if shard_of is not None:
            # this rank's boxes of the full tree (afh_tree_create_sharded)
            full, self._keep_full = tree_desc(shard_of[0], n_var_cell, n_var_face)
            owner = np.ascontiguousarray(shard_of[1], np.int32)
            pown, rank = owner.ctypes.data_as(capi.P_i32), int(shard_of[2])
            n = C.c_int32()
            lib.call("dist_local_ids", C.byref(full), pown, rank, None, 0, C.byref(n))
            gids = np.zeros(n.value, np.int32)
            lib.call("dist_local_ids", C.byref(full), pown, rank,
                     gids.ctypes.data_as(capi.P_i32), n.value, C.byref(n))
            self.global_ids = gids
            self.n_global = self.n_boxes
            self.n_boxes = n.value + 1
            lib.call("tree_create_sharded", C.byref(full), pown, rank, device, C.byref(h))
        elif _regrid_of is None:
            lib.call("tree_create", C.byref(d), device, C.byref(h))
        else:
            lib.call("tree_regrid", _regrid_of.h, C.byref(d), C.byref(h))
        self.h = h

    def regrid(self, topo):
        """af_adjust_refinement's data movement onto the new topology `topo`
        (afh_tree_regrid): a new Tree. When the new tree fits this one's
        pools (box_capacity) the data stay in place and this tree keeps only
        its topology; otherwise it stays valid."""
        return Tree(self.lib, topo, self.n_var_cell, self.n_var_face,
                    _regrid_of=self, box_capacity=self.box_capacity)

    def set_cc_prolong(self, iv, method, limiter=None):
        """tree%cc_methods(iv)%prolong (capi.PROLONG_LINEAR / PROLONG_LIMIT)
        and prolong_limiter; iv becomes an automatic variable. The default
        limiter is af_set_cc_methods' own: MC in 2-D, gminmod43 in 3-D
        (m_af_core.f90:399-408)."""
        if limiter is None:
            limiter = capi.LIM_MC if self.ndim < 3 else capi.LIM_GMINMOD43
        self.lib.call("set_cc_prolong", self.h, iv, method, limiter)

    # -- lifetime
    def close(self):
        for d in list(self._deps):
            d.close()
        if self.h:
            self.lib.call("tree_destroy", self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def sync(self):
        self.lib.call("tree_sync", self.h)

    # -- methods / data
    @property
    def cc_shape(self):
        return (self.n_boxes,) + (self.nc + 2,) * self.ndim

    @property
    def fc_shape(self):
        return (self.n_boxes, self.ndim) + (self.nc + 1,) * self.ndim

    def set_cc_methods(self, iv, bc, rb=capi.RB_GC_INTERP, prolong_limiter=None):
        """af_set_cc_methods; bc is a list of 2 ndim (type, value) pairs. The
        default prolong_limiter is af_set_cc_methods' own: MC in 2-D,
        gminmod43 in 3-D (m_af_core.f90:399-408)."""
        if prolong_limiter is None:
            prolong_limiter = capi.LIM_MC if self.ndim < 3 else capi.LIM_GMINMOD43
        arr = (capi.BC * 6)()
        for n, (t, v) in enumerate(bc[:2 * self.ndim]):
            arr[n].type, arr[n].value = int(t), float(v)
        self.lib.call("set_cc_methods", self.h, iv, arr, rb, prolong_limiter)

    def set_bc(self, iv, nb, bc_type, value):
        self.lib.call("set_bc", self.h, iv, nb, bc_type, float(value))

    def local_id(self, box_id):
        """The library's id of global box id (0: a sharded tree does not store it)."""
        if self.global_ids is None:
            return int(box_id)
        k = int(np.searchsorted(self.global_ids, box_id))
        return k + 1 if k < len(self.global_ids) and self.global_ids[k] == box_id else 0

    def _to_local(self, a):
        """A whole-tree array -> the stored boxes (the unused last id NaN)."""
        if self.global_ids is None or a.shape[0] == self.n_boxes:
            return a
        assert a.shape[0] == self.n_global, (a.shape, self.n_global)
        out = np.full((self.n_boxes,) + a.shape[1:], np.nan)
        out[:-1] = a[self.global_ids - 1]
        return out

    def _to_global(self, a):
        """Stored boxes -> a whole-tree array (NaN where not stored)."""
        if self.global_ids is None:
            return a
        out = np.full((self.n_global,) + a.shape[1:], np.nan)
        out[self.global_ids - 1] = a[:-1]
        return out

    def put_cc(self, iv, arr):
        """Whole-tree array (n_boxes, ng, ng, ng); a sharded tree takes the
        whole tree's array (or its stored boxes', local_shape)."""
        a = np.ascontiguousarray(self._to_local(np.asarray(arr, np.float64)))
        assert a.shape == self.cc_shape, (a.shape, self.cc_shape)
        self.lib.call("cc_put", self.h, iv, a.ctypes.data_as(capi.P_f64))

    def get_cc(self, iv):
        a = np.empty(self.cc_shape)
        self.lib.call("cc_get", self.h, iv, a.ctypes.data_as(capi.P_f64))
        return self._to_global(a)

    def row_width(self, n_cc, n_fc):
        """Doubles per box row of pack_boxes / unpack_boxes."""
        return (n_cc * int(np.prod(self.cc_shape[1:])) +
                n_fc * int(np.prod(self.fc_shape[1:])))

    def pack_boxes(self, lids, n_cc, n_fc, buf):
        """Boxes `lids` (local ids, 1-based) into the rows of `buf`, a
        contiguous float64 device tensor of len(lids) x row_width(n_cc, n_fc)
        on the tree's device: cell variables 1..n_cc, then face variables
        1..n_fc (afh_tree_pack_boxes; no host copy)."""
        ids = np.ascontiguousarray(lids, np.int32)
        assert buf.is_contiguous() and tuple(buf.shape) == (len(ids), self.row_width(n_cc, n_fc))
        self.lib.call("tree_pack_boxes", self.h, ids.ctypes.data_as(capi.P_i32), len(ids),
                      n_cc, n_fc, C.cast(buf.data_ptr(), capi.P_f64))

    def unpack_boxes(self, lids, n_cc, n_fc, buf):
        """The rows of `buf` into boxes `lids` (afh_tree_unpack_boxes)."""
        ids = np.ascontiguousarray(lids, np.int32)
        assert buf.is_contiguous() and tuple(buf.shape) == (len(ids), self.row_width(n_cc, n_fc))
        self.lib.call("tree_unpack_boxes", self.h, ids.ctypes.data_as(capi.P_i32), len(ids),
                      n_cc, n_fc, C.cast(buf.data_ptr(), capi.P_f64))

    def get_cc_local(self, iv):
        """The stored boxes' array (a sharded tree's local ids; the unused
        last id NaN) -- no whole-tree array."""
        a = np.empty(self.cc_shape)
        self.lib.call("cc_get", self.h, iv, a.ctypes.data_as(capi.P_f64))
        return a

    def get_fc_local(self, ivf):
        a = np.empty(self.fc_shape)
        self.lib.call("fc_get", self.h, ivf, a.ctypes.data_as(capi.P_f64))
        return a

    def put_fc(self, ivf, arr):
        a = np.ascontiguousarray(self._to_local(np.asarray(arr, np.float64)))
        assert a.shape == self.fc_shape
        self.lib.call("fc_put", self.h, ivf, a.ctypes.data_as(capi.P_f64))

    def get_fc(self, ivf):
        a = np.empty(self.fc_shape)
        self.lib.call("fc_get", self.h, ivf, a.ctypes.data_as(capi.P_f64))
        return self._to_global(a)

    # -- afivo tree operations
    def gc_lvl(self, lvl, iv, corners=True):
        self.lib.call("gc_lvl", self.h, lvl, iv, int(corners))

    def gc_tree(self, iv, corners=True):
        self.lib.call("gc_tree", self.h, iv, int(corners))

    def restrict_tree(self, iv):
        self.lib.call("restrict_tree", self.h, iv)

    def copy_cc(self, iv_from, iv_to):
        self.lib.call("tree_copy_cc", self.h, iv_from, iv_to)

    def maxabs_cc(self, iv):
        out = C.c_double()
        self.lib.call("tree_maxabs_cc", self.h, iv, C.byref(out))
        return out.value

    def fetch_reduced(self, *slots):
        """The |x| maxima folded on the device by the deferred entry points
        (capi.SLOT_MAXRES, capi.SLOT_RHS), read in one transfer."""
        sl = _i32(slots)
        out = (C.c_double * len(sl))()
        self.lib.call("tree_fetch_reduced", self.h, len(sl), sl.ctypes.data_as(capi.P_i32), out)
        return list(out)

    def sum_cc(self, iv, power=1):
        """af_tree_sum_cc (m_af_utils.f90:966-1026): volume-weighted sum of
        cc(iv)**power over the leaf interiors."""
        out = C.c_double()
        self.lib.call("tree_sum_cc", self.h, iv, int(power), C.byref(out))
        return out.value

    def reduce_loc(self, iv, op, with_loc=True):
        """af_tree_max_cc / af_tree_min_cc / af_tree_maxabs_cc (op =
        capi.RED_MAX / RED_MIN / RED_MAXABS): (value, (id, i, j, k)) -- the
        af_loc_t of the first extremum in the reference's loop order."""
        out = C.c_double()
        loc = np.zeros(4, np.int32)
        self.lib.call("tree_reduce_loc", self.h, iv, int(op), C.byref(out),
                      loc.ctypes.data_as(capi.P_i32) if with_loc else None)
        return out.value, (tuple(int(x) for x in loc) if with_loc else None)

    def max_cc(self, iv):
        return self.reduce_loc(iv, capi.RED_MAX, with_loc=False)[0]

    def min_cc(self, iv):
        return self.reduce_loc(iv, capi.RED_MIN, with_loc=False)[0]


class Multigrid:
    """mg_t bound to a tree (mg_init / mg_fas_vcycle)."""

    def __init__(self, tree, i_phi, i_rhs, i_tmp, n_cycle_down=2, n_cycle_up=2,
                 helmholtz_lambda=0.0, coarse_cycles=20, coarse_mode=None,
                 coarse_tol=0.0):
        """coarse_mode: capi.COARSE_CYCLES (coarse_cycles MG cycles on the
        level-1 grid) or capi.COARSE_DIRECT (exact separable solve); None
        picks COARSE_DIRECT when coarse_cycles == 0. coarse_tol > 0 (cycles
        only): HYPRE PFMG's stopping rule, |r|_2 < coarse_tol |b|_2 within at
        most coarse_cycles cycles."""
        if coarse_mode is None:
            coarse_mode = capi.COARSE_DIRECT if coarse_cycles == 0 else capi.COARSE_CYCLES
        self.tree = tree
        self.lib = tree.lib
        d = capi.MgDesc(i_phi, i_rhs, i_tmp, n_cycle_down, n_cycle_up,
                        helmholtz_lambda, coarse_mode, coarse_cycles, coarse_tol)
        self.i_phi, self.i_rhs, self.i_tmp = i_phi, i_rhs, i_tmp
        h = C.c_void_p()
        self.lib.call("mg_create", tree.h, C.byref(d), C.byref(h))
        self.h = h
        tree._deps.append(self)

    def close(self):
        if self.h:
            self.lib.call("mg_destroy", self.h)
            self.h = C.c_void_p()
        if self in self.tree._deps:
            self.tree._deps.remove(self)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def fas_vcycle(self, set_residual=True, highest_lvl=0):
        self.lib.call("mg_fas_vcycle", self.h, int(set_residual), highest_lvl)

    def fas_vcycle_maxres(self, highest_lvl=0):
        """mg_fas_vcycle(set_residual) + af_tree_maxabs_cc(i_tmp), fused."""
        out = C.c_double()
        self.lib.call("mg_fas_vcycle_maxres", self.h, highest_lvl, C.byref(out))
        return out.value

    def fas_vcycle_fold(self, highest_lvl=0):
        """fas_vcycle_maxres without reading the maximum: it stays folded in
        capi.SLOT_MAXRES (Tree.fetch_reduced, Fluid.fetch_step) and the call
        does not wait for the device."""
        self.lib.call("mg_fas_vcycle_fold", self.h, highest_lvl)

    def set_box_stencil(self, box_id, v, bc_correction=None):
        """The electrode operator stencil of box `box_id` as afivo stores it
        (mg_box_lsf_stencil): v(7, nc, nc, nc) -- here an array of shape
        (nc, nc, nc, 7), [k][j][i][c] -- and bc_correction (nc, nc, nc) or
        None; v = None removes it."""
        vp = None if v is None else np.ascontiguousarray(v, dtype=np.float64)
        bp = None if bc_correction is None else np.ascontiguousarray(
            bc_correction, dtype=np.float64)
        self.lib.call("mg_set_box_stencil", self.h, int(box_id),
                      None if vp is None else vp.ctypes.data_as(capi.P_f64),
                      None if bp is None else bp.ctypes.data_as(capi.P_f64))

    def set_box_lsf(self, box_id, ix, dd, bval, i_lsf):
        """Boundary distances of box `box_id` for mg_box_lpllsf_gradient:
        ix (n, 3) 1-based (i, j, k), dd (n, 6), bval (nc, nc, nc) the
        electrode potential per cell; n = 0 removes."""
        ix = _i32(ix).reshape(-1)
        dd = np.ascontiguousarray(dd, dtype=np.float64).reshape(-1)
        bv = np.ascontiguousarray(bval, dtype=np.float64)
        self.lib.call("mg_set_box_lsf", self.h, int(box_id), len(ix) // 3,
                      ix.ctypes.data_as(capi.P_i32), dd.ctypes.data_as(capi.P_f64),
                      bv.ctypes.data_as(capi.P_f64), int(i_lsf))

    def fas_fmg(self, set_residual=True, have_guess=True):
        """mg_fas_fmg (m_af_multigrid.f90:137-180)."""
        self.lib.call("mg_fas_fmg", self.h, int(set_residual), int(have_guess))

    def coarse_iterations(self):
        """Level-1 cycles of the last coarse solve (PFMG's GetNumIteration)."""
        n = C.c_int32()
        self.lib.call("mg_coarse_iterations", self.h, C.byref(n))
        return n.value

    def graph_stats(self):
        """(V-cycles replayed from hipGraphs, of them segmented) -- diagnostics."""
        r, s = C.c_int64(), C.c_int64()
        self.lib.call("mg_graph_stats", self.h, C.byref(r), C.byref(s))
        return r.value, s.value

    def set_gradient_output(self, i_norm, fac=-1.0):
        """afh_mg_set_gradient_output: the final residual pass of every later
        V-cycle also stores |E| into i_norm (0: off); compute_phi_gradient(0,
        fac, i_norm) after it then launches nothing."""
        self.lib.call("mg_set_gradient_output", self.h, int(i_norm), float(fac))

    def compute_phi_gradient(self, i_fc, fac=-1.0, i_norm=0):
        self.lib.call("mg_compute_phi_gradient", self.h, i_fc, fac, i_norm)

    # oracle-only stage hooks
    def _stage(self, name, *args):
        self.lib.call(name, self.h, *args)


class Fluid:
    """The m_fluid / m_chemistry state (LFA). A variable gas density
    (gas_constant_density = .false.) is cc variable `i_gas_dens`; the gas
    species (densities gas_fractions * N) then come first in the reactions'
    species indices, as in m_chemistry.f90:193-197."""

    def __init__(self, tree, species_iv, species_charge, i_electron, i_efld,
                 f_flux, f_field, gas_number_density, td, chem, reactions,
                 limiter=capi.LIM_KOREN, dt_chemistry_nmin=-1.0,
                 gas_temperature=300.0, td_energy_col=0, i_gas_dens=0,
                 gas_fractions=(), i_photo=0, photo_species=0, ions=()):
        """ions: the mobile ions, [(species index (1-based into species_iv),
        face flux variable, mobility x N)] (afh_fluid_desc n_ions ...)."""
        self.tree = tree
        self.lib = tree.lib
        d = capi.FluidDesc()
        d.n_species = len(species_iv)
        d.species_iv[:len(species_iv)] = list(species_iv)
        d.species_charge[:len(species_iv)] = list(species_charge)
        d.i_electron, d.i_efld, d.f_flux, d.f_field = i_electron, i_efld, f_flux, f_field
        d.limiter = limiter
        d.gas_number_density = gas_number_density
        self._tables = []
        for name, lt in (("td", td), ("chem", chem)):
            rc = np.asfortranarray(lt["rows_cols"], dtype=np.float64)
            flat = np.ascontiguousarray(rc.T.reshape(-1))  # column-major
            self._tables.append(flat)
            s = getattr(d, name)
            s.n_points, s.n_cols = rc.shape
            s.x_min, s.inv_fac = float(lt["x_min"]), float(lt["inv_fac"])
            s.rows_cols = flat.ctypes.data_as(capi.P_f64)
        arr = (capi.Reaction * max(1, len(reactions)))()
        for n, r in enumerate(reactions):
            a = arr[n]
            a.rate_type = r.get("rate_type", capi.RATE_TABULATED_FIELD)
            a.table_col = r.get("table_col", 0)
            a.rate_factor = r.get("rate_factor", 1.0)
            for q, c in enumerate(r.get("c", [])):
                a.c[q] = c
            a.n_in = len(r["ix_in"])
            a.ix_in[:a.n_in] = r["ix_in"]
            a.n_out = len(r["ix_out"])
            a.ix_out[:a.n_out] = r["ix_out"]
            a.mult_out[:a.n_out] = r["mult_out"]
        self._reactions = arr
        d.n_reactions = len(reactions)
        d.reactions = C.cast(arr, C.POINTER(capi.Reaction))
        d.dt_chemistry_nmin = dt_chemistry_nmin
        d.gas_temperature = gas_temperature
        d.td_energy_col = td_energy_col
        d.i_gas_dens = i_gas_dens
        d.n_gas_species = len(gas_fractions)
        d.gas_fractions[:len(gas_fractions)] = list(gas_fractions)
        d.i_photo, d.photo_species = int(i_photo), int(photo_species)
        d.n_ions = len(ions)  # (more than AFH_MAX_IONS: the library refuses it)
        for q, (sp, fv, mob) in enumerate(ions[:capi.MAX_IONS]):
            d.ion_species[q], d.f_ion_flux[q], d.ion_mobility[q] = int(sp), int(fv), float(mob)
        h = C.c_void_p()
        self.lib.call("fluid_create", tree.h, C.byref(d), C.byref(h))
        self.h = h
        tree._deps.append(self)

    def close(self):
        if self.h:
            self.lib.call("fluid_destroy", self.h)
            self.h = C.c_void_p()
        if self in self.tree._deps:
            self.tree._deps.remove(self)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def electrode_species_bc(self, i_lsf, i_1pos_ion, box_ids, neumann_zero=True):
        """electrode_species_bc over the electrode boxes (src/streamer.f90:578-636)."""
        ids = _i32(box_ids)
        self.lib.call("electrode_species_bc", self.h, i_lsf, i_1pos_ion,
                      int(neumann_zero), len(ids), ids.ctypes.data_as(capi.P_i32))

    def set_update_mask(self, i_lsf):
        """set_box_mask's electrode part (src/m_fluid.f90:469-483): cells
        whose level set cc(i_lsf) is <= 0 are not updated, and boxes of such
        cells only add no chemistry limit (afh_fluid_set_update_mask; 0:
        off)."""
        self.lib.call("fluid_set_update_mask", self.h, int(i_lsf))

    def set_rhs_output(self, i_rhs, ghosts=True):
        """Fold field_set_rhs(i_rhs, s_out) into every density update (0: off);
        ghosts=False leaves the rhs ghost cells alone (no solver reads them)."""
        self.lib.call("fluid_set_rhs_output", self.h, i_rhs, int(ghosts))

    def set_field_source(self, i_phi, fac=-1.0):
        """The flux evaluates the face field from the potential i_phi
        (fac / dr * (phi_f - phi_{f-1}), mg_box_lpl_gradient) instead of
        reading f_field; 0 restores f_field (afh_fluid_set_field_source)."""
        self.lib.call("fluid_set_field_source", self.h, i_phi, float(fac))

    def set_ion_se_yield(self, y):
        """input_data%ion_se_yield: forward_euler applies handle_ion_se_flux
        between the flux and the update (afh_fluid_set_ion_se_yield)."""
        self.lib.call("fluid_set_ion_se_yield", self.h, float(y))

    def ion_se_flux(self):
        """handle_ion_se_flux over the leaves (afh_fluid_ion_se_flux)."""
        self.lib.call("fluid_ion_se_flux", self.h)

    def rhs_maxabs(self, s_out):
        """max|rhs| of the rhs the last update wrote for state s_out."""
        out = C.c_double()
        self.lib.call("fluid_rhs_maxabs", self.h, s_out, C.byref(out))
        return out.value

    def photoi_set_src(self, i_rhs, coeff, alpha_col=3):
        """photoi_set_src's Zheleznyak source (photoionization_rate_from_alpha,
        src/m_photoi.f90:217-253) into i_rhs on the leaf interiors."""
        self.lib.call("photoi_set_src", self.h, int(i_rhs), int(alpha_col), float(coeff))

    def rhs_valid(self, s_out):
        """Whether the rhs the last update wrote for state s_out is still
        current (afh_fluid_rhs_valid: tracked in the library)."""
        out = C.c_int32()
        self.lib.call("fluid_rhs_valid", self.h, s_out, C.byref(out))
        return bool(out.value)

    def field_set_rhs(self, i_rhs, s_in):
        self.lib.call("field_set_rhs", self.h, i_rhs, s_in)

    def field_set_rhs_maxabs(self, i_rhs, s_in):
        """field_set_rhs + af_tree_maxabs_cc(i_rhs), fused; returns max|rhs|."""
        out = C.c_double()
        self.lib.call("field_set_rhs_maxabs", self.h, i_rhs, s_in, C.byref(out))
        return out.value

    def flux_upwind_tree(self, s_deriv):
        dt = (C.c_double * 2)()
        self.lib.call("flux_upwind_tree", self.h, s_deriv, dt)
        return dt[0], dt[1]

    def flux_update_densities(self, dt, s_deriv, s_prev, w_prev, s_out, last_step):
        sp = _i32(s_prev)
        wp = np.ascontiguousarray(w_prev, dtype=np.float64)
        out = (C.c_double * 2)()
        self.lib.call("flux_update_densities", self.h, float(dt), s_deriv, len(sp),
                      sp.ctypes.data_as(capi.P_i32), wp.ctypes.data_as(capi.P_f64),
                      s_out, int(last_step), out)
        return out[0], out[1]

    def refine_flags(self, desc, electrode_box=None):
        """default_refinement reduced per box (afh_refine_flags): (flags,
        masks) arrays over the tree's boxes."""
        nb = self.tree.n_boxes
        flags = np.zeros(nb, np.int32)
        masks = np.zeros(nb, np.uint32)
        eb = None if electrode_box is None else np.ascontiguousarray(electrode_box, np.uint8)
        self.lib.call("refine_flags", self.h, C.byref(desc),
                      None if eb is None else eb.ctypes.data_as(C.POINTER(C.c_uint8)),
                      flags.ctypes.data_as(capi.P_i32),
                      masks.ctypes.data_as(C.POINTER(C.c_uint32)))
        return flags, masks

    def forward_euler(self, dt, s_deriv, s_prev, w_prev, s_out, last_step,
                      store_flux=False):
        """flux_upwind_tree + flux_update_densities (forward_euler,
        src/m_fluid.f90:56-70), fused on the device where the tree allows;
        returns dt_limits(1:4)."""
        sp = _i32(s_prev)
        wp = np.ascontiguousarray(w_prev, dtype=np.float64)
        out = (C.c_double * 4)()
        self.lib.call("fluid_forward_euler", self.h, float(dt), s_deriv, len(sp),
                      sp.ctypes.data_as(capi.P_i32), wp.ctypes.data_as(capi.P_f64),
                      s_out, int(last_step), int(store_flux), out)
        return out[0], out[1], out[2], out[3]

    def forward_euler_fold(self, dt, s_deriv, s_prev, w_prev, s_out, last_step,
                           store_flux=False):
        """forward_euler without reading the limits (fetch_step reads them);
        does not wait for the device."""
        sp = _i32(s_prev)
        wp = np.ascontiguousarray(w_prev, dtype=np.float64)
        self.lib.call("fluid_forward_euler_fold", self.h, float(dt), s_deriv, len(sp),
                      sp.ctypes.data_as(capi.P_i32), wp.ctypes.data_as(capi.P_f64),
                      s_out, int(last_step), int(store_flux))

    def fetch_step(self, last_step, *extra_slots):
        """(dt_limits(1:4) of the last forward_euler_fold, [extra slot
        values]) in one transfer."""
        sl = _i32(extra_slots) if extra_slots else np.zeros(1, np.int32)
        lim = (C.c_double * 4)()
        ext = (C.c_double * max(1, len(extra_slots)))()
        self.lib.call("fluid_fetch_step", self.h, int(last_step), len(extra_slots),
                      sl.ctypes.data_as(capi.P_i32), lim, ext)
        return (lim[0], lim[1], lim[2], lim[3]), list(ext)[:len(extra_slots)]


def photoi_helmh_compute(modes, coeffs, i_photo, max_rel_res=1e-2, max_fmg=10):
    """photoi_helmh_compute (src/m_photoi_helmh.f90:162-204) over the
    Helmholtz multigrid modes (Multigrid objects sharing one tree); returns the
    FMG cycles each mode took."""
    lib = modes[0].lib
    hs = (C.c_void_p * len(modes))(*[m.h.value for m in modes])
    cf = np.ascontiguousarray(coeffs, dtype=np.float64)
    n = np.zeros(len(modes), np.int32)
    lib.call("photoi_helmh_compute", hs, len(modes), cf.ctypes.data_as(capi.P_f64),
             int(i_photo), float(max_rel_res), int(max_fmg), n.ctypes.data_as(capi.P_i32))
    return list(n)
