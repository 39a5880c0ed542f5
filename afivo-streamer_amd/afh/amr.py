"""Host-side af_t topology: af_init and af_adjust_refinement restated.

The octree mesh changes only at a regrid (every refine_per_steps steps), so
its topology bookkeeping stays on the host, as afivo keeps it in af_t; the
box data never leave the device (afh_tree_regrid moves them). ``AfTree``
restates, routine by routine, what afivo/src/m_af_core.f90 does to the
topology:

* af_init / af_set_coarse_grid (138-340, create_index_array 436-501): coarse
  boxes with ids 1..N in k, j, i order, neighbours from the index array
  (periodic dimensions wrap);
* af_adjust_refinement (697-822) with consistent_ref_flags (929-1013),
  ensure_two_one_balance (1016-1057), handle_derefinement_flags
  (1059-1090), cell_to_ref_flags (1095-1148), add_children (1188-1233),
  remove_children (1151-1185), set_neighbs / find_neighb (595-661),
  get_free_ids (885-922), set_leaves_parents (504-535), set_child_ids
  (1237-1254);
* af_refine_up_to_lvl (664-689).

Box ids, level lists and their order are exactly afivo's, so a device tree
built from ``topology()`` lists boxes in the reference's loop order, and a
regrid keeps the ids of persisting boxes (the device moves data by id).

The refinement routine is the per-box summary cell_to_ref_flags makes of a
box's cell flags: ``flags_fn(ids) -> (flag, mask)`` with flag in
{RM_REF, KEEP_REF, DO_REF} and mask bit (dk+1)*9 + (dj+1)*3 + (di+1) set
when a cell within the buffer width of the side towards neighbour
(di, dj, dk) asks for refinement -- what ``afh_refine_flags`` computes on
the device from default_refinement (src/m_refine.f90:198-298).
"""
import numpy as np

# afivo/src/m_af_types.f90:14-45
MAX_LVL = 30
RM_REF, KEEP_REF, DO_REF = -1, 0, 1
DEREFINE, REFINE = -2, 2
NO_BOX, PHYS_BOUNDARY = 0, -1
_UNSET = -(2 ** 31 - 1)

# m_af_types.f90:167-236 (NDIM = 3); child c (0-based) has offset CHILD_DIX[c]
CHILD_DIX = ((0, 0, 0), (1, 0, 0), (0, 1, 0), (1, 1, 0),
             (0, 0, 1), (1, 0, 1), (0, 1, 1), (1, 1, 1))
NEIGHB_DIX = ((-1, 0, 0), (1, 0, 0), (0, -1, 0), (0, 1, 0), (0, 0, -1), (0, 0, 1))
NEIGHB_REV = (1, 0, 3, 2, 5, 4)  # 0-based af_neighb_rev
CHILD_ADJ_NB = ((0, 2, 4, 6), (1, 3, 5, 7), (0, 1, 4, 5), (2, 3, 6, 7),
                (0, 1, 2, 3), (4, 5, 6, 7))  # 0-based af_child_adj_nb


class _Dim:
    """afivo's per-NDIM constants (m_af_types.f90:114-236): child offsets,
    neighbour offsets, af_neighb_rev, af_child_adj_nb, the neighbor_mat
    directions in KJI_DO(-1,1) order (k outer, i inner)."""

    def __init__(self, ndim):
        self.ndim = ndim
        self.n_children = 2 ** ndim
        self.n_neighbors = 2 * ndim
        self.n_mat = 3 ** ndim
        self.center = (self.n_mat - 1) // 2
        if ndim == 3:
            self.child_dix, self.neighb_dix = CHILD_DIX, NEIGHB_DIX
            self.neighb_rev, self.child_adj_nb = NEIGHB_REV, CHILD_ADJ_NB
            self.dirs = [(di, dj, dk) for dk in (-1, 0, 1) for dj in (-1, 0, 1)
                         for di in (-1, 0, 1)]
        elif ndim == 2:
            self.child_dix = ((0, 0), (1, 0), (0, 1), (1, 1))
            self.neighb_dix = ((-1, 0), (1, 0), (0, -1), (0, 1))
            self.neighb_rev = (1, 0, 3, 2)
            self.child_adj_nb = ((0, 2), (1, 3), (0, 1), (2, 3))
            self.dirs = [(di, dj) for dj in (-1, 0, 1) for di in (-1, 0, 1)]
        else:
            raise ValueError("NDIM = %d not supported" % ndim)

    def nmat_index(self, d):
        """Index of neighbor_mat(d) in the flat 3^NDIM list (i fastest)."""
        return sum((d[q] + 1) * 3 ** q for q in range(self.ndim))

    def ix_to_ichild(self, ix):
        """af_ix_to_ichild (m_af_types.f90:1012-1023), 0-based."""
        return sum((1 - (ix[q] & 1)) << q for q in range(self.ndim))


def nmat_index(di, dj, dk):
    """Index of neighbor_mat(di, dj, dk) in a flat 27-list (i fastest)."""
    return (di + 1) + 3 * (dj + 1) + 9 * (dk + 1)


def ix_to_ichild(ix):
    """af_ix_to_ichild (m_af_types.f90:1012-1023), 0-based."""
    return (1 - (ix[0] & 1)) + 2 * (1 - (ix[1] & 1)) + 4 * (1 - (ix[2] & 1))


class RefInfo:
    """ref_info_t: boxes added per level and removed ids."""

    def __init__(self):
        self.add = {}
        self.rm = []

    @property
    def n_add(self):
        return sum(len(v) for v in self.add.values())

    @property
    def n_rm(self):
        return len(self.rm)


class AfTree:
    """The af_t topology (m_af_types.f90:326-393) of a Cartesian tree, NDIM = 3
    (the default) or 2 (len(grid_size) == 2: afivo/lib_2d, BASELINE config 1)."""

    def __init__(self, n_cell, r_max, grid_size, periodic=None, r_min=None,
                 box_limit=10 ** 7):
        nc = int(n_cell)
        if nc < 2 or nc % 2:
            raise ValueError("n_cell should be even and >= 2")
        grid_size = [int(g) for g in grid_size]
        nd = len(grid_size)
        self.D = _Dim(nd)
        self.ndim = nd
        if any(g < nc or g % nc for g in grid_size):
            raise ValueError("coarse_grid_size must be a multiple of n_cell")
        self.nc = nc
        self.r_base = np.zeros(nd) if r_min is None else np.asarray(r_min, float)[:nd]
        self.domain = np.asarray(r_max, float)[:nd]
        # dr_base = (r_max - r_min) / grid_size (af_init, 174)
        self.dr_base = (self.domain - self.r_base) / np.asarray(grid_size, float)
        self.coarse_grid_size = grid_size
        self.periodic = tuple(bool(p) for p in (periodic or (False,) * nd))
        self.box_limit = int(box_limit)
        # per-box records, indexed by id (index 0 unused)
        self.lvl, self.ix, self.parent = [0], [None], [0]
        self.children, self.neighbors, self.nmat = [None], [None], [None]
        self.r_min, self.dr, self.in_use = [None], [None], [False]
        self.lvls = [None] + [{"ids": [], "leaves": [], "parents": []}
                              for _ in range(MAX_LVL)]
        self.highest_id = 0
        self.highest_lvl = 0
        self.removed_ids = []
        self._set_coarse_grid()

    # ------------------------------------------------------------ helpers
    def _grow(self, n):
        while len(self.lvl) <= n:
            self.lvl.append(0)
            self.ix.append(None)
            self.parent.append(0)
            self.children.append(None)
            self.neighbors.append(None)
            self.nmat.append(None)
            self.r_min.append(None)
            self.dr.append(None)
            self.in_use.append(False)

    def has_children(self, bid):
        return self.children[bid][0] > NO_BOX

    def _set_coarse_grid(self):
        """af_set_coarse_grid (m_af_core.f90:206-340)."""
        D, nd = self.D, self.ndim
        nx = [g // self.nc for g in self.coarse_grid_size]

        def index(q):  # create_index_array (436-501)
            q = list(q)
            for d in range(nd):
                if q[d] < 1 or q[d] > nx[d]:
                    if not self.periodic[d]:
                        return PHYS_BOUNDARY
                    q[d] = nx[d] if q[d] < 1 else 1
            bid, stride = 0, 1
            for d in range(nd):
                bid += (q[d] - 1) * stride
                stride *= nx[d]
            return bid + 1

        n = int(np.prod(nx))
        ids = self.get_free_ids(n)
        self.lvls[1]["ids"] = list(ids)
        self.lvls[1]["leaves"] = list(ids)
        # box ids i fastest (KJI order)
        for q in np.ndindex(*reversed(nx)):
            ixq = tuple(int(x) + 1 for x in reversed(q))
            bid = index(ixq)
            self.lvl[bid] = 1
            self.ix[bid] = ixq
            self.dr[bid] = self.dr_base.copy()
            self.r_min[bid] = self.r_base + (np.array(ixq) - 1) * self.dr_base * self.nc
            self.parent[bid] = NO_BOX
            self.children[bid] = [NO_BOX] * D.n_children
            self.neighbors[bid] = [index([ixq[d] + dd[d] for d in range(nd)])
                                   for dd in D.neighb_dix]
            self.nmat[bid] = [index([ixq[d] + dd[d] for d in range(nd)]) for dd in D.dirs]
            self.in_use[bid] = True
        self.highest_lvl = 1

    def get_free_ids(self, n):
        """get_free_ids (m_af_core.f90:885-922)."""
        if n <= len(self.removed_ids):
            ids = self.removed_ids[len(self.removed_ids) - n:]
            del self.removed_ids[len(self.removed_ids) - n:]
            return ids
        prev = self.highest_id
        self.highest_id += n
        if self.highest_id > self.box_limit:
            raise MemoryError("get_free_ids: exceeding the box limit (%d)" % self.box_limit)
        self._grow(self.highest_id)
        return list(range(prev + 1, prev + n + 1))

    # ------------------------------------------------------- connectivity
    def _find_neighb(self, bid, dix):
        """find_neighb (m_af_core.f90:636-661)."""
        D, nd = self.D, self.ndim
        p_id = self.parent[bid]
        low = D.child_dix[D.ix_to_ichild(self.ix[bid])]
        dix_c = [dix[d] if ((dix[d] == -1) == (low[d] == 0)) else 0 for d in range(nd)]
        p_nb = self.nmat[p_id][D.nmat_index(dix_c)]
        if p_nb <= NO_BOX:
            return p_nb
        q = [self.ix[bid][d] + dix[d] for d in range(nd)]
        return self.children[p_nb][D.ix_to_ichild(q)]

    def _set_neighbs(self, bid):
        """set_neighbs (m_af_core.f90:595-633)."""
        D = self.D
        nm = self.nmat[bid]
        for dd in D.dirs:
            m = D.nmat_index(dd)
            if nm[m] == NO_BOX:
                nb_id = self._find_neighb(bid, dd)
                if nb_id > NO_BOX:
                    nm[m] = nb_id
                    self.nmat[nb_id][D.nmat_index([-x for x in dd])] = bid
        nbs = self.neighbors[bid]
        for nb in range(D.n_neighbors):
            if nbs[nb] == NO_BOX:
                nb_id = nm[D.nmat_index(D.neighb_dix[nb])]
                if nb_id > NO_BOX:
                    nbs[nb] = nb_id
                    self.neighbors[nb_id][D.neighb_rev[nb]] = bid

    def _add_children(self, bid, c_ids):
        """add_children (m_af_core.f90:1188-1233)."""
        D, nd = self.D, self.ndim
        self.children[bid] = list(c_ids)
        base = [2 * x - 1 for x in self.ix[bid]]
        for c in range(D.n_children):
            cid = c_ids[c]
            dix = D.child_dix[c]
            self.ix[cid] = tuple(base[d] + dix[d] for d in range(nd))
            self.lvl[cid] = self.lvl[bid] + 1
            self.parent[cid] = bid
            self.children[cid] = [NO_BOX] * D.n_children
            self.neighbors[cid] = [NO_BOX] * D.n_neighbors
            nm = [NO_BOX] * D.n_mat
            nm[D.center] = cid
            self.nmat[cid] = nm
            self.dr[cid] = 0.5 * self.dr[bid]
            self.r_min[cid] = self.r_min[bid] + 0.5 * self.dr[bid] * \
                np.asarray(dix, float) * self.nc
        for nb in range(D.n_neighbors):
            pnb = self.neighbors[bid][nb]
            if pnb < NO_BOX:  # physical boundary
                for c in D.child_adj_nb[nb]:
                    cid = c_ids[c]
                    self.neighbors[cid][nb] = pnb
                    self.nmat[cid][D.nmat_index(D.neighb_dix[nb])] = pnb
        for cid in c_ids:  # af_init_box: data zeroed on the device
            self.in_use[cid] = True

    def _remove_children(self, bid):
        """remove_children (m_af_core.f90:1151-1185)."""
        D = self.D
        for cid in self.children[bid]:
            for nb in range(D.n_neighbors):
                nb_id = self.neighbors[cid][nb]
                if nb_id > NO_BOX:
                    self.neighbors[nb_id][D.neighb_rev[nb]] = NO_BOX
            for dd in D.dirs:
                nb_id = self.nmat[cid][D.nmat_index(dd)]
                if nb_id > NO_BOX:
                    self.nmat[nb_id][D.nmat_index([-x for x in dd])] = NO_BOX
            self.in_use[cid] = False  # af_deactivate_box
        self.children[bid] = [NO_BOX] * D.n_children

    def _set_leaves_parents(self, lvl):
        """set_leaves_parents (m_af_core.f90:504-535)."""
        L = self.lvls[lvl]
        L["parents"] = [b for b in L["ids"] if self.has_children(b)]
        L["leaves"] = [b for b in L["ids"] if not self.has_children(b)]

    # --------------------------------------------------------- refinement
    def _cell_to_ref_flags(self, ref, bid, flag, mask):
        """cell_to_ref_flags (m_af_core.f90:1095-1148) from a box summary;
        every update is a max, so the per-thread arrays of the reference
        (maxed at the end) give the same result."""
        if flag == DO_REF:
            ref[bid] = DO_REF
        elif flag == KEEP_REF:
            ref[bid] = max(ref[bid], KEEP_REF)
        else:
            ref[bid] = max(ref[bid], RM_REF)
        if mask:
            nm = self.nmat[bid]
            for m in range(self.D.n_mat):
                if (mask >> m) & 1 and m != self.D.center:
                    nb_id = nm[m]
                    if nb_id > NO_BOX:
                        ref[nb_id] = DO_REF

    def _consistent_ref_flags(self, flags_fn):
        """consistent_ref_flags (m_af_core.f90:929-1013), without ref_links."""
        D = self.D
        ref = [_UNSET] * (self.highest_id + 1)
        ids, parents_of = [], []
        for lvl in range(1, self.highest_lvl + 1):
            for bid in self.lvls[lvl]["leaves"]:
                ids.append(bid)
                if self.lvl[bid] > 1:
                    p = self.parent[bid]
                    c = D.ix_to_ichild(self.ix[bid])
                    if all(self.has_children(self.children[p][q]) for q in range(c)):
                        parents_of.append((len(ids) - 1, p))
        # the refinement routine for every box it is called on, in one call
        need = sorted(set(ids) | set(p for _, p in parents_of))
        flag, mask = flags_fn(need)
        summ = {b: (int(flag[q]), int(mask[q])) for q, b in enumerate(need)}
        pq = dict(parents_of)
        for q, bid in enumerate(ids):
            self._cell_to_ref_flags(ref, bid, *summ[bid])
            if q in pq:
                self._cell_to_ref_flags(ref, pq[q], *summ[pq[q]])
        ref = [KEEP_REF if r == _UNSET else r for r in ref]
        for bid in self.lvls[MAX_LVL]["ids"]:
            if ref[bid] == DO_REF:
                ref[bid] = KEEP_REF
        self._ensure_two_one_balance(ref)
        self._handle_derefinement_flags(ref)
        return ref

    def _ensure_two_one_balance(self, ref):
        """ensure_two_one_balance (m_af_core.f90:1016-1057)."""
        n_nb = self.D.n_neighbors
        for lvl in range(self.highest_lvl, 0, -1):
            for bid in self.lvls[lvl]["leaves"]:
                if ref[bid] in (DO_REF, REFINE):
                    ref[bid] = REFINE
                    for nb in range(n_nb):
                        if self.neighbors[bid][nb] == NO_BOX:
                            p_nb = self.neighbors[self.parent[bid]][nb]
                            if p_nb > NO_BOX:  # always, in a balanced tree
                                ref[p_nb] = REFINE
                elif ref[bid] == RM_REF:
                    for nb in range(n_nb):
                        nb_id = self.neighbors[bid][nb]
                        if nb_id > NO_BOX and (self.has_children(nb_id) or
                                               ref[nb_id] > KEEP_REF):
                            ref[bid] = KEEP_REF
                            break

    def _handle_derefinement_flags(self, ref):
        """handle_derefinement_flags (m_af_core.f90:1059-1090)."""
        for lvl in range(self.highest_lvl - 1, 0, -1):
            for bid in self.lvls[lvl]["parents"]:
                c_ids = self.children[bid]
                if all(self.has_children(c) for c in c_ids):
                    continue
                if all(ref[c] == RM_REF for c in c_ids) and ref[bid] <= KEEP_REF:
                    ref[bid] = DEREFINE
                else:
                    ref[bid] = KEEP_REF
                    for c in c_ids:
                        if ref[c] != DEREFINE:
                            ref[c] = max(ref[c], KEEP_REF)

    def adjust_refinement(self, flags_fn):
        """af_adjust_refinement (m_af_core.f90:697-822): returns a RefInfo.
        The data movement (auto_restrict / auto_prolong) is the device's
        afh_tree_regrid, driven by the topology before and after."""
        ref = self._consistent_ref_flags(flags_fn)
        info = RefInfo()
        n_ref = len(ref) - 1
        lvl = 1
        while lvl <= MAX_LVL - 1:
            add = []
            for bid in list(self.lvls[lvl]["ids"]):
                if bid > n_ref:
                    continue  # a newly added box
                if ref[bid] == REFINE:
                    c_ids = self.get_free_ids(self.D.n_children)
                    self._add_children(bid, c_ids)
                    add += self.children[bid]
                elif ref[bid] == DEREFINE:
                    info.rm += self.children[bid]
                    self._remove_children(bid)
            info.add[lvl + 1] = add
            self._set_leaves_parents(lvl)
            nxt = []
            for p in self.lvls[lvl]["parents"]:  # set_child_ids
                nxt += self.children[p]
            self.lvls[lvl + 1]["ids"] = nxt
            for p in self.lvls[lvl]["parents"]:
                if ref[p] == REFINE:
                    for c in self.children[p]:
                        self._set_neighbs(c)
            if not nxt:
                break
            lvl += 1
        self.highest_lvl = lvl
        self.removed_ids += info.rm
        bid = self.highest_id
        while bid >= 1 and not self.in_use[bid]:
            bid -= 1
        self.highest_id = bid
        self.removed_ids = [r for r in self.removed_ids if r <= self.highest_id]
        self._set_leaves_parents(min(lvl + 1, MAX_LVL))
        return info

    def refine_up_to_lvl(self, lvl):
        """af_refine_up_to_lvl (m_af_core.f90:664-689)."""
        if lvl < self.highest_lvl:
            raise ValueError("tree already above level")

        def fn(ids):
            f = np.array([DO_REF if self.lvl[b] < lvl else KEEP_REF for b in ids])
            return f, np.zeros(len(ids), np.uint32)

        while self.adjust_refinement(fn).n_add > 0:
            pass

    # ------------------------------------------------------------- export
    def lvl_dr(self, lvl):
        """af_lvl_dr: dr_base / 2^(lvl-1) (the bits every box of the level
        carries, halved exactly per level)."""
        return self.dr_base * 0.5 ** (lvl - 1)

    def total_volume(self):
        """af_total_volume (m_af_utils.f90): the coarse boxes' volume (area
        in 2-D)."""
        v = 0.0
        for bid in self.lvls[1]["ids"]:
            v += float(np.prod(self.dr[bid] * self.nc))
        return v

    def min_dr(self):
        """af_min_dr: the finest level's smallest spacing."""
        return float(np.min(self.lvl_dr(self.highest_lvl)))

    def topology(self):
        """The topology dict the device tree is created from (afh/tree.py
        conventions; ids not in use have level 0; a 2-D tree has ndim = 2)."""
        D, nd = self.D, self.ndim
        nb = self.highest_id
        out = {"nc": np.int32(self.nc), "n_boxes": np.int32(nb),
               "highest_lvl": np.int32(self.highest_lvl),
               "coarse_grid_size": np.array(self.coarse_grid_size, np.int32),
               "r_base": self.r_base.copy(), "dr_base": self.dr_base.copy(),
               "domain": self.domain.copy()}
        if nd != 3:
            out["ndim"] = np.int32(nd)
        lvl = np.zeros(nb, np.int32)
        ix = np.zeros((nb, nd), np.int32)
        parent = np.zeros(nb, np.int32)
        children = np.zeros((nb, D.n_children), np.int32)
        neighbors = np.zeros((nb, D.n_neighbors), np.int32)
        nmat = np.zeros((nb, D.n_mat), np.int32)
        r_min = np.zeros((nb, nd))
        dr = np.zeros((nb, nd))
        for b in range(1, nb + 1):
            if not self.in_use[b]:
                continue
            lvl[b - 1] = self.lvl[b]
            ix[b - 1] = self.ix[b]
            parent[b - 1] = self.parent[b]
            children[b - 1] = self.children[b]
            neighbors[b - 1] = self.neighbors[b]
            nmat[b - 1] = self.nmat[b]
            r_min[b - 1] = self.r_min[b]
            dr[b - 1] = self.dr[b]
        out.update(meta_lvl=lvl, meta_ix=ix, meta_parent=parent,
                   meta_children=children, meta_neighbors=neighbors,
                   meta_neighbor_mat=nmat, meta_r_min=r_min, meta_dr=dr)
        for l in range(1, self.highest_lvl + 1):
            L = self.lvls[l]
            out["lvl_ids_%d" % l] = np.array(L["ids"], np.int32)
            out["lvl_leaves_%d" % l] = np.array(L["leaves"], np.int32)
            out["lvl_parents_%d" % l] = np.array(L["parents"], np.int32)
        return out

    def leaves(self):
        return [b for l in range(1, self.highest_lvl + 1) for b in self.lvls[l]["leaves"]]

    def n_leaf_cells(self):
        return len(self.leaves()) * self.nc ** self.ndim
