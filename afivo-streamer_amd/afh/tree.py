"""Octree topology in afivo's conventions (afivo/src/m_af_types.f90:286-393).

``build_tree`` creates the box_t topology that af_init + af_refine_up_to_lvl /
af_adjust_refinement produce (afivo/src/m_af_core.f90:138-340, 697-822,
add_children 1180-1228, set_neighbs 596-630), without the physics. The result
is a plain dict of numpy arrays (the same keys the golden fixtures use), so a
reference-generated tree and a locally built one are interchangeable.
"""
import numpy as np

# afivo/src/m_af_types.f90:167-236 (NDIM = 3)
CHILD_DIX = np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0], [1, 1, 0],
                      [0, 0, 1], [1, 0, 1], [0, 1, 1], [1, 1, 1]], np.int32)
NEIGHB_DIX = np.array([[-1, 0, 0], [1, 0, 0], [0, -1, 0], [0, 1, 0],
                       [0, 0, -1], [0, 0, 1]], np.int32)


def build_tree(n_cell, coarse_grid_size, domain, max_lvl, refine=None,
               r_base=(0.0, 0.0, 0.0)):
    """Return an afivo-style topology dict.

    Boxes at levels < ``max_lvl`` are refined everywhere; beyond that a box is
    refined while ``refine(lvl, r_min, r_max)`` is true (and its level is
    below the level ``refine`` returns as second value, if it returns a tuple).
    The refinement is 2:1 balanced like af_adjust_refinement.
    """
    nc = int(n_cell)
    cgs = np.array(coarse_grid_size, np.int64)
    nbox0 = cgs // nc
    assert np.all(nbox0 * nc == cgs), "coarse_grid_size must be a multiple of n_cell"
    domain = np.asarray(domain, float)
    r_base = np.asarray(r_base, float)
    dr_base = (domain - r_base) / cgs

    # boxes keyed by (lvl, ix) -> id; ids assigned in creation order
    key2id = {}
    recs = []

    def add(lvl, ix, parent):
        bid = len(recs) + 1
        key2id[(lvl, tuple(ix))] = bid
        recs.append({"lvl": lvl, "ix": np.array(ix, np.int32), "parent": parent,
                     "children": np.zeros(8, np.int32)})
        return bid

    for k in range(1, nbox0[2] + 1):
        for j in range(1, nbox0[1] + 1):
            for i in range(1, nbox0[0] + 1):
                add(1, (i, j, k), 0)

    def nboxes_at(lvl):
        return nbox0 * (2 ** (lvl - 1))

    def inside(lvl, ix):
        n = nboxes_at(lvl)
        return all(1 <= ix[d] <= n[d] for d in range(3))

    def box_extent(lvl, ix):
        dr = dr_base / 2 ** (lvl - 1)
        r_min = r_base + (np.asarray(ix) - 1) * nc * dr
        return r_min, r_min + nc * dr, dr

    def wants(lvl, ix):
        if lvl < max_lvl:
            return True
        if refine is None:
            return False
        r0, r1, _ = box_extent(lvl, ix)
        return bool(refine(lvl, r0, r1))

    lvl = 1
    while True:
        cur = [(key, bid) for key, bid in key2id.items() if key[0] == lvl]
        flag = {key: wants(*key) for key, _ in cur}
        # 2:1 balance: a box whose same-level neighbour (incl. diagonal) is
        # being refined and has a refined neighbour... afivo keeps levels of
        # adjacent leaves within one; enforce by refining parents of marked
        # boxes' neighbours at the coarser level is implicit here because we
        # refine level by level and mark neighbours of boxes whose children
        # will be refined next (see below).
        if not any(flag.values()):
            break
        for key, bid in sorted(cur, key=lambda kv: kv[1]):
            if not flag[key]:
                continue
            base = 2 * np.array(key[1]) - 1
            for c in range(8):
                cix = base + CHILD_DIX[c]
                recs[bid - 1]["children"][c] = add(lvl + 1, cix, bid)
        lvl += 1
        _balance(key2id, recs, lvl)

    return _finish(nc, cgs, domain, r_base, dr_base, key2id, recs, inside,
                   box_extent)


def _balance(key2id, recs, lvl):
    """Refine coarse leaves so that leaves adjacent (incl. diagonally) to a
    box at ``lvl`` exist at level >= lvl-1 (afivo's 2:1 balance)."""
    changed = True
    while changed:
        changed = False
        for (l, ix), bid in list(key2id.items()):
            if l != lvl:
                continue
            p = np.array(ix)
            for dz in (-1, 0, 1):
                for dy in (-1, 0, 1):
                    for dx in (-1, 0, 1):
                        q = p + (dx, dy, dz)
                        # parent-level neighbour region must exist
                        pq = (q + 1) // 2
                        if (l - 1, tuple(pq)) in key2id:
                            continue
                        gq = (pq + 1) // 2
                        gid = key2id.get((l - 2, tuple(gq)))
                        if gid is None or recs[gid - 1]["children"][0] != 0:
                            continue
                        base = 2 * gq - 1
                        for c in range(8):
                            cix = base + CHILD_DIX[c]
                            nid = len(recs) + 1
                            key2id[(l - 1, tuple(cix))] = nid
                            recs.append({"lvl": l - 1, "ix": cix.astype(np.int32),
                                         "parent": gid,
                                         "children": np.zeros(8, np.int32)})
                            recs[gid - 1]["children"][c] = nid
                        changed = True


def _finish(nc, cgs, domain, r_base, dr_base, key2id, recs, inside, box_extent):
    nb = len(recs)
    out = {"nc": np.int32(nc), "n_boxes": np.int32(nb)}
    lvl = np.array([r["lvl"] for r in recs], np.int32)
    highest = int(lvl.max())
    out["highest_lvl"] = np.int32(highest)
    out["coarse_grid_size"] = cgs.astype(np.int32)
    out["r_base"] = r_base
    out["dr_base"] = dr_base
    out["domain"] = domain
    ix = np.array([r["ix"] for r in recs], np.int32)
    parent = np.array([r["parent"] for r in recs], np.int32)
    children = np.array([r["children"] for r in recs], np.int32)
    neighbors = np.zeros((nb, 6), np.int32)
    nmat = np.zeros((nb, 27), np.int32)
    r_min = np.zeros((nb, 3))
    dr = np.zeros((nb, 3))
    for b in range(nb):
        l, p = int(lvl[b]), ix[b]
        rmn, _, d = box_extent(l, p)
        # r_min as afivo accumulates it: parent r_min + 0.5*dr_p*dix*nc
        r_min[b] = rmn
        dr[b] = d
        for n in range(6):
            q = p + NEIGHB_DIX[n]
            if not inside(l, q):
                neighbors[b, n] = -1
            else:
                neighbors[b, n] = key2id.get((l, tuple(q)), 0)
        for dz in (-1, 0, 1):
            for dy in (-1, 0, 1):
                for dx in (-1, 0, 1):
                    q = p + (dx, dy, dz)
                    m = (dx + 1) + 3 * (dy + 1) + 9 * (dz + 1)
                    if not inside(l, q):
                        nmat[b, m] = -1
                    else:
                        nmat[b, m] = key2id.get((l, tuple(q)), 0)
    # afivo computes children's r_min/dr recursively from the parent
    for b in np.argsort(lvl, kind="stable"):
        if parent[b] > 0:
            pb = parent[b] - 1
            dr[b] = 0.5 * dr[pb]
            c = list(children[pb]).index(b + 1)
            r_min[b] = r_min[pb] + 0.5 * dr[pb] * CHILD_DIX[c] * nc
        else:
            dr[b] = dr_base
            r_min[b] = r_base + (ix[b] - 1) * nc * dr_base
    out.update(meta_lvl=lvl, meta_ix=ix, meta_parent=parent,
               meta_children=children, meta_neighbors=neighbors,
               meta_neighbor_mat=nmat, meta_r_min=r_min, meta_dr=dr)
    for l in range(1, highest + 1):
        ids = np.where(lvl == l)[0] + 1
        has_ch = children[ids - 1, 0] > 0
        out["lvl_ids_%d" % l] = ids.astype(np.int32)
        out["lvl_leaves_%d" % l] = ids[~has_ch].astype(np.int32)
        out["lvl_parents_%d" % l] = ids[has_ch].astype(np.int32)
    return out


def uniform_tree(n_cell, coarse_grid_size, domain, max_lvl):
    """Uniformly refined tree (af_refine_up_to_lvl)."""
    return build_tree(n_cell, coarse_grid_size, domain, max_lvl)


def uniform_tree_2d(n_cell, coarse_grid_size, domain, max_lvl):
    """The 2-D topology af_init + af_refine_up_to_lvl build with NDIM = 2
    (m_af_core.f90:138-340; children in af_child_dix order (0,0), (1,0),
    (0,1), (1,1), m_af_types.f90:134): ids level by level, the level-1 boxes
    i fastest, children in parent-id order. topo["ndim"] = 2; neighbors
    (lowx, highx, lowy, highy), neighbor_mat(-1:1, -1:1) i fastest, -1 =
    physical boundary, as in the reference's 2-D box_t."""
    nc = int(n_cell)
    cgs = np.array(coarse_grid_size, np.int64)
    nbox0 = cgs // nc
    assert np.all(nbox0 * nc == cgs), "coarse_grid_size must be a multiple of n_cell"
    domain = np.asarray(domain, float)
    dr_base = domain / cgs
    cdix = np.array([[0, 0], [1, 0], [0, 1], [1, 1]], np.int32)
    key2id, lvl, ix, parent, children = {}, [], [], [], []

    def add(l, p, par):
        key2id[(l, tuple(int(v) for v in p))] = len(lvl) + 1
        lvl.append(l), ix.append(np.asarray(p, np.int32)), parent.append(par)
        children.append(np.zeros(4, np.int32))
        return len(lvl)

    for j in range(1, nbox0[1] + 1):
        for i in range(1, nbox0[0] + 1):
            add(1, (i, j), 0)
    for l in range(1, max_lvl):
        for bid in [b for b in range(1, len(lvl) + 1) if lvl[b - 1] == l]:
            for c in range(4):
                children[bid - 1][c] = add(l + 1, 2 * ix[bid - 1] - 1 + cdix[c], bid)
    nb = len(lvl)
    out = {"nc": np.int32(nc), "n_boxes": np.int32(nb), "ndim": np.int32(2),
           "highest_lvl": np.int32(max_lvl), "coarse_grid_size": cgs.astype(np.int32),
           "r_base": np.zeros(2), "dr_base": dr_base, "domain": domain}
    lv, ixa = np.array(lvl, np.int32), np.array(ix, np.int32)
    nbs = np.zeros((nb, 4), np.int32)
    nmat = np.zeros((nb, 9), np.int32)
    r_min, dr = np.zeros((nb, 2)), np.zeros((nb, 2))
    ndix = np.array([[-1, 0], [1, 0], [0, -1], [0, 1]])
    for b in range(nb):
        l, p = int(lv[b]), ixa[b]
        n = nbox0 * 2 ** (l - 1)
        inside = lambda q: bool(np.all(q >= 1) and np.all(q <= n))  # noqa: E731
        for m in range(4):
            q = p + ndix[m]
            nbs[b, m] = key2id.get((l, tuple(int(v) for v in q)), 0) if inside(q) else -1
        for dy in (-1, 0, 1):
            for dx in (-1, 0, 1):
                q = p + (dx, dy)
                # a diagonal outside the domain: -1 on level 1, 0 (no box)
                # below, where afivo finds it through the parent's neighbours
                out_v = -1 if l == 1 or dx == 0 or dy == 0 else 0
                nmat[b, (dx + 1) + 3 * (dy + 1)] = (
                    key2id.get((l, tuple(int(v) for v in q)), 0) if inside(q) else out_v)
    # r_min / dr accumulated from the parent as afivo does (add_children)
    for b in range(nb):
        if parent[b] > 0:
            pb = parent[b] - 1
            c = list(children[pb]).index(b + 1)
            dr[b] = 0.5 * dr[pb]
            r_min[b] = r_min[pb] + 0.5 * dr[pb] * cdix[c] * nc
        else:
            dr[b] = dr_base
            r_min[b] = (ixa[b] - 1) * nc * dr_base
    ch = np.array(children, np.int32)
    out.update(meta_lvl=lv, meta_ix=ixa, meta_parent=np.array(parent, np.int32),
               meta_children=ch, meta_neighbors=nbs, meta_neighbor_mat=nmat,
               meta_r_min=r_min, meta_dr=dr)
    for l in range(1, max_lvl + 1):
        ids = np.where(lv == l)[0] + 1
        has_ch = ch[ids - 1, 0] > 0
        out["lvl_ids_%d" % l] = ids.astype(np.int32)
        out["lvl_leaves_%d" % l] = ids[~has_ch].astype(np.int32)
        out["lvl_parents_%d" % l] = ids[has_ch].astype(np.int32)
    return out


def leaf_cells(topo):
    nc = int(topo["nc"])
    n = 0
    for l in range(1, int(topo["highest_lvl"]) + 1):
        n += len(topo["lvl_leaves_%d" % l])
    return n * nc ** int(topo.get("ndim", 3))
