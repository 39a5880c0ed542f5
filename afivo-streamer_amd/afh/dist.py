"""Box sharding over ranks.

Partition (round 4: a weighted Morton split of a partition frontier). The
frontier starts as the boxes of level 2 (level 1 -- the coarse grid and its
solver -- is replicated on every rank). Its boxes are ordered by the Morton
index of their lower corner at the finest level's resolution (a Z-order
walk over boxes of several levels, which cover disjoint blocks) and cut into
contiguous chunks of about equal leaf weight (the leaf boxes of the subtree:
the species step and the finest V-cycle work). While the heaviest rank
carries more than (1 + TOL) of the mean, or the frontier has fewer boxes than
ranks, the heaviest refined frontier box is replaced by its children and
becomes replicated. Every descendant belongs to the rank of its frontier
ancestor, so restriction and prolongation stay rank-local below the
frontier; the replicated boxes above it (ancestors of frontier boxes, never
leaves, except level-1 leaves) are computed by every rank. On a uniform tree
the first frontier (level 2 or the first level with a box per rank) is
already balanced, so the split is the round-3 one.

Every rank allocates storage for the whole tree; the boxes of other ranks are
replicas, refreshed by exchanges where the library's hooks say a replica is
read after its owner wrote it (include/afivo_hip.h, AFH_HOOK_*):

* HALO(l, iv): the cells of each remote neighbour (26 directions) within two
  layers of a box the rank computes (owned or replicated), before a
  ghost-cell fill of level l;
* RIMS(l, iv): the same regions extended over the neighbour's ghost layers,
  after the fill (read by the fused smoother's neighbour recomputation and
  by refinement-boundary interpolation);
* RESTRICT(l, iv): the parent octants restricted from owned boxes of level l
  into their replicated parents (all-gather);
* CFLUX: the face fluxes af_consistent_fluxes copies from a refined box's
  children into a coarse leaf neighbour on another rank;
* MAX / MIN / SUM: all-reduce of reduction results.

Transport: torch.distributed point-to-point (batch_isend_irecv) -- RCCL
("nccl") with device buffers on the GPU, gloo with host buffers in the CPU
tests (and for several ranks sharing one GPU, staged through the host).
"""
import ctypes as C
import traceback

import numpy as np

from . import capi

# 26 neighbour directions, neighbor_mat index (dx+1) + 3(dy+1) + 9(dz+1)
DIRS = [(dx, dy, dz) for dz in (-1, 0, 1) for dy in (-1, 0, 1) for dx in (-1, 0, 1)
        if (dx, dy, dz) != (0, 0, 0)]
DEPTH = 2
# the frontier is refined while the heaviest rank carries more than
# (100 + TOL_PCT) % of the mean leaf weight (afh_dist_core.h TOL_PCT)
TOL_PCT = 10
MORTON_BITS = 21  # per dimension (int64 codes)


def morton3(ix):
    """Interleaved-bit (Z-order) index of 0-based integer positions."""
    ix = np.asarray(ix, dtype=np.int64)
    code = np.zeros(len(ix), dtype=np.int64)
    for b in range(MORTON_BITS):
        for d in range(3):
            code |= ((ix[:, d] >> b) & 1) << (3 * b + d)
    return code


def local_topology(topo, owner, rank):
    """The topology dict with rank's level lists: its own boxes and the
    replicated ones (owner -1); what afh_tree_create_sharded builds."""
    owner = np.asarray(owner)
    t = dict(topo)
    for l in range(1, int(topo["highest_lvl"]) + 1):
        for k in ("ids", "leaves", "parents"):
            key = "lvl_%s_%d" % (k, l)
            ids = np.asarray(topo[key], np.int64)
            o = owner[ids - 1]
            t[key] = ids[(o == rank) | (o < 0)].astype(np.int32)
    return t


def compact_topology(topo, present, space):
    """The topology dict of the boxes `present` (global ids) renumbered by
    their position in `space` (sorted global ids, a superset shared by
    several such trees: a box keeps its id in each), plus one unused id
    (len(space) + 1) that every reference to a box outside `present` points
    to -- the convention of afh_tree_create_sharded. Ids of `space` not
    present are holes (level 0)."""
    space = np.asarray(space, np.int64)
    present = np.asarray(sorted(set(int(b) for b in present)), np.int64)
    n = len(space)
    unused = n + 1
    nb = int(topo["n_boxes"])
    g2c = np.zeros(nb + 2, np.int64)
    pos = np.searchsorted(space, present)
    g2c[present] = pos + 1
    inset = np.zeros(nb + 2, bool)
    inset[present] = True

    def remap(a):
        a = np.asarray(a, np.int64)
        out = a.copy()
        pos_ = a > 0
        ok = np.zeros_like(pos_)
        ok[pos_] = inset[a[pos_]]
        out[pos_ & ok] = g2c[a[pos_ & ok]]
        out[pos_ & ~ok] = unused
        return out.astype(np.int32)

    out = {k: v for k, v in topo.items() if not k.startswith(("meta_", "lvl_"))}
    out["n_boxes"] = np.int32(n + 1)
    rows = pos  # compact index (0-based) of each present box
    src = present - 1
    for key in ("meta_lvl", "meta_ix", "meta_r_min", "meta_dr"):
        a = np.asarray(topo[key])
        b = np.zeros((n + 1,) + a.shape[1:], a.dtype)
        b[rows] = a[src]
        out[key] = b
    for key in ("meta_parent", "meta_children", "meta_neighbors", "meta_neighbor_mat"):
        a = np.asarray(topo[key])
        b = np.zeros((n + 1,) + a.shape[1:], np.int32)
        b[rows] = remap(a[src])
        out[key] = b
    for l in range(1, int(topo["highest_lvl"]) + 1):
        for k in ("ids", "leaves", "parents"):
            key = "lvl_%s_%d" % (k, l)
            ids = np.asarray(topo[key], np.int64)
            ids = ids[inset[ids]]
            out[key] = g2c[ids].astype(np.int32)
    return out


class Partition:
    """Ownership of every box for n_ranks (owner -1: replicated)."""

    def __init__(self, topo, n_ranks, min_level_cells=0):
        self.topo = topo
        self.min_level_cells = int(min_level_cells)
        self.n_ranks = n_ranks
        self.nc = int(topo["nc"])
        self.nb = int(topo["n_boxes"])
        self.nlvl = int(topo["highest_lvl"])
        self.lvl = np.asarray(topo["meta_lvl"])
        self.parent = np.asarray(topo["meta_parent"])
        self.children = np.asarray(topo["meta_children"])
        self.nmat = np.asarray(topo["meta_neighbor_mat"]).reshape(self.nb, 27)
        self.ix = np.asarray(topo["meta_ix"])
        ids = {l: np.asarray(topo["lvl_ids_%d" % l], np.int64)
               for l in range(1, self.nlvl + 1)}
        self.owner = np.full(self.nb, -1, np.int64)
        self.lp = None
        if n_ranks > 1:
            self._partition(ids, n_ranks)
        self.ids = ids

    def _partition(self, ids, n):
        """The weighted Morton split of the partition frontier (module
        docstring); afh_dist_core.h partition() is the same algorithm."""
        nlvl = self.nlvl
        # leaf weight of every subtree
        w = np.zeros(self.nb + 1, np.int64)
        for l in range(nlvl, 0, -1):
            for i in ids[l]:
                ch = self.children[i - 1]
                w[i] = 1 if ch[0] == 0 else w[ch].sum()
        if nlvl < 2:
            if self.min_level_cells > 0:
                return
            raise ValueError("no level >= 2 has enough boxes to shard over %d ranks" % n)
        ls = 2
        if self.min_level_cells > 0:
            # the frontier starts at the first level holding min_level_cells
            # cells (and n boxes); the levels below are replicated; none such:
            # the whole tree replicated (lp None)
            big = [l for l in range(2, nlvl + 1)
                   if len(ids[l]) * self.nc ** 3 >= self.min_level_cells and len(ids[l]) >= n]
            if not big:
                return
            ls = big[0]
        roots = [int(i) for i in ids[ls]]

        def code(b):  # Morton index of the lower corner at the finest resolution
            sh = nlvl - int(self.lvl[b - 1])
            return int(morton3((self.ix[b - 1][None] - 1) << sh)[0])

        def split(rs):
            order = sorted(rs, key=code)
            ww = w[np.asarray(order, np.int64)]
            cum = np.cumsum(ww)
            target = cum[-1] / n
            rk = np.minimum((np.ceil(cum / target) - 1).astype(np.int64), n - 1)
            ok = len(np.unique(rk)) == n
            loads = np.bincount(rk, weights=ww, minlength=n).astype(np.int64)
            return order, rk, ok, int(loads.max()), int(cum[-1])

        while True:
            if len(roots) >= n:
                order, rk, ok, mx, total = split(roots)
                if ok and mx * n * 100 <= (100 + TOL_PCT) * total:
                    break
            cand = [r for r in roots if self.children[r - 1][0] > 0]
            if not cand:
                if len(roots) < n:
                    raise ValueError("no level >= 2 has enough boxes to shard over %d ranks" % n)
                break
            h = max(cand, key=lambda r: (w[r], -r))  # heaviest, then lowest id
            roots.remove(h)
            roots += [int(c) for c in self.children[h - 1]]
        order, rk, ok, _, _ = split(roots)
        # every rank gets at least one frontier box: fall back to an even split
        if not ok:
            rk = (np.arange(len(order)) * n) // len(order)
        self.owner[np.asarray(order, np.int64) - 1] = rk
        for l in range(ls + 1, nlvl + 1):
            for i in ids[l]:
                p = self.parent[i - 1]
                if self.owner[p - 1] >= 0:
                    self.owner[i - 1] = self.owner[p - 1]
        self.lp = min(int(self.lvl[r - 1]) for r in roots)

    def owned(self, rank, box_ids):
        o = self.owner[np.asarray(box_ids, np.int64) - 1]
        return np.asarray(box_ids)[(o == rank) | (o < 0)]

    def local_topology(self, rank):
        """The topology dict with this rank's level lists."""
        return local_topology(self.topo, self.owner, rank)

    # ---------------------------------------------------------------- plans
    def _region(self, b, d, rims, depth=DEPTH):
        """Cells of box b within `depth` layers of the box in direction -d
        (b lies at direction d of the owned box); with rims, b's ghost
        layers are included (along d and across it)."""
        nc = self.nc
        lo, hi = [], []
        for x in d:
            if x < 0:
                lo.append(nc - depth + 1), hi.append(nc + 1 if rims else nc)
            elif x > 0:
                lo.append(0 if rims else 1), hi.append(depth)
            else:
                lo.append(0 if rims else 1), hi.append(nc + 1 if rims else nc)
        return (int(b), *lo, *hi)

    def halo_regions(self, recv_rank, send_rank, level, rims, depth=DEPTH):
        """Regions of boxes owned by send_rank that recv_rank reads around its
        boxes of `level` (sorted, duplicates and contained regions removed),
        `depth` layers deep (the library asks for one layer where no fused
        pair reads the second: the hook's n)."""
        if self.lp is None or level < self.lp:
            return []
        regs = set()
        for a in self.ids[level]:
            # the boxes recv_rank computes: its own and the replicated ones
            if self.owner[a - 1] != recv_rank and self.owner[a - 1] >= 0:
                continue
            for d in DIRS:
                b = self.nmat[a - 1][(d[0] + 1) + 3 * (d[1] + 1) + 9 * (d[2] + 1)]
                if b > 0 and self.owner[b - 1] == send_rank:
                    regs.add(self._region(b, d, rims, depth))
        out = []
        by_box = {}
        for r in regs:
            by_box.setdefault(r[0], []).append(r)
        nc = self.nc
        for b in sorted(by_box):
            rs = by_box[b]
            for r in sorted(rs):
                inside = any(q != r and all(q[1 + k] <= r[1 + k] and r[4 + k] <= q[4 + k]
                                            for k in range(3)) for q in rs)
                if inside:
                    continue
                if not rims:
                    out.append(r)
                    continue
                # RIMS follows the HALO of the same variable and level with
                # only a ghost fill between: the interior arrived with the
                # HALO, only the ghost cells travel -- the region less
                # [1, nc]^3 as disjoint slabs (afh_dist_core.h halo_regions;
                # a rank's fills do not write its replicas' ghost cells, so
                # all of them travel)
                for k in range(3):
                    for side in (0, 1):
                        g = list(r)
                        for j in range(k):
                            g[1 + j], g[4 + j] = max(r[1 + j], 1), min(r[4 + j], nc)
                        if side == 0:
                            if r[1 + k] >= 1:
                                continue
                            g[4 + k] = 0
                        else:
                            if r[4 + k] <= nc:
                                continue
                            g[1 + k] = nc + 1
                        out.append(tuple(g))
        return out

    def cflux_regions(self, recv_rank, send_rank):
        """Face-flux faces of recv_rank's leaves that af_consistent_fluxes
        sets from send_rank's refined neighbours (8 ints: id, dim, lo, hi;
        face indices), in (refined box, face) order."""
        if self.lp is None:
            return []
        nc = self.nc
        out = []
        for l in range(1, self.nlvl + 1):
            for p in np.asarray(self.topo["lvl_parents_%d" % l], np.int64):
                if self.owner[p - 1] != send_rank:
                    continue
                for nb in range(1, 7):
                    q = int(np.asarray(self.topo["meta_neighbors"])[p - 1][nb - 1])
                    if q <= 0 or self.children[q - 1][0] != 0 or self.owner[q - 1] != recv_rank:
                        continue
                    d = (nb - 1) // 2
                    f = nc + 1 if (nb - 1) % 2 == 0 else 1  # the neighbour's face
                    lo, hi = [1, 1, 1], [nc, nc, nc]
                    lo[d] = hi[d] = f
                    out.append((q, d, *lo, *hi))
        # a replicated refined box whose children are sharded: the face
        # quarter each child covers on the coarse leaf neighbour goes from
        # the child's owner to the neighbour's owner (every other rank when
        # the neighbour is replicated)
        h = nc // 2
        nbs = np.asarray(self.topo["meta_neighbors"])
        for l in range(1, self.nlvl + 1):
            for p in np.asarray(self.topo["lvl_parents_%d" % l], np.int64):
                if self.owner[p - 1] >= 0 or recv_rank == send_rank:
                    continue
                for nb in range(1, 7):
                    q = int(nbs[p - 1][nb - 1])
                    if q <= 0 or self.children[q - 1][0] != 0:
                        continue
                    if self.owner[q - 1] >= 0 and self.owner[q - 1] != recv_rank:
                        continue
                    d, side = (nb - 1) // 2, (nb - 1) % 2
                    f = nc + 1 if side == 0 else 1
                    for ch in range(8):
                        c = int(self.children[p - 1][ch])
                        cd = (ch & 1, (ch >> 1) & 1, (ch >> 2) & 1)
                        if cd[d] != side or c <= 0 or self.owner[c - 1] != send_rank:
                            continue
                        lo = [h * cd[k] + 1 for k in range(3)]
                        hi = [h * cd[k] + h for k in range(3)]
                        lo[d] = hi[d] = f
                        out.append((q, d, *lo, *hi))
        return out

    def restrict_levels(self):
        """Levels with an owned box whose parent is replicated (a RESTRICT
        exchange after their restriction)."""
        if self.lp is None:
            return []
        return [l for l in range(max(2, self.lp), self.nlvl + 1)
                if any(self.owner[c - 1] >= 0 and self.owner[self.parent[c - 1] - 1] < 0
                       for c in self.ids[l])]

    def octant_regions(self, send_rank, level=None):
        """Parent octants written by send_rank's boxes of `level` (default
        Lp) into their replicated parents, in box order."""
        if self.lp is None:
            return []
        level = self.lp if level is None else level
        hnc = self.nc // 2
        out = []
        for c in self.ids[level]:
            if self.owner[c - 1] != send_rank:
                continue
            p = self.parent[c - 1]
            if self.owner[p - 1] >= 0:
                continue
            co = [((self.ix[c - 1][k] - 1) & 1) * hnc for k in range(3)]
            out.append((int(p), co[0] + 1, co[1] + 1, co[2] + 1,
                        co[0] + hnc, co[1] + hnc, co[2] + hnc))
        return out


class Shard:
    """Executes the library's exchange hooks for one rank of a sharded tree."""

    def __init__(self, part, rank, backend="gloo", device=None):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.part = part
        self.rank = rank
        self.n = part.n_ranks
        self.backend = backend
        self.device = device  # torch device of the library's buffers (HIP) or None
        self.tree = None
        self.plans = {}
        self.n_exchanges = 0

    def make_tree(self, lib, topo, n_var_cell, n_var_face, device=-1, box_capacity=0):
        """This rank's Tree: storage for the whole tree, its level lists."""
        from .model import Tree
        return Tree(lib, self.part.local_topology(self.rank), n_var_cell, n_var_face,
                    device=device, box_capacity=box_capacity)

    def attach(self, tree):
        """Register plans and the hook on a Tree built from local_topology."""
        self.tree = tree
        lib = tree.lib
        part = self.part
        peers = [q for q in range(self.n) if q != self.rank]
        if part.lp is not None:
            for lvl in range(part.lp, part.nlvl + 1):
                for rims in (False, True):
                    send, recv = {}, {}
                    for q in peers:
                        send[q] = self._plan(part.halo_regions(q, self.rank, lvl, rims))
                        recv[q] = self._plan(part.halo_regions(self.rank, q, lvl, rims))
                    self.plans[("rims" if rims else "halo", lvl)] = (send, recv)
            self.plans[("cflux", 0)] = (
                {q: self._plan(part.cflux_regions(q, self.rank), fc=True) for q in peers},
                {q: self._plan(part.cflux_regions(self.rank, q), fc=True) for q in peers})
            for lvl in part.restrict_levels():
                mine = self._plan(part.octant_regions(self.rank, lvl))
                self.plans[("octant", lvl)] = (
                    {q: mine for q in peers},
                    {q: self._plan(part.octant_regions(q, lvl)) for q in peers})
        self._bufs = {}
        self.stream = None
        if self.device is not None and self.backend == "nccl":
            self.stream = self.torch.cuda.Stream(device=self.device)
            lib.call("tree_set_stream", tree.h, C.c_void_p(self.stream.cuda_stream))
        self._cb = capi.HOOK_FN(self._hook)
        lib.call("tree_set_hook", tree.h, C.cast(self._cb, C.c_void_p), None)

    def detach(self):
        if self.tree is not None and self.tree.h:
            self.tree.lib.call("tree_set_hook", self.tree.h, None, None)

    def _plan(self, regions, fc=False):
        lib, t = self.tree.lib, self.tree.h
        arr = np.ascontiguousarray(np.asarray(regions, np.int32).reshape(-1, 8 if fc else 7))
        pid, nval = C.c_int32(), C.c_int64()
        lib.call("plan_create_fc" if fc else "plan_create", t,
                 arr.ctypes.data_as(capi.P_i32), len(arr), C.byref(pid), C.byref(nval))
        return (pid.value, nval.value)

    # ----------------------------------------------------------- transport
    def _buf(self, key, n, device):
        """Persistent exchange buffer (reused by every exchange of a plan)."""
        torch = self.torch
        b = self._bufs.get(key)
        if b is None:
            b = torch.empty(max(n, 1), dtype=torch.float64, device=device)
            self._bufs[key] = b
        return b[:n]

    def _exchange(self, send, recv, iv):
        torch, dist = self.torch, self.dist
        lib, t = self.tree.lib, self.tree.h
        peers = sorted(set(send) | set(recv))
        if self.device is not None and self.backend == "nccl":
            # device buffers, everything on the tree's stream: pack, RCCL
            # send/recv (ordered after the pack, and the stream waits for
            # them), unpack -- no host synchronisation
            with torch.cuda.stream(self.stream):
                ops = []
                for q in peers:
                    (sp, sn), (rp, rn) = send[q], recv[q]
                    if sn:
                        b = self._buf(("s", sp), sn, self.device)
                        lib.call("plan_pack", t, sp, iv, C.c_void_p(b.data_ptr()))
                        ops.append(dist.P2POp(dist.isend, b, q))
                    if rn:
                        ops.append(dist.P2POp(dist.irecv, self._buf(("r", rp), rn, self.device), q))
                if ops:
                    for r in dist.batch_isend_irecv(ops):
                        r.wait()
                for q in peers:
                    rp, rn = recv[q]
                    if rn:
                        lib.call("plan_unpack", t, rp, iv,
                                 C.c_void_p(self._buf(("r", rp), rn, self.device).data_ptr()))
            self.n_exchanges += 1
            return
        # host transport (gloo): a device library stages through the host
        staged = self.device is not None
        ops = []
        for q in peers:
            sp, sn = send[q]
            if sn:
                hb = self._buf(("s", sp), sn, None)
                if staged:
                    db = self._buf(("ds", sp), sn, self.device)
                    lib.call("plan_pack", t, sp, iv, C.c_void_p(db.data_ptr()))
                    self.tree.sync()
                    hb.copy_(db)
                else:
                    lib.call("plan_pack", t, sp, iv, C.c_void_p(hb.data_ptr()))
                ops.append(dist.P2POp(dist.isend, hb, q))
            rp, rn = recv[q]
            if rn:
                ops.append(dist.P2POp(dist.irecv, self._buf(("r", rp), rn, None), q))
        if ops:
            for r in dist.batch_isend_irecv(ops):
                r.wait()
        for q in peers:
            rp, rn = recv[q]
            if not rn:
                continue
            hb = self._buf(("r", rp), rn, None)
            if staged:
                db = self._buf(("dr", rp), rn, self.device)
                db.copy_(hb)
                torch.cuda.synchronize(self.device)
                lib.call("plan_unpack", t, rp, iv, C.c_void_p(db.data_ptr()))
                self.tree.sync()
            else:
                lib.call("plan_unpack", t, rp, iv, C.c_void_p(hb.data_ptr()))
        self.n_exchanges += 1

    def _reduce(self, vals, n, op):
        torch, dist = self.torch, self.dist
        rop = {capi.HOOK_MAX: dist.ReduceOp.MAX, capi.HOOK_MIN: dist.ReduceOp.MIN,
               capi.HOOK_SUM: dist.ReduceOp.SUM}[op]
        host = [vals[i] for i in range(n)]
        if self.device is not None and self.backend == "nccl":
            with torch.cuda.stream(self.stream):
                x = torch.tensor(host, dtype=torch.float64, device=self.device)
                dist.all_reduce(x, op=rop)
                out = x.tolist()
        else:
            x = torch.tensor(host, dtype=torch.float64)
            dist.all_reduce(x, op=rop)
            out = x.tolist()
        for i in range(n):
            vals[i] = out[i]

    def _hook(self, ctx, kind, level, iv, vals, n):
        try:
            if kind in (capi.HOOK_MAX, capi.HOOK_MIN, capi.HOOK_SUM):
                self._reduce(vals, n, kind)
            elif kind == capi.HOOK_HALO:
                p = self.plans.get(("halo", level))
                if p:
                    self._exchange(p[0], p[1], iv)
            elif kind == capi.HOOK_RIMS:
                p = self.plans.get(("rims", level))
                if p:
                    self._exchange(p[0], p[1], iv)
            elif kind == capi.HOOK_CFLUX:
                p = self.plans.get(("cflux", 0))
                if p:
                    self._exchange(p[0], p[1], iv)
            elif kind == capi.HOOK_RESTRICT:
                p = self.plans.get(("octant", level))
                if p:
                    self._exchange(p[0], p[1], iv)
            return 0
        except Exception:  # a Python error must not unwind through C
            traceback.print_exc()
            return 1

    # ----------------------------------------------------------- results
    def owned_mask(self):
        o = self.part.owner
        return (o == self.rank) | (o < 0)


# ---------------------------------------------------------------- native
class NativeGroup:
    """afh_dist_group: the ranks of one process sharing a sharded tree
    (AFH_DIST_LOCAL; one thread per rank)."""

    def __init__(self, lib, n_ranks):
        import threading
        self.lib = lib
        self.n_ranks = n_ranks
        h = C.c_void_p()
        lib.call("dist_group_create", n_ranks, C.byref(h))
        self.h = h
        # host-side all-gather of Python objects among the thread ranks
        self._barrier = threading.Barrier(n_ranks)
        self._slots = [None] * n_ranks

    def allgather(self, rank, obj):
        """Every thread rank's obj, in rank order (a collective of the group)."""
        self._slots[rank] = obj
        self._barrier.wait()
        out = list(self._slots)
        self._barrier.wait()
        return out

    def close(self):
        if self.h:
            self.lib.call("dist_group_destroy", self.h)
            self.h = C.c_void_p()


def broadcast_bytes(data, src=0):
    """Rank src's bytes on every rank of the torch.distributed group (a device
    tensor under the nccl backend, which carries no host tensors)."""
    import torch
    import torch.distributed as tdist
    dev = "cuda" if tdist.get_backend() == "nccl" else "cpu"
    t = torch.tensor(list(data), dtype=torch.uint8, device=dev)
    tdist.broadcast(t, src=src)
    return bytes(t.cpu().tolist())


def rccl_comm(lib, rank, n_ranks, device):
    """An RCCL communicator for the library's AFH_DIST_RCCL transport; the
    unique id travels over the torch.distributed process group."""
    uid = (C.c_uint8 * 128)()
    if rank == 0:
        lib.call("dist_rccl_unique_id", C.cast(uid, C.c_void_p))
    if n_ranks > 1:
        uid = (C.c_uint8 * 128)(*broadcast_bytes(bytes(uid)))
    comm = C.c_void_p()
    lib.call("dist_rccl_comm", C.cast(uid, C.c_void_p), rank, n_ranks, device, C.byref(comm))
    return comm


class NativeShard:
    """One rank of a tree sharded by the library itself (afh_dist_*): the
    partition, the plans and the exchange hook are native; no Python runs
    during a step. Same interface as Shard (make_tree / attach / detach).

    transport: capi.DIST_LOCAL with `group` (a NativeGroup; ranks are
    threads of this process) or capi.DIST_RCCL with `comm` (rccl_comm)."""

    def __init__(self, lib, topo, n_ranks, rank, transport=capi.DIST_LOCAL, group=None,
                 comm=None, min_level_cells=0):
        from .model import tree_desc
        self.lib = lib
        self.topo = topo
        self.n = n_ranks
        self.rank = rank
        self.transport = transport
        self.group, self.comm = group, comm
        self.link = group.h if transport == capi.DIST_LOCAL else comm
        self._desc, self._keep = tree_desc(topo, 1, 1)
        self.owner = np.zeros(int(topo["n_boxes"]), np.int32)
        lp = C.c_int32()
        # min_level_cells: levels smaller than that replicated (afh_dist_partition_levels)
        self.min_level_cells = int(min_level_cells)
        lib.call("dist_partition_levels", C.byref(self._desc), n_ranks, self.min_level_cells,
                 self.owner.ctypes.data_as(capi.P_i32), C.byref(lp))
        self.lp = lp.value or None
        self.tree = None
        self.h = C.c_void_p()

    def plan(self, kind, level, recv_rank, send_rank):
        """The regions one exchange moves (afh_dist_plan), n x 7 (x 8 CFLUX)."""
        n = C.c_int32()
        pown = self.owner.ctypes.data_as(capi.P_i32)
        self.lib.call("dist_plan", C.byref(self._desc), pown, kind, level, recv_rank,
                      send_rank, None, 0, C.byref(n))
        w = 8 if kind == capi.HOOK_CFLUX else 7
        out = np.zeros((n.value, w), np.int32)
        self.lib.call("dist_plan", C.byref(self._desc), pown, kind, level, recv_rank,
                      send_rank, out.ctypes.data_as(capi.P_i32), n.value, C.byref(n))
        return out

    def local_topology(self):
        return local_topology(self.topo, self.owner, self.rank)

    def local_ids(self, rank):
        """Global ids of the boxes rank stores (afh_dist_local_ids: owned,
        replicated, replicas), sorted."""
        n = C.c_int32()
        pown = self.owner.ctypes.data_as(capi.P_i32)
        self.lib.call("dist_local_ids", C.byref(self._desc), pown, rank, None, 0, C.byref(n))
        out = np.zeros(n.value, np.int32)
        self.lib.call("dist_local_ids", C.byref(self._desc), pown, rank,
                      out.ctypes.data_as(capi.P_i32), n.value, C.byref(n))
        return out

    def make_tree(self, lib, topo, n_var_cell, n_var_face, device=-1, box_capacity=0):
        from .model import Tree
        return Tree(lib, self.local_topology(), n_var_cell, n_var_face, device=device,
                    box_capacity=box_capacity, shard_of=(topo, self.owner, self.rank))

    def attach(self, tree):
        self.tree = tree
        h = C.c_void_p()
        self.lib.call("dist_create", tree.h, C.byref(self._desc),
                      self.owner.ctypes.data_as(capi.P_i32), self.rank, self.n,
                      self.transport, self.link, C.byref(h))
        self.h = h

    def detach(self):
        if self.h:
            self.lib.call("dist_destroy", self.h)
            self.h = C.c_void_p()

    def renew(self, topo):
        """A shard of a new topology (after a regrid) over the same ranks and
        transport: a fresh partition."""
        return NativeShard(self.lib, topo, self.n, self.rank, self.transport,
                           group=self.group, comm=self.comm,
                           min_level_cells=self.min_level_cells)

    def allgather(self, obj):
        """Every rank's obj, in rank order: the thread ranks' group (objects
        shared in-process), or the torch.distributed process group (RCCL
        transport: one rank per process; small host objects only)."""
        if self.transport == capi.DIST_LOCAL:
            return self.group.allgather(self.rank, obj)
        import torch.distributed as tdist
        out = [None] * self.n
        tdist.all_gather_object(out, obj)
        return out

    def allgather_rows(self, ids, rows):
        """Every rank's (ids, rows) -- int box ids and float64 rows of equal
        width -- in rank order, as numeric collectives: the thread ranks'
        group in-process; with the RCCL transport two all_gathers of device
        tensors (the counts, then the rows padded to the longest), no pickling
        of data."""
        ids = np.ascontiguousarray(ids, np.int64)
        rows = np.ascontiguousarray(rows, np.float64).reshape(len(ids), -1)
        if self.transport == capi.DIST_LOCAL:
            return self.group.allgather(self.rank, (ids, rows))
        import torch
        import torch.distributed as tdist
        dev = "cuda" if tdist.get_backend() == "nccl" else "cpu"
        n = torch.tensor([len(ids)], dtype=torch.int64, device=dev)
        counts = [torch.zeros_like(n) for _ in range(self.n)]
        tdist.all_gather(counts, n)
        counts = [int(c.item()) for c in counts]
        m, w = max(counts), rows.shape[1]
        pid = torch.zeros(max(m, 1), dtype=torch.int64, device=dev)
        pid[:len(ids)] = torch.from_numpy(ids).to(dev)
        prow = torch.zeros((max(m, 1), w), dtype=torch.float64, device=dev)
        prow[:len(ids)] = torch.from_numpy(rows).to(dev)
        gid = [torch.zeros_like(pid) for _ in range(self.n)]
        grow = [torch.zeros_like(prow) for _ in range(self.n)]
        tdist.all_gather(gid, pid)
        tdist.all_gather(grow, prow)
        return [(gid[q][:counts[q]].cpu().numpy(), grow[q][:counts[q]].cpu().numpy())
                for q in range(self.n)]

    def exchange_rows(self, sends):
        """Point to point: sends = {rank q: (ids, rows)} (int box ids, float64
        rows of equal width); returns {rank q: (ids, rows)} received from q.
        The thread ranks hand over arrays in-process; with the RCCL transport
        the counts go in one all_gather and the data in batched send/recv of
        device tensors (only the pairs that exchange rows)."""
        norm = {}
        for q, (ids, rows) in sends.items():
            ids = np.ascontiguousarray(ids, np.int64)
            norm[q] = (ids, np.ascontiguousarray(rows, np.float64).reshape(len(ids), -1))
        if self.transport == capi.DIST_LOCAL:
            every = self.group.allgather(self.rank, norm)
            return {q: every[q][self.rank] for q in range(self.n)
                    if q != self.rank and self.rank in every[q]}
        import torch
        import torch.distributed as tdist
        dev = "cuda" if tdist.get_backend() == "nccl" else "cpu"
        mine = torch.zeros((self.n, 2), dtype=torch.int64, device=dev)
        for q, (ids, rows) in norm.items():
            mine[q, 0], mine[q, 1] = len(ids), rows.shape[1]
        counts = [torch.zeros_like(mine) for _ in range(self.n)]
        tdist.all_gather(counts, mine)
        counts = [c.cpu().numpy() for c in counts]
        ops, bufs = [], {}
        for q, (ids, rows) in norm.items():
            if len(ids):
                ops.append(tdist.P2POp(tdist.isend, torch.from_numpy(ids).to(dev), q))
                ops.append(tdist.P2POp(tdist.isend, torch.from_numpy(rows).to(dev), q))
        for q in range(self.n):
            m, w = counts[q][self.rank]
            if q != self.rank and m:
                bi = torch.zeros(int(m), dtype=torch.int64, device=dev)
                br = torch.zeros((int(m), int(w)), dtype=torch.float64, device=dev)
                bufs[q] = (bi, br)
                ops.append(tdist.P2POp(tdist.irecv, bi, q))
                ops.append(tdist.P2POp(tdist.irecv, br, q))
        if ops:
            for r in tdist.batch_isend_irecv(ops):
                r.wait()
        return {q: (bi.cpu().numpy(), br.cpu().numpy()) for q, (bi, br) in bufs.items()}

    def exchange_rows_dev(self, sends, device):
        """exchange_rows with the rows as device tensors (float64, on the
        tree's device `device`, from Tree.pack_boxes): the thread ranks hand the
        tensors over in-process; the RCCL transport sends and receives them
        as they are -- the box data never visit the host. Returns {rank q:
        (ids, rows tensor)}; the received rows are complete on return."""
        import torch
        norm = {q: (np.ascontiguousarray(ids, np.int64), rows) for q, (ids, rows) in sends.items()}
        if self.transport == capi.DIST_LOCAL:
            every = self.group.allgather(self.rank, norm)
            return {q: every[q][self.rank] for q in range(self.n)
                    if q != self.rank and self.rank in every[q]}
        import torch.distributed as tdist
        cuda = tdist.get_backend() == "nccl"
        dev = device if cuda else "cpu"
        mine = torch.zeros((self.n, 2), dtype=torch.int64, device=dev)
        for q, (ids, rows) in norm.items():
            mine[q, 0], mine[q, 1] = len(ids), rows.shape[1]
        counts = [torch.zeros_like(mine) for _ in range(self.n)]
        tdist.all_gather(counts, mine)
        counts = [c.cpu().numpy() for c in counts]
        ops, bufs = [], {}
        for q, (ids, rows) in norm.items():
            if len(ids):
                ops.append(tdist.P2POp(tdist.isend, torch.from_numpy(ids).to(dev), q))
                # a backend without device tensors (gloo) sends host copies
                ops.append(tdist.P2POp(tdist.isend, rows if cuda else rows.cpu(), q))
        for q in range(self.n):
            m, w = counts[q][self.rank]
            if q != self.rank and m:
                bi = torch.zeros(int(m), dtype=torch.int64, device=dev)
                br = torch.empty((int(m), int(w)), dtype=torch.float64, device=dev)
                bufs[q] = (bi, br)
                ops.append(tdist.P2POp(tdist.irecv, bi, q))
                ops.append(tdist.P2POp(tdist.irecv, br, q))
        if ops:
            for r in tdist.batch_isend_irecv(ops):
                r.wait()
        if cuda:
            # the receives complete on the communicator's stream; the
            # library's unpack runs on the tree's
            torch.cuda.synchronize(device)
        return {q: (bi.cpu().numpy(), br if cuda else br.to(device)) for q, (bi, br) in bufs.items()}

    def stats(self):
        n, b = C.c_int64(), C.c_int64()
        self.lib.call("dist_stats", self.h, C.byref(n), C.byref(b))
        return n.value, b.value

    @property
    def n_exchanges(self):
        return self.stats()[0]

    def owned_mask(self):
        return (self.owner == self.rank) | (self.owner < 0)
