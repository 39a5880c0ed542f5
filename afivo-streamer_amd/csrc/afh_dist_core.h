// Native box sharding: the partition and the exchange plans (host code
// shared by libafivo_hip (afh_dist.hip) and the C oracle's CPU twin
// (oracle/c/afo_dist.cpp), which runs the same sharded semantics on host
// buffers). The Python reference these restate: afivo-streamer_amd/afh/dist.py
// (Partition); tests/test_dist_native.py compares them.
#pragma once
#include <stdint.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <condition_variable>
#include <map>
#include <mutex>
#include <set>
#include <vector>

#include "../../include/afivo_hip.h"

namespace afhd {

using Region = std::array<int32_t, 8>;  // cc: id, lo[3], hi[3] (7 used); fc: id, dim, lo, hi

constexpr int DEPTH = 2;  // halo layers (dist.py DEPTH)
constexpr int TOL_PCT = 10;  // frontier refined while max load > (100 + TOL_PCT) % of the mean
constexpr int MORTON_BITS = 21;

struct Topo {
  int nc, nb, nlvl;
  const afh_box_meta *m;
  std::vector<std::vector<int32_t>> ids, leaves, parents;  // per level 1..nlvl (index l-1)
};

inline Topo topo_of(const afh_tree_desc *d) {
  Topo t;
  t.nc = d->n_cell, t.nb = d->n_boxes, t.nlvl = d->highest_lvl, t.m = d->boxes;
  auto lists = [&](const int32_t *a, const int32_t *off) {
    std::vector<std::vector<int32_t>> v(t.nlvl);
    for (int l = 0; l < t.nlvl; l++) v[l].assign(a + off[l], a + off[l + 1]);
    return v;
  };
  t.ids = lists(d->lvl_ids, d->lvl_ids_off);
  t.leaves = lists(d->lvl_leaves, d->lvl_leaves_off);
  t.parents = lists(d->lvl_parents, d->lvl_parents_off);
  return t;
}

// Z-order index of the box's lower corner at `shift` levels finer
inline int64_t morton3(const int32_t ix[3], int shift = 0) {
  int64_t code = 0;
  for (int b = 0; b < MORTON_BITS; b++)
    for (int d = 0; d < 3; d++)
      code |= (int64_t)((((int64_t)(ix[d] - 1) << shift) >> b) & 1) << (3 * b + d);
  return code;
}

// Partition._partition (afh/dist.py): the weighted Morton split of a
// partition frontier. The frontier starts as level 2 (level 1 replicated);
// its boxes, in Z-order of their lower corners at the finest resolution, are
// cut into chunks of about equal leaf weight; while the heaviest rank carries
// more than (100 + TOL_PCT) % of the mean (or the frontier has fewer boxes
// than ranks), its heaviest refined box is replaced by its children and
// becomes replicated. Descendants follow their frontier box. Returns the
// first level with an owned box, or -1.
//
// min_level_cells > 0 (round 6): the frontier starts at the first level >= 2
// whose boxes hold at least that many cells; the levels below it, leaves
// included, are replicated -- computed by every rank, with no exchange. A
// level smaller than that is launch-bound on one GPU already: sharding it
// saves no kernel time and adds its exchanges. When no level
// is that large the whole tree is replicated (returns 0: every rank computes
// every box, as one GPU would).
inline int partition(const Topo &t, int n, std::vector<int32_t> &owner,
                     int64_t min_level_cells = 0) {
  owner.assign(t.nb, -1);
  if (n <= 1) return 0;
  if (t.nlvl < 2) return min_level_cells > 0 ? 0 : -1;
  int ls = 2;
  if (min_level_cells > 0) {
    const int64_t box_cells = (int64_t)t.nc * t.nc * t.nc;
    ls = 0;
    for (int l = 2; l <= t.nlvl && !ls; l++)
      if ((int64_t)t.ids[l - 1].size() * box_cells >= min_level_cells &&
          (int)t.ids[l - 1].size() >= n)
        ls = l;
    if (!ls) return 0;
  }
  std::vector<int64_t> w(t.nb + 1, 0);
  for (int l = t.nlvl; l >= 1; l--)
    for (int32_t i : t.ids[l - 1]) {
      const int32_t *ch = t.m[i - 1].children;
      if (ch[0] == 0) {
        w[i] = 1;
      } else {
        int64_t s = 0;
        for (int c = 0; c < 8; c++) s += w[ch[c]];
        w[i] = s;
      }
    }
  std::vector<int32_t> roots = t.ids[ls - 1];
  auto code = [&](int32_t b) { return morton3(t.m[b - 1].ix, t.nlvl - t.m[b - 1].lvl); };
  std::vector<int32_t> order;
  std::vector<int64_t> rk;
  // chunks of the frontier; true when every rank gets a box
  auto split = [&](int64_t &mx, int64_t &total) {
    order = roots;
    std::vector<int64_t> key(t.nb + 1, 0);
    for (int32_t b : order) key[b] = code(b);
    std::stable_sort(order.begin(), order.end(),
                     [&](int32_t a, int32_t b) { return key[a] < key[b]; });
    const int no = (int)order.size();
    std::vector<int64_t> cum(no);
    int64_t s = 0;
    for (int q = 0; q < no; q++) cum[q] = (s += w[order[q]]);
    total = s;
    const double target = (double)s / n;
    rk.assign(no, 0);
    std::vector<int64_t> load(n, 0);
    for (int q = 0; q < no; q++) {
      const int64_t r = (int64_t)std::ceil((double)cum[q] / target) - 1;
      rk[q] = std::min<int64_t>(r, n - 1);
      load[rk[q]] += w[order[q]];
    }
    mx = *std::max_element(load.begin(), load.end());
    return (int)std::set<int64_t>(rk.begin(), rk.end()).size() == n;
  };
  int64_t mx = 0, total = 0;
  for (;;) {
    if ((int)roots.size() >= n && split(mx, total) && mx * n * 100 <= (100 + TOL_PCT) * total)
      break;
    int32_t h = 0;
    for (int32_t r : roots)
      if (t.m[r - 1].children[0] > 0 && (!h || w[r] > w[h] || (w[r] == w[h] && r < h))) h = r;
    if (!h) {
      if ((int)roots.size() < n) return -1;
      break;
    }
    roots.erase(std::find(roots.begin(), roots.end(), h));
    for (int c = 0; c < 8; c++) roots.push_back(t.m[h - 1].children[c]);
  }
  if (!split(mx, total))  // every rank gets a frontier box: an even split
    for (size_t q = 0; q < order.size(); q++) rk[q] = ((int64_t)q * n) / (int64_t)order.size();
  for (size_t q = 0; q < order.size(); q++) owner[order[q] - 1] = (int32_t)rk[q];
  for (int l = ls + 1; l <= t.nlvl; l++)
    for (int32_t i : t.ids[l - 1]) {
      const int32_t p = t.m[i - 1].parent;
      if (owner[p - 1] >= 0) owner[i - 1] = owner[p - 1];
    }
  int lp = t.nlvl;
  for (int32_t r : roots) lp = std::min(lp, t.m[r - 1].lvl);
  return lp;
}

// Partition._region: cells of box b within `depth` layers (DEPTH unless the
// reader needs fewer), b at direction d
inline Region region(const Topo &t, int32_t b, const int d[3], bool rims, int depth = DEPTH) {
  Region r{};
  r[0] = b;
  for (int k = 0; k < 3; k++) {
    int lo, hi;
    if (d[k] < 0)
      lo = t.nc - depth + 1, hi = rims ? t.nc + 1 : t.nc;
    else if (d[k] > 0)
      lo = rims ? 0 : 1, hi = depth;
    else
      lo = rims ? 0 : 1, hi = rims ? t.nc + 1 : t.nc;
    r[1 + k] = lo, r[4 + k] = hi;
  }
  return r;
}

// Partition.halo_regions
// local_faces (RIMS after a fill of every box of the level): a ghost slab
// facing a box the receiver computes is left out (below)
// pair (round 6: RIMS before a fused pair on a level no finer level
// interpolates from): of the ghost slabs only the face parts ([1, nc] in
// both tangential directions; the 6-point stencil of the pair's recomputed
// neighbour cells reads no edge or corner ghost) of faces the receiver
// cannot fill itself -- faces at a refinement boundary, or whose same-level
// neighbour it does not store (`stored`, by global id); a face next to a
// stored box or the domain boundary it fills itself (afh_dist.hip
// k_face_fill)
inline std::vector<Region> halo_regions(const Topo &t, const std::vector<int32_t> &owner, int lp,
                                 int recv, int send, int level, bool rims,
                                 int depth = DEPTH, bool local_faces = false,
                                 const std::vector<char> *pair = nullptr) {
  std::vector<Region> out;
  if (!lp || level < lp) return out;
  std::set<Region> regs;
  for (int32_t a : t.ids[level - 1]) {
    // the boxes recv computes: its own and the replicated ones
    if (owner[a - 1] != recv && owner[a - 1] >= 0) continue;
    for (int dz = -1; dz <= 1; dz++)
      for (int dy = -1; dy <= 1; dy++)
        for (int dx = -1; dx <= 1; dx++) {
          if (!dx && !dy && !dz) continue;
          const int b = t.m[a - 1].neighbor_mat[(dx + 1) + 3 * (dy + 1) + 9 * (dz + 1)];
          const int d[3] = {dx, dy, dz};
          if (b > 0 && owner[b - 1] == send) regs.insert(region(t, b, d, rims, depth));
        }
  }
  std::map<int32_t, std::vector<Region>> by_box;
  for (const Region &r : regs) by_box[r[0]].push_back(r);
  for (auto &kv : by_box) {
    auto &rs = kv.second;
    std::sort(rs.begin(), rs.end());
    for (const Region &r : rs) {
      bool inside = false;
      for (const Region &q : rs)
        if (q != r && q[1] <= r[1] && q[2] <= r[2] && q[3] <= r[3] && r[4] <= q[4] &&
            r[5] <= q[5] && r[6] <= q[6])
          inside = true;
      if (inside) continue;
      if (!rims) {
        out.push_back(r);
        continue;
      }
      // RIMS follows the HALO exchange of the same variable and level, with
      // only a ghost-cell fill between them: the region's interior cells
      // arrived with the HALO and are unchanged, so only its ghost cells
      // travel (round 6) -- the region less the box interior [1, nc]^3, as
      // disjoint slabs: along dimension k, the cells outside [1, nc] whose
      // coordinates in the dimensions before k lie inside it. And with
      // local_faces (the level fills of the multigrid, not the flux's
      // leaves-only fill), of a slab whose face neighbour the receiver
      // computes (its own box or a replicated one) the part facing that
      // neighbour is left out too: the receiver copies it from that
      // neighbour itself after the exchange (afh_dist.hip face_copies, a
      // same-level face copy as the owner's fill made); only the slab's
      // rims (edge and corner ghosts) travel
      const afh_box_meta &mb = t.m[r[0] - 1];
      for (int k = 0; k < 3; k++)
        for (int side = 0; side < 2; side++) {
          Region g = r;
          for (int j = 0; j < k; j++)
            g[1 + j] = std::max(r[1 + j], 1), g[4 + j] = std::min(r[4 + j], t.nc);
          if (side == 0) {
            if (r[1 + k] >= 1) continue;
            g[4 + k] = 0;
          } else {
            if (r[4 + k] <= t.nc) continue;
            g[1 + k] = t.nc + 1;
          }
          const int nb = mb.neighbors[2 * k + side];
          if (pair) {
            if (nb < 0 || (nb > 0 && (*pair)[nb])) continue;  // filled by the receiver
            for (int j = 0; j < 3; j++)
              if (j != k) g[1 + j] = std::max(g[1 + j], 1), g[4 + j] = std::min(g[4 + j], t.nc);
            out.push_back(g);
            continue;
          }
          if (!local_faces || !(nb > 0 && (owner[nb - 1] == recv || owner[nb - 1] < 0))) {
            out.push_back(g);
            continue;
          }
          // the slab less its face part (transverse coordinates in [1, nc])
          int jj = 0;
          for (int j = 0; j < 3; j++) {
            if (j == k) continue;
            for (int s2 = 0; s2 < 2; s2++) {
              Region h = g;
              for (int q = 0; q < 3; q++)
                if (q != k && q != j && (jj > 0 && q < j))
                  h[1 + q] = std::max(g[1 + q], 1), h[4 + q] = std::min(g[4 + q], t.nc);
              if (s2 == 0) {
                if (g[1 + j] >= 1) continue;
                h[4 + j] = 0;
              } else {
                if (g[4 + j] <= t.nc) continue;
                h[1 + j] = t.nc + 1;
              }
              out.push_back(h);
            }
            jj++;
          }
        }
    }
  }
  return out;
}

// The boxes of `level` a rank holds current data of around its boxes: the
// ones it computes and the HALO replicas (by global id; RIMS pair mode)
inline std::vector<char> level_stored(const Topo &t, const std::vector<int32_t> &owner, int lp,
                                      int rank, int n_ranks, int level) {
  std::vector<char> st(t.nb + 1, 0);
  for (int32_t a : t.ids[level - 1])
    if (owner[a - 1] == rank || owner[a - 1] < 0) st[a] = 1;
  for (int q = 0; q < n_ranks; q++)
    if (q != rank)
      for (const Region &r : halo_regions(t, owner, lp, rank, q, level, false)) st[r[0]] = 1;
  return st;
}

// Partition.cflux_regions (8 ints: id, dim, lo, hi; face indices)
inline std::vector<Region> cflux_regions(const Topo &t, const std::vector<int32_t> &owner, int lp,
                                  int recv, int send) {
  std::vector<Region> out;
  if (!lp) return out;
  for (int l = 1; l <= t.nlvl; l++)
    for (int32_t p : t.parents[l - 1]) {
      if (owner[p - 1] != send) continue;
      for (int nb = 1; nb <= 6; nb++) {
        const int q = t.m[p - 1].neighbors[nb - 1];
        if (q <= 0 || t.m[q - 1].children[0] != 0 || owner[q - 1] != recv) continue;
        const int d = (nb - 1) / 2;
        const int f = (nb - 1) % 2 == 0 ? t.nc + 1 : 1;
        int lo[3] = {1, 1, 1}, hi[3] = {t.nc, t.nc, t.nc};
        lo[d] = hi[d] = f;
        out.push_back(Region{q, d, lo[0], lo[1], lo[2], hi[0], hi[1], hi[2]});
      }
    }
  // a replicated refined box whose children are sharded: only the owner of
  // a child has that child's fluxes -- the face quarter each child covers on
  // the coarse leaf neighbour goes from the child's owner to the neighbour's
  // owner (to every other rank when the neighbour is replicated)
  const int h = t.nc / 2;
  for (int l = 1; l <= t.nlvl; l++)
    for (int32_t p : t.parents[l - 1]) {
      if (owner[p - 1] >= 0) continue;
      for (int nb = 1; nb <= 6; nb++) {
        const int q = t.m[p - 1].neighbors[nb - 1];
        if (q <= 0 || t.m[q - 1].children[0] != 0 || recv == send) continue;
        if (owner[q - 1] >= 0 && owner[q - 1] != recv) continue;
        const int d = (nb - 1) / 2, side = (nb - 1) % 2;  // side 0: q below p
        const int f = side == 0 ? t.nc + 1 : 1;
        for (int ch = 0; ch < 8; ch++) {
          const int c = t.m[p - 1].children[ch];
          const int cd[3] = {ch & 1, (ch >> 1) & 1, (ch >> 2) & 1};  // af_child_dix
          if (cd[d] != side || c <= 0 || owner[c - 1] != send) continue;
          int lo[3], hi[3];
          for (int k = 0; k < 3; k++) lo[k] = h * cd[k] + 1, hi[k] = h * cd[k] + h;
          lo[d] = hi[d] = f;
          out.push_back(Region{q, d, lo[0], lo[1], lo[2], hi[0], hi[1], hi[2]});
        }
      }
    }
  return out;
}

// Partition.octant_regions: parent octants written by send's boxes of
// `level` into their replicated parents
inline std::vector<Region> octant_regions(const Topo &t, const std::vector<int32_t> &owner, int lp,
                                   int send, int level) {
  std::vector<Region> out;
  if (!lp || level < 2 || level > t.nlvl) return out;
  const int h = t.nc / 2;
  for (int32_t c : t.ids[level - 1]) {
    if (owner[c - 1] != send) continue;
    const afh_box_meta &m = t.m[c - 1];
    if (owner[m.parent - 1] >= 0) continue;
    int co[3];
    for (int k = 0; k < 3; k++) co[k] = ((m.ix[k] - 1) & 1) * h;
    out.push_back(Region{m.parent, co[0] + 1, co[1] + 1, co[2] + 1, co[0] + h, co[1] + h,
                         co[2] + h, 0});
  }
  return out;
}

// Partition.restrict_levels: levels with an owned box whose parent is
// replicated (a RESTRICT exchange follows their restriction)
inline std::vector<int> restrict_levels(const Topo &t, const std::vector<int32_t> &owner, int lp) {
  std::vector<int> out;
  if (!lp) return out;
  for (int l = std::max(2, lp); l <= t.nlvl; l++)
    for (int32_t c : t.ids[l - 1])
      if (owner[c - 1] >= 0 && owner[t.m[c - 1].parent - 1] < 0) {
        out.push_back(l);
        break;
      }
  return out;
}

inline std::vector<Region> plan_regions(const Topo &t, const std::vector<int32_t> &owner, int lp,
                                 int kind, int level, int recv, int send,
                                 int depth = DEPTH, bool local_faces = false,
                                 const std::vector<char> *pair = nullptr) {
  switch (kind) {
  case AFH_HOOK_HALO: return halo_regions(t, owner, lp, recv, send, level, false, depth);
  case AFH_HOOK_RIMS:
    return halo_regions(t, owner, lp, recv, send, level, true, depth, local_faces, pair);
  case AFH_HOOK_CFLUX: return cflux_regions(t, owner, lp, recv, send);
  case AFH_HOOK_RESTRICT: return octant_regions(t, owner, lp, send, level);
  default: return {};
  }
}

// A reusable barrier for the threads of an AFH_DIST_LOCAL group
struct Barrier {
  std::mutex mu;
  std::condition_variable cv;
  int n, waiting = 0;
  uint64_t gen = 0;
  explicit Barrier(int n_) : n(n_) {}
  void wait() {
    std::unique_lock<std::mutex> lk(mu);
    const uint64_t g = gen;
    if (++waiting == n) {
      waiting = 0;
      gen++;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return gen != g; });
    }
  }
};

// the partition level: the first level with an owned (non-replicated) box
inline int first_owned_level(const Topo &t, const int32_t *owner) {
  for (int l = 1; l <= t.nlvl; l++)
    for (int32_t i : t.ids[l - 1])
      if (owner[i - 1] >= 0) return l;
  return 0;
}

// The boxes a rank stores (owned-box allocation): its own boxes, the
// replicated levels below Lp, every box an exchange plan of the rank names
// (as sender or receiver: halo / rim replicas, the faces it writes for the
// consistent fluxes, the parents of the restriction) and, on a level where
// that leaves none, one box of the level (its grid spacing). Ascending
// global ids; the local id of ids[k] is k + 1.
inline std::vector<int32_t> local_boxes(const Topo &t, const std::vector<int32_t> &owner,
                                        int rank) {
  int lp = 0, n = 1;
  for (int l = 1; l <= t.nlvl && !lp; l++)
    for (int32_t i : t.ids[l - 1])
      if (owner[i - 1] >= 0) {
        lp = l;
        break;
      }
  for (int32_t o : owner) n = std::max(n, o + 1);
  std::vector<char> keep(t.nb + 1, 0);
  for (int i = 1; i <= t.nb; i++) keep[i] = owner[i - 1] == rank || owner[i - 1] < 0;
  auto add = [&](const std::vector<Region> &rs) {
    for (const Region &r : rs) keep[r[0]] = 1;
  };
  if (lp)
    for (int q = 0; q < n; q++) {
      if (q == rank) continue;
      for (int l = lp; l <= t.nlvl; l++) {
        add(plan_regions(t, owner, lp, AFH_HOOK_RIMS, l, rank, q));
        add(plan_regions(t, owner, lp, AFH_HOOK_RIMS, l, q, rank));
      }
      add(plan_regions(t, owner, lp, AFH_HOOK_CFLUX, 0, rank, q));
      add(plan_regions(t, owner, lp, AFH_HOOK_CFLUX, 0, q, rank));
      for (int l : restrict_levels(t, owner, lp)) {
        add(plan_regions(t, owner, lp, AFH_HOOK_RESTRICT, l, rank, q));
        add(plan_regions(t, owner, lp, AFH_HOOK_RESTRICT, l, q, rank));
      }
    }
  for (int l = 1; l <= t.nlvl; l++) {
    bool any = false;
    for (int32_t i : t.ids[l - 1]) any |= keep[i] != 0;
    if (!any && !t.ids[l - 1].empty()) keep[t.ids[l - 1][0]] = 1;
  }
  std::vector<int32_t> ids;
  for (int i = 1; i <= t.nb; i++)
    if (keep[i]) ids.push_back(i);
  return ids;
}

// A rank's compacted tree: the boxes of local_boxes renumbered 1..n, and a
// last, unused id (level 0, no data anyone reads) that stands for every box
// a stored box names but the rank does not store.
struct Compact {
  std::vector<int32_t> ids, g2l;  // local -> global (ids[k] = global id of k+1); global -> local
  std::vector<afh_box_meta> meta;
  std::vector<int32_t> lists[3], offs[3];
  afh_tree_desc desc;
};

inline void compact(const Topo &t, const afh_tree_desc *full, const std::vector<int32_t> &owner,
                    int rank, Compact &c) {
  c.ids = local_boxes(t, owner, rank);
  const int n = (int)c.ids.size(), absent = n + 1;
  c.g2l.assign(t.nb + 1, 0);
  for (int k = 0; k < n; k++) c.g2l[c.ids[k]] = k + 1;
  auto map = [&](int32_t g) { return g <= 0 ? g : c.g2l[g] ? c.g2l[g] : absent; };
  c.meta.assign(n + 1, afh_box_meta{});
  for (int k = 0; k < n; k++) {
    afh_box_meta m = t.m[c.ids[k] - 1];
    m.parent = map(m.parent);
    for (int q = 0; q < 8; q++) m.children[q] = map(m.children[q]);
    for (int q = 0; q < 6; q++) m.neighbors[q] = map(m.neighbors[q]);
    for (int q = 0; q < 27; q++) m.neighbor_mat[q] = map(m.neighbor_mat[q]);
    c.meta[k] = m;
  }
  const std::vector<std::vector<int32_t>> *src[3] = {&t.ids, &t.leaves, &t.parents};
  for (int k = 0; k < 3; k++) {
    c.lists[k].clear(), c.offs[k].assign(1, 0);
    for (int l = 0; l < t.nlvl; l++) {
      for (int32_t i : (*src[k])[l])
        if (owner[i - 1] == rank || owner[i - 1] < 0) c.lists[k].push_back(c.g2l[i]);
      c.offs[k].push_back((int32_t)c.lists[k].size());
    }
  }
  c.desc = *full;
  c.desc.n_boxes = n + 1;
  c.desc.box_capacity = 0;
  c.desc.boxes = c.meta.data();
  c.desc.lvl_ids = c.lists[0].data(), c.desc.lvl_ids_off = c.offs[0].data();
  c.desc.lvl_leaves = c.lists[1].data(), c.desc.lvl_leaves_off = c.offs[1].data();
  c.desc.lvl_parents = c.lists[2].data(), c.desc.lvl_parents_off = c.offs[2].data();
}

}  // namespace afhd
