// Native box sharding: the partition, the exchange plans
// and the exchange hook inside the library, so a driver in any language
// shards a tree without a collective library of its own.
//
// Partition (as afivo-streamer_amd/afh/dist.py states it, the tests compare
// the two): a weighted Morton split of a partition frontier, refined until
// the heaviest rank carries at most 110 % of the mean leaf weight
// (afh_dist_core.h partition()); descendants follow their frontier box; the
// frontier's ancestors and level 1 are replicated (owner -1).
//
// Plans: for every exchange the library's hooks request (HALO / RIMS per
// level, CFLUX, RESTRICT), the regions this rank sends to and receives from
// every peer, packed and unpacked by afh_plan_pack / afh_plan_unpack on the
// tree's stream.
//
// Transports: AFH_DIST_LOCAL -- the ranks are threads of one process (one
// tree each, on one or several GPUs): pack, a group barrier, peer copies of
// the peers' packed buffers, unpack, a barrier; AFH_DIST_RCCL -- one rank per
// process: grouped ncclSend / ncclRecv on the tree's stream (no host
// synchronisation) and ncclAllReduce for the reductions.
#include <rccl/rccl.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <condition_variable>
#include <map>
#include <mutex>
#include <set>
#include <tuple>

#include "afh_internal.h"

using namespace afh;

#include "afh_dist_core.h"

using namespace afhd;

struct afh_dist;

struct afh_dist_group {
  int n;
  Barrier bar;
  std::vector<afh_dist *> rank;
  std::vector<std::array<double, 16>> vals;
  explicit afh_dist_group(int n_) : n(n_), bar(n_), rank(n_, nullptr), vals(n_) {}
};

struct afh_dist {
  afh_tree *t = nullptr;
  int rank = 0, n = 1, transport = 0, device = 0;
  afh_dist_group *group = nullptr;
  ncclComm_t comm = nullptr;
  // One exchange: the regions this rank sends to every peer as ONE plan
  // (packed by one launch into one buffer, peer q's values at send_off[q]),
  // the regions it receives likewise (one unpack launch) -- instead of a
  // pack and an unpack launch per peer (round 5: 1586 plan-copy launches
  // per S5 step on 8 ranks, profiles/r05_scaling_*.json)
  struct Plan {
    int32_t send_plan = -1, recv_plan = -1;
    double *send_buf = nullptr, *recv_buf = nullptr;
    std::vector<int64_t> send_off, send_n, recv_off, recv_n;  // per peer
    // RIMS with local faces: (local box, face 1..6) pairs whose face ghosts
    // this rank copies from its own face neighbour after the exchange
    int32_t *d_fc = nullptr;
    int32_t n_fc = 0;
    bool local_only = false;  // the same on every rank: nothing to send anywhere
  };
  std::map<std::tuple<int, int, int>, Plan> plans;  // (hook kind, level, layers)
  double *d_red = nullptr;
  int64_t n_exchanges = 0, bytes = 0;
  std::vector<int64_t> peer_sent, peer_recv;  // bytes per peer (afh_dist_peer_bytes)
};

namespace {

// (hook kind, level, layers): HALO / RIMS plans exist for one and two
// layers -- the hook's n: the layers the next reader needs after a fill of
// every box of the level (RIMS then leaves out the face ghosts of replicas
// next to a box this rank computes, afh_dist_core.h halo_regions, and
// copies them here: k_face_copy); n = 0: DEPTH layers after any fill (key
// layers 0 for RIMS: every ghost cell travels)
using Key = std::tuple<int, int, int>;

// The face part ([1, nc]^2) of the ghost layer of face nb of box list[2 q],
// nb = list[2 q + 1], filled by the receiver: copied from the same-level
// neighbour's boundary layer, or the domain boundary's condition from the
// box's own cells (af_gc_box, m_af_ghostcell.f90:64-120, bc_to_gc 173-279).
// One thread per cell, one block row per pair.
__global__ void k_face_fill(double *__restrict__ v, const afh_box_meta *__restrict__ meta,
                            const int32_t *__restrict__ list, int nc, size_t bsz, GcArgs ga) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nc * nc) return;
  const int id = list[2 * blockIdx.y], nb = list[2 * blockIdx.y + 1];
  const int d = (nb - 1) >> 1;
  const bool low = ((nb - 1) & 1) == 0;
  const afh_box_meta &m = meta[id - 1];
  const int src = m.neighbors[nb - 1];
  const int a = t % nc + 1, b = t / nc + 1;
  const int ta = (d == 0) ? 1 : 0, tb = (d == 2) ? 1 : 2;
  int p[3];
  p[ta] = a;
  p[tb] = b;
  p[d] = low ? 0 : nc + 1;
  const int ng = nc + 2;
  double *c = v + (size_t)(id - 1) * bsz;
  if (src > 0) {
    int q[3] = {p[0], p[1], p[2]};
    q[d] = low ? nc : 1;
    c[ix3(ng, p[0], p[1], p[2])] = v[(size_t)(src - 1) * bsz + ix3(ng, q[0], q[1], q[2])];
    return;
  }
  c[ix3(ng, p[0], p[1], p[2])] =
      gc_face_nocopy(v, meta, m, nb, p, a, b, nc, bsz, ga.bc[nb - 1], ga.rb,
                     [&](const int *q) { return c[ix3(ng, q[0], q[1], q[2])]; });
}

// the receiver's own face fills of a RIMS plan (k_face_fill); the bc of the
// alt image is its source variable's
int32_t face_fill(afh_tree *t, const afh_dist::Plan &p, int iv) {
  const GcArgs ga = t->gc_args(iv ? iv : t->alt_of);
  for (int q0 = 0; q0 < p.n_fc; q0 += 65535) {
    hipLaunchKernelGGL(k_face_fill, dim3((t->nc * t->nc + 255) / 256, std::min(65535, p.n_fc - q0)),
                       dim3(256), 0, t->stream, t->var(iv), t->d_boxes, p.d_fc + 2 * (size_t)q0,
                       t->nc, t->bsz, ga);
    AFH_LAUNCH_CHECK("k_face_fill");
  }
  return AFH_OK;
}

int32_t exchange(afh_dist *d, const Key &key, int iv) {
  auto it = d->plans.find(key);
  if (it == d->plans.end()) return AFH_OK;
  const afh_dist::Plan &p = it->second;
  afh_tree *t = d->t;
  // no rank sends anything (every rank fills the faces itself): no exchange
  if (p.local_only) return face_fill(t, p, iv);
  // AFH_DIST_LOG=1: one stderr line per exchange (rank, kind, level,
  // layers, variable, doubles sent) -- what a step exchanges, for the
  // scaling work
  static const bool log = getenv("AFH_DIST_LOG") && atoi(getenv("AFH_DIST_LOG"));
  if (log) {
    int64_t n = 0;
    for (int q = 0; q < d->n; q++) n += p.send_n[q];
    fprintf(stderr, "XCHG r%d k%d l%d n%d v%d %lld\n", d->rank, std::get<0>(key),
            std::get<1>(key), std::get<2>(key), iv, (long long)n);
  }
  int32_t e = AFH_OK;
  if (p.send_plan >= 0) e = afh_plan_pack(t, p.send_plan, iv, p.send_buf);
  if (d->transport == AFH_DIST_RCCL) {
    // the grouped send/recv is posted even after a failed pack (the buffer
    // then carries stale values), so the peers' matching calls complete and
    // every rank reports an error instead of some of them hanging
    const int32_t e_pack = e;
    bool posted = ncclGroupStart() == ncclSuccess;
    for (int q = 0; q < d->n && posted; q++) {
      if (p.send_n[q] && ncclSend(p.send_buf + p.send_off[q], p.send_n[q], ncclDouble, q,
                                  d->comm, t->stream) != ncclSuccess)
        posted = false;
      if (posted && p.recv_n[q] &&
          ncclRecv(p.recv_buf + p.recv_off[q], p.recv_n[q], ncclDouble, q, d->comm,
                   t->stream) != ncclSuccess)
        posted = false;
    }
    if (ncclGroupEnd() != ncclSuccess) posted = false;
    if (!posted)
      return set_error(AFH_ERR_DEVICE, "exchange %d/%d: posting the RCCL send/recv failed",
                       std::get<0>(key), std::get<1>(key));
    if (e_pack) return e_pack;
  } else {
    // every rank's packs complete, then each copies the peers' packed
    // buffers; nobody packs again before every peer has copied. The
    // barriers are passed on every path, so a failing rank cannot strand
    // its peers.
    if (!e && hipStreamSynchronize(t->stream) != hipSuccess)
      e = set_error(AFH_ERR_DEVICE, "stream sync");
    d->group->bar.wait();
    for (int q = 0; q < d->n && !e; q++) {
      if (!p.recv_n[q]) continue;
      const afh_dist *peer = d->group->rank[q];
      const afh_dist::Plan &src = peer->plans.at(key);
      const int64_t n = src.send_n[d->rank];
      if (n != p.recv_n[q])
        e = set_error(AFH_ERR_STATE, "exchange %d/%d: rank %d sends %lld values, rank %d "
                      "expects %lld", std::get<0>(key), std::get<1>(key), q, (long long)n, d->rank,
                      (long long)p.recv_n[q]);
      else if (hipMemcpyPeerAsync(p.recv_buf + p.recv_off[q], d->device,
                                  src.send_buf + src.send_off[d->rank], peer->device,
                                  sizeof(double) * n, t->stream) != hipSuccess)
        e = set_error(AFH_ERR_DEVICE, "peer copy");
    }
    if (!e && hipStreamSynchronize(t->stream) != hipSuccess)
      e = set_error(AFH_ERR_DEVICE, "stream sync");
    d->group->bar.wait();
    if (e) return e;
  }
  if (p.recv_plan >= 0) e = afh_plan_unpack(t, p.recv_plan, iv, p.recv_buf);
  if (e) return e;
  if ((e = face_fill(t, p, iv))) return e;
  d->n_exchanges++;
  for (int q = 0; q < d->n; q++) {
    d->bytes += 8 * (p.send_n[q] + p.recv_n[q]);
    d->peer_sent[q] += 8 * p.send_n[q];
    d->peer_recv[q] += 8 * p.recv_n[q];
  }
  return AFH_OK;
}

int32_t reduce(afh_dist *d, int kind, double *vals, int n) {
  if (n > 16) return set_error(AFH_ERR_ARG, "reduction of %d values", n);
  if (d->transport == AFH_DIST_RCCL) {
    afh_tree *t = d->t;
    const ncclRedOp_t op = kind == AFH_HOOK_MAX ? ncclMax : kind == AFH_HOOK_MIN ? ncclMin : ncclSum;
    AFH_HIP(hipMemcpyAsync(d->d_red, vals, sizeof(double) * n, hipMemcpyHostToDevice, t->stream));
    if (ncclAllReduce(d->d_red, d->d_red, n, ncclDouble, op, d->comm, t->stream) != ncclSuccess)
      return set_error(AFH_ERR_DEVICE, "ncclAllReduce");
    AFH_HIP(hipMemcpyAsync(vals, d->d_red, sizeof(double) * n, hipMemcpyDeviceToHost, t->stream));
    AFH_HIP(hipStreamSynchronize(t->stream));
    return AFH_OK;
  }
  afh_dist_group *g = d->group;
  for (int k = 0; k < n; k++) g->vals[d->rank][k] = vals[k];
  g->bar.wait();
  for (int k = 0; k < n; k++) {
    double v = g->vals[0][k];  // rank order: the same result on every rank
    for (int q = 1; q < d->n; q++) {
      const double w = g->vals[q][k];
      v = kind == AFH_HOOK_MAX ? std::max(v, w) : kind == AFH_HOOK_MIN ? std::min(v, w) : v + w;
    }
    vals[k] = v;
  }
  g->bar.wait();
  return AFH_OK;
}

// RCCL: all-reduce n ordered keys (dbl_to_ord: max / min of the keys is that
// of the doubles) in place on the tree's stream
int32_t dist_dev_reduce(void *ctx, int kind, unsigned long long *keys, int n) {
  afh_dist *d = static_cast<afh_dist *>(ctx);
  if (ncclAllReduce(keys, keys, n, ncclUint64, kind == AFH_HOOK_MIN ? ncclMin : ncclMax,
                    d->comm, d->t->stream) != ncclSuccess)
    return set_error(AFH_ERR_DEVICE, "ncclAllReduce (device keys)");
  return AFH_OK;
}

// RCCL: the SUM of afh_tree_sum_cc, all-reduced in place on the device
int32_t dist_dev_sum(void *ctx, double *val) {
  afh_dist *d = static_cast<afh_dist *>(ctx);
  if (ncclAllReduce(val, val, 1, ncclDouble, ncclSum, d->comm, d->t->stream) != ncclSuccess)
    return set_error(AFH_ERR_DEVICE, "ncclAllReduce (device sum)");
  return AFH_OK;
}

int32_t dist_hook(void *ctx, int32_t kind, int32_t level, int32_t iv, double *vals, int32_t n) {
  afh_dist *d = static_cast<afh_dist *>(ctx);
  switch (kind) {
  case AFH_HOOK_MAX:
  case AFH_HOOK_MIN:
  case AFH_HOOK_SUM: return reduce(d, kind, vals, n);
  case AFH_HOOK_CFLUX: return exchange(d, Key(kind, 0, DEPTH), iv);
  case AFH_HOOK_HALO: return exchange(d, Key(kind, level, n == 1 ? 1 : DEPTH), iv);
  case AFH_HOOK_RIMS:
    return exchange(d, Key(kind, level, (n >= 1 && n <= 2) || (n >= 11 && n <= 12) ? n : 0), iv);
  default: return exchange(d, Key(kind, level, DEPTH), iv);
  }
}

}  // namespace

extern "C" {

int32_t afh_dist_partition(const afh_tree_desc *desc, int32_t n_ranks, int32_t *owner,
                           int32_t *lp) {
  return afh_dist_partition_levels(desc, n_ranks, 0, owner, lp);
}

int32_t afh_dist_partition_levels(const afh_tree_desc *desc, int32_t n_ranks,
                                  int64_t min_level_cells, int32_t *owner, int32_t *lp) {
  if (!desc || !owner || n_ranks < 1 || min_level_cells < 0)
    return set_error(AFH_ERR_ARG, "afh_dist_partition");
  const Topo t = topo_of(desc);
  std::vector<int32_t> own;
  const int l = partition(t, n_ranks, own, min_level_cells);
  if (l < 0)
    return set_error(AFH_ERR_ARG, "no level >= 2 has enough boxes to shard over %d ranks",
                     n_ranks);
  std::copy(own.begin(), own.end(), owner);
  if (lp) *lp = l;
  return AFH_OK;
}

int32_t afh_dist_plan(const afh_tree_desc *desc, const int32_t *owner, int32_t kind,
                      int32_t level, int32_t recv_rank, int32_t send_rank, int32_t *regions,
                      int32_t cap, int32_t *n) {
  if (!desc || !owner || !n) return set_error(AFH_ERR_ARG, "afh_dist_plan");
  const Topo t = topo_of(desc);
  const std::vector<int32_t> own(owner, owner + t.nb);
  const auto rs = plan_regions(t, own, first_owned_level(t, owner), kind, level, recv_rank,
                               send_rank);
  const int w = kind == AFH_HOOK_CFLUX ? 8 : 7;
  *n = (int32_t)rs.size();
  if (regions) {
    if ((int)rs.size() > cap) return set_error(AFH_ERR_ARG, "afh_dist_plan: %d regions > cap %d",
                                               (int)rs.size(), cap);
    for (size_t k = 0; k < rs.size(); k++)
      for (int c = 0; c < w; c++) regions[k * w + c] = rs[k][c];
  }
  return AFH_OK;
}

int32_t afh_dist_local_ids(const afh_tree_desc *desc, const int32_t *owner, int32_t rank,
                          int32_t *ids, int32_t cap, int32_t *n) {
  if (!desc || !owner || !n) return set_error(AFH_ERR_ARG, "afh_dist_local_ids");
  const Topo t = topo_of(desc);
  const auto v = local_boxes(t, std::vector<int32_t>(owner, owner + t.nb), rank);
  *n = (int32_t)v.size();
  if (ids) {
    if ((int)v.size() > cap)
      return set_error(AFH_ERR_ARG, "afh_dist_local_ids: %d boxes > cap %d", (int)v.size(), cap);
    std::copy(v.begin(), v.end(), ids);
  }
  return AFH_OK;
}

int32_t afh_tree_create_sharded(const afh_tree_desc *desc, const int32_t *owner, int32_t rank,
                                int32_t device, afh_tree **out) {
  if (!desc || !owner || !out) return set_error(AFH_ERR_ARG, "afh_tree_create_sharded");
  const Topo t = topo_of(desc);
  Compact c;
  compact(t, desc, std::vector<int32_t>(owner, owner + t.nb), rank, c);
  int32_t e = afh_tree_create(&c.desc, device, out);
  if (e) return e;
  // the choices every rank must make alike (which exchanges a ghost-cell
  // fill requests, the smoother per level) follow the whole topology, as in
  // an unsharded tree, not this rank's boxes
  afh_tree *tr = *out;
  // the unused id reads as NaN in every variable: a kernel that reaches a
  // box the rank does not store fails the parity tests loudly
  for (int iv = 1; iv <= tr->nvc; iv++)
    AFH_HIP(hipMemsetAsync(tr->ccv(iv) + (size_t)(tr->nb - 1) * tr->bsz, 0xff,
                           sizeof(double) * tr->bsz, tr->stream));
  for (int iv = 1; iv <= tr->nvf; iv++)
    AFH_HIP(hipMemsetAsync(tr->fcv(iv) + (size_t)(tr->nb - 1) * tr->fsz, 0xff,
                           sizeof(double) * tr->fsz, tr->stream));
  AFH_HIP(hipStreamSynchronize(tr->stream));
  // a replicated leaf (levels below the partition level) is summed by rank 0
  // only, so the SUM all-reduce counts it once
  tr->sum_skip.assign(tr->nb, 0);
  if (rank != 0)
    for (size_t k = 0; k < c.ids.size(); k++) tr->sum_skip[k] = owner[c.ids[k] - 1] < 0;
  tr->lvl_total.assign(t.nlvl, 0);
  tr->lvl_leaves_total.assign(t.nlvl, 0);
  tr->lvl_rb_coarse.assign(t.nlvl, 0);
  tr->any_cflux = false;
  for (int id = 1; id <= t.nb; id++) {
    const afh_box_meta &m = t.m[id - 1];
    if (m.lvl < 1) continue;
    tr->lvl_total[m.lvl - 1]++;
    if (m.children[0] == 0) tr->lvl_leaves_total[m.lvl - 1]++;
    for (int q = 0; q < 6; q++) {
      if (m.lvl >= 2 && m.neighbors[q] == 0) tr->lvl_rb_coarse[m.lvl - 2] = 1;
      if (m.children[0] && m.neighbors[q] > 0 && t.m[m.neighbors[q] - 1].children[0] == 0)
        tr->any_cflux = true;
    }
  }
  return AFH_OK;
}

int32_t afh_dist_group_create(int32_t n_ranks, afh_dist_group **out) {
  if (n_ranks < 1 || !out) return set_error(AFH_ERR_ARG, "afh_dist_group_create");
  *out = new afh_dist_group(n_ranks);
  return AFH_OK;
}

int32_t afh_dist_group_destroy(afh_dist_group *g) {
  delete g;
  return AFH_OK;
}

int32_t afh_dist_rccl_unique_id(void *id) {
  if (!id) return set_error(AFH_ERR_ARG, "null id");
  ncclUniqueId u;
  if (ncclGetUniqueId(&u) != ncclSuccess) return set_error(AFH_ERR_DEVICE, "ncclGetUniqueId");
  memcpy(id, &u, sizeof(u));
  return AFH_OK;
}

int32_t afh_dist_rccl_comm(const void *id, int32_t rank, int32_t n_ranks, int32_t device,
                           void **comm) {
  if (!id || !comm) return set_error(AFH_ERR_ARG, "afh_dist_rccl_comm");
  AFH_HIP(hipSetDevice(device));
  ncclUniqueId u;
  memcpy(&u, id, sizeof(u));
  ncclComm_t c;
  if (ncclCommInitRank(&c, n_ranks, u, rank) != ncclSuccess)
    return set_error(AFH_ERR_DEVICE, "ncclCommInitRank");
  *comm = c;
  return AFH_OK;
}

int32_t afh_dist_rccl_comm_destroy(void *comm) {
  if (comm) ncclCommDestroy(static_cast<ncclComm_t>(comm));
  return AFH_OK;
}

int32_t afh_dist_create(afh_tree *t, const afh_tree_desc *desc, const int32_t *owner,
                        int32_t rank, int32_t n_ranks, int32_t transport, void *group_or_comm,
                        afh_dist **out) {
  if (!t || !desc || !owner || !out || rank < 0 || rank >= n_ranks || !group_or_comm)
    return set_error(AFH_ERR_ARG, "afh_dist_create");
  AFH_LIVE(t, "afh_dist_create");
  if (transport != AFH_DIST_LOCAL && transport != AFH_DIST_RCCL)
    return set_error(AFH_ERR_UNSUPPORTED, "transport %d", transport);
  const Topo tp = topo_of(desc);
  const std::vector<int32_t> own(owner, owner + tp.nb);
  const int lp = first_owned_level(tp, owner);
  // region box ids -> the rank's compacted ids (afh_tree_create_sharded)
  const auto local = local_boxes(tp, own, rank);
  if ((int)local.size() + 1 != t->nb || tp.nc != t->nc)
    return set_error(AFH_ERR_ARG, "afh_dist_create: the tree is not rank %d's part of this "
                     "topology (afh_tree_create_sharded)", rank);
  std::vector<int32_t> g2l(tp.nb + 1, 0);
  for (size_t k = 0; k < local.size(); k++) g2l[local[k]] = (int32_t)k + 1;
  afh_dist *d = new afh_dist;
  d->t = t, d->rank = rank, d->n = n_ranks, d->transport = transport;
  d->peer_sent.assign(n_ranks, 0), d->peer_recv.assign(n_ranks, 0);
  hipGetDevice(&d->device);
  if (transport == AFH_DIST_LOCAL) {
    d->group = static_cast<afh_dist_group *>(group_or_comm);
    if (d->group->n != n_ranks) {
      delete d;
      return set_error(AFH_ERR_ARG, "group of %d ranks, n_ranks %d", d->group->n, n_ranks);
    }
  } else {
    d->comm = static_cast<ncclComm_t>(group_or_comm);
  }
  auto add = [&](int kind, int level, int depth = DEPTH) -> int32_t {
    afh_dist::Plan p;
    p.send_off.assign(n_ranks, 0), p.send_n.assign(n_ranks, 0);
    p.recv_off.assign(n_ranks, 0), p.recv_n.assign(n_ranks, 0);
    const bool fc = kind == AFH_HOOK_CFLUX;
    const int w = fc ? 8 : 7, lo = fc ? 2 : 1;
    std::set<int32_t> fc_boxes;
    const bool pair = kind == AFH_HOOK_RIMS && depth > 10;
    std::map<int, std::vector<char>> stored;
    auto stored_of = [&](int r) -> const std::vector<char> & {
      auto it = stored.find(r);
      if (it == stored.end())
        it = stored.emplace(r, level_stored(tp, own, lp, r, n_ranks, level)).first;
      return it->second;
    };
    for (int side = 0; side < 2; side++) {
      // the regions of every peer, peer after peer, in one plan
      std::vector<int32_t> flat;
      int64_t total = 0;
      std::vector<int64_t> &off = side == 0 ? p.send_off : p.recv_off;
      std::vector<int64_t> &cnt = side == 0 ? p.send_n : p.recv_n;
      for (int q = 0; q < n_ranks; q++) {
        off[q] = total;
        if (q == rank) continue;
        const int dep = depth > 10 ? depth - 10 : depth > 0 ? depth : DEPTH;
        const bool lf = kind == AFH_HOOK_RIMS && depth > 0 && depth < 10;
        // (pair mode, layers 11 / 12: the sender's regions follow the
        // receiver's stored boxes)
        const std::vector<char> *pm = nullptr;
        if (pair) pm = side == 0 ? &stored_of(q) : &stored_of(rank);
        const auto rs = side == 0 ? plan_regions(tp, own, lp, kind, level, q, rank, dep, lf, pm)
                                  : plan_regions(tp, own, lp, kind, level, rank, q, dep, lf, pm);
        // the faces this rank fills itself: of the boxes whose ghost cells
        // it receives, the faces next to a box it computes (local faces), or
        // next to a stored box or the domain boundary (pair mode)
        if (lf && side == 1)
          for (const Region &r : rs) fc_boxes.insert(r[0]);
        if (pair && side == 1)
          for (const Region &r : halo_regions(tp, own, lp, rank, q, level, true, dep))
            fc_boxes.insert(r[0]);
        for (const Region &r : rs) {
          flat.insert(flat.end(), r.begin(), r.begin() + w);
          flat[flat.size() - w] = g2l[r[0]];
          int64_t cells = 1;
          for (int dd = 0; dd < 3; dd++) cells *= r[lo + 3 + dd] - r[lo + dd] + 1;
          cnt[q] += cells;
        }
        total += cnt[q];
      }
      if (flat.empty()) continue;
      int32_t &plan = side == 0 ? p.send_plan : p.recv_plan;
      double *&buf = side == 0 ? p.send_buf : p.recv_buf;
      int64_t n = 0;
      const int32_t nr = (int32_t)(flat.size() / w);
      int32_t e = fc ? afh_plan_create_fc(t, flat.data(), nr, &plan, &n)
                     : afh_plan_create(t, flat.data(), nr, &plan, &n);
      if (e) return e;
      if (n != total) return set_error(AFH_ERR_STATE, "exchange plan: %lld != %lld values",
                                       (long long)n, (long long)total);
      if (n && hipMalloc(&buf, sizeof(double) * n) != hipSuccess)
        return set_error(AFH_ERR_DEVICE, "exchange buffer");
    }
    std::vector<int32_t> fcl;
    for (int32_t b : fc_boxes)
      for (int f = 0; f < 6; f++) {
        const int nb = tp.m[b - 1].neighbors[f];
        const bool fill = pair ? (nb < 0 || (nb > 0 && stored_of(rank)[nb]))
                               : (nb > 0 && (own[nb - 1] == rank || own[nb - 1] < 0));
        if (fill) fcl.push_back(g2l[b]), fcl.push_back(f + 1);
      }
    if (pair) {
      // nothing to send between any two ranks: every rank only fills
      bool any = false;
      for (int r = 0; r < n_ranks && !any; r++)
        for (int q = 0; q < n_ranks && !any; q++)
          if (q != r)
            any = !halo_regions(tp, own, lp, r, q, level, true, depth - 10, false, &stored_of(r))
                       .empty();
      p.local_only = !any;
    }
    if (!fcl.empty()) {
      if (hipMalloc(&p.d_fc, sizeof(int32_t) * fcl.size()) != hipSuccess ||
          hipMemcpy(p.d_fc, fcl.data(), sizeof(int32_t) * fcl.size(), hipMemcpyHostToDevice) !=
              hipSuccess)
        return set_error(AFH_ERR_DEVICE, "face copy list");
      p.n_fc = (int32_t)(fcl.size() / 2);
    }
    d->plans[Key(kind, level, depth)] = std::move(p);
    return AFH_OK;
  };
  int32_t e = AFH_OK;
  if (lp) {
    for (int l = lp; l <= tp.nlvl && !e; l++)
      for (int depth = 0; depth <= DEPTH && !e; depth++) {
        if (!(e = depth ? add(AFH_HOOK_HALO, l, depth) : AFH_OK)) e = add(AFH_HOOK_RIMS, l, depth);
        if (!e && depth) e = add(AFH_HOOK_RIMS, l, 10 + depth);
      }
    if (!e) e = add(AFH_HOOK_CFLUX, 0);
    for (int l : restrict_levels(tp, own, lp))
      if (!e) e = add(AFH_HOOK_RESTRICT, l);
  }
  if (!e && transport == AFH_DIST_RCCL && hipMalloc(&d->d_red, 16 * sizeof(double)) != hipSuccess)
    e = set_error(AFH_ERR_DEVICE, "reduction buffer");
  if (!e) e = afh_tree_set_hook(t, dist_hook, d);
  if (!e && transport == AFH_DIST_RCCL) {
    t->dev_reduce = dist_dev_reduce;
    t->dev_sum = dist_dev_sum;
    t->hook_capturable = true;  // exchanges are stream operations
  }
  if (e) {
    afh_dist_destroy(d);
    return e;
  }
  if (transport == AFH_DIST_LOCAL) d->group->rank[rank] = d;
  *out = d;
  return AFH_OK;
}

int32_t afh_dist_destroy(afh_dist *d) {
  if (!d) return AFH_OK;
  if (d->t && !d->t->retired && d->t->hook_ctx == d) {
    afh_tree_set_hook(d->t, nullptr, nullptr);
    d->t->dev_reduce = nullptr;
    d->t->dev_sum = nullptr;
    d->t->hook_capturable = false;
  }
  if (d->t) hipStreamSynchronize(d->t->stream);
  for (auto &kv : d->plans) {
    hipFree(kv.second.send_buf);
    hipFree(kv.second.recv_buf);
    hipFree(kv.second.d_fc);
  }
  hipFree(d->d_red);
  if (d->group && d->group->rank[d->rank] == d) d->group->rank[d->rank] = nullptr;
  delete d;
  return AFH_OK;
}

int32_t afh_dist_stats(afh_dist *d, int64_t *n_exchanges, int64_t *bytes) {
  if (!d) return set_error(AFH_ERR_ARG, "null dist");
  if (n_exchanges) *n_exchanges = d->n_exchanges;
  if (bytes) *bytes = d->bytes;
  return AFH_OK;
}

int32_t afh_dist_peer_bytes(afh_dist *d, int64_t *sent, int64_t *received) {
  if (!d) return set_error(AFH_ERR_ARG, "null dist");
  for (int q = 0; q < d->n; q++) {
    if (sent) sent[q] = d->peer_sent[q];
    if (received) received[q] = d->peer_recv[q];
  }
  return AFH_OK;
}

}  // extern "C"
