// ORACLE TEST INFRASTRUCTURE -- not product code.
//
// The CPU twin of libafivo_hip's native box sharding (afivo-streamer_amd/csrc/
// afh_dist.hip): the same partition and exchange plans (the shared host code
// in afh_dist_core.h), the same hook, on host buffers. AFH_DIST_LOCAL only:
// the ranks are threads of one process, each with its own oracle tree; an
// exchange packs, waits for the group, copies the peers' packed buffers and
// unpacks. AFH_DIST_RCCL has no CPU meaning and is refused.
//
// tests/test_dist_native.py runs the sharded oracle (threads) against the
// single-rank oracle, bitwise, and the HIP library against both.
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <map>
#include <utility>
#include <vector>

#include "afo.h"
#include "../../afivo-streamer_amd/csrc/afh_dist_core.h"

extern "C" int32_t afo_fail_msg(int32_t code, const char *msg);
extern "C" void afo_poison_box(afh_tree *t, int id);
extern "C" void afo_set_sum_skip(afh_tree *t, const unsigned char *skip);

using namespace afhd;

namespace {
int32_t fail(int32_t code, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  return afo_fail_msg(code, buf);
}
}  // namespace

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
  int rank = 0, n = 1;
  afh_dist_group *group = nullptr;
  struct Side {
    int32_t plan = -1;
    int64_t n = 0;
    std::vector<double> buf;
  };
  struct Plan {
    std::vector<Side> send, recv;
  };
  std::map<std::pair<int, int>, Plan> plans;
  int64_t n_exchanges = 0, bytes = 0;
  std::vector<int64_t> peer_sent, peer_recv;
};

namespace {

using Key = std::pair<int, int>;

int32_t exchange(afh_dist *d, const Key &key, int iv) {
  auto it = d->plans.find(key);
  if (it == d->plans.end()) return AFH_OK;
  afh_dist::Plan &p = it->second;
  int32_t e = AFH_OK;
  for (int q = 0; q < d->n && !e; q++)
    if (p.send[q].n) e = afo_plan_pack(d->t, p.send[q].plan, iv, p.send[q].buf.data());
  // the barriers are passed on every path, so a failing rank cannot strand
  // its peers
  d->group->bar.wait();
  for (int q = 0; q < d->n && !e; q++) {
    if (!p.recv[q].n) continue;
    const afh_dist::Side &src = d->group->rank[q]->plans.at(key).send[d->rank];
    if (src.n != p.recv[q].n)
      e = fail(AFH_ERR_STATE, "exchange %d/%d: rank %d sends %lld values, rank %d expects %lld",
               key.first, key.second, q, (long long)src.n, d->rank, (long long)p.recv[q].n);
    else
      memcpy(p.recv[q].buf.data(), src.buf.data(), sizeof(double) * src.n);
  }
  d->group->bar.wait();
  for (int q = 0; q < d->n && !e; q++)
    if (p.recv[q].n) e = afo_plan_unpack(d->t, p.recv[q].plan, iv, p.recv[q].buf.data());
  if (e) return e;
  d->n_exchanges++;
  if ((int)d->peer_sent.size() != d->n) d->peer_sent.assign(d->n, 0), d->peer_recv.assign(d->n, 0);
  for (int q = 0; q < d->n; q++) {
    d->bytes += 8 * (p.send[q].n + p.recv[q].n);
    d->peer_sent[q] += 8 * p.send[q].n;
    d->peer_recv[q] += 8 * p.recv[q].n;
  }
  return AFH_OK;
}

int32_t reduce(afh_dist *d, int kind, double *vals, int n) {
  if (n > 16) return fail(AFH_ERR_ARG, "reduction of %d values", n);
  afh_dist_group *g = d->group;
  for (int k = 0; k < n; k++) g->vals[d->rank][k] = vals[k];
  g->bar.wait();
  for (int k = 0; k < n; k++) {
    double v = g->vals[0][k];
    for (int q = 1; q < d->n; q++) {
      const double w = g->vals[q][k];
      v = kind == AFH_HOOK_MAX ? std::max(v, w) : kind == AFH_HOOK_MIN ? std::min(v, w) : v + w;
    }
    vals[k] = v;
  }
  g->bar.wait();
  return AFH_OK;
}

int32_t dist_hook(void *ctx, int32_t kind, int32_t level, int32_t iv, double *vals, int32_t n) {
  afh_dist *d = static_cast<afh_dist *>(ctx);
  switch (kind) {
  case AFH_HOOK_MAX:
  case AFH_HOOK_MIN:
  case AFH_HOOK_SUM: return reduce(d, kind, vals, n);
  case AFH_HOOK_CFLUX: return exchange(d, Key(kind, 0), iv);
  default: return exchange(d, Key(kind, level), iv);
  }
}

}  // namespace

extern "C" {

int32_t afo_dist_partition_levels(const afh_tree_desc *desc, int32_t n_ranks,
                                  int64_t min_level_cells, int32_t *owner, int32_t *lp) {
  if (!desc || !owner || n_ranks < 1 || min_level_cells < 0)
    return fail(AFH_ERR_ARG, "afo_dist_partition");
  const Topo t = topo_of(desc);
  std::vector<int32_t> own;
  const int l = partition(t, n_ranks, own, min_level_cells);
  if (l < 0)
    return fail(AFH_ERR_ARG, "no level >= 2 has enough boxes to shard over %d ranks", n_ranks);
  std::copy(own.begin(), own.end(), owner);
  if (lp) *lp = l;
  return AFH_OK;
}

int32_t afo_dist_partition(const afh_tree_desc *desc, int32_t n_ranks, int32_t *owner,
                           int32_t *lp) {
  return afo_dist_partition_levels(desc, n_ranks, 0, owner, lp);
}

int32_t afo_dist_plan(const afh_tree_desc *desc, const int32_t *owner, int32_t kind,
                      int32_t level, int32_t recv_rank, int32_t send_rank, int32_t *regions,
                      int32_t cap, int32_t *n) {
  if (!desc || !owner || !n) return fail(AFH_ERR_ARG, "afo_dist_plan");
  const Topo t = topo_of(desc);
  const std::vector<int32_t> own(owner, owner + t.nb);
  const auto rs = plan_regions(t, own, first_owned_level(t, owner), kind, level, recv_rank,
                               send_rank);
  const int w = kind == AFH_HOOK_CFLUX ? 8 : 7;
  *n = (int32_t)rs.size();
  if (regions) {
    if ((int)rs.size() > cap)
      return fail(AFH_ERR_ARG, "afo_dist_plan: %d regions > cap %d", (int)rs.size(), cap);
    for (size_t k = 0; k < rs.size(); k++)
      for (int c = 0; c < w; c++) regions[k * w + c] = rs[k][c];
  }
  return AFH_OK;
}

int32_t afo_dist_local_ids(const afh_tree_desc *desc, const int32_t *owner, int32_t rank,
                          int32_t *ids, int32_t cap, int32_t *n) {
  if (!desc || !owner || !n) return fail(AFH_ERR_ARG, "afo_dist_local_ids");
  const Topo t = topo_of(desc);
  const auto v = local_boxes(t, std::vector<int32_t>(owner, owner + t.nb), rank);
  *n = (int32_t)v.size();
  if (ids) {
    if ((int)v.size() > cap)
      return fail(AFH_ERR_ARG, "afo_dist_local_ids: %d boxes > cap %d", (int)v.size(), cap);
    std::copy(v.begin(), v.end(), ids);
  }
  return AFH_OK;
}

int32_t afo_tree_create_sharded(const afh_tree_desc *desc, const int32_t *owner, int32_t rank,
                                int32_t device, afh_tree **out) {
  if (!desc || !owner || !out) return fail(AFH_ERR_ARG, "afo_tree_create_sharded");
  const Topo t = topo_of(desc);
  Compact c;
  compact(t, desc, std::vector<int32_t>(owner, owner + t.nb), rank, c);
  const int32_t e = afo_tree_create(&c.desc, device, out);
  if (e) return e;
  afo_poison_box(*out, c.desc.n_boxes);
  // a replicated leaf is summed by rank 0 only (the SUM reduction counts it once)
  std::vector<unsigned char> skip(c.desc.n_boxes, 0);
  if (rank != 0)
    for (size_t k = 0; k < c.ids.size(); k++) skip[k] = owner[c.ids[k] - 1] < 0;
  afo_set_sum_skip(*out, skip.data());
  return AFH_OK;
}

int32_t afo_dist_group_create(int32_t n_ranks, afh_dist_group **out) {
  if (n_ranks < 1 || !out) return fail(AFH_ERR_ARG, "afo_dist_group_create");
  *out = new afh_dist_group(n_ranks);
  return AFH_OK;
}

int32_t afo_dist_group_destroy(afh_dist_group *g) {
  delete g;
  return AFH_OK;
}

int32_t afo_dist_rccl_unique_id(void *) {
  return fail(AFH_ERR_UNSUPPORTED, "the CPU oracle has no RCCL transport");
}

int32_t afo_dist_rccl_comm(const void *, int32_t, int32_t, int32_t, void **) {
  return fail(AFH_ERR_UNSUPPORTED, "the CPU oracle has no RCCL transport");
}

int32_t afo_dist_rccl_comm_destroy(void *) { return AFH_OK; }

int32_t afo_dist_create(afh_tree *t, const afh_tree_desc *desc, const int32_t *owner,
                        int32_t rank, int32_t n_ranks, int32_t transport, void *group_or_comm,
                        afh_dist **out) {
  if (!t || !desc || !owner || !out || rank < 0 || rank >= n_ranks || !group_or_comm)
    return fail(AFH_ERR_ARG, "afo_dist_create");
  if (transport != AFH_DIST_LOCAL)
    return fail(AFH_ERR_UNSUPPORTED, "the CPU oracle shards over AFH_DIST_LOCAL only");
  afh_dist_group *g = static_cast<afh_dist_group *>(group_or_comm);
  if (g->n != n_ranks) return fail(AFH_ERR_ARG, "group of %d ranks, n_ranks %d", g->n, n_ranks);
  const Topo tp = topo_of(desc);
  const std::vector<int32_t> own(owner, owner + tp.nb);
  const int lp = first_owned_level(tp, owner);
  const auto local = local_boxes(tp, own, rank);
  std::vector<int32_t> g2l(tp.nb + 1, 0);
  for (size_t k = 0; k < local.size(); k++) g2l[local[k]] = (int32_t)k + 1;
  afh_dist *d = new afh_dist;
  d->t = t, d->rank = rank, d->n = n_ranks, d->group = g;
  auto add = [&](int kind, int level) -> int32_t {
    afh_dist::Plan p;
    p.send.resize(n_ranks), p.recv.resize(n_ranks);
    const bool fc = kind == AFH_HOOK_CFLUX;
    for (int q = 0; q < n_ranks; q++) {
      if (q == rank) continue;
      for (int side = 0; side < 2; side++) {
        const auto rs = side == 0 ? plan_regions(tp, own, lp, kind, level, q, rank)
                                  : plan_regions(tp, own, lp, kind, level, rank, q);
        afh_dist::Side &sd = side == 0 ? p.send[q] : p.recv[q];
        if (rs.empty()) continue;
        std::vector<int32_t> flat;
        for (const Region &r : rs) {
          flat.insert(flat.end(), r.begin(), r.begin() + (fc ? 8 : 7));
          flat[flat.size() - (fc ? 8 : 7)] = g2l[r[0]];
        }
        const int32_t e = fc ? afo_plan_create_fc(t, flat.data(), (int32_t)rs.size(), &sd.plan, &sd.n)
                             : afo_plan_create(t, flat.data(), (int32_t)rs.size(), &sd.plan, &sd.n);
        if (e) return e;
        sd.buf.resize(sd.n);
      }
    }
    d->plans[Key(kind, level)] = std::move(p);
    return AFH_OK;
  };
  int32_t e = AFH_OK;
  if (lp) {
    for (int l = lp; l <= tp.nlvl && !e; l++)
      if (!(e = add(AFH_HOOK_HALO, l))) e = add(AFH_HOOK_RIMS, l);
    if (!e) e = add(AFH_HOOK_CFLUX, 0);
    for (int l : restrict_levels(tp, own, lp))
      if (!e) e = add(AFH_HOOK_RESTRICT, l);
  }
  if (!e) e = afo_tree_set_hook(t, dist_hook, d);
  if (e) {
    delete d;
    return e;
  }
  g->rank[rank] = d;
  *out = d;
  return AFH_OK;
}

int32_t afo_dist_destroy(afh_dist *d) {
  if (!d) return AFH_OK;
  afo_tree_set_hook(d->t, nullptr, nullptr);
  if (d->group && d->group->rank[d->rank] == d) d->group->rank[d->rank] = nullptr;
  delete d;
  return AFH_OK;
}

int32_t afo_dist_stats(afh_dist *d, int64_t *n_exchanges, int64_t *bytes) {
  if (!d) return fail(AFH_ERR_ARG, "null dist");
  if (n_exchanges) *n_exchanges = d->n_exchanges;
  if (bytes) *bytes = d->bytes;
  return AFH_OK;
}

int32_t afo_dist_peer_bytes(afh_dist *d, int64_t *sent, int64_t *received) {
  if (!d) return fail(AFH_ERR_ARG, "null dist");
  for (int q = 0; q < d->n; q++) {
    const bool any = (int)d->peer_sent.size() == d->n;
    if (sent) sent[q] = any ? d->peer_sent[q] : 0;
    if (received) received[q] = any ? d->peer_recv[q] : 0;
  }
  return AFH_OK;
}

}  // extern "C"
