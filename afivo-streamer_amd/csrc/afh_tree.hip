// Box pool, topology upload, ghost cells, restriction, reductions.
//
// Ghost-cell kernels restate afivo/src/m_af_ghostcell.f90 (af_gc_box 64-120,
// copy_from_nb 654-669, bc_to_gc 173-279, af_gc_interp 394-498,
// af_gc_interp_lim 503-612, corners/edges 125-170 + 860-924) and
// mg_sides_rb (afivo/src/m_af_multigrid.f90:294-461). One level is filled by
// two launches: all faces of all boxes (one thread per ghost cell), then
// edges and corners (one workgroup per box), because edge extrapolation reads
// face ghosts and corner extrapolation reads edge ghosts.
#include <stdarg.h>
#include <stdio.h>

#include <float.h>
#include <math.h>

#include <algorithm>
#include <cmath>

#include "afh_internal.h"

namespace afh {

static thread_local char g_err[512];

int32_t set_error(int32_t code, const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof g_err, fmt, ap);
  va_end(ap);
  return code;
}

int32_t check_hip(hipError_t e, const char *what) {
  return set_error(AFH_ERR_DEVICE, "%s: %s", what, hipGetErrorString(e));
}

int32_t pool_alloc(void **p, size_t bytes, const char *what) {
  (void)what;
  *p = nullptr;
  AFH_HIP(hipMalloc(p, bytes));
  return AFH_OK;
}

static hipEvent_t next_event(afh_tree *t) {
  if (t->ev_used == t->ev_pool.size()) {
    hipEvent_t e;
    hipEventCreate(&e);
    t->ev_pool.push_back(e);
  }
  return t->ev_pool[t->ev_used++];
}

void prof_begin(afh_tree *t, int kc) {
  if (t->prof_class != kc) return;
  hipEventRecord(next_event(t), t->stream);
}

bool prof_ext(afh_tree *t, int kc, hipEvent_t &e0, hipEvent_t &e1) {
  if (t->prof_class != kc) return false;
  e0 = next_event(t);
  e1 = next_event(t);
  return true;
}

void prof_count(afh_tree *t, double bytes) {
  t->prof_bytes += bytes;
  t->prof_launches++;
}

void prof_end(afh_tree *t, int kc, double bytes) {
  if (t->prof_class != kc) return;
  hipEventRecord(next_event(t), t->stream);
  t->prof_bytes += bytes;
  t->prof_launches++;
}

// ------------------------------------------------------------ faces
// One thread per ghost cell of face (blockIdx.y+1) of box ids[blockIdx.z].
// Coarse data (refinement boundaries) are read from vc.
__global__ void k_gc_faces(double *__restrict__ v,
                           const double *__restrict__ vc,
                           const afh_box_meta *__restrict__ meta,
                           const int32_t *__restrict__ ids, int nc, size_t bsz,
                           GcArgs ga) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nc * nc) return;
  const int id = ids[blockIdx.z];
  const int nb = blockIdx.y + 1;
  const int d = (nb - 1) >> 1;
  const bool low = ((nb - 1) & 1) == 0;
  const int ta = (d == 0) ? 1 : 0, tb = (d == 2) ? 1 : 2;
  int a, b;
  if ((nc & (nc - 1)) == 0) {
    a = (t & (nc - 1)) + 1;
    b = (t >> __builtin_ctz(nc)) + 1;
  } else {
    a = t % nc + 1;
    b = t / nc + 1;
  }
  const int ng = nc + 2;
  const afh_box_meta &m = meta[id - 1];
  double *c = v + (size_t)(id - 1) * bsz;
  const int nb_id = m.neighbors[nb - 1];
  int p[3];
  p[ta] = a;
  p[tb] = b;
  p[d] = low ? 0 : nc + 1;
  const size_t dst = ix3(ng, p[0], p[1], p[2]);

  if (nb_id > 0) {
    // copy_from_nb: ghost(lo) = neighbor(lo - dnb * nc)
    int q[3] = {p[0], p[1], p[2]};
    q[d] = low ? nc : 1;
    c[dst] = v[(size_t)(nb_id - 1) * bsz + ix3(ng, q[0], q[1], q[2])];
    return;
  }
  c[dst] = gc_face_nocopy(vc, meta, m, nb, p, a, b, nc, bsz, ga.bc[nb - 1], ga.rb,
                          [&](const int *q) {
                            return c[ix3(ng, q[0], q[1], q[2])];
                          });
}


// ------------------------------------------------------------ edges+corners
__constant__ int c_edge_dim[12] = {0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2};
__constant__ int c_edge_dir[12][3] = {
    {0, -1, -1}, {0, 1, -1}, {0, -1, 1}, {0, 1, 1}, {-1, 0, -1}, {1, 0, -1},
    {-1, 0, 1},  {1, 0, 1},  {-1, -1, 0}, {1, -1, 0}, {-1, 1, 0}, {1, 1, 0}};
__constant__ int c_edge_min[12][3] = {
    {0, 0, 0}, {0, 1, 0}, {0, 0, 1}, {0, 1, 1}, {0, 0, 0}, {1, 0, 0},
    {0, 0, 1}, {1, 0, 1}, {0, 0, 0}, {1, 0, 0}, {0, 1, 0}, {1, 1, 0}};
__constant__ int c_child_dix[8][3] = {{0, 0, 0}, {1, 0, 0}, {0, 1, 0},
                                      {1, 1, 0}, {0, 0, 1}, {1, 0, 1},
                                      {0, 1, 1}, {1, 1, 1}};

__global__ void k_gc_corners(double *__restrict__ v,
                             const afh_box_meta *__restrict__ meta,
                             const int32_t *__restrict__ ids, int nc,
                             size_t bsz) {
  const int id = ids[blockIdx.x];
  const int ng = nc + 2;
  const afh_box_meta &m = meta[id - 1];
  double *c = v + (size_t)(id - 1) * bsz;
  // edges (af_gc_box_corner, first loop)
  for (int e = threadIdx.x; e < 12 * nc; e += blockDim.x) {
    const int n = e / nc, pos = e % nc + 1;
    const int dim = c_edge_dim[n];
    const int dx = c_edge_dir[n][0], dy = c_edge_dir[n][1], dz = c_edge_dir[n][2];
    const int nb_id = m.neighbor_mat[(dx + 1) + 3 * (dy + 1) + 9 * (dz + 1)];
    int x[3];
    for (int q = 0; q < 3; q++) x[q] = c_edge_min[n][q] * (nc + 1);
    x[dim] = pos;
    if (nb_id > 0) {
      // dnb = offsets of the two adjacent neighbours = edge direction
      int s[3] = {x[0] - dx * nc, x[1] - dy * nc, x[2] - dz * nc};
      c[ix3(ng, x[0], x[1], x[2])] =
          v[(size_t)(nb_id - 1) * bsz + ix3(ng, s[0], s[1], s[2])];
    } else {
      // af_edge_gc_extrap
      const int o1 = (dim + 1) % 3, o2 = (dim + 2) % 3;
      int di[3];
      for (int q = 0; q < 3; q++) di[q] = 1 - 2 * (x[q] & 1);
      di[dim] = 0;
      int ia[3] = {x[0], x[1], x[2]}, ib[3] = {x[0], x[1], x[2]};
      ia[o1] += di[o1];
      ib[o2] += di[o2];
      int ic[3] = {x[0] + di[0], x[1] + di[1], x[2] + di[2]};
      c[ix3(ng, x[0], x[1], x[2])] = c[ix3(ng, ia[0], ia[1], ia[2])] +
                                     c[ix3(ng, ib[0], ib[1], ib[2])] -
                                     c[ix3(ng, ic[0], ic[1], ic[2])];
    }
  }
  __syncthreads();
  if (threadIdx.x < 8) {
    const int n = threadIdx.x;
    int dnb[3], x[3];
    for (int q = 0; q < 3; q++) {
      dnb[q] = 2 * c_child_dix[n][q] - 1;
      x[q] = c_child_dix[n][q] * (nc + 1);
    }
    const int nb_id =
        m.neighbor_mat[(dnb[0] + 1) + 3 * (dnb[1] + 1) + 9 * (dnb[2] + 1)];
    if (nb_id > 0) {
      c[ix3(ng, x[0], x[1], x[2])] =
          v[(size_t)(nb_id - 1) * bsz +
            ix3(ng, x[0] - dnb[0] * nc, x[1] - dnb[1] * nc, x[2] - dnb[2] * nc)];
    } else {
      int di[3];
      for (int q = 0; q < 3; q++) di[q] = 1 - 2 * (x[q] & 1);
      c[ix3(ng, x[0], x[1], x[2])] =
          c[ix3(ng, x[0], x[1] + di[1], x[2] + di[2])] +
          c[ix3(ng, x[0] + di[0], x[1], x[2] + di[2])] +
          c[ix3(ng, x[0] + di[0], x[1] + di[1], x[2])] -
          2 * c[ix3(ng, x[0] + di[0], x[1] + di[1], x[2] + di[2])];
    }
  }
}

// A small box's whole fill in one workgroup (NC <= 16: NC^2 threads, one
// per (a, b)): the six faces as k_gc_faces6, then -- with corners -- the
// edges and corners as k_gc_corners, behind workgroup barriers (edge
// extrapolation reads this box's face ghosts, corner extrapolation its edge
// ghosts). One launch per level fill instead of two; the same values.
template <int NC>
__global__ void __launch_bounds__(NC * NC)
    k_gc_box(double *__restrict__ v, const double *__restrict__ vc,
             const afh_box_meta *__restrict__ meta, const int32_t *__restrict__ ids,
             size_t bsz, GcArgs ga, int corners) {
  constexpr int NG = NC + 2;
  const int t = threadIdx.x;
  const int id = ids[blockIdx.x];
  const int a = t % NC + 1, b = t / NC + 1;
  const afh_box_meta &m = meta[id - 1];
  double *c = v + (size_t)(id - 1) * bsz;
  {
    double val[6];
    int dst[6];
#pragma unroll
    for (int nb = 1; nb <= 6; nb++) {
      const int d = (nb - 1) >> 1;
      const bool low = ((nb - 1) & 1) == 0;
      const int ta = (d == 0) ? 1 : 0, tb = (d == 2) ? 1 : 2;
      int p[3];
      p[ta] = a;
      p[tb] = b;
      p[d] = low ? 0 : NC + 1;
      dst[nb - 1] = ix3(NG, p[0], p[1], p[2]);
      const int nb_id = m.neighbors[nb - 1];
      if (nb_id > 0) {
        int q[3] = {p[0], p[1], p[2]};
        q[d] = low ? NC : 1;
        val[nb - 1] = v[(size_t)(nb_id - 1) * bsz + ix3(NG, q[0], q[1], q[2])];
      } else {
        val[nb - 1] = gc_face_nocopy(vc, meta, m, nb, p, a, b, NC, bsz, ga.bc[nb - 1], ga.rb,
                                     [&](const int *q) { return c[ix3(NG, q[0], q[1], q[2])]; });
      }
    }
#pragma unroll
    for (int nb = 0; nb < 6; nb++) c[dst[nb]] = val[nb];
  }
  if (!corners) return;
  __syncthreads();
  for (int e = t; e < 12 * NC; e += NC * NC) {
    const int n = e / NC, pos = e % NC + 1;
    const int dim = c_edge_dim[n];
    const int dx = c_edge_dir[n][0], dy = c_edge_dir[n][1], dz = c_edge_dir[n][2];
    const int nb_id = m.neighbor_mat[(dx + 1) + 3 * (dy + 1) + 9 * (dz + 1)];
    int x[3];
    for (int q = 0; q < 3; q++) x[q] = c_edge_min[n][q] * (NC + 1);
    x[dim] = pos;
    if (nb_id > 0) {
      int s[3] = {x[0] - dx * NC, x[1] - dy * NC, x[2] - dz * NC};
      c[ix3(NG, x[0], x[1], x[2])] = v[(size_t)(nb_id - 1) * bsz + ix3(NG, s[0], s[1], s[2])];
    } else {
      const int o1 = (dim + 1) % 3, o2 = (dim + 2) % 3;
      int di[3];
      for (int q = 0; q < 3; q++) di[q] = 1 - 2 * (x[q] & 1);
      di[dim] = 0;
      int ia[3] = {x[0], x[1], x[2]}, ib[3] = {x[0], x[1], x[2]};
      ia[o1] += di[o1];
      ib[o2] += di[o2];
      int ic[3] = {x[0] + di[0], x[1] + di[1], x[2] + di[2]};
      c[ix3(NG, x[0], x[1], x[2])] = c[ix3(NG, ia[0], ia[1], ia[2])] +
                                     c[ix3(NG, ib[0], ib[1], ib[2])] -
                                     c[ix3(NG, ic[0], ic[1], ic[2])];
    }
  }
  __syncthreads();
  if (t < 8) {
    const int n = t;
    int dnb[3], x[3];
    for (int q = 0; q < 3; q++) {
      dnb[q] = 2 * c_child_dix[n][q] - 1;
      x[q] = c_child_dix[n][q] * (NC + 1);
    }
    const int nb_id = m.neighbor_mat[(dnb[0] + 1) + 3 * (dnb[1] + 1) + 9 * (dnb[2] + 1)];
    if (nb_id > 0) {
      c[ix3(NG, x[0], x[1], x[2])] =
          v[(size_t)(nb_id - 1) * bsz +
            ix3(NG, x[0] - dnb[0] * NC, x[1] - dnb[1] * NC, x[2] - dnb[2] * NC)];
    } else {
      int di[3];
      for (int q = 0; q < 3; q++) di[q] = 1 - 2 * (x[q] & 1);
      c[ix3(NG, x[0], x[1], x[2])] = c[ix3(NG, x[0], x[1] + di[1], x[2] + di[2])] +
                                     c[ix3(NG, x[0] + di[0], x[1], x[2] + di[2])] +
                                     c[ix3(NG, x[0] + di[0], x[1] + di[1], x[2])] -
                                     2 * c[ix3(NG, x[0] + di[0], x[1] + di[1], x[2] + di[2])];
    }
  }
}

int32_t call_hook(afh_tree *t, int kind, int lvl, int iv, double *vals, int n) {
  if (!t->hook) return AFH_OK;
  if (afh_tree::SegRec *r = t->seg_rec) {
    // inside a segmented capture: the exchange runs between the segments'
    // replays; a reduction needs host values now and cannot be deferred
    if (vals || kind == AFH_HOOK_MAX || kind == AFH_HOOK_MIN || kind == AFH_HOOK_SUM) {
      r->bad = true;
      return set_error(AFH_ERR_STATE, "reduction inside a captured V-cycle");
    }
    hipGraph_t g = nullptr;
    AFH_HIP(hipStreamEndCapture(t->stream, &g));
    r->graphs.push_back(g);
    r->ops.push_back({kind, lvl, iv, n});
    AFH_HIP(hipStreamBeginCapture(t->stream, hipStreamCaptureModeThreadLocal));
    return AFH_OK;
  }
  int32_t e = t->hook(t->hook_ctx, kind, lvl, iv, vals, n);
  if (e) return set_error(AFH_ERR_STATE, "sharding hook %d failed (%d)", kind, e);
  return AFH_OK;
}

int32_t gc_lvl_var(afh_tree *t, int lvl, int iv, const double *vc,
                   const GcArgs &ga, int corners, bool rims, int depth) {
  const int n = t->ids.n(lvl);
  double *v = t->var(iv);
  int32_t e;
  if ((e = call_hook(t, AFH_HOOK_HALO, lvl, iv, nullptr, depth))) return e;
  if (n > 0) {
    const int nc = t->nc;
    prof_begin(t, AFH_PROF_GHOST);
    if (nc == 4 || nc == 8 || nc == 16) {
      // small boxes: faces, then edges and corners, one workgroup per box
      const int cr = corners ? 1 : 0;
      if (nc == 4)
        hipLaunchKernelGGL(k_gc_box<4>, dim3(n), dim3(16), 0, t->stream, v, vc, t->d_boxes,
                           t->ids.at(lvl), t->bsz, ga, cr);
      else if (nc == 8)
        hipLaunchKernelGGL(k_gc_box<8>, dim3(n), dim3(64), 0, t->stream, v, vc, t->d_boxes,
                           t->ids.at(lvl), t->bsz, ga, cr);
      else
        hipLaunchKernelGGL(k_gc_box<16>, dim3(n), dim3(256), 0, t->stream, v, vc, t->d_boxes,
                           t->ids.at(lvl), t->bsz, ga, cr);
      prof_end(t, AFH_PROF_GHOST, 16.0 * 6 * nc * nc * n);
      AFH_LAUNCH_CHECK("k_gc_box");
    } else {
      hipLaunchKernelGGL(k_gc_faces, dim3((nc * nc + 255) / 256, 6, n), dim3(256), 0,
                         t->stream, v, vc, t->d_boxes, t->ids.at(lvl), nc, t->bsz, ga);
      // algorithmic bytes: read one interior layer + write one ghost layer
      prof_end(t, AFH_PROF_GHOST, 16.0 * 6 * nc * nc * n);
      AFH_LAUNCH_CHECK("k_gc_faces");
      if (corners) {
        hipLaunchKernelGGL(k_gc_corners, dim3(n), dim3(fit_blk(12 * nc)), 0, t->stream, v,
                           t->d_boxes, t->ids.at(lvl), nc, t->bsz);
        AFH_LAUNCH_CHECK("k_gc_corners");
      }
    }
  }
  // replicas' ghost cells: a finer level's fill interpolates from this
  // level's (every ghost cell), or only a fused pair reads them (their face
  // ghosts next to its box: n = 10 + depth, most filled by the receiver)
  if (t->lvl_rb_coarse[lvl - 1]) return call_hook(t, AFH_HOOK_RIMS, lvl, iv, nullptr, depth);
  if (rims) return call_hook(t, AFH_HOOK_RIMS, lvl, iv, nullptr, 10 + depth);
  return AFH_OK;
}

int32_t gc_lvl_corners(afh_tree *t, int lvl, int iv) {
  const int n = t->ids.n(lvl);
  if (!n) return AFH_OK;
  hipLaunchKernelGGL(k_gc_corners, dim3(n), dim3(fit_blk(12 * t->nc)), 0, t->stream, t->var(iv), t->d_boxes,
                     t->ids.at(lvl), t->nc, t->bsz);
  AFH_LAUNCH_CHECK("k_gc_corners");
  return AFH_OK;
}

int32_t gc_lvl(afh_tree *t, int lvl, int iv, int corners, bool rims, int depth) {
  return gc_lvl_var(t, lvl, iv, t->ccv(iv), t->gc_args(iv), corners, rims, depth);
}

// ------------------------------------------------------------ plans
// Copy the cells of a list of box regions between a variable and a packed
// buffer (region r at off[r], i fastest). One block row per region.
__global__ void k_plan_copy(double *__restrict__ v, double *__restrict__ buf,
                            const int32_t *__restrict__ reg,
                            const int64_t *__restrict__ off, int ng, size_t bsz,
                            int unpack) {
  const int32_t *q = reg + 7 * blockIdx.y;
  const int nx = q[4] - q[1] + 1, ny = q[5] - q[2] + 1, nz = q[6] - q[3] + 1;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nx * ny * nz) return;
  const int i = q[1] + t % nx, j = q[2] + (t / nx) % ny, k = q[3] + t / (nx * ny);
  double *c = v + (size_t)(q[0] - 1) * bsz + ix3(ng, i, j, k);
  double *b = buf + off[blockIdx.y] + t;
  if (unpack) *c = *b;
  else *b = *c;
}

__global__ void k_plan_copy_fc(double *__restrict__ v, double *__restrict__ buf,
                               const int32_t *__restrict__ reg,
                               const int64_t *__restrict__ off, int nf,
                               size_t fsz, int unpack) {
  const int32_t *q = reg + 8 * blockIdx.y;
  const int nx = q[5] - q[2] + 1, ny = q[6] - q[3] + 1, nz = q[7] - q[4] + 1;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nx * ny * nz) return;
  const int i = q[2] + t % nx, j = q[3] + (t / nx) % ny, k = q[4] + t / (nx * ny);
  double *c = v + (size_t)(q[0] - 1) * fsz + (size_t)q[1] * nf * nf * nf +
              ((size_t)(k - 1) * nf + (j - 1)) * nf + (i - 1);
  double *b = buf + off[blockIdx.y] + t;
  if (unpack) *c = *b;
  else *b = *c;
}

// ------------------------------------------------------------ restriction
// af_restrict_box (m_af_restrict.f90:62-136): parent octant cell = 0.125 *
// sum of its 8 children in column-major order. One thread per parent cell.
__global__ void k_restrict(double *__restrict__ v,
                           const afh_box_meta *__restrict__ meta,
                           const int32_t *__restrict__ ids, int nc,
                           size_t bsz) {
  const int hnc = nc >> 1;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= hnc * hnc * hnc) return;
  const int id = ids[blockIdx.y];
  const afh_box_meta &m = meta[id - 1];
  int i, j, k;
  cell3(t, hnc, i, j, k);
  const int ng = nc + 2;
  const double *c = v + (size_t)(id - 1) * bsz;
  double *p = v + (size_t)(m.parent - 1) * bsz;
  const int fi = 2 * i - 1, fj = 2 * j - 1, fk = 2 * k - 1;
  double s = c[ix3(ng, fi, fj, fk)];
  s += c[ix3(ng, fi + 1, fj, fk)];
  s += c[ix3(ng, fi, fj + 1, fk)];
  s += c[ix3(ng, fi + 1, fj + 1, fk)];
  s += c[ix3(ng, fi, fj, fk + 1)];
  s += c[ix3(ng, fi + 1, fj, fk + 1)];
  s += c[ix3(ng, fi, fj + 1, fk + 1)];
  s += c[ix3(ng, fi + 1, fj + 1, fk + 1)];
  const int o0 = ((m.ix[0] - 1) & 1) * hnc, o1 = ((m.ix[1] - 1) & 1) * hnc,
            o2 = ((m.ix[2] - 1) & 1) * hnc;
  p[ix3(ng, o0 + i, o1 + j, o2 + k)] = 0.125 * s;
}

int32_t restrict_boxes(afh_tree *t, const int32_t *d_ids, int n, int iv) {
  if (n == 0) return AFH_OK;
  const int hnc = t->nc / 2, cells = hnc * hnc * hnc;
  hipLaunchKernelGGL(k_restrict, dim3((cells + 255) / 256, n), dim3(256), 0,
                     t->stream, t->ccv(iv), t->d_boxes, d_ids, t->nc, t->bsz);
  AFH_LAUNCH_CHECK("k_restrict");
  return AFH_OK;
}

// ------------------------------------------------------------ reductions
__global__ void k_red_fill(unsigned long long *r, unsigned long long v) {
  r[blockIdx.x * blockDim.x + threadIdx.x] = v;
}
// Slots folded by one launch of k_red_fold: block b folds slots[b]
struct RedFold {
  int slot[RED_SLOTS];
  int is_max[RED_SLOTS];
  unsigned long long reset[RED_SLOTS];
};
__global__ void k_red_fold(unsigned long long *red, RedFold F) {
  // one block of RED_SHARDS threads per slot; ordered integers fold like the
  // doubles; the shards are left at `reset` for the slot's next use
  __shared__ unsigned long long s[RED_SHARDS];
  const int slot = F.slot[blockIdx.x], is_max = F.is_max[blockIdx.x];
  unsigned long long *r = red + (size_t)slot * RED_SHARDS;
  unsigned long long *out = red + (size_t)RED_SLOTS * RED_SHARDS + slot;
  s[threadIdx.x] = r[threadIdx.x];
  r[threadIdx.x] = F.reset[blockIdx.x];
  __syncthreads();
  for (int o = RED_SHARDS / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      unsigned long long a = s[threadIdx.x], b = s[threadIdx.x + o];
      s[threadIdx.x] = is_max ? (a > b ? a : b) : (a < b ? a : b);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) *out = s[0];
}

// Each slot has a canonical start value (red_canon, set at tree creation);
// a fold resets the shards to it, so a red_init with that value finds them
// ready and launches nothing (V-cycle graphs captured in that state replay
// in it: every fold in them re-arms the slot). Another start value fills.
int32_t red_init(afh_tree *t, int slot, double v) {
  const unsigned long long o = host_dbl_to_ord(v);
  if (t->red_ready[slot] && o == t->red_canon[slot]) {
    t->red_ready[slot] = false;
    return AFH_OK;
  }
  auto *r = reinterpret_cast<unsigned long long *>(t->scratch);
  hipLaunchKernelGGL(k_red_fill, dim3(RED_SHARDS / 256), dim3(256), 0,
                     t->stream, r + (size_t)slot * RED_SHARDS, o);
  AFH_LAUNCH_CHECK("k_red_fill");
  t->red_ready[slot] = false;
  return AFH_OK;
}
int32_t red_finish(afh_tree *t, int slot, bool is_max) {
  const int slots[1] = {slot};
  const bool mx[1] = {is_max};
  return red_finish_n(t, 1, slots, mx);
}
// n slots folded in one launch (one block each)
int32_t red_finish_n(afh_tree *t, int n, const int *slots, const bool *is_max) {
  if (n < 1 || n > RED_SLOTS) return set_error(AFH_ERR_ARG, "fold of %d slots", n);
  RedFold F;
  for (int q = 0; q < n; q++) {
    F.slot[q] = slots[q];
    F.is_max[q] = is_max[q] ? 1 : 0;
    F.reset[q] = (unsigned long long)t->red_canon[slots[q]];
  }
  auto *r = reinterpret_cast<unsigned long long *>(t->scratch);
  hipLaunchKernelGGL(k_red_fold, dim3(n), dim3(RED_SHARDS), 0, t->stream, r, F);
  AFH_LAUNCH_CHECK("k_red_fold");
  for (int q = 0; q < n; q++) t->red_ready[slots[q]] = true;
  return AFH_OK;
}
int32_t red_fetch(afh_tree *t, int slot, int n, double *out) {
  auto *r = reinterpret_cast<unsigned long long *>(t->scratch);
  auto *h = reinterpret_cast<unsigned long long *>(t->h_scratch);
  AFH_HIP(hipMemcpyAsync(h, r + (size_t)RED_SLOTS * RED_SHARDS + slot,
                         n * sizeof(unsigned long long), hipMemcpyDeviceToHost,
                         t->stream));
  AFH_HIP(hipStreamSynchronize(t->stream));
  for (int q = 0; q < n; q++) out[q] = ord_to_dbl(h[q]);
  return AFH_OK;
}

int32_t red_reduce_fetch(afh_tree *t, int slot, int n_max, int n_min, double *out, int iv,
                         int level) {
  int32_t e;
  if (t->hook && t->dev_reduce) {
    auto *keys = reinterpret_cast<unsigned long long *>(t->scratch) +
                 (size_t)RED_SLOTS * RED_SHARDS + slot;
    if (n_max && (e = t->dev_reduce(t->hook_ctx, AFH_HOOK_MAX, keys, n_max))) return e;
    if (n_min && (e = t->dev_reduce(t->hook_ctx, AFH_HOOK_MIN, keys + n_max, n_min))) return e;
    return red_fetch(t, slot, n_max + n_min, out);
  }
  if ((e = red_fetch(t, slot, n_max + n_min, out))) return e;
  if (n_max && (e = call_hook(t, AFH_HOOK_MAX, level, iv, out, n_max))) return e;
  if (n_min && (e = call_hook(t, AFH_HOOK_MIN, level, iv, out + n_max, n_min))) return e;
  return AFH_OK;
}

// Any folded slots in one transfer (the deferred reductions of a step):
// with a device all-reduce, each run of consecutive slots of one kind is
// all-reduced in place first; with a host hook, each kind's values are
// reduced in one call after the fetch. Slot AFH_SLOT_CHEM is a minimum,
// every other slot a maximum.
int32_t red_fetch_slots(afh_tree *t, int n, const int32_t *slots, double *out) {
  if (n < 1 || n > RED_SLOTS) return set_error(AFH_ERR_ARG, "fetch of %d slots", n);
  int lo = RED_SLOTS, hi = -1;
  for (int q = 0; q < n; q++) {
    if (slots[q] < 0 || slots[q] >= RED_SLOTS)
      return set_error(AFH_ERR_ARG, "bad reduction slot %d", slots[q]);
    lo = std::min(lo, (int)slots[q]), hi = std::max(hi, (int)slots[q]);
  }
  auto is_min = [](int s) { return s == AFH_SLOT_CHEM; };
  auto *keys = reinterpret_cast<unsigned long long *>(t->scratch) +
               (size_t)RED_SLOTS * RED_SHARDS;
  int32_t e;
  if (t->hook && t->dev_reduce) {
    bool want[RED_SLOTS] = {};
    for (int q = 0; q < n; q++) want[slots[q]] = true;
    for (int s = lo; s <= hi;) {
      if (!want[s]) { s++; continue; }
      int r = s + 1;
      while (r <= hi && want[r] && is_min(r) == is_min(s)) r++;
      if ((e = t->dev_reduce(t->hook_ctx, is_min(s) ? AFH_HOOK_MIN : AFH_HOOK_MAX, keys + s,
                             r - s)))
        return e;
      s = r;
    }
  }
  double v[RED_SLOTS];
  if ((e = red_fetch(t, lo, hi - lo + 1, v))) return e;
  for (int q = 0; q < n; q++) out[q] = v[slots[q] - lo];
  if (t->hook && !t->dev_reduce) {
    for (int kind = 0; kind < 2; kind++) {
      double w[RED_SLOTS];
      int m = 0;
      for (int q = 0; q < n; q++)
        if (is_min(slots[q]) == (kind == 1)) w[m++] = out[q];
      if (m && (e = call_hook(t, kind ? AFH_HOOK_MIN : AFH_HOOK_MAX, 0, 0, w, m))) return e;
      m = 0;
      for (int q = 0; q < n; q++)
        if (is_min(slots[q]) == (kind == 1)) out[q] = w[m++];
    }
  }
  return AFH_OK;
}

// max |x| over the interiors of the listed boxes -> sharded atomicMax
__global__ void k_maxabs(const double *__restrict__ v,
                         const int32_t *__restrict__ ids, int nc, size_t bsz,
                         unsigned long long *out) {
  const int ng = nc + 2;
  const int id = ids[blockIdx.y];
  const double *c = v + (size_t)(id - 1) * bsz;
  const int n3 = nc * nc * nc;
  double mx = 0.0;
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < n3;
       t += gridDim.x * blockDim.x) {
    int i, j, k;
    cell3(t, nc, i, j, k);
    mx = fmax(mx, fabs(c[ix3(ng, i, j, k)]));
  }
  for (int o = 32; o > 0; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o, 64));
  __shared__ double red[16];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) red[w] = mx;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int q = 1; q < (int)(blockDim.x >> 6); q++) mx = fmax(mx, red[q]);
    atomicMax(&out[red_shard()], dbl_to_ord(mx));
  }
}

// af_tree_sum_cc / af_reduction_loc, per box (m_af_utils.f90:694-754,
// 840-874, 966-1026): one workgroup per leaf box reduces its interior. The
// sum folds each thread's cells in order, then a fixed butterfly and the
// waves in order (deterministic); max / min keep the first cell (i fastest)
// of the extremum, as Fortran's maxloc / minloc. The boxes are folded on the
// host in the reference's loop order.
__device__ __forceinline__ double ipow(double x, int n) {
  // gfortran's real ** integer (_gfortran_pow_r8_i4): binary powering
  double p = 1.0;
  for (;;) {
    if (n & 1) p *= x;
    n >>= 1;
    if (!n) break;
    x *= x;
  }
  return p;
}
template <int OP>
__global__ void k_box_reduce(const double *__restrict__ v,
                             const int32_t *__restrict__ ids, int nc, size_t bsz,
                             int power, double *__restrict__ out) {
  const int ng = nc + 2, n3 = nc * nc * nc;
  const double *c = v + (size_t)(ids[blockIdx.x] - 1) * bsz;
  double best = OP == 0 ? 0.0 : (OP == AFH_RED_MIN ? HUGE_VAL : -HUGE_VAL);
  int bix = 0x7fffffff;
  for (int t = threadIdx.x; t < n3; t += blockDim.x) {
    int i, j, k;
    cell3(t, nc, i, j, k);
    double x = c[ix3(ng, i, j, k)];
    if (OP == 0) {
      best += ipow(x, power);
    } else {
      if (OP == AFH_RED_MAXABS) x = fabs(x);
      if (OP == AFH_RED_MIN ? x < best : x > best) best = x, bix = t;
    }
  }
  auto comb = [&](double b, int ib) {
    if (OP == 0) {
      best += b;
    } else if ((OP == AFH_RED_MIN ? b < best : b > best) || (b == best && ib < bix)) {
      best = b, bix = ib;
    }
  };
  for (int o = 32; o > 0; o >>= 1) {
    const double b = __shfl_xor(best, o, 64);
    const int ib = __shfl_xor(bix, o, 64);
    comb(b, ib);
  }
  __shared__ double s_v[16];
  __shared__ int s_i[16];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) s_v[w] = best, s_i[w] = bix;
  __syncthreads();
  if (threadIdx.x == 0) {
    best = s_v[0], bix = s_i[0];
    for (int q = 1; q < (int)(blockDim.x >> 6); q++) comb(s_v[q], s_i[q]);
    out[2 * blockIdx.x] = best;
    out[2 * blockIdx.x + 1] = (double)bix;
  }
}

int32_t upload_list(afh_tree *t, LevelList &L,
                    const std::vector<std::vector<int32_t>> &lists) {
  if (L.d) hipFree(L.d), L.d = nullptr;
  L.off.assign(lists.size() + 1, 0);
  std::vector<int32_t> flat;
  for (size_t l = 0; l < lists.size(); l++) {
    flat.insert(flat.end(), lists[l].begin(), lists[l].end());
    L.off[l + 1] = (int32_t)flat.size();
  }
  AFH_HIP(hipMalloc(&L.d, sizeof(int32_t) * (flat.size() + 1)));
  if (!flat.empty())
    AFH_HIP(hipMemcpy(L.d, flat.data(), sizeof(int32_t) * flat.size(),
                      hipMemcpyHostToDevice));
  return AFH_OK;
}


// ------------------------------------------------------------ regrid
// af_prolong_limit / af_prolong_linear (m_af_prolong.f90:311-420, 531-679),
// add = .false.: one thread per parent cell of the child's octant writes
// its 8 child cells (value + 0, the child interior starting at 0)
template <int METHOD>
__global__ void k_prolong_new(double *__restrict__ v,
                              const afh_box_meta *__restrict__ meta,
                              const int32_t *__restrict__ ids, int nc, size_t bsz,
                              int lim) {
  const int hn = nc >> 1;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= hn * hn * hn) return;
  const int id = ids[blockIdx.y];
  const afh_box_meta &m = meta[id - 1];
  int i, j, k;
  cell3(t, hn, i, j, k);
  const int ng = nc + 2;
  const int ic = i + ((m.ix[0] - 1) & 1) * hn, jc = j + ((m.ix[1] - 1) & 1) * hn,
            kc = k + ((m.ix[2] - 1) & 1) * hn;
  const double *p = v + (size_t)(m.parent - 1) * bsz;
  double *c = v + (size_t)(id - 1) * bsz;
  const int fi = 2 * i - 1, fj = 2 * j - 1, fk = 2 * k - 1;
  auto P = [&](int a, int b, int d) { return p[ix3(ng, ic + a, jc + b, kc + d)]; };
  if (METHOD == AFH_PROLONG_LIMIT) {
    const double f0 = P(0, 0, 0);
    const double f1 = 0.25 * limiter(lim, f0 - P(-1, 0, 0), P(1, 0, 0) - f0);
    const double f2 = 0.25 * limiter(lim, f0 - P(0, -1, 0), P(0, 1, 0) - f0);
    const double f3 = 0.25 * limiter(lim, f0 - P(0, 0, -1), P(0, 0, 1) - f0);
#pragma unroll
    for (int q = 0; q < 8; q++) {
      double x = (q & 1) ? f0 + f1 : f0 - f1;
      x = ((q >> 1) & 1) ? x + f2 : x - f2;
      x = (q >> 2) ? x + f3 : x - f3;
      c[ix3(ng, fi + (q & 1), fj + ((q >> 1) & 1), fk + (q >> 2))] = x + 0.0;
    }
  } else {
    const double f1 = 1 / 64.0, f3 = 3 / 64.0, f9 = 9 / 64.0, f27 = 27 / 64.0;
    const double f000 = f27 * P(0, 0, 0);
    const double f00l = f9 * P(0, 0, -1), f0l0 = f9 * P(0, -1, 0), f0ll = f3 * P(0, -1, -1);
    const double fl00 = f9 * P(-1, 0, 0), fl0l = f3 * P(-1, 0, -1), fll0 = f3 * P(-1, -1, 0);
    const double flll = f1 * P(-1, -1, -1);
    const double f00h = f9 * P(0, 0, 1), f0h0 = f9 * P(0, 1, 0), f0hh = f3 * P(0, 1, 1);
    const double fh00 = f9 * P(1, 0, 0), fh0h = f3 * P(1, 0, 1), fhh0 = f3 * P(1, 1, 0);
    const double fhhh = f1 * P(1, 1, 1);
    const double fl0h = f3 * P(-1, 0, 1), fh0l = f3 * P(1, 0, -1), flh0 = f3 * P(-1, 1, 0);
    const double fhl0 = f3 * P(1, -1, 0), f0lh = f3 * P(0, -1, 1), f0hl = f3 * P(0, 1, -1);
    const double fllh = f1 * P(-1, -1, 1), flhl = f1 * P(-1, 1, -1), fhll = f1 * P(1, -1, -1);
    const double fhhl = f1 * P(1, 1, -1), fhlh = f1 * P(1, -1, 1), flhh = f1 * P(-1, 1, 1);
    auto W = [&](int a, int b, int d, double x) { c[ix3(ng, fi + a, fj + b, fk + d)] = x + 0.0; };
    W(0, 0, 0, f000 + fl00 + f0l0 + f00l + fll0 + fl0l + f0ll + flll);
    W(1, 0, 0, f000 + fh00 + f0l0 + f00l + fhl0 + fh0l + f0ll + fhll);
    W(0, 1, 0, f000 + fl00 + f0h0 + f00l + flh0 + fl0l + f0hl + flhl);
    W(1, 1, 0, f000 + fh00 + f0h0 + f00l + fhh0 + fh0l + f0hl + fhhl);
    W(0, 0, 1, f000 + fl00 + f0l0 + f00h + fll0 + fl0h + f0lh + fllh);
    W(1, 0, 1, f000 + fh00 + f0l0 + f00h + fhl0 + fh0h + f0lh + fhlh);
    W(0, 1, 1, f000 + fl00 + f0h0 + f00h + flh0 + fl0h + f0hh + flhh);
    W(1, 1, 1, f000 + fh00 + f0h0 + f00h + fhh0 + fh0h + f0hh + fhhh);
  }
}

// box ids[blockIdx.y] of variable blockIdx.z: src pool -> dst pool (the two
// pools of a regrid may hold different box counts: different variable
// strides); src null: zero
__global__ void k_copy_boxes(const double *__restrict__ src, double *__restrict__ dst,
                             const int32_t *__restrict__ ids, size_t per_box,
                             size_t src_var, size_t dst_var) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= per_box) return;
  const size_t b = (size_t)(ids[blockIdx.y] - 1) * per_box + t;
  dst[blockIdx.z * dst_var + b] = src ? src[blockIdx.z * src_var + b] : 0.0;
}
}  // namespace afh

using namespace afh;

extern "C" {

const char *afh_last_error(void) { return afh::g_err; }


static int32_t tree_create_impl(const afh_tree_desc *d, int32_t device,
                                afh_tree **out, afh_tree *adopt) {
  if (!d || !out || d->n_cell < 2 || (d->n_cell & 1) || d->n_boxes < 1 ||
      d->highest_lvl < 1 || d->n_var_cell < 1)
    return set_error(AFH_ERR_ARG, "afh_tree_create: bad descriptor");
  if (d->n_cell > 128)
    return set_error(AFH_ERR_UNSUPPORTED, "n_cell > 128 not supported");
  if (d->periodic[0] || d->periodic[1] || d->periodic[2])
    return set_error(AFH_ERR_UNSUPPORTED, "periodic domains not supported");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1)
    return set_error(AFH_ERR_DEVICE, "no HIP device available");
  afh_tree *t = new afh_tree();
  if (const char *env = getenv("AFH_ALL_LVL")) t->all_lvl_launch = atoi(env) != 0;
  if (device >= 0) {
    AFH_HIP(hipSetDevice(device));
    t->device = device;
  } else {
    AFH_HIP(hipGetDevice(&t->device));
  }
  AFH_HIP(hipStreamCreateWithFlags(&t->stream, hipStreamNonBlocking));
  t->nc = d->n_cell;
  t->ng = d->n_cell + 2;
  t->nb = d->n_boxes;
  t->cap = std::max(d->n_boxes, d->box_capacity);
  t->nlvl = d->highest_lvl;
  t->nvc = d->n_var_cell;
  t->nvf = d->n_var_face;
  t->bsz = (size_t)t->ng * t->ng * t->ng;
  t->fsz = 3 * (size_t)(t->nc + 1) * (t->nc + 1) * (t->nc + 1);
  for (int q = 0; q < 3; q++) {
    t->cgs[q] = d->coarse_grid_size[q];
    t->r_base[q] = d->r_base[q];
    t->dr_base[q] = d->dr_base[q];
  }
  t->boxes.assign(d->boxes, d->boxes + t->nb);
  t->meth.assign(t->nvc + 1, CcMethod());
  t->gen.assign(t->nvc + 1, 0);
  auto split = [&](const int32_t *arr, const int32_t *off) {
    std::vector<std::vector<int32_t>> v(t->nlvl);
    for (int l = 0; l < t->nlvl; l++) v[l].assign(arr + off[l], arr + off[l + 1]);
    return v;
  };
  t->h_ids = split(d->lvl_ids, d->lvl_ids_off);
  t->h_leaves = split(d->lvl_leaves, d->lvl_leaves_off);
  t->h_parents = split(d->lvl_parents, d->lvl_parents_off);
  // grid spacing per level over ALL boxes of the topology (a sharded tree
  // lists only this rank's boxes, possibly none on some level)
  t->lvl_dr.assign(3 * t->nlvl, 0.0);
  std::vector<int> seen(t->nlvl, 0);
  t->lvl_total.assign(t->nlvl, 0);
  for (int id = 1; id <= t->nb; id++) {
    const afh_box_meta &m = t->boxes[id - 1];
    if (m.lvl < 1) continue;  // unused id
    if (m.lvl > t->nlvl) return set_error(AFH_ERR_ARG, "box %d level %d", id, m.lvl);
    const int l = m.lvl - 1;
    for (int q = 0; q < 3; q++) {
      if (!seen[l]) t->lvl_dr[3 * l + q] = m.dr[q];
      if (memcmp(&m.dr[q], &t->lvl_dr[3 * l + q], sizeof(double)) != 0)
        return set_error(AFH_ERR_UNSUPPORTED, "non-uniform dr on level %d", l + 1);
    }
    seen[l] = 1;
    t->lvl_total[l]++;
  }
  t->lvl_leaves_total.assign(t->nlvl, 0);
  for (int l = 0; l < t->nlvl; l++)
    t->lvl_leaves_total[l] = (int)t->h_leaves[l].size();
  t->lvl_rb_coarse.assign(t->nlvl, 0);
  for (int id = 1; id <= t->nb; id++) {
    const afh_box_meta &m = t->boxes[id - 1];
    if (m.lvl < 2) continue;
    for (int nb = 0; nb < 6; nb++)
      if (m.neighbors[nb] == 0) t->lvl_rb_coarse[m.lvl - 2] = 1;
  }
  for (int l = 0; l < t->nlvl; l++) {
    if (!seen[l]) return set_error(AFH_ERR_ARG, "empty level %d", l + 1);
    for (int32_t id : t->h_ids[l]) {
      if (id < 1 || id > t->nb) return set_error(AFH_ERR_ARG, "bad box id %d", id);
      if (t->boxes[id - 1].lvl != l + 1)
        return set_error(AFH_ERR_ARG, "box %d level mismatch", id);
    }
  }
  t->any_cflux = false;
  for (int id = 1; id <= t->nb; id++) {
    const afh_box_meta &m = t->boxes[id - 1];
    if (m.children[0] == 0) continue;
    for (int nb = 0; nb < 6; nb++) {
      const int nb_id = m.neighbors[nb];
      if (nb_id > 0 && t->boxes[nb_id - 1].children[0] == 0) t->any_cflux = true;
    }
  }
  // derived task lists
  std::vector<std::vector<int32_t>> refb(t->nlvl), cfl(t->nlvl);
  for (int l = 0; l < t->nlvl; l++) {
    for (int32_t id : t->h_leaves[l]) {
      const afh_box_meta &m = t->boxes[id - 1];
      bool any = false;
      for (int nb = 0; nb < 6; nb++) any |= (m.neighbors[nb] == 0);
      if (m.parent > 0 && any) refb[l].push_back(id);
    }
    for (int32_t id : t->h_parents[l]) {
      const afh_box_meta &m = t->boxes[id - 1];
      for (int nb = 1; nb <= 6; nb++) {
        int nb_id = m.neighbors[nb - 1];
        if (nb_id > 0 && t->boxes[nb_id - 1].children[0] == 0)
          cfl[l].push_back(id * 8 + nb);
      }
    }
  }
  int32_t e;
  if ((e = upload_list(t, t->ids, t->h_ids)) ||
      (e = upload_list(t, t->leaves, t->h_leaves)) ||
      (e = upload_list(t, t->parents, t->h_parents)) ||
      (e = upload_list(t, t->refb, refb)) || (e = upload_list(t, t->cflux, cfl)))
    return e;
  AFH_HIP(hipMalloc(&t->d_boxes, sizeof(afh_box_meta) * t->nb));
  AFH_HIP(hipMemcpy(t->d_boxes, t->boxes.data(), sizeof(afh_box_meta) * t->nb,
                    hipMemcpyHostToDevice));
  if (adopt) {  // afh_tree_regrid in place: the old tree's pools
    t->cap = adopt->cap;
    t->vstride = adopt->vstride;
    t->cc = adopt->cc, t->fc = adopt->fc, t->gc2 = adopt->gc2;
    adopt->cc = adopt->fc = adopt->gc2 = nullptr;
    adopt->retired = true;
  } else {
    t->vstride = (size_t)t->cap * t->bsz;
    size_t ncc = (size_t)t->nvc * t->vstride;
    size_t nfc = (size_t)std::max(1, t->nvf) * t->cap * t->fsz;
    if (int32_t e2 = pool_alloc((void **)&t->cc, ncc * sizeof(double), "cc")) return e2;
    if (int32_t e2 = pool_alloc((void **)&t->fc, nfc * sizeof(double), "fc")) return e2;
    AFH_HIP(hipMemsetAsync(t->cc, 0, ncc * sizeof(double), t->stream));
    AFH_HIP(hipMemsetAsync(t->fc, 0, nfc * sizeof(double), t->stream));
    if (int32_t e2 = pool_alloc((void **)&t->gc2,
                                sizeof(double) * (size_t)t->cap * 6 * t->nc * t->nc, "gc2"))
      return e2;
  }
  AFH_HIP(hipMalloc(&t->scratch, (size_t)(RED_SLOTS + 1) * RED_SHARDS * sizeof(double)));
  AFH_HIP(hipHostMalloc(&t->h_scratch, RED_SLOTS * sizeof(double)));
  // canonical start values of the reduction slots: the flux maxima (0, 1),
  // the chemistry time-step minimum (2), max|x| (3, 4)
  static_assert(RED_SLOTS == 8, "red_canon / red_ready sizes");
  const double canon[RED_SLOTS] = {-HUGE_VAL, -HUGE_VAL, 1e100, 0.0, 0.0, 0.0, 0.0, 0.0};
  for (int q = 0; q < RED_SLOTS; q++) {
    t->red_canon[q] = host_dbl_to_ord(canon[q]);
    t->red_ready[q] = false;
    if (int32_t e2 = red_init(t, q, canon[q])) return e2;
    t->red_ready[q] = true;
  }
  AFH_HIP(hipStreamSynchronize(t->stream));
  *out = t;
  return AFH_OK;
}

int32_t afh_tree_create(const afh_tree_desc *d, int32_t device,
                        afh_tree **out) {
  return tree_create_impl(d, device, out, nullptr);
}

int32_t afh_profile_enable(afh_tree *t, int32_t kclass) {
  AFH_LIVE(t, "afh_profile_enable");
  AFH_HIP(hipStreamSynchronize(t->stream));
  t->prof_class = kclass;
  t->ev_used = 0;
  t->prof_bytes = 0;
  t->prof_launches = 0;
  return AFH_OK;
}

int32_t afh_profile_read(afh_tree *t, double *total_ms, int64_t *launches,
                         double *bytes) {
  if (!t || !total_ms || !launches || !bytes)
    return set_error(AFH_ERR_ARG, "null argument");
  AFH_HIP(hipStreamSynchronize(t->stream));
  double ms = 0;
  for (size_t q = 0; q + 1 < t->ev_used; q += 2) {
    float e = 0;
    AFH_HIP(hipEventElapsedTime(&e, t->ev_pool[q], t->ev_pool[q + 1]));
    ms += e;
  }
  *total_ms = ms;
  *launches = t->prof_launches;
  *bytes = t->prof_bytes;
  t->ev_used = 0;
  t->prof_bytes = 0;
  t->prof_launches = 0;
  return AFH_OK;
}

int32_t afh_tree_destroy(afh_tree *t) {
  if (!t) return AFH_OK;
  hipStreamSynchronize(t->stream);
  for (hipEvent_t e : t->ev_pool) hipEventDestroy(e);
  for (LevelList *L : {&t->ids, &t->leaves, &t->parents, &t->refb, &t->cflux})
    hipFree(L->d);
  for (auto &p : t->plans) {
    hipFree(p.d_reg);
    hipFree(p.d_off);
  }
  hipFree(t->d_boxes);
  hipFree(t->cc);
  hipFree(t->fc);
  hipFree(t->gc2);
  hipFree(t->scratch);
  hipFree(t->d_sumw);
  for (hipStream_t &q : t->side)
    if (q) hipStreamDestroy(q);
  for (hipEvent_t &q : t->side_ev)
    if (q) hipEventDestroy(q);
  hipFree(t->d_boxred);
  hipHostFree(t->h_scratch);
  if (t->own_stream) hipStreamDestroy(t->stream);
  delete t;
  return AFH_OK;
}

int32_t afh_tree_sync(afh_tree *t) {
  AFH_LIVE(t, "afh_tree_sync");
  AFH_HIP(hipStreamSynchronize(t->stream));
  return AFH_OK;
}

int32_t afh_set_cc_methods(afh_tree *t, int32_t iv, const afh_bc *bc6,
                           int32_t rb, int32_t lim) {
  AFH_LIVE(t, "afh_set_cc_methods");
  if (!t || iv < 1 || iv > t->nvc || !bc6)
    return set_error(AFH_ERR_ARG, "afh_set_cc_methods: bad argument");
  if (rb < AFH_RB_GC_INTERP || rb > AFH_RB_MG_SIDES)
    return set_error(AFH_ERR_UNSUPPORTED, "refinement-boundary method %d", rb);
  if (lim < AFH_LIM_NONE || lim > AFH_LIM_ZERO)
    return set_error(AFH_ERR_UNSUPPORTED, "limiter %d", lim);
  CcMethod &m = t->meth[iv];
  m.set = 1;
  t->meth_gen++;
  for (int n = 0; n < 6; n++) {
    if (bc6[n].type < AFH_BC_DIRICHLET_COPY || bc6[n].type > AFH_BC_DIRICHLET)
      return set_error(AFH_ERR_UNSUPPORTED, "bc type %d", bc6[n].type);
    m.bc[n] = bc6[n];
  }
  m.rb = rb;
  m.lim = lim;
  return AFH_OK;
}

int32_t afh_set_bc(afh_tree *t, int32_t iv, int32_t nb, int32_t type,
                   double value) {
  AFH_LIVE(t, "afh_set_bc");
  if (!t || iv < 1 || iv > t->nvc || nb < 1 || nb > 6)
    return set_error(AFH_ERR_ARG, "afh_set_bc: bad argument");
  if (type < AFH_BC_DIRICHLET_COPY || type > AFH_BC_DIRICHLET)
    return set_error(AFH_ERR_UNSUPPORTED, "bc type %d", type);
  // captured V-cycles hold the boundary values (and the coarse-solve tables
  // the types): drop them, as afh_set_cc_methods does
  t->meth_gen++;
  t->meth[iv].bc[nb - 1].type = type;
  t->meth[iv].bc[nb - 1].value = value;
  return AFH_OK;
}

int32_t afh_cc_put(afh_tree *t, int32_t iv, const double *h) {
  AFH_LIVE(t, "afh_cc_put");
  if (!t || iv < 1 || iv > t->nvc || !h)
    return set_error(AFH_ERR_ARG, "afh_cc_put: bad argument");
  t->touch(iv);
  AFH_HIP(hipMemcpyAsync(t->ccv(iv), h, sizeof(double) * t->bsz * t->nb,
                         hipMemcpyHostToDevice, t->stream));
  AFH_HIP(hipStreamSynchronize(t->stream));
  return AFH_OK;
}
int32_t afh_cc_get(afh_tree *t, int32_t iv, double *h) {
  AFH_LIVE(t, "afh_cc_get");
  if (!t || iv < 1 || iv > t->nvc || !h)
    return set_error(AFH_ERR_ARG, "afh_cc_get: bad argument");
  AFH_HIP(hipMemcpyAsync(h, t->ccv(iv), sizeof(double) * t->bsz * t->nb,
                         hipMemcpyDeviceToHost, t->stream));
  AFH_HIP(hipStreamSynchronize(t->stream));
  return AFH_OK;
}
int32_t afh_fc_put(afh_tree *t, int32_t ivf, const double *h) {
  AFH_LIVE(t, "afh_fc_put");
  if (!t || ivf < 1 || ivf > t->nvf || !h)
    return set_error(AFH_ERR_ARG, "afh_fc_put: bad argument");
  AFH_HIP(hipMemcpyAsync(t->fcv(ivf), h, sizeof(double) * t->fsz * t->nb,
                         hipMemcpyHostToDevice, t->stream));
  AFH_HIP(hipStreamSynchronize(t->stream));
  return AFH_OK;
}
int32_t afh_fc_get(afh_tree *t, int32_t ivf, double *h) {
  AFH_LIVE(t, "afh_fc_get");
  if (!t || ivf < 1 || ivf > t->nvf || !h)
    return set_error(AFH_ERR_ARG, "afh_fc_get: bad argument");
  AFH_HIP(hipMemcpyAsync(h, t->fcv(ivf), sizeof(double) * t->fsz * t->nb,
                         hipMemcpyDeviceToHost, t->stream));
  AFH_HIP(hipStreamSynchronize(t->stream));
  return AFH_OK;
}

// Box rows in device memory: row r of buf = box ids[r]'s cell-centred
// variables 1..n_cc, then its face variables 1..n_fc (the host arrays'
// per-box layout). One launch per variable, a block row per box.
__global__ void k_box_rows(double *__restrict__ v, double *__restrict__ buf,
                           const int32_t *__restrict__ ids, size_t blk, size_t row_w,
                           size_t off, int unpack) {
  const int r = blockIdx.y;
  double *b = buf + (size_t)r * row_w + off;
  double *c = v + (size_t)(ids[r] - 1) * blk;
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < blk;
       e += (size_t)gridDim.x * blockDim.x) {
    if (unpack) c[e] = b[e];
    else b[e] = c[e];
  }
}

static int32_t box_rows(afh_tree *t, const int32_t *ids, int32_t n, int32_t n_cc,
                        int32_t n_fc, double *buf, int unpack) {
  if (!t || n < 0 || (n && (!ids || !buf)) || n_cc < 0 || n_cc > t->nvc || n_fc < 0 ||
      n_fc > t->nvf)
    return set_error(AFH_ERR_ARG, "afh_tree_%spack_boxes: bad argument", unpack ? "un" : "");
  for (int r = 0; r < n; r++)
    if (ids[r] < 1 || ids[r] > t->nb)
      return set_error(AFH_ERR_ARG, "afh_tree_%spack_boxes: box %d", unpack ? "un" : "", ids[r]);
  if (!n) return AFH_OK;
  int32_t *d_ids = nullptr;
  AFH_HIP(hipMalloc(&d_ids, sizeof(int32_t) * n));
  AFH_HIP(hipMemcpyAsync(d_ids, ids, sizeof(int32_t) * n, hipMemcpyHostToDevice, t->stream));
  const size_t row_w = (size_t)n_cc * t->bsz + (size_t)n_fc * t->fsz;
  for (int q = 0; q < n_cc + n_fc; q++) {
    const bool cc = q < n_cc;
    const size_t blk = cc ? t->bsz : t->fsz;
    const size_t off = cc ? (size_t)q * t->bsz : (size_t)n_cc * t->bsz + (size_t)(q - n_cc) * t->fsz;
    double *v = cc ? t->ccv(q + 1) : t->fcv(q - n_cc + 1);
    if (unpack && cc) t->touch(q + 1);
    const int gx = (int)std::min<size_t>((blk + 255) / 256, 64);
    for (int r0 = 0; r0 < n; r0 += 65535) {
      const int nr = std::min(65535, n - r0);
      hipLaunchKernelGGL(k_box_rows, dim3(gx, nr), dim3(256), 0, t->stream, v,
                         buf + (size_t)r0 * row_w, d_ids + r0, blk, row_w, off, unpack);
      AFH_LAUNCH_CHECK("k_box_rows");
    }
  }
  const hipError_t e = hipStreamSynchronize(t->stream);
  hipFree(d_ids);
  if (e != hipSuccess) return check_hip(e, "k_box_rows");
  return AFH_OK;
}

int32_t afh_tree_pack_boxes(afh_tree *t, const int32_t *ids, int32_t n, int32_t n_cc,
                            int32_t n_fc, double *buf) {
  AFH_LIVE(t, "afh_tree_pack_boxes");
  return box_rows(t, ids, n, n_cc, n_fc, buf, 0);
}

int32_t afh_tree_unpack_boxes(afh_tree *t, const int32_t *ids, int32_t n, int32_t n_cc,
                              int32_t n_fc, const double *buf) {
  AFH_LIVE(t, "afh_tree_unpack_boxes");
  return box_rows(t, ids, n, n_cc, n_fc, const_cast<double *>(buf), 1);
}

int32_t afh_device_alloc(int32_t device, int64_t n_bytes, void **out) {
  if (!out || n_bytes < 0) return set_error(AFH_ERR_ARG, "afh_device_alloc: bad argument");
  *out = nullptr;
  int cur = 0;
  AFH_HIP(hipGetDevice(&cur));
  AFH_HIP(hipSetDevice(device));
  const hipError_t e = hipMalloc(out, n_bytes > 0 ? (size_t)n_bytes : 8);
  hipSetDevice(cur);
  if (e != hipSuccess) return check_hip(e, "afh_device_alloc");
  return AFH_OK;
}

int32_t afh_device_free(void *p) {
  if (p) AFH_HIP(hipFree(p));
  return AFH_OK;
}

int32_t afh_gc_lvl(afh_tree *t, int32_t lvl, int32_t iv, int32_t corners) {
  AFH_LIVE(t, "afh_gc_lvl");
  if (!t || lvl < 1 || lvl > t->nlvl || iv < 1 || iv > t->nvc ||
      !t->meth[iv].set)
    return set_error(AFH_ERR_ARG, "afh_gc_lvl: bad argument / no methods");
  t->touch(iv);
  return gc_lvl(t, lvl, iv, corners);
}

int32_t afh_gc_tree(afh_tree *t, int32_t iv, int32_t corners) {
  AFH_LIVE(t, "afh_gc_tree");
  for (int l = 1; l <= (t ? t->nlvl : 0); l++) {
    int32_t e = afh_gc_lvl(t, l, iv, corners);
    if (e) return e;
  }
  return t ? AFH_OK : set_error(AFH_ERR_ARG, "null tree");
}

int32_t afh_restrict_tree(afh_tree *t, int32_t iv) {
  AFH_LIVE(t, "afh_restrict_tree");
  if (iv < 1 || iv > t->nvc) return set_error(AFH_ERR_ARG, "bad iv");
  t->touch(iv);
  // af_restrict_tree: parents of levels highest-1..1, i.e. children of
  // levels highest..2, coarsest last
  for (int l = t->nlvl; l >= 2; l--) {
    int32_t e = restrict_boxes(t, t->ids.at(l), t->ids.n(l), iv);
    if (e || (e = call_hook(t, AFH_HOOK_RESTRICT, l, iv))) return e;
  }
  return AFH_OK;
}

int32_t afh_tree_copy_cc(afh_tree *t, int32_t a, int32_t b) {
  AFH_LIVE(t, "afh_tree_copy_cc");
  if (a < 1 || a > t->nvc || b < 1 || b > t->nvc)
    return set_error(AFH_ERR_ARG, "bad iv");
  t->touch(b);
  AFH_HIP(hipMemcpyAsync(t->ccv(b), t->ccv(a), sizeof(double) * t->bsz * t->nb,
                         hipMemcpyDeviceToDevice, t->stream));
  return AFH_OK;
}

int32_t afh_tree_maxabs_cc(afh_tree *t, int32_t iv, double *out) {
  AFH_LIVE(t, "afh_tree_maxabs_cc");
  if (!t || iv < 1 || iv > t->nvc || !out) return set_error(AFH_ERR_ARG, "bad iv");
  int32_t e;
  if ((e = red_init(t, 3, 0.0))) return e;
  auto *d = reinterpret_cast<unsigned long long *>(t->scratch) + 3 * RED_SHARDS;
  const int nc = t->nc, n3 = nc * nc * nc;
  int bx = std::min(64, (n3 + 255) / 256);
  for (int l = 1; l <= t->nlvl; l++) {
    int n = t->leaves.n(l);
    if (!n) continue;
    hipLaunchKernelGGL(k_maxabs, dim3(bx, n), dim3(256), 0, t->stream,
                       t->ccv(iv), t->leaves.at(l), nc, t->bsz, d);
    AFH_LAUNCH_CHECK("k_maxabs");
  }
  if ((e = red_finish(t, 3, true))) return e;
  return red_reduce_fetch(t, 3, 1, 0, out, iv);
}

// per-box partial results over all leaves (level order), on the host
static int32_t box_reduce(afh_tree *t, int iv, int op, int power,
                          std::vector<double> &res, bool fetch = true) {
  const int nl = t->leaves.off[t->nlvl];
  res.assign(2 * (size_t)nl, 0.0);
  if (!nl) return AFH_OK;
  if (nl > t->boxred_cap) {
    AFH_HIP(hipStreamSynchronize(t->stream));
    hipFree(t->d_boxred);
    t->d_boxred = nullptr;
    AFH_HIP(hipMalloc(&t->d_boxred, sizeof(double) * 2 * nl));
    t->boxred_cap = nl;
  }
  const dim3 grid(nl), blk(256);
  switch (op) {
  case 0:
    hipLaunchKernelGGL(k_box_reduce<0>, grid, blk, 0, t->stream, t->ccv(iv),
                       t->leaves.d, t->nc, t->bsz, power, t->d_boxred);
    break;
  case AFH_RED_MAX:
    hipLaunchKernelGGL(k_box_reduce<AFH_RED_MAX>, grid, blk, 0, t->stream,
                       t->ccv(iv), t->leaves.d, t->nc, t->bsz, power, t->d_boxred);
    break;
  case AFH_RED_MIN:
    hipLaunchKernelGGL(k_box_reduce<AFH_RED_MIN>, grid, blk, 0, t->stream,
                       t->ccv(iv), t->leaves.d, t->nc, t->bsz, power, t->d_boxred);
    break;
  default:
    hipLaunchKernelGGL(k_box_reduce<AFH_RED_MAXABS>, grid, blk, 0, t->stream,
                       t->ccv(iv), t->leaves.d, t->nc, t->bsz, power, t->d_boxred);
  }
  AFH_LAUNCH_CHECK("k_box_reduce");
  if (!fetch) return AFH_OK;
  AFH_HIP(hipMemcpyAsync(res.data(), t->d_boxred, sizeof(double) * 2 * nl,
                         hipMemcpyDeviceToHost, t->stream));
  AFH_HIP(hipStreamSynchronize(t->stream));
  return AFH_OK;
}

// afh_tree_sum_cc's fold on the device: the host loop's order and operations
// (sum = sum + fac * box sum, leaves in level order, skipped boxes left out)
// in one thread
__global__ void k_sum_fold(const double *__restrict__ res, const double *__restrict__ w,
                           int n, double *__restrict__ out) {
  if (threadIdx.x != 0) return;
  double sum = 0.0;
  for (int q = 0; q < n; q++)
    if (w[q] != 0.0) sum = sum + w[q] * res[2 * q];
  *out = sum;
}

int32_t afh_tree_sum_cc(afh_tree *t, int32_t iv, int32_t power, double *out) {
  AFH_LIVE(t, "afh_tree_sum_cc");
  if (iv < 1 || iv > t->nvc || power < 1 || !out)
    return set_error(AFH_ERR_ARG, "afh_tree_sum_cc: bad argument");
  std::vector<double> res;
  int32_t e;
  if (t->hook && t->dev_sum) {
    // sharded over RCCL: box sums, their fold and the all-reduce on the
    // device, one transfer at the end (bitwise the host path below)
    const int nl = t->leaves.off[t->nlvl];
    if (t->sumw_n != nl) {
      std::vector<double> w(nl > 0 ? nl : 1, 0.0);
      size_t q = 0;
      for (int l = 1; l <= t->nlvl; l++) {
        const double *dr = &t->lvl_dr[3 * (l - 1)];
        const double fac = dr[0] * dr[1] * dr[2];
        for (int b = 0; b < t->leaves.n(l); b++, q++)
          w[q] = (t->sum_skip.empty() || !t->sum_skip[t->h_leaves[l - 1][b] - 1]) ? fac : 0.0;
      }
      AFH_HIP(hipStreamSynchronize(t->stream));
      hipFree(t->d_sumw);
      t->d_sumw = nullptr;
      AFH_HIP(hipMalloc(&t->d_sumw, sizeof(double) * w.size()));
      AFH_HIP(hipMemcpy(t->d_sumw, w.data(), sizeof(double) * w.size(), hipMemcpyHostToDevice));
      t->sumw_n = nl;
    }
    if ((e = box_reduce(t, iv, 0, power, res, false))) return e;
    // (after the slots' shards and their fold outputs)
    double *d_out = t->scratch + (size_t)RED_SLOTS * RED_SHARDS + RED_SLOTS;
    hipLaunchKernelGGL(k_sum_fold, dim3(1), dim3(64), 0, t->stream, t->d_boxred, t->d_sumw, nl,
                       d_out);
    AFH_LAUNCH_CHECK("k_sum_fold");
    if ((e = t->dev_sum(t->hook_ctx, d_out))) return e;
    AFH_HIP(hipMemcpyAsync(out, d_out, sizeof(double), hipMemcpyDeviceToHost, t->stream));
    AFH_HIP(hipStreamSynchronize(t->stream));
    return AFH_OK;
  }
  if ((e = box_reduce(t, iv, 0, power, res))) return e;
  // my_sum = my_sum + fac * tmp, fac = product(af_lvl_dr(tree, lvl))
  double sum = 0.0;
  size_t q = 0;
  for (int l = 1; l <= t->nlvl; l++) {
    const double *dr = &t->lvl_dr[3 * (l - 1)];
    const double fac = dr[0] * dr[1] * dr[2];
    for (int b = 0; b < t->leaves.n(l); b++, q++)
      if (t->sum_skip.empty() || !t->sum_skip[t->h_leaves[l - 1][b] - 1])
        sum = sum + fac * res[2 * q];
  }
  *out = sum;
  return call_hook(t, AFH_HOOK_SUM, 0, iv, out, 1);
}

int32_t afh_tree_reduce_loc(afh_tree *t, int32_t iv, int32_t op, double *out,
                            int32_t *loc) {
  AFH_LIVE(t, "afh_tree_reduce_loc");
  if (iv < 1 || iv > t->nvc || !out || op < AFH_RED_MAX || op > AFH_RED_MAXABS)
    return set_error(AFH_ERR_ARG, "afh_tree_reduce_loc: bad argument");
  if (t->hook && loc)
    return set_error(AFH_ERR_UNSUPPORTED, "location of a sharded reduction");
  std::vector<double> res;
  int32_t e;
  if ((e = box_reduce(t, iv, op, 1, res))) return e;
  // af_reduction_loc: init -huge/10 (max) or huge/10 (min); a box replaces
  // the running value when reduction(tmp, val) differs from val
  const bool is_min = op == AFH_RED_MIN;
  double val = (is_min ? 1 : -1) * (DBL_MAX / 10);
  int32_t lid = -1, lix = -1;
  size_t q = 0;
  for (int l = 1; l <= t->nlvl; l++)
    for (int b = 0; b < t->leaves.n(l); b++, q++) {
      const double tmp = res[2 * q];
      const double nv = is_min ? std::min(tmp, val) : std::max(tmp, val);
      if (std::fabs(nv - val) > 0) {
        val = tmp;
        lid = t->h_leaves[l - 1][b];
        lix = (int32_t)res[2 * q + 1];
      }
    }
  *out = val;
  if (loc) {
    loc[0] = lid;
    const int nc = t->nc;
    loc[1] = lix < 0 ? -1 : lix % nc + 1;
    loc[2] = lix < 0 ? -1 : (lix / nc) % nc + 1;
    loc[3] = lix < 0 ? -1 : lix / (nc * nc) + 1;
  }
  return call_hook(t, is_min ? AFH_HOOK_MIN : AFH_HOOK_MAX, 0, iv, out, 1);
}

int32_t afh_tree_fetch_reduced(afh_tree *t, int32_t n, const int32_t *slots, double *out) {
  if (!t || !slots || !out) return set_error(AFH_ERR_ARG, "afh_tree_fetch_reduced: null");
  AFH_LIVE(t, "afh_tree_fetch_reduced");
  if (n < 1 || n > 2) return set_error(AFH_ERR_ARG, "afh_tree_fetch_reduced: %d slots", n);
  for (int q = 0; q < n; q++)
    if (slots[q] != AFH_SLOT_MAXRES && slots[q] != AFH_SLOT_RHS)
      return set_error(AFH_ERR_ARG, "afh_tree_fetch_reduced: slot %d", slots[q]);
  return red_fetch_slots(t, n, slots, out);
}

int32_t afh_tree_set_stream(afh_tree *t, void *stream) {
  AFH_LIVE(t, "afh_tree_set_stream");
  AFH_HIP(hipStreamSynchronize(t->stream));
  if (t->own_stream) AFH_HIP(hipStreamDestroy(t->stream));
  t->stream = (hipStream_t)stream;
  t->own_stream = false;
  return AFH_OK;
}

int32_t afh_tree_set_hook(afh_tree *t, afh_hook_fn fn, void *ctx) {
  AFH_LIVE(t, "afh_tree_set_hook");
  t->hook = fn;
  t->hook_ctx = ctx;
  t->dev_reduce = nullptr;  // the library's RCCL transport sets its own
  t->dev_sum = nullptr;
  t->hook_capturable = false;
  t->meth_gen++;            // captured V-cycles recorded the old exchanges
  return AFH_OK;
}

static int32_t plan_create(afh_tree *t, const int32_t *reg, int32_t n,
                           int32_t *plan, int64_t *n_values, int fc) {
  AFH_LIVE(t, "afh_plan_create");
  if (!t || n < 0 || (n > 0 && !reg) || !plan || !n_values)
    return set_error(AFH_ERR_ARG, "afh_plan_create: bad argument");
  const int w = fc ? 8 : 7, lo = fc ? 2 : 1;
  const int vmin = fc ? 1 : 0, vmax = t->nc + 1;
  afh_tree::Plan p;
  p.n = n;
  p.fc = fc;
  std::vector<int64_t> off(n + 1, 0);
  for (int r = 0; r < n; r++) {
    const int32_t *q = reg + w * r;
    if (q[0] < 1 || q[0] > t->nb) return set_error(AFH_ERR_ARG, "plan: bad box id");
    if (fc && (q[1] < 0 || q[1] > 2)) return set_error(AFH_ERR_ARG, "plan: bad dim");
    int64_t cells = 1;
    for (int d = 0; d < 3; d++) {
      if (q[lo + d] < vmin || q[lo + 3 + d] > vmax || q[lo + 3 + d] < q[lo + d])
        return set_error(AFH_ERR_ARG, "plan: bad region");
      cells *= q[lo + 3 + d] - q[lo + d] + 1;
    }
    off[r + 1] = off[r] + cells;
    p.max_cells = std::max(p.max_cells, (int)cells);
  }
  p.n_values = off[n];
  AFH_HIP(hipMalloc(&p.d_reg, sizeof(int32_t) * w * std::max(n, 1)));
  AFH_HIP(hipMalloc(&p.d_off, sizeof(int64_t) * (n + 1)));
  if (n > 0)
    AFH_HIP(hipMemcpy(p.d_reg, reg, sizeof(int32_t) * w * n, hipMemcpyHostToDevice));
  AFH_HIP(hipMemcpy(p.d_off, off.data(), sizeof(int64_t) * (n + 1),
                    hipMemcpyHostToDevice));
  t->plans.push_back(p);
  *plan = (int32_t)t->plans.size() - 1;
  *n_values = p.n_values;
  return AFH_OK;
}

int32_t afh_plan_create(afh_tree *t, const int32_t *reg, int32_t n,
                        int32_t *plan, int64_t *n_values) {
  return plan_create(t, reg, n, plan, n_values, 0);
}

int32_t afh_plan_create_fc(afh_tree *t, const int32_t *reg, int32_t n,
                           int32_t *plan, int64_t *n_values) {
  return plan_create(t, reg, n, plan, n_values, 1);
}

static int32_t plan_copy(afh_tree *t, int32_t plan, int32_t iv, double *buf,
                         int unpack) {
  AFH_LIVE(t, "afh_plan_pack/unpack");
  if (!t || plan < 0 || plan >= (int)t->plans.size())
    return set_error(AFH_ERR_ARG, "afh_plan_pack/unpack: bad plan");
  const afh_tree::Plan &p = t->plans[plan];
  if (p.fc ? (iv < 1 || iv > t->nvf) : (iv < 0 || iv > t->nvc || (iv == 0 && !t->alt)))
    return set_error(AFH_ERR_ARG, "afh_plan_pack/unpack: bad variable");
  if (p.n == 0) return AFH_OK;
  // one block row per region, in chunks of the grid's 65535 rows (a plan
  // merges every peer's regions of an exchange)
  for (int r0 = 0; r0 < p.n; r0 += 65535) {
    const int nr = std::min(65535, p.n - r0);
    if (p.fc) {
      hipLaunchKernelGGL(k_plan_copy_fc, dim3((p.max_cells + 255) / 256, nr), dim3(256), 0,
                         t->stream, t->fcv(iv), buf, p.d_reg + 8 * (size_t)r0, p.d_off + r0,
                         t->nc + 1, t->fsz, unpack);
      AFH_LAUNCH_CHECK("k_plan_copy_fc");
    } else {
      hipLaunchKernelGGL(k_plan_copy, dim3((p.max_cells + 255) / 256, nr), dim3(256), 0,
                         t->stream, t->var(iv), buf, p.d_reg + 7 * (size_t)r0, p.d_off + r0,
                         t->ng, t->bsz, unpack);
      AFH_LAUNCH_CHECK("k_plan_copy");
    }
  }
  return AFH_OK;
}

int32_t afh_plan_pack(afh_tree *t, int32_t plan, int32_t iv, double *buf) {
  return plan_copy(t, plan, iv, buf, 0);
}

int32_t afh_plan_unpack(afh_tree *t, int32_t plan, int32_t iv,
                        const double *buf) {
  // a caller unpacking into phi or a species state: ghost cells and a fused
  // rhs derived from the old values are no longer current (the hook path
  // runs inside calls that touch the variable themselves)
  if (t && !t->retired && t->plans.size() > (size_t)std::max(plan, 0) &&
      !t->plans[plan].fc && iv > 0)
    t->touch(iv);
  return plan_copy(t, plan, iv, const_cast<double *>(buf), 1);
}

}  // extern "C"

// device id list for one launch (freed by the caller after a sync)
static int32_t device_list(const std::vector<int32_t> &h, int32_t **d) {
  AFH_HIP(hipMalloc(d, sizeof(int32_t) * std::max<size_t>(1, h.size())));
  if (!h.empty())
    AFH_HIP(hipMemcpy(*d, h.data(), sizeof(int32_t) * h.size(), hipMemcpyHostToDevice));
  return AFH_OK;
}

extern "C" {

int32_t afh_set_cc_prolong(afh_tree *t, int32_t iv, int32_t method, int32_t limiter) {
  if (t) t->meth_gen++;
  AFH_LIVE(t, "afh_set_cc_prolong");
  if (!t || iv < 1 || iv > t->nvc) return set_error(AFH_ERR_ARG, "bad variable index");
  if (method < AFH_PROLONG_NONE || method > AFH_PROLONG_LIMIT)
    return set_error(AFH_ERR_UNSUPPORTED, "prolongation method %d", method);
  if (!t->meth[iv].set) return set_error(AFH_ERR_STATE, "set cc methods first");
  if (method != AFH_PROLONG_NONE &&
      std::find(t->auto_vars.begin(), t->auto_vars.end(), iv) == t->auto_vars.end())
    t->auto_vars.push_back(iv);
  t->meth[iv].prolong = method;
  t->meth[iv].prolong_lim = limiter;
  return AFH_OK;
}

int32_t afh_tree_regrid(afh_tree *o, const afh_tree_desc *d, afh_tree **out) {
  if (!o || !d || !out) return set_error(AFH_ERR_ARG, "afh_tree_regrid: null");
  AFH_LIVE(o, "afh_tree_regrid");
  if (d->n_cell != o->nc || d->n_var_cell != o->nvc || d->n_var_face != o->nvf)
    return set_error(AFH_ERR_ARG, "afh_tree_regrid: box size / variables differ");
  if (o->hook) return set_error(AFH_ERR_UNSUPPORTED, "regrid of a sharded tree");
  afh_tree *t = nullptr;
  int32_t e;
  // in place when the new tree fits the old pools (box ids index them)
  const bool in_place = std::max(d->n_boxes, d->box_capacity) <= o->cap;
  const int nc = o->nc;
  // boxes that persist: same id, level and index in both topologies
  std::vector<char> in_old(o->nb + 1, 0), keep(d->n_boxes + 1, 0);
  for (const auto &L : o->h_ids)
    for (int32_t id : L) in_old[id] = 1;
  std::vector<int32_t> kept, rchild, fresh;
  for (int q = 0; q < d->lvl_ids_off[d->highest_lvl]; q++) {
      const int32_t id = d->lvl_ids[q];
      if (id < 1 || id > d->n_boxes) return set_error(AFH_ERR_ARG, "bad box id %d", id);
      if (id > o->nb || !in_old[id]) {
        fresh.push_back(id);
        continue;
      }
      const afh_box_meta &a = o->boxes[id - 1], &b = d->boxes[id - 1];
      if (a.lvl != b.lvl || a.ix[0] != b.ix[0] || a.ix[1] != b.ix[1] || a.ix[2] != b.ix[2]) {
        fresh.push_back(id);
        continue;
      }
      keep[id] = 1;
      kept.push_back(id);
      // auto_restrict (m_af_core.f90:826-840): the box lost its children
      if (a.children[0] > 0 && b.children[0] == 0)
        for (int c = 0; c < 8; c++) rchild.push_back(a.children[c]);
  }
  int32_t *d_list = nullptr;
  if (!rchild.empty()) {
    if ((e = device_list(rchild, &d_list))) return e;
    for (int iv : o->auto_vars)
      if ((e = restrict_boxes(o, d_list, (int)rchild.size(), iv))) return e;
  }
  AFH_HIP(hipStreamSynchronize(o->stream));
  hipFree(d_list);
  d_list = nullptr;
  if ((e = tree_create_impl(d, o->device, &t, in_place ? o : nullptr))) return e;
  t->meth = o->meth;
  t->auto_vars = o->auto_vars;
  if (in_place && !fresh.empty()) {
    // new boxes start at 0 in every variable (af_init_box, m_af_core.f90:556-557)
    if ((e = device_list(fresh, &d_list))) return e;
    const unsigned n = (unsigned)fresh.size();
    hipLaunchKernelGGL(k_copy_boxes, dim3((unsigned)((t->bsz + 255) / 256), n, t->nvc),
                       dim3(256), 0, t->stream, nullptr, t->cc, d_list, t->bsz,
                       (size_t)0, t->vstride);
    AFH_LAUNCH_CHECK("k_copy_boxes");
    if (t->nvf > 0) {
      hipLaunchKernelGGL(k_copy_boxes, dim3((unsigned)((t->fsz + 255) / 256), n, t->nvf),
                         dim3(256), 0, t->stream, nullptr, t->fc, d_list, t->fsz,
                         (size_t)0, (size_t)t->cap * t->fsz);
      AFH_LAUNCH_CHECK("k_copy_boxes");
    }
    AFH_HIP(hipStreamSynchronize(t->stream));
    hipFree(d_list);
    d_list = nullptr;
  }
  if (!in_place && !kept.empty()) {
    if ((e = device_list(kept, &d_list))) return e;
    const unsigned n = (unsigned)kept.size();
    hipLaunchKernelGGL(k_copy_boxes, dim3((unsigned)((t->bsz + 255) / 256), n, t->nvc),
                       dim3(256), 0, t->stream, o->cc, t->cc, d_list, t->bsz,
                       o->vstride, t->vstride);
    AFH_LAUNCH_CHECK("k_copy_boxes");
    if (t->nvf > 0) {
      hipLaunchKernelGGL(k_copy_boxes, dim3((unsigned)((t->fsz + 255) / 256), n, t->nvf),
                         dim3(256), 0, t->stream, o->fc, t->fc, d_list, t->fsz,
                         (size_t)o->cap * o->fsz, (size_t)t->cap * t->fsz);
      AFH_LAUNCH_CHECK("k_copy_boxes");
    }
    AFH_HIP(hipStreamSynchronize(t->stream));
    hipFree(d_list);
    d_list = nullptr;
  }
  // auto_prolong (m_af_core.f90:843-881): level by level, every automatic
  // variable of the new boxes, then their ghost cells (corners included)
  const int hn = nc / 2;
  for (int l = 2; l <= t->nlvl; l++) {
    std::vector<int32_t> add;
    for (int32_t id : t->h_ids[l - 1])
      if (!keep[id]) add.push_back(id);
    if (add.empty()) continue;
    if ((e = device_list(add, &d_list))) return e;
    const unsigned n = (unsigned)add.size();
    for (int iv : t->auto_vars) {
      const CcMethod &m = t->meth[iv];
      auto kern = m.prolong == AFH_PROLONG_LIMIT ? k_prolong_new<AFH_PROLONG_LIMIT>
                                                 : k_prolong_new<AFH_PROLONG_LINEAR>;
      hipLaunchKernelGGL(kern, dim3((hn * hn * hn + 255) / 256, n), dim3(256), 0,
                         t->stream, t->ccv(iv), t->d_boxes, d_list, nc, t->bsz,
                         m.prolong_lim);
      AFH_LAUNCH_CHECK("k_prolong_new");
    }
    for (int iv : t->auto_vars) {
      hipLaunchKernelGGL(k_gc_faces, dim3((nc * nc + 255) / 256, 6, n), dim3(256), 0,
                         t->stream, t->ccv(iv), t->ccv(iv), t->d_boxes, d_list, nc,
                         t->bsz, t->gc_args(iv));
      AFH_LAUNCH_CHECK("k_gc_faces");
      hipLaunchKernelGGL(k_gc_corners, dim3(n), dim3(fit_blk(12 * nc)), 0, t->stream, t->ccv(iv),
                         t->d_boxes, d_list, nc, t->bsz);
      AFH_LAUNCH_CHECK("k_gc_corners");
    }
    AFH_HIP(hipStreamSynchronize(t->stream));
    hipFree(d_list);
    d_list = nullptr;
  }
  *out = t;
  return AFH_OK;
}

}  // extern "C"

extern "C" {

/* Cell flags with the box summary (flag, mask) of afh_refine_flags, for the
 * driver's refinement routine (af_subr_ref) in af_adjust_refinement: a set
 * of cells asking for refinement whose cell_to_ref_flags result
 * (m_af_core.f90:1095-1148) is exactly (flag, mask); the other cells keep
 * (flag >= keep) or remove (flag = remove) the refinement. Per dimension a
 * cell index is in the low buffer slab, the high one, both or neither; one
 * representative cell per class combination whose neighbour slabs all lie in
 * the mask is marked when it adds a direction (or, for a box refining only
 * away from its sides, a cell in no slab). */
int32_t afh_refine_cell_flags(int32_t flag, uint32_t mask, int32_t nc, int32_t bw,
                               int32_t *cf) {
  if (nc < 1 || bw < 0 || bw > nc || !cf || flag < AFH_RM_REF || flag > AFH_DO_REF)
    return set_error(AFH_ERR_ARG, "refine_cell_flags: bad argument");
  const size_t n3 = (size_t)nc * nc * nc;
  for (size_t q = 0; q < n3; q++) cf[q] = flag == AFH_RM_REF ? AFH_RM_REF : AFH_KEEP_REF;
  if (flag != AFH_DO_REF) return mask ? set_error(AFH_ERR_ARG, "mask without refinement") : AFH_OK;
  int rep[4]; /* class -> first index (1-based) or 0; class = lo | hi << 1 */
  for (int c = 0; c < 4; c++) rep[c] = 0;
  for (int i = nc; i >= 1; i--) rep[(i <= bw) | ((i > nc - bw) << 1)] = i;
  uint32_t need = mask;
  int placed = 0;
  for (int pass = 0; pass < 2; pass++)
    for (int cz = 0; cz < 4; cz++)
      for (int cy = 0; cy < 4; cy++)
        for (int cx = 0; cx < 4; cx++) {
          if (!rep[cx] || !rep[cy] || !rep[cz]) continue;
          const int cl[3] = {cx, cy, cz};
          uint32_t mem = 0;
          for (int dk = -1; dk <= 1; dk++)
            for (int dj = -1; dj <= 1; dj++)
              for (int di = -1; di <= 1; di++) {
                if (!di && !dj && !dk) continue;
                const int dd[3] = {di, dj, dk};
                int in = 1;
                for (int d = 0; d < 3; d++)
                  in = in && (dd[d] == 0 || (cl[d] & (dd[d] < 0 ? 1 : 2)));
                if (in) mem |= 1u << ((dk + 1) * 9 + (dj + 1) * 3 + (di + 1));
              }
          if ((mem & ~mask) != 0) continue;
          /* pass 0: cells that add a direction; pass 1: any cell if none yet */
          if (pass == 0 ? (mem & need) == 0 : placed) continue;
          cf[((size_t)(rep[cz] - 1) * nc + (rep[cy] - 1)) * nc + (rep[cx] - 1)] = AFH_DO_REF;
          need &= ~mem;
          placed = 1;
        }
  if (need || !placed) return set_error(AFH_ERR_ARG, "refine_cell_flags: inconsistent mask");
  return AFH_OK;
}

}  // extern "C"
