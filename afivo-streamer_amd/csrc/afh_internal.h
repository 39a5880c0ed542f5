// Internal declarations shared by the HIP translation units of libafivo_hip.
//
// Device layout (HBM):
//   cc pool  [iv][box][k][j][i], (nc+2)^3 doubles per box, i fastest: each
//            box of a variable is the exact image of the Fortran array
//            box%cc(0:nc+1,0:nc+1,0:nc+1,iv), boxes contiguous per variable.
//   fc pool  [ivf][box][dim][k][j][i], (nc+1)^3 per dim (box%fc layout).
//   meta     afh_box_meta[n_boxes] (topology), per-level id lists.
// All kernels evaluate floating-point expressions in the order the reference
// Fortran writes them; the library is compiled with -ffp-contract=off so the
// results are bitwise those of the C oracle (oracle/c/afo.c).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <string>
#include <array>
#include <vector>
#include <map>
#include <mutex>
#include <utility>

#include "../../include/afivo_hip.h"

namespace afh {

int32_t set_error(int32_t code, const char *fmt, ...);
int32_t check_hip(hipError_t e, const char *what);
// Data pools (cc, fc, gc2, the spare image). (Round 4's placement
// experiments -- contiguous allocations, padding between variables, an
// offset spare image -- changed nothing measurable and were removed.)
int32_t pool_alloc(void **p, size_t bytes, const char *what);
#define AFH_HIP(call)                                                         \
  do {                                                                        \
    hipError_t _e = (call);                                                   \
    if (_e != hipSuccess) return ::afh::check_hip(_e, #call);                 \
  } while (0)
#define AFH_LAUNCH_CHECK(what)                                                \
  do {                                                                        \
    hipError_t _e = hipGetLastError();                                        \
    if (_e != hipSuccess) return ::afh::check_hip(_e, what);                  \
  } while (0)

struct CcMethod {
  int set = 0;
  afh_bc bc[6];
  int rb = AFH_RB_GC_INTERP;
  int lim = AFH_LIM_GMINMOD43;
  int prolong = AFH_PROLONG_NONE;  // afh_set_cc_prolong
  int prolong_lim = AFH_LIM_GMINMOD43;
};

// Per-variable methods as the kernels see them (passed by value).
struct GcArgs {
  afh_bc bc[6];
  int rb;
  int lim;
};

struct LevelList {
  std::vector<int32_t> off;  // highest_lvl + 1 offsets
  int32_t *d = nullptr;      // device, concatenated 1-based ids
  int n(int lvl) const { return off[lvl] - off[lvl - 1]; }
  const int32_t *at(int lvl) const { return d + off[lvl - 1]; }
};

}  // namespace afh

struct afh_tree {
  int device = 0;
  hipStream_t stream = nullptr;
  int nc = 0, ng = 0, nb = 0, nlvl = 0, nvc = 0, nvf = 0;
  int cap = 0;  // boxes the data pools hold (variable stride), >= nb
  size_t bsz = 0, fsz = 0;
  int cgs[3] = {0, 0, 0};
  double r_base[3], dr_base[3];
  std::vector<afh_box_meta> boxes;  // host copy
  afh_box_meta *d_boxes = nullptr;
  afh::LevelList ids, leaves, parents;
  std::vector<std::vector<int32_t>> h_ids, h_leaves, h_parents;
  // leaves next to a refinement boundary, per level (af_restrict_ref_boundary)
  afh::LevelList refb;
  // (parent id, nb) tasks of af_consistent_fluxes, per level
  afh::LevelList cflux;
  // af_consistent_fluxes has a task anywhere in the whole topology (all
  // ranks): the fused forward-Euler kernel needs every face flux final
  bool any_cflux = false;
  double *cc = nullptr, *fc = nullptr;
  double *gc2 = nullptr;     // 2nd ghost layer for the flux: [box][6][nc][nc]
  double *scratch = nullptr; // reductions etc.
  // reduction slots (red_init / red_finish): a fold leaves the slot's shards
  // at its canonical start value, so the next red_init with that value needs
  // no fill launch
  uint64_t red_canon[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  bool red_ready[8] = {false, false, false, false, false, false, false, false};
  double *h_scratch = nullptr;
  std::vector<afh::CcMethod> meth;
  std::vector<int> auto_vars;  // tree%cc_auto_vars (afh_set_cc_prolong order)
  // grid spacing per level (afivo halves dr exactly per level, so every box
  // of a level has the same bits; verified at tree creation)
  std::vector<double> lvl_dr;  // 3 per level
  std::vector<int> lvl_total;  // boxes per level over all ranks (topology)
  std::vector<int> lvl_leaves_total;  // leaves per level over all ranks
  // level l+1 has a refinement boundary (a face without same-level neighbour)
  std::vector<int> lvl_rb_coarse;
  bool own_stream = true;
  // kernel timing (afh_profile_*)
  int prof_class = 0;
  std::vector<hipEvent_t> ev_pool;
  size_t ev_used = 0;
  double prof_bytes = 0;
  int64_t prof_launches = 0;
  // box sharding (afh_tree_set_hook, afh_plan_*): exchange hook, the
  // smoother's spare phi image (variable 0 in hooks and plans), plans
  afh_hook_fn hook = nullptr;
  void *hook_ctx = nullptr;
  // sharded over RCCL (afh_dist_create): MAX / MIN of the reduction slots are
  // all-reduced on the device, on the ordered keys in place (stream-ordered,
  // no host round trip); the one fetch afterwards reads the global value
  int32_t (*dev_reduce)(void *ctx, int kind, unsigned long long *keys, int n) = nullptr;
  // and the SUM of afh_tree_sum_cc (a double on the device, summed in place)
  int32_t (*dev_sum)(void *ctx, double *val) = nullptr;
  // the hook's exchanges are stream operations only (RCCL): a V-cycle may be
  // captured with them inside (AFH_RCCL_CAPTURE)
  bool hook_capturable = false;
  // side streams of concurrent multigrid solves (afh_photoi_helmh_compute:
  // one per Helmholtz mode) and their fork / join events, created on use
  hipStream_t side[4] = {nullptr, nullptr, nullptr, nullptr};
  hipEvent_t side_ev[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
  // afh_tree_sum_cc on the device: per leaf (level order) the level's cell
  // volume, or 0 where sum_skip drops the box (built on first use)
  double *d_sumw = nullptr;
  int sumw_n = -1;
  // segmented capture of a sharded V-cycle (afh_mg.hip vcycle_graph): while
  // seg_rec is set the stream is capturing, and call_hook ends the capture at
  // each exchange, records the exchange and begins the next segment; a
  // reduction (host values) marks the recording unusable
  struct SegRec {
    std::vector<hipGraph_t> graphs;
    std::vector<std::array<int32_t, 4>> ops;  // (kind, level, iv, n) after graphs[k]
    bool bad = false;
  };
  SegRec *seg_rec = nullptr;
  // shared by every multigrid on the tree (one stream: the image is only
  // live inside one fused pair); freed with the last of them
  double *alt = nullptr;
  int alt_of = 0;  // the variable whose image alt holds (its ghost-cell methods)
  int alt_refs = 0;
  // independent per-box work of every leaf level in one launch where the
  // kernel reads the box's level data from its meta record (flux of small
  // boxes, density update, residual; AFH_ALL_LVL=0: one launch per level)
  bool all_lvl_launch = true;
  struct Plan {
    int32_t *d_reg = nullptr;  // n x 7 (id, lo[3], hi[3])
    int64_t *d_off = nullptr;  // n + 1 value offsets
    int n = 0, max_cells = 0;
    int64_t n_values = 0;
    int fc = 0;                // face-variable plan (8 ints per region)
  };
  std::vector<Plan> plans;
  // afh_tree_regrid in place handed this tree's pools to the new tree: every
  // entry point on this handle (or on a fluid / multigrid bound to it) fails
  bool retired = false;
  // write generation of every cc variable, bumped by the public calls that
  // may change it (afh_fluid_rhs_valid: is a fused rhs still current?)
  std::vector<uint64_t> gen;
  // bumped by afh_set_cc_methods / afh_set_cc_prolong: graphs captured with
  // the old boundary values are replayed no more
  uint64_t meth_gen = 0;
  void touch(int iv) {
    if (iv >= 0 && iv < (int)gen.size()) gen[iv]++;
  }
  // per-box partial results of afh_tree_sum_cc / afh_tree_reduce_loc
  double *d_boxred = nullptr;
  int boxred_cap = 0;
  // sharded tree: boxes whose leaf sum another rank contributes (the
  // replicated levels below the partition level count on rank 0 only);
  // empty on an unsharded tree
  std::vector<char> sum_skip;

  // cc variable stride (doubles): cap * bsz
  size_t vstride = 0;
  double *alt_base = nullptr;  // allocation of alt (alt = alt_base)
  double *ccv(int iv) const { return cc + (size_t)(iv - 1) * vstride; }
  // cc variable iv, or the smoother's spare image of phi for iv == 0
  double *var(int iv) const { return iv == 0 ? alt : ccv(iv); }
  double *fcv(int ivf) const { return fc + (size_t)(ivf - 1) * cap * fsz; }
  afh::GcArgs gc_args(int iv) const {
    afh::GcArgs a;
    for (int n = 0; n < 6; n++) a.bc[n] = meth[iv].bc[n];
    a.rb = meth[iv].rb;
    a.lim = meth[iv].lim;
    return a;
  }
};

namespace afh {
// entry-point guard: a null or retired tree handle is an error
// Workgroup lanes for a per-box launch of `work` items: the work rounded up
// to whole waves, at most 256 (an 8^3 box's 64-cell face or 96 edge cells
// without the idle waves of a 256-lane workgroup).
inline int fit_blk(int work) {
  return work < 256 ? ((work + 63) / 64) * 64 : 256;
}

// hipFuncAttributeMaxDynamicSharedMemorySize is per kernel (and device), not
// per object: several multigrids in one process each need their own LDS size,
// so the limit is only ever raised
inline hipError_t raise_dyn_lds(const void *f, int bytes) {
  static std::mutex m;
  static std::map<std::pair<int, const void *>, int> top;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  std::lock_guard<std::mutex> g(m);
  int &cur = top[{dev, f}];
  if (bytes <= cur) return hipSuccess;
  e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  if (e == hipSuccess) cur = bytes;
  return e;
}

inline int32_t live(const afh_tree *t, const char *what) {
  if (!t) return set_error(AFH_ERR_ARG, "%s: null tree", what);
  if (t->retired)
    return set_error(AFH_ERR_STATE,
                     "%s: tree handle retired by an in-place afh_tree_regrid", what);
  return AFH_OK;
}
#define AFH_LIVE(t, what)                                                     \
  do {                                                                        \
    int32_t _e = ::afh::live((t), (what));                                     \
    if (_e) return _e;                                                        \
  } while (0)
// per-level id lists -> one device array with offsets (frees L's old array)
int32_t upload_list(afh_tree *t, LevelList &L,
                    const std::vector<std::vector<int32_t>> &lists);
// Kernel timing: bracket one launch of class `kc` (no-op unless enabled).
void prof_begin(afh_tree *t, int kc);
void prof_end(afh_tree *t, int kc, double bytes);
// or: a start / end event pair for a launch that records them itself
// (hipExtLaunchKernelGGL; false: class not timed), then prof_count
bool prof_ext(afh_tree *t, int kc, hipEvent_t &e0, hipEvent_t &e1);
void prof_count(afh_tree *t, double bytes);
// Host launchers shared between translation units (afh_tree.hip).
int32_t gc_lvl(afh_tree *t, int lvl, int iv, int corners, bool rims = false, int depth = 2);
// ghost fill of level lvl of variable iv (0: the spare phi image), with the
// coarse data of refinement boundaries read from vc; calls the sharding
// hooks: HALO before, RIMS after when `rims` (the fused smoother reads the
// replicas' ghost cells next) or when the next level has refinement
// boundaries (its ghost cells read this level's replicas, ghosts included)
// depth: the replica layers the next reader of the level needs (2: a fused
// pair follows -- it recomputes neighbours' boundary cells --, 1: only
// ghost cells are read), handed to the hooks as their n
// xrim: the x ghost cells facing same-level neighbours are current except
// on rows 1, nc and planes 1, nc (k_gsrb_pair2<..., XR> stored them): only
// those are filled
int32_t gc_lvl_var(afh_tree *t, int lvl, int iv, const double *vc,
                   const GcArgs &ga, int corners, bool rims = false, int depth = 2);
// edges and corners only of level lvl (k_gc_corners), for a level whose
// faces a producer kernel filled (the fused pair's pushed faces)
int32_t gc_lvl_corners(afh_tree *t, int lvl, int iv);
// sharding hook (no-op without one)
int32_t call_hook(afh_tree *t, int kind, int lvl, int iv, double *vals = nullptr,
                  int n = 0);
int32_t restrict_boxes(afh_tree *t, const int32_t *d_ids, int n, int iv);
// Sharded max/min reductions: each block folds its value into one of
// RED_SHARDS words of a slot (no single-address contention), a one-block
// kernel folds the shards. Slots: 0 cfl, 1 conductivity, 2 chemistry dt,
// 3 maxabs.
constexpr int RED_SHARDS = 1024;
constexpr int RED_SLOTS = 8;
int32_t red_init(afh_tree *t, int slot, double v);
int32_t red_finish(afh_tree *t, int slot, bool is_max);
int32_t red_finish_n(afh_tree *t, int n, const int *slots, const bool *is_max);
// fetch the folded values of `n` consecutive slots starting at `slot`
int32_t red_fetch(afh_tree *t, int slot, int n, double *out);
// the folded values of slots slot .. slot+n_max-1 (maxima) and the next
// n_min (minima), reduced over the ranks of a sharded tree: on the device
// before the fetch (dev_reduce), or through the host hook after it
// several folded slots in one transfer (sharded: all-reduced first)
int32_t red_fetch_slots(afh_tree *t, int n, const int32_t *slots, double *out);
int32_t red_reduce_fetch(afh_tree *t, int slot, int n_max, int n_min, double *out,
                         int iv = 0, int level = 0);
__device__ __forceinline__ int red_shard() {
  return (int)((blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z)) &
               (RED_SHARDS - 1));
}
// Orderable encoding of doubles for atomicMax/Min on 64-bit integers.
__device__ __forceinline__ unsigned long long dbl_to_ord(double x) {
  unsigned long long u = __double_as_longlong(x);
  return (u & 0x8000000000000000ull) ? ~u : (u | 0x8000000000000000ull);
}
// Fold a per-thread max into shard red_shard() of `red` (one atomic per
// workgroup; blockDim.x a multiple of 64, at most 1024). Every thread calls.
__device__ __forceinline__ void block_max_to_shard(double v,
                                                   unsigned long long *red) {
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  __shared__ double s_red[16];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) s_red[w] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int q = 1; q < (int)(blockDim.x >> 6); q++) v = fmax(v, s_red[q]);
    atomicMax(&red[red_shard()], dbl_to_ord(v));
  }
}
inline double ord_to_dbl(unsigned long long o) {
  unsigned long long u =
      (o & 0x8000000000000000ull) ? (o & ~0x8000000000000000ull) : ~o;
  double d;
  memcpy(&d, &u, sizeof d);
  return d;
}
inline unsigned long long host_dbl_to_ord(double x) {
  unsigned long long u;
  memcpy(&u, &x, sizeof u);
  return (u & 0x8000000000000000ull) ? ~u : (u | 0x8000000000000000ull);
}

// A store of a kernel's output, streaming (nontemporal: no reuse expected
// before eviction) when NT. The big per-level outputs are read back only by
// the next kernel, from HBM anyway (a leaf level is GBs, the L2 + MALL a few
// hundred MB). Per-kernel-class switches (-DAFH_NT_*=0 for plain stores),
// measured with scripts/grad_ab.py / scripts/ab_bench.sh: S1-64 14.1-14.9
// -> 13.9 ms/step over three alternating rounds:
#ifndef AFH_NT_FLUX
#define AFH_NT_FLUX 1
#endif
#ifndef AFH_NT_UPD
#define AFH_NT_UPD 1
#endif
#ifndef AFH_NT_PAIR
#define AFH_NT_PAIR 1
#endif
#ifndef AFH_NT_MG
#define AFH_NT_MG 1
#endif
template <bool NT>
__device__ __forceinline__ void st_nt(double *p, double v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// Workgroup b of n -> work item: workgroups are dispatched round-robin over
// the 8 XCDs (b % 8); this gives each XCD a contiguous run of work items
// (bijective for any n), so neighbouring boxes of a level list share an L2.
__device__ __forceinline__ int xcd_swizzle(int b, int n) {
  const int q = n >> 3, r = n & 7, x = b & 7, slot = b >> 3;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + slot;
}

// A 2-D grid (the blocks of a box in x, the boxes of a level list in y)
// remapped by xcd_swizzle: the blocks of a box run on one XCD, in order, so
// the planes and rows that neighbouring blocks both read meet in one L2.
// Used where it measured faster (k_gradient_t -8 %; k_flux_lds's 1-D tiles
// -1 %); k_update, k_residual, k_prolong and k_rstr_fas measured 2-8 %
// slower with it (scripts/ab_kernels.sh) and keep the hardware order.
struct Blk {
  int x, y;
};
__device__ __forceinline__ Blk xcd_block() {
  const int gx = gridDim.x;
  const int w = xcd_swizzle(blockIdx.y * gx + blockIdx.x, gx * gridDim.y);
  return {w % gx, w / gx};
}

__device__ __forceinline__ size_t ix3(int ng, int i, int j, int k) {
  return ((size_t)k * ng + j) * ng + i;
}

// af_limiter_apply (m_af_limiters.f90:41-149)
__device__ __forceinline__ double limiter(int lim, double a, double b) {
  const double third = 1 / 3.0;
  switch (lim) {
  case AFH_LIM_KOREN: {
    const double aa = a * a, ab = a * b;
    if (ab <= 0) return 0;
    if (aa <= 0.25 * ab) return 2 * a;
    if (aa <= 2.5 * ab) return third * (b + 2 * a);
    return 2 * b;
  }
  case AFH_LIM_VANLEER: {
    const double ab = a * b;
    return ab > 0 ? 2 * ab / (a + b) : 0;
  }
  case AFH_LIM_NONE: return 0.5 * (a + b);
  case AFH_LIM_ZERO: return 0.0;
  default: {
    const double th =
        lim == AFH_LIM_MINMOD ? 1.0 : lim == AFH_LIM_MC ? 2.0 : 4 / 3.0;
    if (a * b > 0) {
      double m = fabs(th * a);
      const double y = fabs(th * b), z = fabs(0.5 * (a + b));
      if (y < m) m = y;
      if (z < m) m = z;
      return copysign(m, a);
    }
    return 0.0;
  }
  }
}

// Linear index t -> (i, j, k), 1-based, of an n x n x n block, i fastest.
// n is uniform (a kernel argument): powers of two (every afivo box size in
// practice) decode with shifts computed in scalar registers; others divide.
__device__ __forceinline__ void cell3(int t, int n, int &i, int &j, int &k) {
  if ((n & (n - 1)) == 0) {
    const int ln = __builtin_ctz(n);
    i = (t & (n - 1)) + 1;
    j = ((t >> ln) & (n - 1)) + 1;
    k = (t >> (2 * ln)) + 1;
  } else {
    i = t % n + 1;
    j = (t / n) % n + 1;
    k = t / (n * n) + 1;
  }
}

// t -> (i, j, k), 0-based, of an ng^3 block (ng = nc + 2, not a power of
// two): float quotient corrected by one step (exact for t < 2^24)
__device__ __forceinline__ int divg(int t, int ng, float inv) {
  int q = (int)((float)t * inv);
  q -= (q * ng > t) ? 1 : 0;
  q += ((q + 1) * ng <= t) ? 1 : 0;
  return q;
}
__device__ __forceinline__ void cell3g(int t, int ng, int &i, int &j, int &k) {
  const float inv = 1.0f / (float)ng;
  const int q = divg(t, ng, inv);
  i = t - q * ng;
  k = divg(q, ng, inv);
  j = q - k * ng;
}

// Face ghost cell p (p[d] = 0 or nc+1, d = dim of face nb) of box m when the
// face has no same-level neighbour (bc: the face's boundary condition, rb:
// the refinement-boundary method): physical boundary (bc_to_gc,
// m_af_ghostcell.f90:173-279) or refinement boundary (mg_sides_rb,
// m_af_multigrid.f90:294-461; af_gc_interp / af_gc_interp_lim,
// m_af_ghostcell.f90:394-612). `own(q)` returns the box's current value at
// interior cell q; coarse data are read from v (the parent's neighbour).
// nb_id / drd: the face's neighbour id and the box's spacing along the
// face normal, passed in by kernels that hold them in registers (no
// per-lane metadata load in their hot loop).
template <class Own>
__device__ __forceinline__ double gc_face_nocopy_k(
    const double *__restrict__ v, const afh_box_meta *__restrict__ meta,
    const afh_box_meta &m, int nb, int nb_id, double drd, const int p[3], int a,
    int b, int nc, size_t bsz, afh_bc bc, int rb, Own own) {
  const int d = (nb - 1) >> 1;
  const bool low = ((nb - 1) & 1) == 0;
  const int ta = (d == 0) ? 1 : 0, tb = (d == 2) ? 1 : 2;
  const int ng = nc + 2;
  const int x1 = low ? 1 : nc;
  const int x2 = low ? 2 : nc - 1;
  int q1[3] = {p[0], p[1], p[2]}, q2[3] = {p[0], p[1], p[2]};
  q1[d] = x1;
  q2[d] = x2;
  if (nb_id < 0) {
    double c0, c1, c2;
    switch (bc.type) {
    case AFH_BC_DIRICHLET: c0 = 2; c1 = -1; c2 = 0; break;
    case AFH_BC_NEUMANN: c0 = drd * (low ? -1 : 1); c1 = 1; c2 = 0; break;
    case AFH_BC_CONTINUOUS: c0 = 0; c1 = 2; c2 = -1; break;
    default: c0 = 1; c1 = 0; c2 = 0; break;
    }
    return c0 * bc.value + c1 * own(q1) + c2 * own(q2);
  }
  // refinement boundary: coarse data from the parent's neighbour
  const int p_id = m.parent;
  const int p_nb_id = meta[p_id - 1].neighbors[nb - 1];
  const double *cp = v + (size_t)(p_nb_id - 1) * bsz;
  const int hnc = nc >> 1;
  int co[3];
  for (int q = 0; q < 3; q++) co[q] = ((m.ix[q] - 1) & 1) * hnc;

  if (rb == AFH_RB_MG_SIDES) {
    // tmp(x, y) = coarse value next to the face, at tangential offsets co;
    // gc = tmp +- g1 +- g2; ghost = 0.5 gc + 0.75 x_i - 0.25 x_i+d
    const int cn = low ? nc : 1;
    const int ii = (a + 1) >> 1, jj = (b + 1) >> 1;
    auto tmp = [&](int x, int y) {
      int q[3];
      q[d] = cn;
      q[ta] = co[ta] + x;
      q[tb] = co[tb] + y;
      return cp[ix3(ng, q[0], q[1], q[2])];
    };
    const double g1 = 0.125 * (tmp(ii + 1, jj) - tmp(ii - 1, jj));
    const double g2 = 0.125 * (tmp(ii, jj + 1) - tmp(ii, jj - 1));
    const double t0 = tmp(ii, jj);
    double gcv;
    if (a & 1) {
      gcv = (b & 1) ? t0 - g1 - g2 : t0 - g1 + g2;
    } else {
      gcv = (b & 1) ? t0 + g1 - g2 : t0 + g1 + g2;
    }
    return 0.5 * gcv + 0.75 * own(q1) - 0.25 * own(q2);
  }
  // af_gc_interp / af_gc_interp_lim; offsets on the parent's neighbour
  const double third = 1 / 3.0, sixth = 1 / 6.0;
  int off[3] = {co[0], co[1], co[2]};
  off[d] -= (low ? -1 : 1) * nc;
  const int ix_c = low ? nc : 1;
  const int a1 = off[ta] + ((a + 1) >> 1), a2 = a1 + 1 - 2 * (a & 1);
  const int b1 = off[tb] + ((b + 1) >> 1), b2 = b1 + 1 - 2 * (b & 1);
  int q[3];
  q[d] = ix_c;
  q[ta] = a1, q[tb] = b1;
  const double cv1 = cp[ix3(ng, q[0], q[1], q[2])];
  double cv2, cv3;
  if (d < 2) {
    q[ta] = a2, q[tb] = b1;
    cv2 = cp[ix3(ng, q[0], q[1], q[2])];
    q[ta] = a1, q[tb] = b2;
    cv3 = cp[ix3(ng, q[0], q[1], q[2])];
  } else {
    // case (3): c(2) uses j_c2 and c(3) uses i_c2 (m_af_ghostcell.f90:479-482)
    q[ta] = a1, q[tb] = b2;
    cv2 = cp[ix3(ng, q[0], q[1], q[2])];
    q[ta] = a2, q[tb] = b1;
    cv3 = cp[ix3(ng, q[0], q[1], q[2])];
  }
  double val = third * cv1 + sixth * cv2 + sixth * cv3 + third * own(q1);
  if (rb == AFH_RB_GC_INTERP_LIM && val > 2 * cv1) val = 2 * cv1;
  return val;
}

template <class Own>
__device__ __forceinline__ double gc_face_nocopy(
    const double *__restrict__ v, const afh_box_meta *__restrict__ meta,
    const afh_box_meta &m, int nb, const int p[3], int a, int b, int nc,
    size_t bsz, afh_bc bc, int rb, Own own) {
  return gc_face_nocopy_k(v, meta, m, nb, m.neighbors[nb - 1], m.dr[(nb - 1) >> 1], p,
                          a, b, nc, bsz, bc, rb, own);
}
}  // namespace afh
