// mcpt_upload.hip — SceneBuild::buildScene's device side built ON the GPU:
// every structure mcpt_scene_upload derives on the host (mcpt_device.hip,
// mcpt_sah.cpp), from a scene already in HBM, bit-identical to the host path.
//
//  * validation (links, material ids, finite vertices) and the reference
//    traversal's stack bound (mcpt_bvh_stack_depth), by depth levels;
//  * the binary child-box nodes (DevNode) and the reference tree collapsed
//    4-wide (DevNode4, breadth-first ids, per-node stack need);
//  * the EXACT path's search tree, mcpt_sah.cpp's algorithm step for step:
//    32-bin SAH splits (double costs, first strict minimum in (axis asc, bin
//    desc) order), stable partitions, node ranges laid out by (lo, hi, base)
//    exactly as Builder::build does, boxes as the host's left-then-right
//    unions, the SAH-optimal 4-wide collapse DP and its preorder emission
//    with the host's allocation order of node ids, its stack need;
//  * the quantized nodes (quantize_node4, whose loops pick the extremal
//    codes, so any initial estimate gives the host's bytes), the triangle
//    records with their Cramer minors.
// Large ranges split level by level with workgroup-local bins merged by
// atomics (min/max and counts: order-free); ranges of <= kSmall leaves are
// finished by one wave each, in LDS.  Compiled with the host's float semantics
// (-ffp-contract=off, IEEE division): Makefile BUILDFLAGS.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/mcpt_hip.h"
#include "mcpt_bvh4.h"
#include "mcpt_upload.h"

namespace mcpt {
int fail(int code, const std::string &msg);  // mcpt_host.cpp
int tree_levels(const mcpt_bvh_node *nodes, int64_t n, hipStream_t st, int32_t *lv, uint32_t *cnt,
                std::vector<uint32_t> &off);  // mcpt_build.hip
}  // namespace mcpt

namespace {

using mcpt::kEmptySlot4;
constexpr int NB = 32;                 // mcpt_sah.cpp split(): bins per axis
constexpr int kSmall = 1024;           // ranges at most this long: one wave builds the subtree (k_small)
constexpr double C_STEP = 1.0, C_TRI = 1.7;  // mcpt_sah.cpp collapse costs (MCPT_COLLAPSE_CTRI)

__device__ __host__ inline float smin(float a, float b) { return (b < a) ? b : a; }  // std::min(a, b)
__device__ __host__ inline float smax(float a, float b) { return (a < b) ? b : a; }  // std::max(a, b)

// order-preserving float <-> uint (for atomic min / max; -0 below +0)
__device__ inline uint32_t f2o(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ inline float o2f(uint32_t o) { return __uint_as_float((o & 0x80000000u) ? (o & 0x7FFFFFFFu) : ~o); }

__device__ inline double area6(const float *b) {  // Builder::area
  const double dx = (double)b[1] - b[0], dy = (double)b[3] - b[2], dz = (double)b[5] - b[4];
  if (dx < 0) return 0.0;
  return 2.0 * (dx * dy + dy * dz + dz * dx);
}
__device__ inline void empty6(float *b) {
  for (int a = 0; a < 3; ++a) b[2 * a] = FLT_MAX, b[2 * a + 1] = -FLT_MAX;
}
__device__ inline void grow6(float *b, const float *x) {  // Builder::grow
  for (int a = 0; a < 3; ++a) {
    b[2 * a] = smin(b[2 * a], x[2 * a]);
    b[2 * a + 1] = smax(b[2 * a + 1], x[2 * a + 1]);
  }
}

// ------------------------------------------------------------ the records
struct __attribute__((aligned(16))) UDevNode {  // DevNode: child boxes + links
  float a[4], b[4], c[4];
  int32_t left, right, pad0, pad1;
};
struct __attribute__((aligned(16))) UDevTri {  // DevTri / DevTriQ
  float v0[4], v1[4], v2[4], nrm[4];
};
static_assert(sizeof(UDevNode) == 64 && sizeof(UDevTri) == 64, "64-B records");

// ------------------------------------------------------- scene checks
// flags: bit 0 negative child, 1 leaf triangle out of range, 2 child out of
// range, 3 material id, 4 non-finite vertex, 5 not the HLBVH layout
__global__ void k_check(const mcpt_bvh_node *__restrict__ nodes, const mcpt_triangle *__restrict__ tris, int64_t n,
                        int32_t n_mats, uint32_t *flags) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t f = 0;
  if (i < 2 * n - 1) {
    const mcpt_bvh_node &b = nodes[i];
    if (b.left < 0 || b.right < 0) f |= 1;
    else if (b.left == b.right) f |= (b.left >= n ? 2 : 0) | (i < n - 1 ? 32 : 0);
    else f |= (b.left >= 2 * n - 1 || b.right >= 2 * n - 1 ? 4 : 0) | (i >= n - 1 ? 32 : 0);
  }
  if (i < n) {
    const mcpt_triangle &t = tris[i];
    const int32_t m = __float_as_int(t.normal[3]);
    if (m < 0 || m >= n_mats) f |= 8;
    for (int k = 0; k < 3; ++k)
      for (int j = 0; j < 3; ++j)
        if (!isfinite(t.v[k][j])) f |= 16;
  }
  if (f) atomicOr(flags, f);
}

// left-first DFS stack bound: d(left) = d + 1, d(right) = d; bound = max d + 1
__global__ void k_stack_depth(const int32_t *__restrict__ lvl, uint32_t count, const mcpt_bvh_node *__restrict__ nodes,
                              int32_t *d, uint32_t *best) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const int32_t x = lvl[i];
  const mcpt_bvh_node &b = nodes[x];
  const int32_t dx = d[x];
  d[b.left] = dx + 1;
  d[b.right] = dx;
  // leaf children end a path: their own entry counts (best = max(d + 1))
  uint32_t m = (uint32_t)dx + 1u;
  if (nodes[b.left].left == nodes[b.left].right) m = max(m, (uint32_t)dx + 2u);
  atomicMax(best, m);
}

// DevNode per internal node (remap = identity on the HLBVH layout)
__global__ void k_devnodes(const mcpt_bvh_node *__restrict__ nodes, int64_t n, UDevNode *out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n - 1) return;
  const mcpt_bvh_node &b = nodes[i], &L = nodes[b.left], &R = nodes[b.right];
  UDevNode d;
  d.a[0] = L.bbmin[0], d.a[1] = L.bbmax[0], d.a[2] = L.bbmin[1], d.a[3] = L.bbmax[1];
  d.b[0] = L.bbmin[2], d.b[1] = L.bbmax[2], d.b[2] = R.bbmin[0], d.b[3] = R.bbmax[0];
  d.c[0] = R.bbmin[1], d.c[1] = R.bbmax[1], d.c[2] = R.bbmin[2], d.c[3] = R.bbmax[2];
  d.left = L.left == L.right ? ~L.left : b.left;
  d.right = R.left == R.right ? ~R.left : b.right;
  d.pad0 = d.pad1 = 0;
  out[i] = d;
}

// triangles: DevTri (Cramer rows and minors) and DevTriQ; leaf boxes vs vertex bounds
__global__ void k_tris(const mcpt_triangle *__restrict__ tris, int64_t n, UDevTri *dt, UDevTri *tq) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const mcpt_triangle &t = tris[i];
  const float b1 = -(t.v[1][0] - t.v[0][0]), b2 = -(t.v[1][1] - t.v[0][1]), b3 = -(t.v[1][2] - t.v[0][2]);
  const float c1 = -(t.v[2][0] - t.v[0][0]), c2 = -(t.v[2][1] - t.v[0][1]), c3 = -(t.v[2][2] - t.v[0][2]);
  const float m0 = fmaf(b2, c3, -(c2 * b3)), m1 = fmaf(b1, c3, -(c1 * b3)), m2 = fmaf(b1, c2, -(c1 * b2));
  UDevTri d;  // DevTri: the normal's xyz in the .w lanes, aux = (material bits, minors)
  d.v0[0] = t.v[0][0], d.v0[1] = t.v[0][1], d.v0[2] = t.v[0][2], d.v0[3] = t.normal[0];
  d.v1[0] = b1, d.v1[1] = b2, d.v1[2] = b3, d.v1[3] = t.normal[1];
  d.v2[0] = c1, d.v2[1] = c2, d.v2[2] = c3, d.v2[3] = t.normal[2];
  d.nrm[0] = t.normal[3], d.nrm[1] = m0, d.nrm[2] = m1, d.nrm[3] = m2;
  dt[i] = d;
  UDevTri q;
  for (int k = 0; k < 3; ++k) q.v0[k] = t.v[0][k], q.v1[k] = t.v[1][k], q.v2[k] = t.v[2][k];
  q.v0[3] = m0, q.v1[3] = m1, q.v2[3] = m2;
  for (int k = 0; k < 4; ++k) q.nrm[k] = t.normal[k];
  tq[i] = q;
}
__global__ void k_leafbox_check(const mcpt_bvh_node *__restrict__ nodes, const mcpt_triangle *__restrict__ tris,
                                int64_t n, uint32_t *flags) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const mcpt_bvh_node &b = nodes[n - 1 + i];
  const mcpt_triangle &t = tris[b.left];
  for (int a = 0; a < 3; ++a) {
    const float lo = smin(smin(t.v[0][a], t.v[1][a]), t.v[2][a]);
    const float hi = smax(smax(t.v[0][a], t.v[1][a]), t.v[2][a]);
    if (!(b.bbmin[a] == lo && b.bbmax[a] == hi)) {
      atomicOr(flags, 64u);
      return;
    }
  }
}

// ------------------------------------------- the reference tree, 4-wide
// one breadth-first level of 4-wide nodes: slot children counted, then placed
__device__ inline int ref4_slots(const mcpt_bvh_node *nodes, int32_t x, int32_t *c) {
  const mcpt_bvh_node &b = nodes[x];
  int s = 0;
  for (int32_t k : {b.left, b.right}) {
    const mcpt_bvh_node &y = nodes[k];
    if (y.left == y.right) {
      c[s++] = k;
    } else {
      c[s++] = y.left;
      c[s++] = y.right;
    }
  }
  return s;
}
__global__ void k_ref4_count(const int32_t *__restrict__ lvl, uint32_t count, const mcpt_bvh_node *__restrict__ nodes,
                             uint32_t *cnt) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  int32_t c[4];
  const int s = ref4_slots(nodes, lvl[i], c);
  uint32_t k = 0;
  for (int j = 0; j < s; ++j) k += nodes[c[j]].left != nodes[c[j]].right;
  cnt[i] = k;
}
// writes the level's records (ids base + i) and the next level's binary ids
__global__ void k_ref4_emit(const int32_t *__restrict__ lvl, uint32_t count, uint32_t base,
                            const uint32_t *__restrict__ pos, uint32_t next_base, const mcpt_bvh_node *__restrict__ nodes,
                            mcpt::Node4Rec *out, int32_t *next, int32_t *child4) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  int32_t c[4];
  const int s = ref4_slots(nodes, lvl[i], c);
  mcpt::Node4Rec q;
  memset(&q, 0, sizeof(q));
  uint32_t p = pos[i];
  for (int j = 0; j < 4; ++j) {
    child4[4 * (base + i) + j] = -1;
    if (j >= s) {
      q.link[j] = kEmptySlot4;
      continue;
    }
    const mcpt_bvh_node &x = nodes[c[j]];
    const float v[6] = {x.bbmin[0], x.bbmax[0], x.bbmin[1], x.bbmax[1], x.bbmin[2], x.bbmax[2]};
    for (int k = 0; k < 6; ++k) q.q[6 * j + k] = v[k];
    if (x.left == x.right) {
      q.link[j] = ~x.left;
    } else {
      q.link[j] = (int32_t)(next_base + p);
      child4[4 * (base + i) + j] = (int32_t)(next_base + p);
      next[p++] = c[j];
    }
  }
  out[base + i] = q;
}
// stack need of one level of 4-wide nodes (children's needs known)
__global__ void k_need4(uint32_t base, uint32_t count, const mcpt::Node4Rec *__restrict__ q, const int32_t *__restrict__ child,
                        int32_t *need) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const uint32_t k = base + i;
  int ns = 0;
  while (ns < 4 && q[k].link[ns] != kEmptySlot4) ++ns;
  int best = ns - 1;
  for (int j = 0; j < ns; ++j)
    if (q[k].link[j] >= 0) best = max(best, ns - 1 - j + need[q[k].link[j]]);
  need[k] = best;
  (void)child;
}

// --------------------------------------------------- the SAH search tree
struct SahNode {            // Builder's BinNode + its range
  float box[6];
  int32_t left, right;      // binary node ids, -1 for a leaf
  int32_t item;             // leaf: index into the leaf list
  int32_t lo, hi;           // idx range
  int32_t depth;
};

struct Split {              // one large range's split state
  uint32_t cmin[3], cmax[3];  // ordered-int centroid bounds
  int32_t node;
};
struct Bins {               // per axis, per bin: box (ordered ints) and count
  uint32_t b[3][NB][6];
  uint32_t c[3][NB];
};

__global__ void k_leaf_init(const mcpt_bvh_node *__restrict__ nodes, int64_t n, float *box, int32_t *tri, float *cen,
                            int32_t *idx, int32_t *owner) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const mcpt_bvh_node &b = nodes[n - 1 + i];  // leaves in node order (HLBVH layout)
  const float bx[6] = {b.bbmin[0], b.bbmax[0], b.bbmin[1], b.bbmax[1], b.bbmin[2], b.bbmax[2]};
  for (int k = 0; k < 6; ++k) box[6 * i + k] = bx[k];
  tri[i] = b.left;
  for (int a = 0; a < 3; ++a) cen[3 * i + a] = 0.5f * (bx[2 * a] + bx[2 * a + 1]);
  idx[i] = (int32_t)i;
  owner[i] = 0;
}

// centroid bounds of the large ranges (owner slot >= 0): a workgroup takes
// a chunk of kBinChunk positions and reduces the chunk's first slot in
// registers, then one atomic per wave into LDS and one per workgroup into
// the slot (a chunk's other slots, where ranges meet, go straight to global)
constexpr int kBinChunk = 4096;
__global__ __launch_bounds__(256) void k_cbounds(const int32_t *__restrict__ idx, const float *__restrict__ cen,
                                                 const int32_t *__restrict__ owner, const int32_t *__restrict__ slot_of,
                                                 int64_t m, Split *sp) {
  __shared__ uint32_t lmn[3], lmx[3];
  __shared__ int32_t s_first;
  const int64_t c0 = (int64_t)blockIdx.x * kBinChunk;
  if (threadIdx.x == 0) s_first = c0 < m ? slot_of[owner[c0]] : -1;
  if (threadIdx.x < 3) lmn[threadIdx.x] = 0xFFFFFFFFu, lmx[threadIdx.x] = 0u;
  __syncthreads();
  const int32_t sf = s_first;
  uint32_t mn[3] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu}, mx[3] = {0u, 0u, 0u};
  for (int64_t i = c0 + threadIdx.x; i < min(c0 + kBinChunk, m); i += blockDim.x) {
    const int32_t s = slot_of[owner[i]];
    if (s < 0) continue;
    const float *c = cen + 3 * (size_t)idx[i];
    for (int a = 0; a < 3; ++a) {
      const uint32_t o = f2o(c[a]);
      if (s == sf)
        mn[a] = min(mn[a], o), mx[a] = max(mx[a], o);
      else
        atomicMin(&sp[s].cmin[a], o), atomicMax(&sp[s].cmax[a], o);
    }
  }
  if (sf < 0) return;  // uniform: no thread of this chunk has a large first slot
  for (int o = 32; o > 0; o >>= 1)
    for (int a = 0; a < 3; ++a) {
      mn[a] = min(mn[a], (uint32_t)__shfl_xor((int)mn[a], o, 64));
      mx[a] = max(mx[a], (uint32_t)__shfl_xor((int)mx[a], o, 64));
    }
  if ((threadIdx.x & 63) == 0)
    for (int a = 0; a < 3; ++a) atomicMin(&lmn[a], mn[a]), atomicMax(&lmx[a], mx[a]);
  __syncthreads();
  if (threadIdx.x < 3) {
    if (lmn[threadIdx.x] != 0xFFFFFFFFu) atomicMin(&sp[sf].cmin[threadIdx.x], lmn[threadIdx.x]);
    if (lmx[threadIdx.x] != 0u) atomicMax(&sp[sf].cmax[threadIdx.x], lmx[threadIdx.x]);
  }
}

__device__ inline int bin_of(float c, float cmin, float scale) {  // split(): min(NB - 1, (int)((c - cmin) * scale))
  return min(NB - 1, (int)((c - cmin) * scale));
}

// bins of the large ranges: a workgroup accumulates a chunk in LDS for the
// chunk's first slot, other slots' elements go straight to global atomics
__global__ __launch_bounds__(256) void k_bins(const int32_t *__restrict__ idx, const float *__restrict__ cen,
                                              const float *__restrict__ box, const int32_t *__restrict__ owner,
                                              const int32_t *__restrict__ slot_of, int64_t m,
                                              const Split *__restrict__ sp, Bins *bins) {
  __shared__ uint32_t lb[3][NB][6];
  __shared__ uint32_t lc[3][NB];
  __shared__ int32_t s_first;
  const int64_t c0 = (int64_t)blockIdx.x * kBinChunk;
  if (threadIdx.x == 0) s_first = c0 < m ? slot_of[owner[c0]] : -1;
  for (int k = threadIdx.x; k < 3 * NB; k += blockDim.x) {
    const int a = k / NB, j = k % NB;
    for (int e = 0; e < 6; ++e) lb[a][j][e] = (e & 1) ? 0u : 0xFFFFFFFFu;
    lc[a][j] = 0;
  }
  __syncthreads();
  const int32_t sf = s_first;
  for (int64_t i = c0 + threadIdx.x; i < min(c0 + kBinChunk, m); i += blockDim.x) {
    const int32_t s = slot_of[owner[i]];
    if (s < 0) continue;
    const int32_t it = idx[i];
    const float *bx = box + 6 * (size_t)it;
    uint32_t ob[6];
    for (int e = 0; e < 6; ++e) ob[e] = f2o(bx[e]);
    for (int a = 0; a < 3; ++a) {
      const float cmn = o2f(sp[s].cmin[a]), cmx = o2f(sp[s].cmax[a]);
      const float ext = cmx - cmn;
      if (!(ext > 0)) continue;
      const float scale = NB / ext;
      const int k = bin_of(cen[3 * it + a], cmn, scale);
      if (s == sf) {
        for (int e = 0; e < 6; ++e) (e & 1) ? atomicMax(&lb[a][k][e], ob[e]) : atomicMin(&lb[a][k][e], ob[e]);
        atomicAdd(&lc[a][k], 1u);
      } else {
        for (int e = 0; e < 6; ++e)
          (e & 1) ? atomicMax(&bins[s].b[a][k][e], ob[e]) : atomicMin(&bins[s].b[a][k][e], ob[e]);
        atomicAdd(&bins[s].c[a][k], 1u);
      }
    }
  }
  __syncthreads();
  if (sf < 0) return;
  for (int k = threadIdx.x; k < 3 * NB; k += blockDim.x) {
    const int a = k / NB, j = k % NB;
    if (lc[a][j] == 0) continue;
    for (int e = 0; e < 6; ++e)
      (e & 1) ? atomicMax(&bins[sf].b[a][j][e], lb[a][j][e]) : atomicMin(&bins[sf].b[a][j][e], lb[a][j][e]);
    atomicAdd(&bins[sf].c[a][j], lc[a][j]);
  }
}

// the SAH sweep of split() on one range's bins: best (axis, bin), or axis -1
struct Choice {
  int axis, bin;
  int64_t left;  // elements with bin < best bin
};
__device__ inline Choice sweep(const float bb[3][NB][6], const uint32_t bc[3][NB], const float *cmin, const float *cmax) {
  double best = DBL_MAX;
  Choice ch{-1, -1, 0};
  for (int a = 0; a < 3; ++a) {
    const float ext = cmax[a] - cmin[a];
    if (!(ext > 0)) continue;
    double left_cost[NB];
    float acc[6];
    empty6(acc);
    int64_t cnt = 0;
    for (int k = 0; k < NB - 1; ++k) {
      grow6(acc, bb[a][k]);
      cnt += bc[a][k];
      left_cost[k] = cnt ? area6(acc) * (double)cnt : -1.0;
    }
    empty6(acc);
    cnt = 0;
    for (int k = NB - 1; k > 0; --k) {
      grow6(acc, bb[a][k]);
      cnt += bc[a][k];
      if (!cnt || left_cost[k - 1] < 0) continue;
      const double c = left_cost[k - 1] + area6(acc) * (double)cnt;
      if (c < best) best = c, ch.axis = a, ch.bin = k;
    }
  }
  if (ch.axis >= 0)
    for (int k = 0; k < ch.bin; ++k) ch.left += bc[ch.axis][k];
  return ch;
}

struct LargeOut {  // per large range this level: the split and its children
  int32_t axis, bin, mid, part;  // part: first right element of the partition
  float cmin, scale;
};

// one thread per large range: sweep, children's nodes and ranges
__global__ void k_large_split(uint32_t count, const Split *__restrict__ sp, const Bins *__restrict__ bins,
                              SahNode *nodes, LargeOut *lo_out, int32_t *next_large, uint32_t *n_next_large,
                              int32_t *small, uint32_t *n_small) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= count) return;
  const int32_t x = sp[s].node;
  SahNode &N = nodes[x];
  float cmin[3], cmax[3];
  for (int a = 0; a < 3; ++a) cmin[a] = o2f(sp[s].cmin[a]), cmax[a] = o2f(sp[s].cmax[a]);
  float bb[3][NB][6];
  uint32_t bc[3][NB];
  for (int a = 0; a < 3; ++a)
    for (int k = 0; k < NB; ++k) {
      bc[a][k] = bins[s].c[a][k];
      for (int e = 0; e < 6; ++e) bb[a][k][e] = bc[a][k] ? o2f(bins[s].b[a][k][e]) : ((e & 1) ? -FLT_MAX : FLT_MAX);
    }
  const Choice ch = sweep(bb, bc, cmin, cmax);
  const int32_t lo = N.lo, hi = N.hi;
  int32_t mid = (int32_t)(((int64_t)lo + hi) / 2);
  LargeOut o{-1, -1, mid, mid, 0.0f, 0.0f};
  if (ch.axis >= 0) {
    const int64_t m2 = lo + ch.left;
    o.part = (int32_t)m2;
    if (m2 > lo && m2 < hi) mid = (int32_t)m2;
    o.axis = ch.axis;
    o.bin = ch.bin;
    o.cmin = cmin[ch.axis];
    o.scale = NB / (cmax[ch.axis] - cmin[ch.axis]);
  }
  o.mid = mid;
  lo_out[s] = o;
  const int32_t lb = x + 1, rb = x + 2 * (mid - lo);
  N.left = lb;
  N.right = rb;
  N.item = -1;
  SahNode &L = nodes[lb], &R = nodes[rb];
  L.lo = lo, L.hi = mid, L.depth = N.depth + 1;
  R.lo = mid, R.hi = hi, R.depth = N.depth + 1;
  for (int32_t c : {lb, rb}) {
    const int32_t sz = nodes[c].hi - nodes[c].lo;
    if (sz > kSmall)
      next_large[atomicAdd(n_next_large, 1u)] = c;
    else
      small[atomicAdd(n_small, 1u)] = c;
  }
}

// the stable partition of every large range: flags, then placement by a scan
__global__ void k_flags(const int32_t *__restrict__ idx, const float *__restrict__ cen, const int32_t *__restrict__ owner,
                        const int32_t *__restrict__ slot_of, const LargeOut *__restrict__ lo_out, int64_t m,
                        uint32_t *flag) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  const int32_t s = slot_of[owner[i]];
  uint32_t f = 0;
  if (s >= 0 && lo_out[s].axis >= 0) {
    const LargeOut o = lo_out[s];
    f = bin_of(cen[3 * idx[i] + o.axis], o.cmin, o.scale) < o.bin;
  }
  flag[i] = f;
}
__global__ void k_place(const int32_t *__restrict__ idx, const int32_t *__restrict__ owner,
                        const int32_t *__restrict__ slot_of, const LargeOut *__restrict__ lo_out,
                        const SahNode *__restrict__ nodes, const uint32_t *__restrict__ flag,
                        const uint32_t *__restrict__ pre, int64_t m, int32_t *idx2, int32_t *owner2) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  const int32_t x = owner[i];
  const int32_t s = slot_of[x];
  if (s < 0) {
    idx2[i] = idx[i];
    owner2[i] = x;
    return;
  }
  const SahNode &N = nodes[x];
  const LargeOut o = lo_out[s];
  int64_t p;
  bool left;
  if (o.axis >= 0) {
    const int64_t rank = (int64_t)pre[i] - pre[N.lo];
    left = flag[i] != 0;
    p = left ? N.lo + rank : o.part + (i - N.lo - rank);
  } else {
    p = i;
    left = i < o.mid;
  }
  idx2[p] = idx[i];
  owner2[p] = left ? N.left : N.right;
}

// ------------------------------------------------------ small ranges
// One wave per range of <= kSmall leaves builds its whole subtree in LDS:
// the range's leaf indices are read once, every split of the subtree
// partitions them in LDS (the global idx order is not needed afterwards),
// pending ranges sit on an LDS stack.  Per node: centroid bounds by wave
// reduction, the 3 x 32 bins by LDS atomics, split()'s sweep with one lane
// per (axis, bin) candidate (sweep_wave), the stable partition by ballot.
// Same result as split() (min / max are exact in any order; only the sign
// of a zero bound can differ, and the costs use differences of bounds, so
// signs of zero never reach them).
struct PendRange {
  int32_t x, lo, hi, depth;  // node id, local range, depth
};
constexpr int kStk = kSmall / 2;  // pending ranges are disjoint with >= 2 leaves each

__device__ inline uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
__device__ inline uint32_t lanes_below(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// split()'s sweep over LDS bins, one lane per (axis, bin k) candidate: the
// left side is bins [0, k) (inclusive prefix of k-1), the right side
// [k, NB) (inclusive suffix), the winner the least cost, ties to the
// earlier candidate of split()'s order (axis ascending, bin descending)
__device__ inline Choice sweep_wave(const uint32_t (*lb)[NB][6], const uint32_t (*lc)[NB], const float *cmin,
                                    const float *cmax) {
  const int lane = (int)lane_id(), j = lane & (NB - 1);
  double best = DBL_MAX;
  int best_ord = INT_MAX, best_left = 0;
  for (int pass = 0; pass < 2; ++pass) {
    const int a = (lane >> 5) + 2 * pass;
    const int ac = a < 3 ? a : 2;
    float pb[6], sb[6];
    const uint32_t n = lc[ac][j];
    for (int e = 0; e < 6; ++e) pb[e] = n ? o2f(lb[ac][j][e]) : ((e & 1) ? -FLT_MAX : FLT_MAX);
    uint32_t pc = n, sc = n;
    for (int e = 0; e < 6; ++e) sb[e] = pb[e];
    for (int o = 1; o < NB; o <<= 1) {  // inclusive prefix / suffix within the 32-lane axis segment
      uint32_t tp = __shfl_up(pc, o, NB), ts = __shfl_down(sc, o, NB);
      float up[6], dn[6];
      for (int e = 0; e < 6; ++e) up[e] = __shfl_up(pb[e], o, NB), dn[e] = __shfl_down(sb[e], o, NB);
      if (j >= o) {
        pc += tp;
        grow6(pb, up);
      }
      if (j + o < NB) {
        sc += ts;
        grow6(sb, dn);
      }
    }
    float lbx[6];
    for (int e = 0; e < 6; ++e) lbx[e] = __shfl_up(pb[e], 1, NB);
    const uint32_t lcnt = __shfl_up(pc, 1, NB);
    const float ext = cmax[ac] - cmin[ac];
    if (a < 3 && ext > 0 && j >= 1 && lcnt && sc) {
      const double c = area6(lbx) * (double)lcnt + area6(sb) * (double)sc;
      const int ord = a * NB + (NB - 1 - j);
      if (c < best || (c == best && ord < best_ord)) best = c, best_ord = ord, best_left = (int)lcnt;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    const double c = __shfl_xor(best, o, 64);
    const int ord = __shfl_xor(best_ord, o, 64), left = __shfl_xor(best_left, o, 64);
    if (c < best || (c == best && ord < best_ord)) best = c, best_ord = ord, best_left = left;
  }
  Choice ch{-1, -1, 0};
  if (best_ord != INT_MAX) ch.axis = best_ord / NB, ch.bin = NB - 1 - best_ord % NB, ch.left = best_left;
  return ch;
}

__global__ __launch_bounds__(64) void k_small(const int32_t *__restrict__ list, uint32_t count,
                                              const int32_t *__restrict__ idx, const float *__restrict__ cen,
                                              const float *__restrict__ box, SahNode *nodes) {
  __shared__ int32_t sidx[kSmall], stmp[kSmall];
  __shared__ PendRange stk[kStk];
  __shared__ uint32_t lb[3][NB][6];
  __shared__ uint32_t lc[3][NB];
  if (blockIdx.x >= count) return;
  const int lane = (int)threadIdx.x;
  const int32_t x0 = list[blockIdx.x];
  const int32_t lo0 = nodes[x0].lo, r0 = nodes[x0].hi - lo0;
  // a leaf: its box, no children, its item (lane e writes word e of the record)
  auto leaf = [&](int32_t x, int32_t it) {
    if (lane < 6) nodes[x].box[lane] = box[6 * (size_t)it + lane];
    if (lane == 6) nodes[x].left = -1;
    if (lane == 7) nodes[x].right = -1;
    if (lane == 8) nodes[x].item = it;
  };
  if (r0 == 1) {
    leaf(x0, idx[lo0]);
    return;
  }
  for (int i = lane; i < r0; i += 64) sidx[i] = idx[lo0 + i];
  if (lane == 0) stk[0] = PendRange{x0, 0, r0, nodes[x0].depth};
  int sp = 1;
  __syncthreads();
  while (sp > 0) {
    const PendRange R = stk[--sp];
    const int32_t lo = R.lo, hi = R.hi;
    // centroid bounds
    float cmin[3], cmax[3];
    for (int a = 0; a < 3; ++a) cmin[a] = FLT_MAX, cmax[a] = -FLT_MAX;
    for (int i = lo + lane; i < hi; i += 64) {
      const float *c = cen + 3 * (size_t)sidx[i];
      for (int a = 0; a < 3; ++a) cmin[a] = smin(cmin[a], c[a]), cmax[a] = smax(cmax[a], c[a]);
    }
    for (int o = 32; o > 0; o >>= 1)
      for (int a = 0; a < 3; ++a) {
        cmin[a] = smin(cmin[a], __shfl_xor(cmin[a], o, 64));
        cmax[a] = smax(cmax[a], __shfl_xor(cmax[a], o, 64));
      }
    // bins
    for (int k = lane; k < 3 * NB; k += 64) {
      const int a = k / NB, j = k % NB;
      for (int e = 0; e < 6; ++e) lb[a][j][e] = (e & 1) ? 0u : 0xFFFFFFFFu;
      lc[a][j] = 0;
    }
    __syncthreads();
    for (int i = lo + lane; i < hi; i += 64) {
      const int32_t it = sidx[i];
      const float *bx = box + 6 * (size_t)it;
      uint32_t ob[6];
      for (int e = 0; e < 6; ++e) ob[e] = f2o(bx[e]);
      for (int a = 0; a < 3; ++a) {
        const float ext = cmax[a] - cmin[a];
        if (!(ext > 0)) continue;
        const int k = bin_of(cen[3 * (size_t)it + a], cmin[a], NB / ext);
        for (int e = 0; e < 6; ++e) (e & 1) ? atomicMax(&lb[a][k][e], ob[e]) : atomicMin(&lb[a][k][e], ob[e]);
        atomicAdd(&lc[a][k], 1u);
      }
    }
    __syncthreads();
    const Choice ch = sweep_wave(lb, lc, cmin, cmax);
    int32_t mid = (lo + hi) / 2;
    if (ch.axis >= 0) {
      const int32_t part = lo + (int32_t)ch.left;
      if (part > lo && part < hi) mid = part;
      // stable partition into stmp, 64 leaves per step
      const float cm = cmin[ch.axis], scale = NB / (cmax[ch.axis] - cmin[ch.axis]);
      int32_t nl = 0, nr = 0;
      for (int base = lo; base < hi; base += 64) {
        const int i = base + lane;
        const bool valid = i < hi;
        const int32_t it = valid ? sidx[i] : 0;
        const bool f = valid && bin_of(cen[3 * (size_t)it + ch.axis], cm, scale) < ch.bin;
        const uint64_t bal = __ballot(f);
        const int32_t before = (int32_t)lanes_below(bal), tot = (int32_t)__popcll(bal);
        if (valid) stmp[f ? lo + nl + before : part + nr + (lane - before)] = it;
        nl += tot;
        nr += min(64, hi - base) - tot;
      }
      __syncthreads();
      for (int i = lo + lane; i < hi; i += 64) sidx[i] = stmp[i];
      __syncthreads();
    }
    const int32_t lx = R.x + 1, rx = R.x + 2 * (mid - lo);
    if (lane == 0) {
      nodes[R.x].left = lx;
      nodes[R.x].right = rx;
      nodes[R.x].item = -1;
      nodes[lx].lo = lo0 + lo, nodes[lx].hi = lo0 + mid, nodes[lx].depth = R.depth + 1;
      nodes[rx].lo = lo0 + mid, nodes[rx].hi = lo0 + hi, nodes[rx].depth = R.depth + 1;
    }
    // right pushed first: the left child is split next
    if (hi - mid == 1)
      leaf(rx, sidx[mid]);
    else {
      if (lane == 0) stk[sp] = PendRange{rx, mid, hi, R.depth + 1};
      ++sp;
    }
    if (mid - lo == 1)
      leaf(lx, sidx[lo]);
    else {
      if (lane == 0) stk[sp] = PendRange{lx, lo, mid, R.depth + 1};
      ++sp;
    }
    __syncthreads();
  }
}

// this level's large ranges: slots, empty bounds and bins (mode 0), or the
// slots cleared again (mode 1)
__global__ void k_large_slots(const int32_t *__restrict__ list, uint32_t count, int mode, int32_t *slot_of, Split *sp,
                              Bins *bins) {
  const uint32_t s = blockIdx.x, t = threadIdx.x;
  if (s >= count) return;
  const int32_t x = list[s];
  if (mode == 1) {
    if (t == 0) slot_of[x] = -1;
    return;
  }
  if (t == 0) {
    slot_of[x] = (int32_t)s;
    sp[s].node = x;
    for (int a = 0; a < 3; ++a) sp[s].cmin[a] = 0xFFFFFFFFu, sp[s].cmax[a] = 0u;
  }
  for (int k = t; k < 3 * NB; k += blockDim.x) {
    const int a = k / NB, j = k % NB;
    for (int e = 0; e < 6; ++e) bins[s].b[a][j][e] = (e & 1) ? 0u : 0xFFFFFFFFu;
    bins[s].c[a][j] = 0;
  }
}

// depth of every node as a sort key (ids ascending within a depth after a stable sort)
__global__ void k_depth_keys(const SahNode *__restrict__ sn, int64_t nb, uint32_t *key, int32_t *id, uint32_t *maxd) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t w = 0;  // every lane stays for the wave reduction: one atomic per wave
  if (i < nb) {
    w = (uint32_t)sn[i].depth;
    key[i] = w;
    id[i] = (int32_t)i;
  }
  for (int o = 32; o > 0; o >>= 1) w = max(w, (uint32_t)__shfl_xor((int)w, o, 64));
  if ((threadIdx.x & 63) == 0) atomicMax(maxd, w);
}
// first position of every depth in the sorted keys (every depth 0..max occurs)
__global__ void k_depth_starts(const uint32_t *__restrict__ key, int64_t nb, uint32_t *start) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nb) return;
  if (i == 0 || key[i] != key[i - 1]) start[key[i]] = (uint32_t)i;
}

// collapse DP (mcpt_sah.cpp build_sah4): f[x][1..4], cut[x][1..4], wide[x]
struct DP {
  double f[5];
  int8_t cut[5];
  int8_t wide[2];
};
// one depth, bottom-up: the box (left box, then grow(right): Builder::build)
// and the collapse DP (children done at the deeper level)
__global__ void k_box_dp_level(const int32_t *__restrict__ ids, uint32_t count, SahNode *nodes, DP *dp) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const int32_t x = ids[i];
  SahNode &N = nodes[x];
  if (N.item < 0) {
    float b[6];
    for (int k = 0; k < 6; ++k) b[k] = nodes[N.left].box[k];
    grow6(b, nodes[N.right].box);
    for (int k = 0; k < 6; ++k) N.box[k] = b[k];
  }
  DP d;
  memset(&d, 0, sizeof(d));
  const double sa = area6(N.box);
  if (N.item >= 0) {
    for (int k = 1; k <= 4; ++k) d.f[k] = sa * C_TRI, d.cut[k] = 0;
    dp[x] = d;
    return;
  }
  const DP &L = dp[N.left], &R = dp[N.right];
  double bw = DBL_MAX;
  for (int a = 1; a <= 3; ++a)
    for (int b = 1; a + b <= 4; ++b)
      if (L.f[a] + R.f[b] < bw) bw = L.f[a] + R.f[b], d.wide[0] = (int8_t)a, d.wide[1] = (int8_t)b;
  d.f[1] = sa * C_STEP + bw;
  d.cut[1] = 0;
  for (int k = 2; k <= 4; ++k) {
    d.f[k] = d.f[k - 1];
    d.cut[k] = d.cut[k - 1];
    for (int a = 1; a < k; ++a)
      if (L.f[a] + R.f[k - a] < d.f[k]) d.f[k] = L.f[a] + R.f[k - a], d.cut[k] = (int8_t)a;
  }
  dp[x] = d;
}

// entries of x's subtree as at most k slots, left to right (build_sah4's `entries`)
__device__ inline void entries(const SahNode *nodes, const DP *dp, int32_t x, int k, int32_t *e, int &ne) {
  int32_t st_x[8];
  int st_k[8];
  int sp = 0;
  st_x[sp] = x, st_k[sp] = k, ++sp;
  while (sp > 0) {  // preorder: left before right
    --sp;
    const int32_t y = st_x[sp];
    const int kk = st_k[sp];
    const int a = dp[y].cut[kk];
    if (a == 0) {
      e[ne++] = y;
      continue;
    }
    st_x[sp] = nodes[y].right, st_k[sp] = kk - a, ++sp;
    st_x[sp] = nodes[y].left, st_k[sp] = a, ++sp;
  }
}
__device__ inline int wide_kids(const SahNode *nodes, const DP *dp, int32_t x, int32_t *kids) {
  int nk = 0;
  entries(nodes, dp, nodes[x].left, dp[x].wide[0], kids, nk);
  entries(nodes, dp, nodes[x].right, dp[x].wide[1], kids, nk);
  return nk;
}
// wide-tree levels: the next frontier (internal entries), counts first
__global__ void k_wide_count(const int32_t *__restrict__ lvl, uint32_t count, const SahNode *__restrict__ nodes,
                             const DP *__restrict__ dp, uint32_t *cnt) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  int32_t kids[4];
  const int nk = wide_kids(nodes, dp, lvl[i], kids);
  uint32_t c = 0;
  for (int k = 0; k < nk; ++k) c += nodes[kids[k]].item < 0;
  cnt[i] = c;
}
// next level's wide nodes in (parent, slot) order; w_parent links them
__global__ void k_wide_next(const int32_t *__restrict__ lvl, uint32_t count, uint32_t base,
                            const uint32_t *__restrict__ pos, uint32_t next_base, const SahNode *__restrict__ nodes,
                            const DP *__restrict__ dp, int32_t *wnode, int32_t *wkid) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  int32_t kids[4];
  const int nk = wide_kids(nodes, dp, lvl[i], kids);
  uint32_t p = pos[i];
  for (int k = 0; k < 4; ++k) wkid[4 * (base + i) + k] = -1;
  for (int k = 0; k < nk; ++k)
    if (nodes[kids[k]].item < 0) {
      wkid[4 * (base + i) + k] = (int32_t)(next_base + p);
      wnode[next_base + p] = kids[k];
      ++p;
    }
}
// subtree sizes of the wide tree (bottom-up by wide level)
__global__ void k_wide_size(uint32_t base, uint32_t count, const int32_t *__restrict__ wkid, uint32_t *size) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  uint32_t s = 1;
  for (int k = 0; k < 4; ++k) {
    const int32_t c = wkid[4 * (base + i) + k];
    if (c >= 0) s += size[c];
  }
  size[base + i] = s;
}
// preorder ranks (top-down): slot k's rank = parent's + 1 + sizes of the earlier slots
__global__ void k_wide_rank(uint32_t base, uint32_t count, const int32_t *__restrict__ wkid,
                            const uint32_t *__restrict__ size, uint32_t *rank, uint32_t *nkids_by_rank) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const uint32_t w = base + i, r = rank[w];
  uint32_t acc = r + 1, nk = 0;
  for (int k = 0; k < 4; ++k) {
    const int32_t c = wkid[4 * w + k];
    if (c < 0) continue;
    rank[c] = acc;
    acc += size[c];
    ++nk;
  }
  nkids_by_rank[r] = nk;
}
// emission: node w's record at its id; its internal slots' ids are the
// allocation base of w (1 + the children of every node emitted before it,
// i.e. earlier in preorder) plus their count so far
__global__ void k_wide_emit(uint32_t base, uint32_t count, const int32_t *__restrict__ wnode,
                            const int32_t *__restrict__ wkid, const uint32_t *__restrict__ rank,
                            const uint32_t *__restrict__ alloc, const SahNode *__restrict__ nodes,
                            const DP *__restrict__ dp, const int32_t *__restrict__ leaf_tri, int32_t *out_id,
                            mcpt::Node4Rec *out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const uint32_t w = base + i;
  int32_t kids[4];
  const int nk = wide_kids(nodes, dp, wnode[w], kids);
  const uint32_t a0 = 1u + alloc[rank[w]];
  mcpt::Node4Rec rec;
  memset(&rec, 0, sizeof(rec));
  uint32_t c = 0;
  for (int k = 0; k < 4; ++k) {
    if (k >= nk) {
      rec.link[k] = kEmptySlot4;
      continue;
    }
    const SahNode &C = nodes[kids[k]];
    for (int e = 0; e < 6; ++e) rec.q[6 * k + e] = C.box[e];
    if (C.item >= 0) {
      rec.link[k] = ~leaf_tri[C.item];
    } else {
      rec.link[k] = (int32_t)(a0 + c);
      out_id[wkid[4 * w + k]] = (int32_t)(a0 + c);
      ++c;
    }
  }
  out[out_id[w]] = rec;
}
// stack need of the emitted tree (bottom-up by wide level, through out ids)
__global__ void k_wide_need(uint32_t base, uint32_t count, const int32_t *__restrict__ out_id,
                            const mcpt::Node4Rec *__restrict__ out, int32_t *need_by_id) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const int32_t id = out_id[base + i];
  const mcpt::Node4Rec &r = out[id];
  int ns = 0, below = 0;
  for (int s = 0; s < 4; ++s) {
    if (r.link[s] == kEmptySlot4) continue;
    ++ns;
    if (r.link[s] >= 0) below = max(below, need_by_id[r.link[s]]);
  }
  need_by_id[id] = ns - 1 + below;
}

// quantize_node4 (mcpt_sah.cpp), per node
__device__ inline float qdec(int q, float s, float o) { return fmaf((float)q, s, o); }
__device__ inline bool normal_or_zero(float x) { return x == 0.0f || (isfinite(x) && fabsf(x) >= FLT_MIN); }
__global__ void k_quantize(const mcpt::Node4Rec *__restrict__ in, int64_t n, mcpt::Node4Q *outq, uint32_t *flags) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const mcpt::Node4Rec &r = in[i];
  mcpt::Node4Q out;
  memset(&out, 0, sizeof(out));
  float scale[3];
  bool ok = true;
  for (int a = 0; a < 3 && ok; ++a) {
    float lo = FLT_MAX, hi = -FLT_MAX;
    for (int k = 0; k < 4; ++k) {
      if (r.link[k] == kEmptySlot4) continue;
      lo = smin(lo, r.q[6 * k + 2 * a]);
      hi = smax(hi, r.q[6 * k + 2 * a + 1]);
    }
    if (lo > hi) lo = hi = 0.0f;
    float org = nextafterf(lo, -FLT_MAX);
    if (!normal_or_zero(org)) org = -FLT_MIN;
    if (!normal_or_zero(org) || !isfinite(hi)) {
      ok = false;
      break;
    }
    const double span = (double)hi - (double)org;
    int e = span > 0 ? (int)ceil(log2(span / 255.0)) : -126;
    e = max(-126, min(e, 127));
    while (e > -126 && qdec(255, ldexpf(1.0f, e - 1), org) > hi) --e;
    while (e <= 127 && !(qdec(255, ldexpf(1.0f, e), org) > hi)) ++e;
    if (e > 127) {
      ok = false;
      break;
    }
    const float s = ldexpf(1.0f, e);
    out.org[a] = org;
    scale[a] = s;
    for (int k = 0; k < 4 && ok; ++k) {
      uint8_t &ql = out.q[6 * k + 2 * a], &qh = out.q[6 * k + 2 * a + 1];
      if (r.link[k] == kEmptySlot4) {
        ql = 0;
        qh = 0;
        continue;
      }
      const float bl = r.q[6 * k + 2 * a], bh = r.q[6 * k + 2 * a + 1];
      int q = (int)fmax(0.0, fmin(255.0, floor(((double)bl - (double)org) / s)));
      while (q > 0 && !(qdec(q, s, org) < bl)) --q;
      while (q < 255 && qdec(q + 1, s, org) < bl) ++q;
      while (q > 0 && !normal_or_zero(qdec(q, s, org))) --q;
      if (!(qdec(q, s, org) < bl) || !normal_or_zero(qdec(q, s, org))) {
        ok = false;
        break;
      }
      ql = (uint8_t)q;
      q = (int)fmax(0.0, fmin(255.0, ceil(((double)bh - (double)org) / s)));
      while (q < 255 && !(qdec(q, s, org) > bh)) ++q;
      while (q > 0 && qdec(q - 1, s, org) > bh) --q;
      while (q < 255 && !normal_or_zero(qdec(q, s, org))) ++q;
      if (!(qdec(q, s, org) > bh) || !normal_or_zero(qdec(q, s, org))) {
        ok = false;
        break;
      }
      qh = (uint8_t)q;
    }
  }
  if (!ok) {
    atomicOr(flags, 1u);
    return;
  }
  out.sx = scale[0];
  out.sy = scale[1];
  out.sz = scale[2];
  for (int k = 0; k < 4; ++k) out.link[k] = r.link[k];
  outq[i] = out;
}

inline unsigned nblk(int64_t n, unsigned b) { return (unsigned)std::max<int64_t>(1, (n + b - 1) / b); }

// device scratch freed on scope exit
struct Scratch {
  std::vector<void *> p;
  template <class T>
  hipError_t alloc(T **x, size_t count) {
    hipError_t e = hipMalloc((void **)x, std::max<size_t>(count, 1) * sizeof(T));
    if (e == hipSuccess) p.push_back((void *)*x);
    return e;
  }
  ~Scratch() {
    for (void *x : p) (void)hipFree(x);
  }
};

}  // namespace

#define UP_OK(expr)                                                                                  \
  do {                                                                                               \
    hipError_t e_ = (expr);                                                                          \
    if (e_ != hipSuccess)                                                                            \
      return mcpt::fail(MCPT_ERR_HIP, std::string("scene_upload_device: ") + #expr + ": " + hipGetErrorString(e_)); \
  } while (0)

namespace mcpt {

// exclusive scan of n u32 (hipCUB)
static int exscan(const uint32_t *in, uint32_t *out, int64_t n, hipStream_t st, Scratch &S) {
  size_t bytes = 0;
  UP_OK(hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, in, out, (int)n, st));
  void *tmp = nullptr;
  UP_OK(S.alloc((char **)&tmp, bytes));
  UP_OK(hipcub::DeviceScan::ExclusiveSum(tmp, bytes, in, out, (int)n, st));
  return MCPT_OK;
}

template <class T>
static int d2h(T *h, const T *d, size_t count, hipStream_t st) {
  UP_OK(hipMemcpyAsync(h, d, count * sizeof(T), hipMemcpyDeviceToHost, st));
  UP_OK(hipStreamSynchronize(st));
  return MCPT_OK;
}

int build_scene_device(const mcpt_triangle *tris, int64_t n, const mcpt_bvh_node *nodes, int32_t n_mats,
                       hipStream_t st, DeviceScene *out) {
  std::memset(out, 0, sizeof(*out));
  if (n <= 0) return fail(MCPT_ERR_ARG, "scene_upload_device: no triangles");
  if (n > (int64_t)0x3FFFFFFF) return fail(MCPT_ERR_LIMIT, "scene_upload_device: too many triangles");
  const int64_t nn = 2 * n - 1;
  Scratch S;
  uint32_t *flags = nullptr;
  UP_OK(S.alloc(&flags, 1));
  UP_OK(hipMemsetAsync(flags, 0, 4, st));
  hipLaunchKernelGGL(k_check, dim3(nblk(nn, 256)), dim3(256), 0, st, nodes, tris, n, n_mats, flags);
  UP_OK(hipGetLastError());
  uint32_t fl = 0;
  if (int rc = d2h(&fl, flags, 1, st)) return rc;
  if (fl & 1) return fail(MCPT_ERR_ARG, "scene_upload: negative child index");
  if (fl & 2) return fail(MCPT_ERR_ARG, "scene_upload: leaf triangle index out of range");
  if (fl & 4) return fail(MCPT_ERR_ARG, "scene_upload: child index out of range");
  if (fl & 8) return fail(MCPT_ERR_ARG, "scene_upload: triangle material id out of range");
  if (fl & 16) return fail(MCPT_ERR_ARG, "scene_upload: non-finite vertex coordinate");
  if (fl & 32)
    return fail(MCPT_ERR_ARG, "scene_upload_device: expected the HLBVH layout (internal [0, n-2], leaves [n-1, 2n-2])");
  if (int rc = d2h(&out->root, nodes, 1, st)) return rc;

  // triangle records, and whether every leaf box is its triangle's vertex bounds
  UP_OK(hipMalloc(&out->tris, n * sizeof(UDevTri)));
  UP_OK(hipMalloc(&out->triq, n * sizeof(UDevTri)));
  hipLaunchKernelGGL(k_tris, dim3(nblk(n, 256)), dim3(256), 0, st, tris, n, (UDevTri *)out->tris, (UDevTri *)out->triq);
  UP_OK(hipGetLastError());
  out->n_int = n - 1;
  if (n == 1) {  // a single leaf: no nodes (mcpt_scene_upload keeps one zeroed record of each)
    out->stack_depth = 1;
    out->depth4 = 1;
    out->n_near4 = out->n_nodes4 = 1;
    UP_OK(hipMalloc(&out->nodes, sizeof(UDevNode)));
    UP_OK(hipMalloc(&out->nodes4, sizeof(Node4Rec)));
    UP_OK(hipMalloc(&out->near4, sizeof(Node4Rec)));
    UP_OK(hipMemsetAsync(out->nodes, 0, sizeof(UDevNode), st));
    UP_OK(hipMemsetAsync(out->nodes4, 0, sizeof(Node4Rec), st));
    UP_OK(hipMemsetAsync(out->near4, 0, sizeof(Node4Rec), st));
    (void)hipFree(out->triq);
    out->triq = nullptr;
    out->quant = false;
    UP_OK(hipStreamSynchronize(st));
    return MCPT_OK;
  }
  hipLaunchKernelGGL(k_leafbox_check, dim3(nblk(n, 256)), dim3(256), 0, st, nodes, tris, n, flags);
  UP_OK(hipGetLastError());

  // binary levels of the reference tree: stack bound, then DevNode
  int32_t *lv = nullptr, *dref = nullptr;
  uint32_t *cnt1 = nullptr, *best = nullptr;
  UP_OK(S.alloc(&lv, n - 1));
  UP_OK(S.alloc(&cnt1, 1));
  UP_OK(S.alloc(&dref, nn));
  UP_OK(S.alloc(&best, 1));
  std::vector<uint32_t> off;
  if (int rc = tree_levels(nodes, n, st, lv, cnt1, off)) return rc;
  UP_OK(hipMemsetAsync(dref, 0, nn * sizeof(int32_t), st));
  UP_OK(hipMemsetAsync(best, 0, 4, st));
  for (size_t k = 0; k + 1 < off.size(); ++k) {
    const uint32_t a = off[k], b = off[k + 1];
    hipLaunchKernelGGL(k_stack_depth, dim3(nblk(b - a, 256)), dim3(256), 0, st, lv + a, b - a, nodes, dref, best);
    UP_OK(hipGetLastError());
  }
  uint32_t best_h = 1;
  if (int rc = d2h(&best_h, best, 1, st)) return rc;
  out->stack_depth = (int32_t)std::max<uint32_t>(best_h, 1);
  if (out->stack_depth > 64)
    return fail(MCPT_ERR_LIMIT, "scene_upload: BVH deeper than the reference's 64-entry stack");
  UP_OK(hipMalloc(&out->nodes, (n - 1) * sizeof(UDevNode)));
  hipLaunchKernelGGL(k_devnodes, dim3(nblk(n - 1, 256)), dim3(256), 0, st, nodes, n, (UDevNode *)out->nodes);
  UP_OK(hipGetLastError());

  // the reference tree 4-wide, breadth-first ids
  {
    std::vector<uint32_t> base(1, 0), cnt(1, 1);  // per level: first id, count
    Node4Rec *q4 = nullptr;
    int32_t *child4 = nullptr, *lvA = nullptr, *lvB = nullptr;
    uint32_t *c4 = nullptr, *p4 = nullptr;
    const int64_t cap = n;  // 4-wide nodes <= internal nodes
    UP_OK(hipMalloc(&q4, cap * sizeof(Node4Rec)));
    out->nodes4 = q4;
    UP_OK(S.alloc(&child4, 4 * cap));
    UP_OK(S.alloc(&lvA, cap));
    UP_OK(S.alloc(&lvB, cap));
    UP_OK(S.alloc(&c4, cap + 1));
    UP_OK(S.alloc(&p4, cap + 1));
    UP_OK(hipMemsetAsync(lvA, 0, 4, st));  // root = binary node 0
    uint32_t total = 1;
    for (;;) {
      const uint32_t b0 = base.back(), c = cnt.back();
      hipLaunchKernelGGL(k_ref4_count, dim3(nblk(c, 256)), dim3(256), 0, st, lvA, c, nodes, c4);
      UP_OK(hipGetLastError());
      UP_OK(hipMemsetAsync(c4 + c, 0, 4, st));
      if (int rc = exscan(c4, p4, (int64_t)c + 1, st, S)) return rc;
      uint32_t nxt = 0;
      if (int rc = d2h(&nxt, p4 + c, 1, st)) return rc;
      hipLaunchKernelGGL(k_ref4_emit, dim3(nblk(c, 256)), dim3(256), 0, st, lvA, c, b0, p4, b0 + c, nodes, q4, lvB,
                         child4);
      UP_OK(hipGetLastError());
      if (nxt == 0) break;
      base.push_back(b0 + c);
      cnt.push_back(nxt);
      total += nxt;
      std::swap(lvA, lvB);
    }
    out->n_nodes4 = total;
    int32_t *need = nullptr;
    UP_OK(S.alloc(&need, total));
    for (size_t k = base.size(); k-- > 0;) {
      hipLaunchKernelGGL(k_need4, dim3(nblk(cnt[k], 256)), dim3(256), 0, st, base[k], cnt[k], q4, child4, need);
      UP_OK(hipGetLastError());
    }
    int32_t need0 = 0;
    if (int rc = d2h(&need0, need, 1, st)) return rc;
    out->depth4 = std::max(need0, 1);
  }

  // ---- the SAH search tree over the reference's leaves
  const int64_t m = n;
  float *lbox = nullptr, *cen = nullptr;
  int32_t *ltri = nullptr, *idx = nullptr, *idx2 = nullptr, *own = nullptr, *own2 = nullptr, *slot_of = nullptr;
  SahNode *sn = nullptr;
  UP_OK(S.alloc(&lbox, 6 * m));
  UP_OK(S.alloc(&cen, 3 * m));
  UP_OK(S.alloc(&ltri, m));
  UP_OK(S.alloc(&idx, m));
  UP_OK(S.alloc(&idx2, m));
  UP_OK(S.alloc(&own, m));
  UP_OK(S.alloc(&own2, m));
  UP_OK(S.alloc(&sn, 2 * m - 1));
  UP_OK(S.alloc(&slot_of, 2 * m - 1));
  hipLaunchKernelGGL(k_leaf_init, dim3(nblk(m, 256)), dim3(256), 0, st, nodes, m, lbox, ltri, cen, idx, own);
  UP_OK(hipGetLastError());
  UP_OK(hipMemsetAsync(slot_of, 0xFF, (2 * m - 1) * sizeof(int32_t), st));  // -1: not a large range
  {
    SahNode root;
    std::memset(&root, 0, sizeof(root));
    root.lo = 0;
    root.hi = (int32_t)m;
    root.depth = 0;
    UP_OK(hipMemcpyAsync(sn, &root, sizeof(root), hipMemcpyHostToDevice, st));
    UP_OK(hipStreamSynchronize(st));  // `root` leaves scope
  }
  const int64_t max_large = m / kSmall + 2;
  int32_t *large = nullptr, *large2 = nullptr, *small = nullptr;
  uint32_t *n_large2 = nullptr, *n_small = nullptr, *flag = nullptr, *pre = nullptr;
  Split *sp = nullptr;
  Bins *bins = nullptr;
  LargeOut *lo_out = nullptr;
  UP_OK(S.alloc(&large, 2 * max_large));
  UP_OK(S.alloc(&large2, 2 * max_large));
  UP_OK(S.alloc(&small, m));
  UP_OK(S.alloc(&n_large2, 1));
  UP_OK(S.alloc(&n_small, 1));
  UP_OK(S.alloc(&flag, m + 1));
  UP_OK(S.alloc(&pre, m + 1));
  UP_OK(S.alloc(&sp, 2 * max_large));
  UP_OK(S.alloc(&bins, 2 * max_large));
  UP_OK(S.alloc(&lo_out, 2 * max_large));
  UP_OK(hipMemsetAsync(n_small, 0, 4, st));
  uint32_t n_large = 0;
  if (m > kSmall) {
    UP_OK(hipMemsetAsync(large, 0, 4, st));  // the root, binary node 0
    n_large = 1;
  } else {
    UP_OK(hipMemsetAsync(small, 0, 4, st));
    UP_OK(hipMemsetD32Async((hipDeviceptr_t)n_small, 1, 1, st));
  }
  while (n_large > 0) {
    hipLaunchKernelGGL(k_large_slots, dim3(n_large), dim3(64), 0, st, large, n_large, 0, slot_of, sp, bins);
    UP_OK(hipGetLastError());
    hipLaunchKernelGGL(k_cbounds, dim3(nblk(m, kBinChunk)), dim3(256), 0, st, idx, cen, own, slot_of, m, sp);
    UP_OK(hipGetLastError());
    hipLaunchKernelGGL(k_bins, dim3(nblk(m, kBinChunk)), dim3(256), 0, st, idx, cen, lbox, own, slot_of, m, sp, bins);
    UP_OK(hipGetLastError());
    UP_OK(hipMemsetAsync(n_large2, 0, 4, st));
    hipLaunchKernelGGL(k_large_split, dim3(nblk(n_large, 64)), dim3(64), 0, st, n_large, sp, bins, sn, lo_out, large2,
                       n_large2, small, n_small);
    UP_OK(hipGetLastError());
    hipLaunchKernelGGL(k_flags, dim3(nblk(m, 256)), dim3(256), 0, st, idx, cen, own, slot_of, lo_out, m, flag);
    UP_OK(hipGetLastError());
    UP_OK(hipMemsetAsync(flag + m, 0, 4, st));
    if (int rc = exscan(flag, pre, m + 1, st, S)) return rc;
    hipLaunchKernelGGL(k_place, dim3(nblk(m, 256)), dim3(256), 0, st, idx, own, slot_of, lo_out, sn, flag, pre, m, idx2,
                       own2);
    UP_OK(hipGetLastError());
    std::swap(idx, idx2);
    std::swap(own, own2);
    hipLaunchKernelGGL(k_large_slots, dim3(n_large), dim3(64), 0, st, large, n_large, 1, slot_of, sp, bins);
    UP_OK(hipGetLastError());
    if (int rc = d2h(&n_large, n_large2, 1, st)) return rc;
    if (n_large > 2 * max_large) return fail(MCPT_ERR_HIP, "scene_upload_device: large-range list overflow");
    std::swap(large, large2);
  }
  uint32_t n_small_h = 0;
  if (int rc = d2h(&n_small_h, n_small, 1, st)) return rc;
  if (n_small_h > 0) {
    hipLaunchKernelGGL(k_small, dim3(n_small_h), dim3(64), 0, st, small, n_small_h, idx, cen, lbox, sn);
    UP_OK(hipGetLastError());
  }
  // the binary SAH tree by depth (stable radix sort of the depths), then
  // boxes and the collapse DP bottom-up
  const int64_t nb = 2 * m - 1;
  uint32_t *dkey = nullptr, *dkey2 = nullptr, *maxd = nullptr, *hist = nullptr;
  int32_t *ids = nullptr, *ids2 = nullptr;
  UP_OK(S.alloc(&dkey, nb));
  UP_OK(S.alloc(&dkey2, nb));
  UP_OK(S.alloc(&ids, nb));
  UP_OK(S.alloc(&ids2, nb));
  UP_OK(S.alloc(&maxd, 1));
  UP_OK(hipMemsetAsync(maxd, 0, 4, st));
  hipLaunchKernelGGL(k_depth_keys, dim3(nblk(nb, 256)), dim3(256), 0, st, sn, nb, dkey, ids, maxd);
  UP_OK(hipGetLastError());
  uint32_t maxd_h = 0;
  if (int rc = d2h(&maxd_h, maxd, 1, st)) return rc;
  {
    int end_bit = 1;
    while (end_bit < 32 && (maxd_h >> end_bit) != 0) ++end_bit;
    size_t bytes = 0;
    UP_OK(hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, dkey, dkey2, ids, ids2, (int)nb, 0, end_bit, st));
    char *tmp = nullptr;
    UP_OK(S.alloc(&tmp, bytes));
    UP_OK(hipcub::DeviceRadixSort::SortPairs(tmp, bytes, dkey, dkey2, ids, ids2, (int)nb, 0, end_bit, st));
  }
  UP_OK(S.alloc(&hist, maxd_h + 1));
  hipLaunchKernelGGL(k_depth_starts, dim3(nblk(nb, 256)), dim3(256), 0, st, dkey2, nb, hist);
  UP_OK(hipGetLastError());
  std::vector<uint32_t> doff(maxd_h + 2, 0);
  if (int rc = d2h(doff.data(), hist, maxd_h + 1, st)) return rc;
  doff[maxd_h + 1] = (uint32_t)nb;
  std::vector<uint32_t> hist_h(maxd_h + 1);
  for (uint32_t d = 0; d <= maxd_h; ++d) hist_h[d] = doff[d + 1] - doff[d];
  DP *dp = nullptr;
  UP_OK(S.alloc(&dp, nb));
  for (int64_t d = maxd_h; d >= 0; --d) {
    const uint32_t c = hist_h[d];
    if (!c) continue;
    hipLaunchKernelGGL(k_box_dp_level, dim3(nblk(c, 256)), dim3(256), 0, st, ids2 + doff[d], c, sn, dp);
    UP_OK(hipGetLastError());
  }

  // the wide tree: levels of wide nodes from the root (internal entries)
  int32_t *wnode = nullptr, *wkid = nullptr, *out_id = nullptr, *need = nullptr;
  uint32_t *wc = nullptr, *wp = nullptr, *wsize = nullptr, *wrank = nullptr, *nk_by_rank = nullptr, *alloc = nullptr;
  const int64_t wcap = m;  // wide nodes <= internal binary nodes
  UP_OK(S.alloc(&wnode, wcap));
  UP_OK(S.alloc(&wkid, 4 * wcap));
  UP_OK(S.alloc(&wc, wcap + 1));
  UP_OK(S.alloc(&wp, wcap + 1));
  UP_OK(hipMemsetAsync(wnode, 0, 4, st));  // wide node 0 = binary root 0
  std::vector<uint32_t> wbase(1, 0), wcnt(1, 1);
  uint32_t nw = 1;
  for (;;) {
    const uint32_t b0 = wbase.back(), c = wcnt.back();
    hipLaunchKernelGGL(k_wide_count, dim3(nblk(c, 256)), dim3(256), 0, st, wnode + b0, c, sn, dp, wc);
    UP_OK(hipGetLastError());
    UP_OK(hipMemsetAsync(wc + c, 0, 4, st));
    if (int rc = exscan(wc, wp, (int64_t)c + 1, st, S)) return rc;
    uint32_t nxt = 0;
    if (int rc = d2h(&nxt, wp + c, 1, st)) return rc;
    hipLaunchKernelGGL(k_wide_next, dim3(nblk(c, 256)), dim3(256), 0, st, wnode + b0, c, b0, wp, b0 + c, sn, dp, wnode,
                       wkid);
    UP_OK(hipGetLastError());
    if (nxt == 0) break;
    wbase.push_back(b0 + c);
    wcnt.push_back(nxt);
    nw += nxt;
  }
  UP_OK(S.alloc(&wsize, nw));
  UP_OK(S.alloc(&wrank, nw));
  UP_OK(S.alloc(&nk_by_rank, nw + 1));
  UP_OK(S.alloc(&alloc, nw + 1));
  UP_OK(S.alloc(&out_id, nw));
  UP_OK(S.alloc(&need, nw));
  for (size_t k = wbase.size(); k-- > 0;) {
    hipLaunchKernelGGL(k_wide_size, dim3(nblk(wcnt[k], 256)), dim3(256), 0, st, wbase[k], wcnt[k], wkid, wsize);
    UP_OK(hipGetLastError());
  }
  UP_OK(hipMemsetAsync(wrank, 0, 4, st));
  UP_OK(hipMemsetAsync(nk_by_rank + nw, 0, 4, st));
  for (size_t k = 0; k < wbase.size(); ++k) {
    hipLaunchKernelGGL(k_wide_rank, dim3(nblk(wcnt[k], 256)), dim3(256), 0, st, wbase[k], wcnt[k], wkid, wsize, wrank,
                       nk_by_rank);
    UP_OK(hipGetLastError());
  }
  if (int rc = exscan(nk_by_rank, alloc, (int64_t)nw + 1, st, S)) return rc;
  Node4Rec *near = nullptr;
  UP_OK(hipMalloc(&near, nw * sizeof(Node4Rec)));
  out->near4 = near;
  out->n_near4 = nw;
  UP_OK(hipMemsetAsync(out_id, 0, 4, st));  // the root's record is node 0
  for (size_t k = 0; k < wbase.size(); ++k) {
    hipLaunchKernelGGL(k_wide_emit, dim3(nblk(wcnt[k], 256)), dim3(256), 0, st, wbase[k], wcnt[k], wnode, wkid, wrank,
                       alloc, sn, dp, ltri, out_id, near);
    UP_OK(hipGetLastError());
  }
  for (size_t k = wbase.size(); k-- > 0;) {
    hipLaunchKernelGGL(k_wide_need, dim3(nblk(wcnt[k], 256)), dim3(256), 0, st, wbase[k], wcnt[k], out_id, near, need);
    UP_OK(hipGetLastError());
  }
  int32_t need0 = 0;
  if (int rc = d2h(&need0, need, 1, st)) return rc;  // need_by_id[0]: the root's
  out->depth4 = std::max(out->depth4, std::max(need0, 1));
  if (out->depth4 > 192) return fail(MCPT_ERR_LIMIT, "scene_upload: 4-wide stack too deep");

  // the quantized tree, when every leaf box is its triangle's vertex bounds
  if (int rc = d2h(&fl, flags, 1, st)) return rc;
  out->quant = (fl & 64) == 0;
  if (out->quant) {
    UP_OK(hipMemsetAsync(flags, 0, 4, st));
    UP_OK(hipMalloc(&out->near4q, nw * sizeof(Node4Q)));
    hipLaunchKernelGGL(k_quantize, dim3(nblk(nw, 128)), dim3(128), 0, st, near, (int64_t)nw, (Node4Q *)out->near4q,
                       flags);
    UP_OK(hipGetLastError());
    if (int rc = d2h(&fl, flags, 1, st)) return rc;
    out->quant = fl == 0;
  }
  if (!out->quant) {
    if (out->near4q) (void)hipFree(out->near4q);
    if (out->triq) (void)hipFree(out->triq);
    out->near4q = nullptr;
    out->triq = nullptr;
  }
  UP_OK(hipStreamSynchronize(st));
  return MCPT_OK;
}

}  // namespace mcpt
