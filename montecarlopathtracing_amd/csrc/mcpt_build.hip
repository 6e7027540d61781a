// mcpt_build.hip — the reference HLBVH built on the GPU.
//
// Same tree, bit for bit, as the host build mcpt_build_hlbvh (mcpt_host.cpp),
// i.e. as MCPT/BVH/hlbvh.cpp:92-200:
//  * triangle boxes min(min(v0,v1),v2) with std::min/std::max semantics,
//    centroids 0.5f*(bbmin+bbmax), the centroid bounds, and the 30-bit Morton
//    code of round((c - gmin) / gsize * 1024) (1024 -> 1023; NaN -> 0 as the
//    reference's MSVC build converts it).  Compiled with -ffp-contract=off and
//    IEEE division, the host's float semantics;
//  * a stable radix sort on the code (hipCUB; hlbvh.cpp's 5 stable 6-bit
//    LSD passes give the same order);
//  * the reference numbers internal nodes by their range (range [lo, hi]
//    split at s has children s / s+1, or leaves s+n-1 / s+n), so the tree
//    does not depend on the order ranges are processed in: each level of
//    ranges is split in parallel with the reference's binary search
//    (hlbvh.cpp:152-161);
//  * refit level by level from the deepest, kernel boundaries ordering the
//    child boxes before their parents (no cross-XCD atomics).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/mcpt_hip.h"

namespace mcpt {
int fail(int code, const std::string &msg);  // mcpt_host.cpp
}

namespace {

__device__ inline float smin(float a, float b) { return (b < a) ? b : a; }  // std::min
__device__ inline float smax(float a, float b) { return (a < b) ? b : a; }  // std::max

struct Bounds {
  float mn[3], mx[3];
};
struct BoundsOp {
  __device__ Bounds operator()(const Bounds &a, const Bounds &b) const {
    Bounds r;
    for (int k = 0; k < 3; ++k) r.mn[k] = smin(a.mn[k], b.mn[k]), r.mx[k] = smax(a.mx[k], b.mx[k]);
    return r;
  }
};

// triangle boxes (w = 0, packFloat zero-initialises it) and centroids
__global__ void k_boxes(const mcpt_triangle *__restrict__ t, int64_t n, float4 *bmin, float4 *bmax, Bounds *cen) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float lo[3], hi[3], c[3];
  for (int k = 0; k < 3; ++k) {
    lo[k] = smin(smin(t[i].v[0][k], t[i].v[1][k]), t[i].v[2][k]);
    hi[k] = smax(smax(t[i].v[0][k], t[i].v[1][k]), t[i].v[2][k]);
    c[k] = 0.5f * (lo[k] + hi[k]);
  }
  bmin[i] = make_float4(lo[0], lo[1], lo[2], 0.0f);
  bmax[i] = make_float4(hi[0], hi[1], hi[2], 0.0f);
  Bounds b;
  for (int k = 0; k < 3; ++k) b.mn[k] = b.mx[k] = c[k];
  cen[i] = b;
}

__device__ inline uint32_t spread_bits10(uint32_t x) {  // hlbvh.cpp:12-23
  if (x == (1u << 10)) --x;
  x = (x | (x << 16)) & 0x030000FFu;
  x = (x | (x << 8)) & 0x0300F00Fu;
  x = (x | (x << 4)) & 0x030C30C3u;
  x = (x | (x << 2)) & 0x09249249u;
  return x;
}
__device__ inline uint32_t to_uint_like_msvc(float v) {  // see mcpt_host.cpp
  const float r = __builtin_roundf(v);
  if (!(r > -9.2233720368547758e18f && r < 9.2233720368547758e18f)) return 0u;
  return (uint32_t)(int64_t)r;
}

__global__ void k_morton(const Bounds *__restrict__ cen, const Bounds *__restrict__ g, int64_t n, uint32_t *code,
                         int32_t *id) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Bounds G = *g;
  uint32_t q[3];
  for (int k = 0; k < 3; ++k) {
    const float gsize = G.mx[k] - G.mn[k];
    float x = (cen[i].mn[k] - G.mn[k]) / gsize;  // IEEE division (this file keeps HIP's default)
    x *= 1024.0f;
    q[k] = to_uint_like_msvc(x);
  }
  code[i] = (spread_bits10(q[2]) << 2) | (spread_bits10(q[1]) << 1) | spread_bits10(q[0]);
  id[i] = (int32_t)i;
}

struct Range {
  uint32_t lo, hi, node;
};

__device__ inline int delta(const uint32_t *c, uint32_t a, uint32_t b) {  // hlbvh.cpp:138-150
  const uint32_t x = c[a] ^ c[b];
  return x == 0 ? 32 : __builtin_clz(x);  // codes < 2^30: the reference's shift loop is clz
}

// one level of the top-down split (hlbvh.cpp:165-188)
__global__ void k_split(const Range *__restrict__ in, uint32_t count, const uint32_t *__restrict__ code, uint32_t n,
                        mcpt_bvh_node *nodes, Range *out, uint32_t *out_count) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const Range r = in[i];
  uint32_t left = r.lo, right = r.hi, s;
  const int target = delta(code, left, right);
  if (target == 32) {
    s = (right + left) >> 1;
  } else {
    do {
      const uint32_t mid = (right + left) >> 1;
      if (delta(code, left, mid) > target)
        left = mid;
      else
        right = mid;
    } while (right > left + 1);
    s = left;
  }
  const uint32_t li = (s != r.lo) ? s : s + n - 1;
  const uint32_t ri = (s + 1 != r.hi) ? s + 1 : s + n;
  nodes[r.node].left = (int32_t)li;
  nodes[li].parent = (int32_t)r.node;
  nodes[r.node].right = (int32_t)ri;
  nodes[ri].parent = (int32_t)r.node;
  const uint32_t k = (li == s) + (ri == s + 1);
  if (k) {
    uint32_t o = atomicAdd(out_count, k);
    if (li == s) out[o++] = Range{r.lo, s, s};
    if (ri == s + 1) out[o] = Range{s + 1, r.hi, s + 1};
  }
}

__global__ void k_leaves(const int32_t *__restrict__ id, const float4 *__restrict__ bmin,
                         const float4 *__restrict__ bmax, int64_t n, mcpt_bvh_node *nodes) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  mcpt_bvh_node &L = nodes[n - 1 + i];
  const int32_t t = id[i];
  L.left = L.right = t;
  const float4 a = bmin[t], b = bmax[t];
  L.bbmin[0] = a.x, L.bbmin[1] = a.y, L.bbmin[2] = a.z, L.bbmin[3] = a.w;
  L.bbmax[0] = b.x, L.bbmax[1] = b.y, L.bbmax[2] = b.z, L.bbmax[3] = b.w;
}

// refit one level (hlbvh.cpp:64-76: min(left, right), max(left, right))
__global__ void k_refit(const Range *__restrict__ lvl, uint32_t count, mcpt_bvh_node *nodes) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  mcpt_bvh_node &P = nodes[lvl[i].node];
  const mcpt_bvh_node &A = nodes[P.left], &B = nodes[P.right];
  for (int k = 0; k < 4; ++k) {
    P.bbmin[k] = smin(A.bbmin[k], B.bbmin[k]);
    P.bbmax[k] = smax(A.bbmax[k], B.bbmax[k]);
  }
}

inline unsigned blocks_for(int64_t n, int b) { return (unsigned)((n + b - 1) / b); }

}  // namespace

#define BUILD_OK(expr)                                                                       \
  do {                                                                                       \
    hipError_t e_ = (expr);                                                                  \
    if (e_ != hipSuccess) {                                                                  \
      rc = mcpt::fail(MCPT_ERR_HIP, std::string("build_hlbvh_device: ") + #expr + ": " + hipGetErrorString(e_)); \
      goto done;                                                                             \
    }                                                                                        \
  } while (0)

extern "C" int mcpt_build_hlbvh_device(const mcpt_triangle *tris, int64_t n, mcpt_bvh_node *nodes, void *stream) {
  if (!tris || !nodes || n <= 0) return mcpt::fail(MCPT_ERR_ARG, "build_hlbvh_device: bad argument");
  if (n > (int64_t)0x3FFFFFFF) return mcpt::fail(MCPT_ERR_LIMIT, "build_hlbvh_device: too many triangles");
  hipStream_t st = (hipStream_t)stream;
  int rc = MCPT_OK;
  float4 *bmin = nullptr, *bmax = nullptr;
  Bounds *cen = nullptr, *gbox = nullptr;
  uint32_t *code = nullptr, *code_s = nullptr, *cnt = nullptr;
  int32_t *id = nullptr, *id_s = nullptr;
  Range *ranges = nullptr;
  void *tmp = nullptr;
  size_t tmp_bytes = 0, red_bytes = 0;
  std::vector<uint32_t> level_off;
  const int64_t nn = 2 * n - 1;
  Bounds init;
  for (int k = 0; k < 3; ++k) init.mn[k] = FLT_MAX, init.mx[k] = -FLT_MAX;

  BUILD_OK(hipMalloc(&bmin, n * sizeof(float4)));
  BUILD_OK(hipMalloc(&bmax, n * sizeof(float4)));
  BUILD_OK(hipMalloc(&cen, n * sizeof(Bounds)));
  BUILD_OK(hipMalloc(&gbox, sizeof(Bounds)));
  BUILD_OK(hipMalloc(&code, n * sizeof(uint32_t)));
  BUILD_OK(hipMalloc(&code_s, n * sizeof(uint32_t)));
  BUILD_OK(hipMalloc(&id, n * sizeof(int32_t)));
  BUILD_OK(hipMalloc(&id_s, n * sizeof(int32_t)));
  BUILD_OK(hipMalloc(&ranges, std::max<int64_t>(n - 1, 1) * sizeof(Range)));
  BUILD_OK(hipMalloc(&cnt, sizeof(uint32_t)));
  BUILD_OK(hipMemsetAsync(nodes, 0, nn * sizeof(mcpt_bvh_node), st));
  hipLaunchKernelGGL(k_boxes, dim3(blocks_for(n, 256)), dim3(256), 0, st, tris, n, bmin, bmax, cen);
  BUILD_OK(hipGetLastError());
  BUILD_OK(hipcub::DeviceReduce::Reduce(nullptr, red_bytes, cen, gbox, (int)n, BoundsOp(), init, st));
  BUILD_OK(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, code, code_s, id, id_s, (int)n, 0, 30, st));
  BUILD_OK(hipMalloc(&tmp, std::max(tmp_bytes, red_bytes)));
  BUILD_OK(hipcub::DeviceReduce::Reduce(tmp, red_bytes, cen, gbox, (int)n, BoundsOp(), init, st));
  hipLaunchKernelGGL(k_morton, dim3(blocks_for(n, 256)), dim3(256), 0, st, cen, gbox, n, code, id);
  BUILD_OK(hipGetLastError());
  BUILD_OK(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, code, code_s, id, id_s, (int)n, 0, 30, st));
  {
    // parent of the root is -1 (hlbvh.cpp:164)
    const int32_t minus1 = -1;
    BUILD_OK(hipMemcpyAsync(&nodes[0].parent, &minus1, sizeof(int32_t), hipMemcpyHostToDevice, st));
  }
  if (n > 1) {
    // levels of ranges are appended to `ranges`: level k = [level_off[k], level_off[k+1])
    const Range root{0, (uint32_t)(n - 1), 0};
    BUILD_OK(hipMemcpyAsync(ranges, &root, sizeof(Range), hipMemcpyHostToDevice, st));
    level_off.push_back(0);
    level_off.push_back(1);
    for (;;) {
      const uint32_t a = level_off[level_off.size() - 2], b = level_off.back();
      if (b == a) break;
      BUILD_OK(hipMemsetAsync(cnt, 0, sizeof(uint32_t), st));
      hipLaunchKernelGGL(k_split, dim3(blocks_for(b - a, 256)), dim3(256), 0, st, ranges + a, b - a, code_s,
                         (uint32_t)n, nodes, ranges + b, cnt);
      BUILD_OK(hipGetLastError());
      uint32_t c = 0;
      BUILD_OK(hipMemcpyAsync(&c, cnt, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
      BUILD_OK(hipStreamSynchronize(st));
      level_off.push_back(b + c);
    }
  }
  hipLaunchKernelGGL(k_leaves, dim3(blocks_for(n, 256)), dim3(256), 0, st, id_s, bmin, bmax, n, nodes);
  BUILD_OK(hipGetLastError());
  for (size_t k = level_off.size() >= 2 ? level_off.size() - 2 : 0; k-- > 0;) {
    const uint32_t a = level_off[k], b = level_off[k + 1];
    hipLaunchKernelGGL(k_refit, dim3(blocks_for(b - a, 256)), dim3(256), 0, st, ranges + a, b - a, nodes);
    BUILD_OK(hipGetLastError());
  }
  BUILD_OK(hipStreamSynchronize(st));
done:
  for (void *p : {(void *)bmin, (void *)bmax, (void *)cen, (void *)gbox, (void *)code, (void *)code_s, (void *)id,
                  (void *)id_s, (void *)ranges, (void *)cnt, tmp})
    if (p) (void)hipFree(p);
  return rc;
}

// ===========================================================================
// Treelet restructuring (MCPT/BVH/treeletBVH.cpp:1-387, TreeletBVH<CPU>), the
// pass the reference applies for "bvhtype": "treelet" (scenebuild.cpp:70-73).
//
// The reference walks up from every leaf along the ORIGINAL parent links and
// rebuilds a node's treelet when its second child walk arrives.  A rebuild of
// node X only rearranges nodes inside X's original subtree, and reads only
// that subtree, so any order that rebuilds a node after all its original
// descendants gives the same tree.  Here: the internal nodes are grouped by
// original depth (top-down frontier), and each depth is one launch, deepest
// first, one wave per node.  Kernel boundaries order a child treelet's writes
// before its ancestors' reads (no cross-XCD flags).  Inside a wave:
//  * lane 0 grows the treelet with the reference's binary heap, written out
//    (pop_heap = Floyd's hole descent + sift-up, push_heap = sift-up, the
//    libstdc++ / MSVC STL algorithms; oracle/mcpt_oracle_treelet.cpp uses
//    std::pop_heap/push_heap and the tests compare bit for bit);
//  * the 2^n - 1 union areas are one subset per lane;
//  * the subset DP runs one popcount class per step, one subset per lane
//    (subsets of equal size never read each other, so the reference's
//    sequential (popcount, value) order gives the same costs);
//  * lane 0 rebuilds and refits (at most 6 nodes).
// getInformation's SAH pass (treeletBVH.cpp:321-347) runs bottom-up by the
// same depth groups; its first-leaf quirk (node n-1 is read as an internal
// node whose children are both node `left`) is evaluated after every other
// node off the root-to-(n-1) path, then that path, deepest first.
// ===========================================================================
namespace {

constexpr int TL_MAX = 7;                           // treeletBVH.cpp:14
constexpr float TL_CINN = 1.2f, TL_CTRI = 1.0f, TL_CLEAF = 0.0f;  // auxiliary.h:9-11

__device__ inline float tl_area(const float *mn, const float *mx) {  // auxiliary.cpp:15-18
  const float x = mx[0] - mn[0], y = mx[1] - mn[1], z = mx[2] - mn[2];
  return 2.0f * (x * y + x * z + y * z);
}
inline float tl_area_host(const mcpt_bvh_node &b) {
  const float x = b.bbmax[0] - b.bbmin[0], y = b.bbmax[1] - b.bbmin[1], z = b.bbmax[2] - b.bbmin[2];
  return 2.0f * (x * y + x * z + y * z);
}

struct TlQ {
  int id;
  float value;
};
__device__ inline bool tl_less(const TlQ &a, const TlQ &b) {  // QueueNode::operator< (:36-41)
  if (a.value < b.value) return true;
  return a.value == b.value && a.id < b.id;
}
__device__ inline void tl_sift_up(TlQ *h, int hole, TlQ v) {  // __push_heap
  int parent = (hole - 1) / 2;
  while (hole > 0 && tl_less(h[parent], v)) {
    h[hole] = h[parent];
    hole = parent;
    parent = (hole - 1) / 2;
  }
  h[hole] = v;
}
__device__ inline void tl_push(TlQ *h, int &n, TlQ v) {  // push_back + push_heap
  h[n] = v;
  ++n;
  tl_sift_up(h, n - 1, v);
}
__device__ inline void tl_pop(TlQ *h, int &n) {  // pop_heap + pop_back
  if (n > 1) {
    const int len = n - 1;  // heap size after the move
    TlQ v = h[len];
    h[len] = h[0];
    int hole = 0, child = 0;
    while (child < (len - 1) / 2) {
      child = 2 * (child + 1);
      if (tl_less(h[child], h[child - 1])) --child;
      h[hole] = h[child];
      hole = child;
    }
    if ((len & 1) == 0 && child == (len - 2) / 2) {
      child = 2 * (child + 1);
      h[hole] = h[child - 1];
      hole = child - 1;
    }
    tl_sift_up(h, hole, v);
  }
  --n;
}

// frontier expansion: the internal children of one depth's internal nodes
__global__ void k_tl_expand(const int32_t *__restrict__ in, uint32_t count, const mcpt_bvh_node *__restrict__ nodes,
                            int32_t *out, uint32_t *out_count) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const mcpt_bvh_node &b = nodes[in[i]];
  int32_t c[2];
  uint32_t k = 0;
  for (int32_t x : {b.left, b.right})
    if (nodes[x].left != nodes[x].right) c[k++] = x;
  if (k) {
    uint32_t o = atomicAdd(out_count, k);
    for (uint32_t j = 0; j < k; ++j) out[o + j] = c[j];
  }
}

// getInformation, leaves (the `id > size/2` test of :327: all but node n-1)
__global__ void k_tl_sah_leaves(const mcpt_bvh_node *__restrict__ nodes, int64_t n, float root_area, float *sah) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x + n;  // [n, 2n-2]
  if (i > 2 * n - 2) return;
  sah[i] = (TL_CTRI + TL_CLEAF) * tl_area(nodes[i].bbmin, nodes[i].bbmax) / root_area;
}

// getInformation, one depth of internal nodes off the (n-1) path
__global__ void k_tl_sah_level(const int32_t *__restrict__ lvl, uint32_t count, const uint8_t *__restrict__ on_path,
                               const mcpt_bvh_node *__restrict__ nodes, float root_area, float *sah) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const int32_t x = lvl[i];
  if (on_path[x]) return;
  const mcpt_bvh_node &b = nodes[x];
  sah[x] = sah[b.left] + sah[b.right] + TL_CINN * (tl_area(b.bbmin, b.bbmax)) / root_area;
}

// marks the root-to-(n-1) path; flags a cycle of the first-leaf quirk
__global__ void k_tl_mark_path(const mcpt_bvh_node *__restrict__ nodes, int64_t n, uint8_t *on_path, int32_t *err) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const int32_t t = nodes[n - 1].left;
  *err = (t == n - 1) ? 1 : 0;
  for (int32_t p = nodes[n - 1].parent; p != -1; p = nodes[p].parent) {
    on_path[p] = 1;
    if (p == t) *err = 1;
  }
}

// the first leaf (read as internal, both children = node t) and its ancestors
__global__ void k_tl_sah_path(const mcpt_bvh_node *__restrict__ nodes, int64_t n, float root_area, float *sah) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const mcpt_bvh_node &f = nodes[n - 1];
  sah[n - 1] = sah[f.left] + sah[f.right] + TL_CINN * (tl_area(f.bbmin, f.bbmax)) / root_area;
  for (int32_t p = f.parent; p != -1; p = nodes[p].parent) {
    const mcpt_bvh_node &b = nodes[p];
    sah[p] = sah[b.left] + sah[b.right] + TL_CINN * (tl_area(b.bbmin, b.bbmax)) / root_area;
  }
}

// reconstructTreelet (:30-318) for one depth's nodes, one 64-lane wave each
__global__ __launch_bounds__(64) void k_tl_rebuild(const int32_t *__restrict__ lvl, uint32_t count,
                                                    mcpt_bvh_node *nodes, float *sah, float root_area) {
  __shared__ TlQ pq[TL_MAX + 1];
  __shared__ int32_t freeN[TL_MAX];
  __shared__ int npq_s, nfree_s;
  __shared__ float area[128], cost[128];
  __shared__ int32_t part[128];
  __shared__ float bmn[TL_MAX][4], bmx[TL_MAX][4];
  if (blockIdx.x >= count) return;
  const int lane = threadIdx.x;
  const int32_t root = lvl[blockIdx.x];

  if (lane == 0) {  // grow the treelet (:44-80)
    int n = 0, nf = 0;
    tl_push(pq, n, TlQ{root, sah[root]});
    while (n < TL_MAX) {
      const TlQ mx = pq[0];
      tl_pop(pq, n);
      if (mx.value < 0.0f) {
        pq[n++] = TlQ{mx.id, -1.0f};  // push_back without push_heap (:55)
        break;
      }
      const int32_t l = nodes[mx.id].left, r = nodes[mx.id].right;
      if (l == r) {
        tl_push(pq, n, TlQ{mx.id, mx.id * (-1.0f)});
        continue;
      }
      tl_push(pq, n, TlQ{l, sah[l]});
      tl_push(pq, n, TlQ{r, sah[r]});
      freeN[nf++] = mx.id;
    }
    npq_s = n;
    nfree_s = nf;
    for (int j = 0; j < n; ++j)
      for (int k = 0; k < 4; ++k) bmn[j][k] = nodes[pq[j].id].bbmin[k], bmx[j][k] = nodes[pq[j].id].bbmax[k];
  }
  for (int s = lane; s < 128; s += 64) cost[s] = 0.0f, part[s] = 0;
  __syncthreads();
  const int NN = npq_s;  // pq.size() never exceeds MAX_NODE, so NOW_NODE == pq.size()
  if (NN < 3) return;
  const int full = (1 << NN) - 1;

  // union areas (:95-119): bit k of the subset <-> pq[NN-1-k]
  for (int s = lane + 1; s <= full; s += 64) {
    float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (int j = 0; j < NN; ++j) {
      if ((s >> (NN - 1 - j)) & 1) {
        for (int k = 0; k < 3; ++k) {
          mx[k] = smax(mx[k], bmx[j][k]);
          mn[k] = smin(mn[k], bmn[j][k]);
        }
      }
    }
    area[s] = tl_area(mn, mx);
  }
  if (lane < NN) cost[1 << lane] = sah[pq[lane].id];  // (:125-127): bit i <-> pq[i]
  __syncthreads();

  // subset DP (:158-199), one popcount class per step
  for (int k = 2; k <= NN; ++k) {
    for (int s = lane + 1; s <= full; s += 64) {
      if (__builtin_popcount(s) != k) continue;
      float cs = FLT_MAX, ps = 0.0f;
      const int delta = (s - 1) & s;
      int p = (-delta) & s;
      do {
        const float c = cost[p] + cost[s ^ p];
        if (c < cs) {
          cs = c;
          ps = (float)p;
        }
        p = (p - delta) & s;
      } while (p != 0);
      cost[s] = TL_CINN * area[s] + cs;
      part[s] = (int32_t)ps;
    }
    __syncthreads();
  }

  if (lane == 0) {  // rebuild (:201-291) breadth-first, then refit (:293-302)
    struct Split {
      int parent_code, self_code, parent_id;
    };
    Split a[TL_MAX], b[TL_MAX];
    Split *cur = a, *nxt = b;
    int ncur = 1, nnxt = 0, fnow = 1;
    cur[0] = Split{full, part[full], freeN[0]};
    auto leaf_of = [&](int code) { return pq[NN - 1 - (31 - __builtin_clz((unsigned)code))].id; };
    while (ncur > 0) {
      for (int x = 0; x < ncur; ++x) {
        const Split i = cur[x];
        const int lcode = part[i.self_code], rcode = part[i.self_code ^ i.parent_code];
        const int pid = i.parent_id;
        if (__builtin_popcount(i.self_code) == 1) {
          const int node = leaf_of(i.self_code);
          nodes[pid].left = node;
          nodes[node].parent = pid;
        } else {
          const int f = freeN[fnow++];
          nodes[pid].left = f;
          nxt[nnxt++] = Split{i.self_code, lcode, f};
          nodes[f].parent = pid;
        }
        const int rc = i.parent_code ^ i.self_code;
        if (__builtin_popcount(rc) == 1) {
          const int node = leaf_of(rc);
          nodes[pid].right = node;
          nodes[node].parent = pid;
        } else {
          const int f = freeN[fnow++];
          nodes[pid].right = f;
          nxt[nnxt++] = Split{rc, rcode, f};
          nodes[f].parent = pid;
        }
      }
      Split *t = cur;
      cur = nxt;
      nxt = t;
      ncur = nnxt;
      nnxt = 0;
    }
    for (int i = nfree_s - 1; i >= 0; --i) {
      mcpt_bvh_node &P = nodes[freeN[i]];
      const mcpt_bvh_node &A = nodes[P.left], &B = nodes[P.right];
      for (int k = 0; k < 4; ++k) {
        P.bbmax[k] = smax(A.bbmax[k], B.bbmax[k]);
        P.bbmin[k] = smin(A.bbmin[k], B.bbmin[k]);
      }
      sah[freeN[i]] = sah[P.left] + sah[P.right] + TL_CINN * (tl_area(P.bbmin, P.bbmax)) / root_area;
    }
  }
}

}  // namespace

#define TL_OK(expr)                                                                          \
  do {                                                                                       \
    hipError_t e_ = (expr);                                                                  \
    if (e_ != hipSuccess) {                                                                  \
      rc = mcpt::fail(MCPT_ERR_HIP, std::string("treelet_device: ") + #expr + ": " + hipGetErrorString(e_)); \
      goto done;                                                                             \
    }                                                                                        \
  } while (0)

namespace mcpt {
// Depth groups of the internal nodes of a 2n-1-node tree rooted at 0, top-down:
// lv[off[k] .. off[k+1]) holds depth k.  lv needs n-1 entries, cnt one word.
// Shared by both treelet passes (this file, mcpt_treelet_gpu.hip).
int tree_levels(const mcpt_bvh_node *nodes, int64_t n, hipStream_t st, int32_t *lv, uint32_t *cnt,
                std::vector<uint32_t> &off) {
  int rc = MCPT_OK;
  const int32_t zero = 0;
  off.clear();
  TL_OK(hipMemcpyAsync(lv, &zero, sizeof(int32_t), hipMemcpyHostToDevice, st));
  off.push_back(0);
  off.push_back(1);
  for (;;) {
    const uint32_t a = off[off.size() - 2], b = off.back();
    if (b == a) break;
    if (b > (uint32_t)(n - 1)) {
      rc = mcpt::fail(MCPT_ERR_ARG, "treelet_device: node links do not form a tree");
      goto done;
    }
    TL_OK(hipMemsetAsync(cnt, 0, sizeof(uint32_t), st));
    hipLaunchKernelGGL(k_tl_expand, dim3(blocks_for(b - a, 256)), dim3(256), 0, st, lv + a, b - a, nodes, lv + b, cnt);
    TL_OK(hipGetLastError());
    uint32_t c = 0;
    TL_OK(hipMemcpyAsync(&c, cnt, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    TL_OK(hipStreamSynchronize(st));
    if ((uint64_t)b + c > (uint64_t)(n - 1)) {
      rc = mcpt::fail(MCPT_ERR_ARG, "treelet_device: node links do not form a tree");
      goto done;
    }
    off.push_back(b + c);
  }
  off.pop_back();  // the empty group
  if (off.back() != (uint32_t)(n - 1))
    rc = mcpt::fail(MCPT_ERR_ARG, "treelet_device: expected n-1 internal nodes reachable from the root");
done:
  return rc;
}
}  // namespace mcpt

extern "C" int mcpt_treelet_device(mcpt_bvh_node *nodes, int64_t n_nodes, void *stream) {
  if (!nodes || n_nodes <= 0 || (n_nodes & 1) == 0)
    return mcpt::fail(MCPT_ERR_ARG, "treelet_device: expected a 2n-1-node BVH");
  const int64_t n = (n_nodes + 1) / 2;
  if (n < 2) return MCPT_OK;  // a single leaf: the leaf loop finds no parent
  if (n > (int64_t)0x3FFFFFFF) return mcpt::fail(MCPT_ERR_LIMIT, "treelet_device: too many triangles");
  hipStream_t st = (hipStream_t)stream;
  int rc = MCPT_OK;
  float *sah = nullptr;
  int32_t *lv = nullptr, *err = nullptr;
  uint8_t *on_path = nullptr;
  uint32_t *cnt = nullptr;
  std::vector<uint32_t> off;
  mcpt_bvh_node root_h;
  int32_t err_h = 0;
  float root_area = 0.0f;

  TL_OK(hipMalloc(&sah, n_nodes * sizeof(float)));
  TL_OK(hipMalloc(&lv, (n - 1) * sizeof(int32_t)));
  TL_OK(hipMalloc(&on_path, n_nodes));
  TL_OK(hipMalloc(&err, sizeof(int32_t)));
  TL_OK(hipMalloc(&cnt, sizeof(uint32_t)));
  TL_OK(hipMemcpyAsync(&root_h, nodes, sizeof(root_h), hipMemcpyDeviceToHost, st));
  TL_OK(hipMemsetAsync(on_path, 0, n_nodes, st));
  TL_OK(hipStreamSynchronize(st));
  if (root_h.left == root_h.right) {
    rc = mcpt::fail(MCPT_ERR_ARG, "treelet_device: node 0 must be the internal root");
    goto done;
  }
  root_area = tl_area_host(root_h);  // ::rootArea, fixed before any rebuild (:351)
  rc = mcpt::tree_levels(nodes, n, st, lv, cnt, off);  // depth groups of internal nodes, top-down
  if (rc != MCPT_OK) goto done;
  // getInformation (:343-347)
  hipLaunchKernelGGL(k_tl_mark_path, dim3(1), dim3(64), 0, st, nodes, n, on_path, err);
  TL_OK(hipGetLastError());
  TL_OK(hipMemcpyAsync(&err_h, err, sizeof(int32_t), hipMemcpyDeviceToHost, st));
  TL_OK(hipStreamSynchronize(st));
  if (err_h) {
    rc = mcpt::fail(MCPT_ERR_ARG,
                    "treelet_device: the reference's getInformation recursion does not terminate on this tree "
                    "(leaf n-1's triangle index names one of its ancestors)");
    goto done;
  }
  if (n > 1) {
    hipLaunchKernelGGL(k_tl_sah_leaves, dim3(blocks_for(n - 1, 256)), dim3(256), 0, st, nodes, n, root_area, sah);
    TL_OK(hipGetLastError());
  }
  for (size_t k = off.size() - 1; k-- > 0;) {
    const uint32_t a = off[k], b = off[k + 1];
    if (b == a) continue;
    hipLaunchKernelGGL(k_tl_sah_level, dim3(blocks_for(b - a, 256)), dim3(256), 0, st, lv + a, b - a, on_path, nodes,
                       root_area, sah);
    TL_OK(hipGetLastError());
  }
  hipLaunchKernelGGL(k_tl_sah_path, dim3(1), dim3(64), 0, st, nodes, n, root_area, sah);
  TL_OK(hipGetLastError());
  // treelets, deepest depth first
  for (size_t k = off.size() - 1; k-- > 0;) {
    const uint32_t a = off[k], b = off[k + 1];
    if (b == a) continue;
    hipLaunchKernelGGL(k_tl_rebuild, dim3(b - a), dim3(64), 0, st, lv + a, b - a, nodes, sah, root_area);
    TL_OK(hipGetLastError());
  }
  TL_OK(hipStreamSynchronize(st));
done:
  for (void *p : {(void *)sah, (void *)lv, (void *)on_path, (void *)err, (void *)cnt})
    if (p) (void)hipFree(p);
  return rc;
}

// ===========================================================================
// LCV, the leaf-count-variance metric of "testbvh" (MCPT/bvhtest.cpp:324-444):
// one un-normalised pixel-centre ray per pixel, (i + 0.5f)/W - 0.5f across
// and (j + 0.5f)/H - 0.5f up, from the camera centre; count the leaves whose
// box (and every ancestor's) the ray's slab test accepts with tmin 0.001f,
// no closest-hit pruning; LCV = standard deviation of the counts.  The count
// is a set size, so the visiting order does not matter.  Host float
// semantics (this file: -ffp-contract=off, IEEE division, std::min/std::max).
// ===========================================================================
namespace {

constexpr int LCV_STACK = 256;

__global__ void k_lcv(const mcpt_bvh_node *__restrict__ nodes, float cx, float cy, float cz, float dx, float dy,
                      float dz, float hx, float hy, float hz, float ux, float uy, float uz, int32_t width,
                      int32_t height, uint32_t *counts, int32_t *overflow) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // i * height + j (push order)
  if (k >= (int64_t)width * height) return;
  const int32_t i = (int32_t)(k / height), j = (int32_t)(k % height);
  const float temp1 = (i + 0.5f) / width - 0.5f;
  const float temp2 = (j + 0.5f) / height - 0.5f;
  // distance * direction + temp1 * horizontal + temp2 * up (cl_float4 operators)
  const float o[3] = {cx, cy, cz};
  const float d[3] = {dx + temp1 * hx + temp2 * ux, dy + temp1 * hy + temp2 * uy, dz + temp1 * hz + temp2 * uz};
  int32_t stack[LCV_STACK];
  int sp = 0;
  int32_t cur = 0;
  uint32_t ans = 0;
  for (;;) {
    const mcpt_bvh_node &b = nodes[cur];
    float tmn[3], tmx[3];
    for (int a = 0; a < 3; ++a) {
      const float off1 = (b.bbmin[a] - o[a]) / d[a];
      const float off2 = (b.bbmax[a] - o[a]) / d[a];
      tmn[a] = smin(off1, off2);
      tmx[a] = smax(off1, off2);
    }
    const float tnear = smax(smax(tmn[0], tmn[1]), tmn[2]);
    const float tfar = smin(smin(tmx[0], tmx[1]), tmx[2]);
    const bool hit = !(tfar < tnear || tfar < 0.001f);
    if (hit && b.left == b.right) {
      ++ans;
    } else if (hit) {
      if (sp == LCV_STACK) {
        *overflow = 1;
        break;
      }
      stack[sp++] = b.right;
      cur = b.left;
      continue;
    }
    if (sp == 0) break;
    cur = stack[--sp];
  }
  counts[k] = ans;
}

}  // namespace

#define LCV_OK(expr)                                                                         \
  do {                                                                                       \
    hipError_t e_ = (expr);                                                                  \
    if (e_ != hipSuccess) {                                                                  \
      rc = mcpt::fail(MCPT_ERR_HIP, std::string("bvh_lcv_device: ") + #expr + ": " + hipGetErrorString(e_)); \
      goto done;                                                                             \
    }                                                                                        \
  } while (0)

extern "C" int mcpt_bvh_lcv_device(const mcpt_bvh_node *nodes_dev, int64_t n_nodes, const mcpt_camera *cam,
                                   int32_t width, int32_t height, uint32_t *counts_dev, double *lcv_out,
                                   void *stream) {
  if (!nodes_dev || n_nodes <= 0 || !cam || width <= 0 || height <= 0 || !counts_dev)
    return mcpt::fail(MCPT_ERR_ARG, "bvh_lcv_device: bad argument");
  hipStream_t st = (hipStream_t)stream;
  int rc = MCPT_OK;
  int32_t *ovf = nullptr, ovf_h = 0;
  const int64_t n = (int64_t)width * height;
  std::vector<uint32_t> c;
  const float distance = 0.5f / std::tan(cam->arg / 2);  // bvhtest.cpp:415 (the float overload)
  float dd[3];
  for (int a = 0; a < 3; ++a) dd[a] = distance * cam->direction[a];
  LCV_OK(hipMalloc(&ovf, sizeof(int32_t)));
  LCV_OK(hipMemsetAsync(ovf, 0, sizeof(int32_t), st));
  hipLaunchKernelGGL(k_lcv, dim3(blocks_for(n, 256)), dim3(256), 0, st, nodes_dev, cam->center[0], cam->center[1],
                     cam->center[2], dd[0], dd[1], dd[2], cam->horizontal[0], cam->horizontal[1], cam->horizontal[2],
                     cam->up[0], cam->up[1], cam->up[2], width, height, counts_dev, ovf);
  LCV_OK(hipGetLastError());
  LCV_OK(hipMemcpyAsync(&ovf_h, ovf, sizeof(int32_t), hipMemcpyDeviceToHost, st));
  LCV_OK(hipStreamSynchronize(st));
  if (ovf_h) {
    rc = mcpt::fail(MCPT_ERR_LIMIT, "bvh_lcv_device: tree deeper than the 256-entry traversal stack");
    goto done;
  }
  if (lcv_out) {  // bvhtest.cpp:430-443
    c.resize(n);
    LCV_OK(hipMemcpy(c.data(), counts_dev, n * sizeof(uint32_t), hipMemcpyDeviceToHost));
    double En = 0.0, En2 = 0.0;
    for (uint32_t x : c) {
      En += (double)x;
      En2 += (double)((uint64_t)x * x);
    }
    En /= (double)n;
    En2 /= (double)n;
    *lcv_out = (double)(float)std::sqrt(En2 - En * En);  // LCV returns float
  }
done:
  if (ovf) (void)hipFree(ovf);
  return rc;
}
