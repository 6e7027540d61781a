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
