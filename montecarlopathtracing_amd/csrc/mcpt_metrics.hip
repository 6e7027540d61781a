// mcpt_metrics.hip — the reference's BVH-quality metric EPO on the GPU
// ("testbvh" mode, MCPT/bvhtest.cpp:288-321 EPO_GPU
// over MCPT/kernels/EPO.cl:133-197 calculateEPO).
//
// EPO = sum over leaves of the triangle area that lies inside every OTHER
// node's box (clipped polygon area, x Ctri for leaves / Cinn for internal
// nodes), divided by the total triangle area.  One lane per triangle walks
// the tree left-first from the root, skipping its own ancestors, exactly as
// calculateEPO; the per-triangle sums are added in the reference's order.
//
// Compiled like mcpt_device.hip (-ffp-contract=on, OpenCL-default division
// and sqrt accuracy) with the OpenCL built-ins of mcpt_refmath.h, so that
// every per-triangle value equals the reference kernel's bit for bit on the
// same GPU (tests/test_gpu_bvh.py runs both).  The host half (double sums in
// index order, EPO_GPU's loop) is mcpt_bvh_epo_device below.
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "../../include/mcpt_hip.h"
#include "mcpt_refmath.h"

namespace mcpt {
int fail(int code, const std::string &msg);  // mcpt_host.cpp
}

namespace {

using mcpt::f3;

constexpr float EPO_CTRI = 1.0f, EPO_CINN = 1.2f;  // EPO.cl:1-2
// The reference clips into MyVec3 points[8] (EPO.cl:117); a triangle clipped
// by six planes can reach 9 vertices (more with vertices exactly on a plane),
// which overflows the reference's private arrays (undefined behaviour there).
// Here the arrays are large enough for every case; inputs that would overflow
// the reference are counted in *overflows.
constexpr int EPO_MAXP = 16;
constexpr int EPO_STACK = 128;  // ancestor[128], toTest[128] (EPO.cl:150,163)

struct V3 {
  float s[3];
};
__device__ inline V3 mk3(f3 v) {  // initVec3
  V3 r;
  r.s[0] = v.x, r.s[1] = v.y, r.s[2] = v.z;
  return r;
}
__device__ inline f3 get3(const V3 &v) {  // getValue
  f3 r;
  r.x = v.s[0], r.y = v.s[1], r.z = v.s[2];
  return r;
}
__device__ inline V3 minus3(const V3 &a, const V3 &b) {  // myVecMinus
  V3 r;
  r.s[0] = a.s[0] - b.s[0], r.s[1] = a.s[1] - b.s[1], r.s[2] = a.s[2] - b.s[2];
  return r;
}
__device__ inline f3 xyz(const float *p) {  // .s012
  f3 r;
  r.x = p[0], r.y = p[1], r.z = p[2];
  return r;
}
// cross(float3), length(float3): opencl.bc _Z5crossDv3_fS_, _Z6lengthDv3_f
__device__ inline f3 cl_cross3(f3 a, f3 b) {
  f3 r;
  r.x = __builtin_fmaf(a.y, b.z, b.y * -a.z);
  r.y = __builtin_fmaf(a.z, b.x, b.z * -a.x);
  r.z = __builtin_fmaf(a.x, b.y, b.x * -a.y);
  return r;
}
__device__ inline float cl_length3(f3 p) {
  const float l2 = mcpt::cl_dot3(p, p);
  if (l2 < 0x1p-126f) {
    const f3 q = p * 0x1p86f;
    return mcpt::cl_sqrt(mcpt::cl_dot3(q, q)) * 0x1p-86f;
  }
  if (l2 == __builtin_inff()) {
    const f3 q = p * 0x1p-66f;
    return mcpt::cl_sqrt(mcpt::cl_dot3(q, q)) * 0x1p66f;
  }
  return mcpt::cl_sqrt(l2);
}

__device__ inline int point_in_box(f3 p, f3 mn, f3 mx) {  // EPO.cl:30-42
  return (p.x >= mn.x && p.x <= mx.x && p.y >= mn.y && p.y <= mx.y && p.z >= mn.z && p.z <= mx.z) ? 1 : 0;
}

// roundTr (EPO.cl:45-87): clip the polygon by the plane axis = pos, keeping
// the side arg > 0 ? >= pos : <= pos
__device__ inline void round_tr(V3 *points, int *size, int axis, float pos, int arg) {
  if (*size == 0) return;
  V3 buffer[EPO_MAXP];
  const int bsize = *size;
  for (int i = 0; i < bsize; ++i) buffer[i] = points[i];
  *size = 0;
  int inside[EPO_MAXP];
  if (arg > 0) {
    for (int i = 0; i < bsize; ++i) inside[i] = (buffer[i].s[axis] >= pos ? 1 : 0);
  } else {
    for (int i = 0; i < bsize; ++i) inside[i] = (buffer[i].s[axis] <= pos ? 1 : 0);
  }
  int n = 0;
  auto emit = [&](const V3 &v) {
    if (n < EPO_MAXP) points[n] = v;
    ++n;
  };
  for (int i = 0; i < bsize; ++i) {
    const int i_1 = ((i + 1) == bsize ? 0 : (i + 1));
    if (!inside[i] && !inside[i_1]) continue;
    if (inside[i] && inside[i_1]) {
      emit(buffer[i]);
      continue;
    }
    if (inside[i]) emit(buffer[i]);
    V3 dir = minus3(buffer[i_1], buffer[i]);
    float tans = (pos - buffer[i].s[axis]) / dir.s[axis];
    f3 final_point = get3(buffer[i]) + tans * get3(dir);
    dir = mk3(final_point);
    emit(dir);
  }
  *size = n;  // > EPO_MAXP only for pathological inputs: the caller flags it
}

__device__ inline float p_area(const V3 *points, int size) {  // EPO.cl:90-100
  float ans = 0.0f;
  if (size < 2) return ans;
  for (int i = 1; i < size - 1; ++i) {
    f3 x1 = get3(points[i]) - get3(points[0]);
    f3 x2 = get3(points[i + 1]) - get3(points[0]);
    ans += cl_length3(cl_cross3(x1, x2)) * 0.5f;
  }
  return ans;
}

// INTERSECT (EPO.cl:102-128); *max_size tracks the largest polygon
__device__ inline float intersect_area(const mcpt_triangle &tr, const float *bbmin, const float *bbmax, int *max_size) {
  const f3 mn = xyz(bbmin), mx = xyz(bbmax);
  const f3 v0 = xyz(tr.v[0]), v1 = xyz(tr.v[1]), v2 = xyz(tr.v[2]);
  const int in0 = point_in_box(v0, mn, mx), in1 = point_in_box(v1, mn, mx), in2 = point_in_box(v2, mn, mx);
  if (in0 && in1 && in2) {
    f3 e1 = v1 - v0;
    f3 e2 = v2 - v0;
    return cl_length3(cl_cross3(e1, e2)) * 0.5f;
  }
  V3 points[EPO_MAXP];
  int now = 3;
  points[0] = mk3(v0), points[1] = mk3(v1), points[2] = mk3(v2);
  round_tr(points, &now, 0, bbmin[0], 1);
  if (now > *max_size) *max_size = now;
  if (now > EPO_MAXP) now = EPO_MAXP;
  round_tr(points, &now, 1, bbmin[1], 1);
  if (now > *max_size) *max_size = now;
  if (now > EPO_MAXP) now = EPO_MAXP;
  round_tr(points, &now, 2, bbmin[2], 1);
  if (now > *max_size) *max_size = now;
  if (now > EPO_MAXP) now = EPO_MAXP;
  round_tr(points, &now, 0, bbmax[0], -1);
  if (now > *max_size) *max_size = now;
  if (now > EPO_MAXP) now = EPO_MAXP;
  round_tr(points, &now, 1, bbmax[1], -1);
  if (now > *max_size) *max_size = now;
  if (now > EPO_MAXP) now = EPO_MAXP;
  round_tr(points, &now, 2, bbmax[2], -1);
  if (now > *max_size) *max_size = now;
  return p_area(points, now < EPO_MAXP ? now : EPO_MAXP);
}

// calculateEPO (EPO.cl:133-197), one lane per triangle (leaf gid + n - 1)
__global__ void k_epo(const mcpt_bvh_node *__restrict__ bvh, const mcpt_triangle *__restrict__ tris,
                      float *__restrict__ tri_epo, float *__restrict__ tri_area, uint32_t num_prims,
                      unsigned long long *flags) {
  const size_t gid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= num_prims) return;
  const size_t my_id = gid + num_prims - 1;
  const mcpt_triangle tr = tris[bvh[my_id].left];
  float epo_area = 0.0f;
  int ancestor[EPO_STACK];
  ancestor[0] = (int)my_id;
  int an_size = 1;
  for (int p = bvh[my_id].parent; p != -1 && an_size < EPO_STACK; p = bvh[p].parent) ancestor[an_size++] = p;
  int to_test[EPO_STACK];
  to_test[0] = 0;
  int test_size = 1;
  int max_poly = 0;
  bool overflow = an_size >= EPO_STACK;
  while (test_size > 0) {
    const int now = to_test[--test_size];
    const mcpt_bvh_node &b = bvh[now];
    bool skip = false;
    for (int i = 0; i < an_size; ++i) {
      if (now == ancestor[i]) {
        if (b.left != b.right) {
          if (test_size + 2 > EPO_STACK) { overflow = true; break; }
          to_test[test_size++] = b.right;
          to_test[test_size++] = b.left;
        }
        skip = true;
        break;
      }
    }
    if (skip) continue;
    const float temp_area = intersect_area(tr, b.bbmin, b.bbmax, &max_poly);
    if (temp_area > 0) {
      epo_area += temp_area * (((uint32_t)now >= (num_prims - 1)) ? EPO_CTRI : EPO_CINN);
      if (b.left != b.right) {
        if (test_size + 2 > EPO_STACK) { overflow = true; continue; }
        to_test[test_size++] = b.right;
        to_test[test_size++] = b.left;
      }
    }
  }
  tri_epo[gid] = epo_area;
  tri_area[gid] = cl_length3(cl_cross3(xyz(tr.v[1]) - xyz(tr.v[0]), xyz(tr.v[2]) - xyz(tr.v[0]))) * 0.5f;
  if (max_poly > 8) atomicAdd(&flags[0], 1ull);  // beyond the reference's points[8]
  if (overflow) atomicAdd(&flags[1], 1ull);
}

}  // namespace

#define EPO_OK(expr)                                                                         \
  do {                                                                                       \
    hipError_t e_ = (expr);                                                                  \
    if (e_ != hipSuccess) {                                                                  \
      rc = mcpt::fail(MCPT_ERR_HIP, std::string("bvh_epo_device: ") + #expr + ": " + hipGetErrorString(e_)); \
      goto done;                                                                             \
    }                                                                                        \
  } while (0)

extern "C" int mcpt_bvh_epo_device(const mcpt_bvh_node *nodes_dev, const mcpt_triangle *tris_dev, int64_t n_tris,
                                   float *epo_dev, float *area_dev, double *epo_out, uint64_t *clip_overflows,
                                   void *stream) {
  if (!nodes_dev || !tris_dev || n_tris <= 0 || !epo_dev || !area_dev)
    return mcpt::fail(MCPT_ERR_ARG, "bvh_epo_device: bad argument");
  if (n_tris > (int64_t)0x7FFFFFFF) return mcpt::fail(MCPT_ERR_LIMIT, "bvh_epo_device: too many triangles");
  hipStream_t st = (hipStream_t)stream;
  int rc = MCPT_OK;
  unsigned long long *flags = nullptr, flags_h[2] = {0, 0};
  std::vector<float> e, a;
  EPO_OK(hipMalloc(&flags, sizeof(flags_h)));
  EPO_OK(hipMemsetAsync(flags, 0, sizeof(flags_h), st));
  hipLaunchKernelGGL(k_epo, dim3((unsigned)((n_tris + 63) / 64)), dim3(64), 0, st, nodes_dev, tris_dev, epo_dev,
                     area_dev, (uint32_t)n_tris, flags);
  EPO_OK(hipGetLastError());
  EPO_OK(hipMemcpyAsync(flags_h, flags, sizeof(flags_h), hipMemcpyDeviceToHost, st));
  EPO_OK(hipStreamSynchronize(st));
  if (flags_h[1]) {
    rc = mcpt::fail(MCPT_ERR_LIMIT, "bvh_epo_device: tree deeper than EPO.cl's 128-entry stacks");
    goto done;
  }
  if (clip_overflows) *clip_overflows = flags_h[0];
  if (epo_out) {  // EPO_GPU's host loop (bvhtest.cpp:306-320): double sums in index order
    e.resize(n_tris);
    a.resize(n_tris);
    EPO_OK(hipMemcpy(e.data(), epo_dev, n_tris * sizeof(float), hipMemcpyDeviceToHost));
    EPO_OK(hipMemcpy(a.data(), area_dev, n_tris * sizeof(float), hipMemcpyDeviceToHost));
    double count = 0.0, area = 0.0;
    for (int64_t i = 0; i < n_tris; ++i) count += e[i];
    for (int64_t i = 0; i < n_tris; ++i) area += a[i];
    count /= area;
    *epo_out = (double)(float)count;  // EPO_GPU returns float
  }
done:
  if (flags) (void)hipFree(flags);
  return rc;
}
