// ref_runner.hip — TEST INFRASTRUCTURE ONLY (never linked into the product).
//
// Runs the reference's own OpenCL kernels — MonteCarloPathTracing/kernels/
// {rayGenerator,intersect,shade,history,EPO}.cl with objdef.h prepended, compiled
// UNMODIFIED for gfx950 by ROCm's OpenCL C compiler (oracle/Makefile, default
// OpenCL build options exactly as OpenCLBasic::createProgramFromFileWithHeader
// passes them, MCPT/oclbasic.cpp:167-183) — on the GPU through the HIP module
// API, in the launch order of OpenCL::update (MCPT/OpenCLApp.cpp:57-82) and
// ColorOut::outputColorCL (MCPT/colorout.cpp:40-73).
//
// It is the pinned oracle for the HIP path: tests/ compare libmcpt_hip.so
// against it bit for bit on the GPU box.  The code objects are built here from
// /root/reference into oracle/_ref/ (git-ignored) and travel with the snapshot.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../include/mcpt_hip.h"

namespace {

std::string g_dir;
std::string g_err;
std::map<std::string, hipModule_t> g_mods;

int err(const std::string &m) {
  g_err = m;
  return -1;
}

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) return err(std::string(#x) + ": " + hipGetErrorString(e_));  \
  } while (0)

int get_fn(const std::string &file, const char *name, hipFunction_t *f) {
  hipModule_t m;
  auto it = g_mods.find(file);
  if (it == g_mods.end()) {
    std::string path = g_dir + "/" + file;
    hipError_t e = hipModuleLoad(&m, path.c_str());
    if (e != hipSuccess) return err("hipModuleLoad(" + path + "): " + hipGetErrorString(e));
    g_mods[file] = m;
  } else {
    m = it->second;
  }
  CK(hipModuleGetFunction(f, m, name));
  return 0;
}

// NDRange with NullRange local size: any work-group size that divides the
// global size gives the same get_global_id / get_global_size.
unsigned pick_block(uint64_t n) {
  for (unsigned b = 256; b > 1; b >>= 1)
    if (n % b == 0) return b;
  return 1;
}

int launch1d(hipFunction_t f, uint64_t n, void **args) {
  unsigned b = pick_block(n);
  CK(hipModuleLaunchKernel(f, (unsigned)(n / b), 1, 1, b, 1, 1, 0, nullptr, args, nullptr));
  return 0;
}
int launch2d(hipFunction_t f, uint32_t w, uint32_t h, void **args) {
  unsigned b = pick_block(w);
  CK(hipModuleLaunchKernel(f, w / b, h, 1, b, 1, 1, 0, nullptr, args, nullptr));
  return 0;
}

template <class T>
struct Dev {
  T *p = nullptr;
  size_t n = 0;
  int alloc(size_t k) {
    n = k;
    CK(hipMalloc(&p, std::max<size_t>(k, 1) * sizeof(T)));
    return 0;
  }
  int up(const T *h) {
    CK(hipMemcpy(p, h, n * sizeof(T), hipMemcpyHostToDevice));
    return 0;
  }
  int down(T *h) {
    CK(hipMemcpy(h, p, n * sizeof(T), hipMemcpyDeviceToHost));
    return 0;
  }
  ~Dev() {
    if (p) (void)hipFree(p);
  }
};

#define TRY(x)             \
  do {                     \
    if ((x) != 0) return -1; \
  } while (0)

__global__ void k_rcp_probe(float *x, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] = __builtin_amdgcn_rcpf(x[i]);
}

}  // namespace

extern "C" {

const char *ref_last_error(void) { return g_err.c_str(); }

int ref_init(const char *code_object_dir) {
  g_dir = code_object_dir;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return err("no HIP device");
  return 0;
}

// rayGenerator.cl over an NDRange {W, H}
int ref_generate(const mcpt_camera *cam, int32_t w, int32_t h, mcpt_ray *rays_out) {
  hipFunction_t f;
  TRY(get_fn("rayGenerator.co", "generateRay", &f));
  Dev<mcpt_camera> dc;
  Dev<mcpt_ray> dr;
  TRY(dc.alloc(1));
  TRY(dc.up(cam));
  TRY(dr.alloc((size_t)w * h));
  void *args[] = {&dc.p, &dr.p};
  TRY(launch2d(f, w, h, args));
  CK(hipDeviceSynchronize());
  TRY(dr.down(rays_out));
  return 0;
}

// intersect.cl on n rays (tmin is the host's EPSILON 1e-3 in the reference)
int ref_intersect(const mcpt_triangle *tris, int64_t nt, const mcpt_bvh_node *nodes, int64_t nn, const mcpt_ray *rays,
                  int64_t n, mcpt_hit *hits_inout, float tmin) {
  hipFunction_t f;
  TRY(get_fn("intersect.co", "intersectRays", &f));
  Dev<mcpt_triangle> dt;
  Dev<mcpt_bvh_node> db;
  Dev<mcpt_ray> dr;
  Dev<mcpt_hit> dh;
  TRY(dt.alloc(nt));
  TRY(dt.up(tris));
  TRY(db.alloc(nn));
  TRY(db.up(nodes));
  TRY(dr.alloc(n));
  TRY(dr.up(rays));
  TRY(dh.alloc(n));
  TRY(dh.up(hits_inout));
  void *args[] = {&dr.p, &db.p, &dt.p, &dh.p, &tmin};
  TRY(launch1d(f, n, args));
  CK(hipDeviceSynchronize());
  TRY(dh.down(hits_inout));
  return 0;
}

// shade.cl (-D MAX_DEPTH=max_depth) on n rays
int ref_shade(const mcpt_material *mats, int32_t nm, mcpt_ray *rays, const mcpt_hit *hits, float *colors,
              uint32_t *seeds, int64_t n, int32_t max_depth) {
  hipFunction_t f;
  TRY(get_fn("shade_d" + std::to_string(max_depth) + ".co", "shade", &f));
  Dev<mcpt_material> dm;
  Dev<mcpt_ray> dr;
  Dev<mcpt_hit> dh;
  Dev<float> dc;
  Dev<uint32_t> ds;
  TRY(dm.alloc(nm));
  TRY(dm.up(mats));
  TRY(dr.alloc(n));
  TRY(dr.up(rays));
  TRY(dh.alloc(n));
  TRY(dh.up(hits));
  TRY(dc.alloc(4 * n));
  TRY(dc.up(colors));
  TRY(ds.alloc(n));
  TRY(ds.up(seeds));
  void *args[] = {&dm.p, &dr.p, &dh.p, &dc.p, &ds.p};
  TRY(launch1d(f, n, args));
  CK(hipDeviceSynchronize());
  TRY(dr.down(rays));
  TRY(dc.down(colors));
  TRY(ds.down(seeds));
  return 0;
}

// history.cl (-D MAX_ATTEMPT=max_attempt) over an NDRange {W, H}
int ref_accumulate(float *colors, float *hist, int32_t *count, int32_t w, int32_t h, int32_t max_attempt) {
  hipFunction_t f;
  TRY(get_fn("history_a" + std::to_string(max_attempt) + ".co", "func", &f));
  size_t n = (size_t)w * h;
  Dev<float> dc, dh;
  Dev<int32_t> dn;
  TRY(dc.alloc(4 * n));
  TRY(dc.up(colors));
  TRY(dh.alloc(4 * n));
  TRY(dh.up(hist));
  TRY(dn.alloc(n));
  TRY(dn.up(count));
  void *args[] = {&dc.p, &dh.p, &dn.p};
  TRY(launch2d(f, w, h, args));
  CK(hipDeviceSynchronize());
  TRY(dc.down(colors));
  TRY(dh.down(hist));
  TRY(dn.down(count));
  return 0;
}

// The whole frame loop, OpenCL::update + ColorOut, for `frames` frames.
// seeds (W*H u32) are read and written back; hist (W*H float4) and count
// (W*H i32) are the accumulated frameBuffer/sampleCount (zero-initialised,
// colorout.cpp:42-53).  The reference's colour buffer is reset to (1,1,1,1)
// every frame (OpenCLApp.cpp:63) and its Hit buffer is never initialised.
int ref_render(const mcpt_camera *cam, const mcpt_triangle *tris, int64_t nt, const mcpt_bvh_node *nodes, int64_t nn,
               const mcpt_material *mats, int32_t nm, int32_t w, int32_t h, int32_t max_depth, int32_t frames,
               int32_t max_attempt, uint32_t *seeds, float *hist_out, int32_t *count_out) {
  hipFunction_t fgen, fint, fsh, fhist;
  TRY(get_fn("rayGenerator.co", "generateRay", &fgen));
  TRY(get_fn("intersect.co", "intersectRays", &fint));
  TRY(get_fn("shade_d" + std::to_string(max_depth) + ".co", "shade", &fsh));
  TRY(get_fn("history_a" + std::to_string(max_attempt) + ".co", "func", &fhist));
  const size_t n = (size_t)w * h;
  Dev<mcpt_camera> dcam;
  Dev<mcpt_triangle> dt;
  Dev<mcpt_bvh_node> db;
  Dev<mcpt_material> dm;
  Dev<mcpt_ray> dr;
  Dev<mcpt_hit> dh;
  Dev<float> dcol, dhist;
  Dev<uint32_t> ds;
  Dev<int32_t> dn;
  TRY(dcam.alloc(1));
  TRY(dcam.up(cam));
  TRY(dt.alloc(nt));
  TRY(dt.up(tris));
  TRY(db.alloc(nn));
  TRY(db.up(nodes));
  TRY(dm.alloc(nm));
  TRY(dm.up(mats));
  TRY(dr.alloc(n));
  TRY(dh.alloc(n));
  TRY(dcol.alloc(4 * n));
  TRY(dhist.alloc(4 * n));
  TRY(ds.alloc(n));
  TRY(ds.up(seeds));
  TRY(dn.alloc(n));
  CK(hipMemset(dhist.p, 0, 16 * n));
  CK(hipMemset(dn.p, 0, 4 * n));
  CK(hipMemset(dh.p, 0xCD, sizeof(mcpt_hit) * n));  // uninitialised in the reference
  std::vector<float> ones(4 * n, 1.0f);
  float tmin = 0.001f;
  int attempt = 0;
  for (int fr = 0; fr < frames; ++fr) {
    TRY(dcol.up(ones.data()));
    void *ag[] = {&dcam.p, &dr.p};
    TRY(launch2d(fgen, w, h, ag));
    for (int i = 0; i < max_depth; ++i) {
      void *ai[] = {&dr.p, &db.p, &dt.p, &dh.p, &tmin};
      TRY(launch1d(fint, n, ai));
      void *as[] = {&dm.p, &dr.p, &dh.p, &dcol.p, &ds.p};
      TRY(launch1d(fsh, n, as));
    }
    if (attempt <= max_attempt) {
      void *ah[] = {&dcol.p, &dhist.p, &dn.p};
      TRY(launch2d(fhist, w, h, ah));
      ++attempt;
    }
  }
  CK(hipDeviceSynchronize());
  TRY(ds.down(seeds));
  TRY(dhist.down(hist_out));
  TRY(dn.down(count_out));
  return 0;
}

// EPO.cl calculateEPO over an NDRange of n_tris (bvhtest.cpp:288-321 EPO_GPU):
// per-leaf EPO area and triangle area, as the reference's host reads them back
int ref_epo(const mcpt_bvh_node *nodes, int64_t nn, const mcpt_triangle *tris, int64_t nt, float *epo_out,
            float *area_out) {
  hipFunction_t f;
  TRY(get_fn("EPO.co", "calculateEPO", &f));
  Dev<mcpt_bvh_node> db;
  Dev<mcpt_triangle> dt;
  Dev<float> de, da;
  TRY(db.alloc(nn));
  TRY(db.up(nodes));
  TRY(dt.alloc(nt));
  TRY(dt.up(tris));
  TRY(de.alloc(nt));
  TRY(da.alloc(nt));
  uint32_t num = (uint32_t)nt;
  void *args[] = {&db.p, &dt.p, &de.p, &da.p, &num};
  TRY(launch1d(f, nt, args));
  CK(hipDeviceSynchronize());
  TRY(de.down(epo_out));
  TRY(da.down(area_out));
  return 0;
}

// Hardware reciprocals (v_rcp_f32) of n floats.  treeletBVH.cl does not
// compile, so its restatement (oracle/mcpt_oracle_treelet_gpu.cpp)
// models the kernel's 2.5-ulp x / rootArea as frexp / v_rcp_f32 / ldexp, the
// sequence ROCm's OpenCL compiler emits for gfx950, and takes v_rcp_f32's
// value of frexp_mant(rootArea) from this probe.
int ref_rcp_f32(const float *in, float *out, int64_t n) {
  Dev<float> d;
  TRY(d.alloc(n));
  TRY(d.up(in));
  hipLaunchKernelGGL(k_rcp_probe, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, d.p, n);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  TRY(d.down(out));
  return 0;
}

}  // extern "C"
