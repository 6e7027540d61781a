// mcpt_device.hip — device half of libmcpt_hip.so: the per-pixel, per-sample
// path-tracing loop for gfx950 (MI355X), behind the C ABI of include/mcpt_hip.h.
//
// Reference kernels restated here (arithmetic in mcpt_refmath.h):
//   generateRay     MCPT/kernels/rayGenerator.cl:1-31
//   intersectRays   MCPT/kernels/intersect.cl:1-28 + MCPT/objdef.h:178-275
//   shade           MCPT/kernels/shade.cl:75-206
//   func (history)  MCPT/kernels/history.cl:3-28
//   frame loop      MCPT/OpenCLApp.cpp:57-82, MCPT/colorout.cpp:40-73
//
// Two ways to run them:
//  * k_render — the fused path: one lane per pixel, the lane walks all of its
//    frames itself (seed chain, running mean and count stay in registers,
//    path regeneration on termination), BVH stack in LDS.  This is the hot
//    path measured by bench.py.
//  * k_generate / k_intersect / k_shade / k_accumulate — one kernel per
//    reference kernel on the reference's AoS records, for drop-in use and for
//    kernel-level parity with the reference code objects.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "../../include/mcpt_hip.h"
#include "mcpt_refmath.h"
#include "mcpt_bvh4.h"
#include "mcpt_upload.h"

using namespace mcpt;

#ifndef MCPT_WAVES_PER_SIMD
#define MCPT_WAVES_PER_SIMD 4  // k_render occupancy target (tools/sweep.py over `make variants`)
#endif
#ifndef MCPT_STACK_WINDOW_K
#define MCPT_STACK_WINDOW_K 16  // 16: room in LDS for the tree's top levels (C2 / C4 even with 32; C3 -1 %)
#endif
constexpr int kStackWindow = MCPT_STACK_WINDOW_K;  // k_render's LDS window when the whole stack would cost occupancy

namespace mcpt {
int fail(int code, const std::string &msg);  // mcpt_host.cpp
}

// ------------------------------------------------------------ device layout
// Internal node n of the reference HLBVH keeps its index; its record stores
// BOTH children's boxes so one 64-B fetch decides where to go next
// (objdef.h:252-273 fetches and tests one 64-B node per step).
struct __attribute__((aligned(16))) DevNode {
  f4 a;  // Lmin.x Lmax.x Lmin.y Lmax.y      (min,max) pairs per axis, so the
  f4 b;  // Lmin.z Lmax.z Rmin.x Rmax.x      slab arithmetic runs on packed
  f4 c;  // Rmin.y Rmax.y Rmin.z Rmax.z      v_pk_add/v_pk_mul_f32
  int32_t left, right, pad0, pad1;  // >= 0 internal node, < 0 leaf: ~triangle
};
// Cramer-ready triangle: v0, -(v1-v0), -(v2-v0) exactly as objdef.h:190-199
// forms them, with the packed normal's xyz in their .w lanes, so a triangle
// test reads the first 48 B: three gathers (the triangle-only minors of
// cramer_reduced are recomputed from nab/nac, the same fma the host used,
// tri_minors).  aux = the material id bits (the packed normal's .w), read once
// per segment for the hit triangle, and the three minors (the quantized
// records copy them).
struct __attribute__((aligned(16))) DevTri {
  f4 v0;   // .w = normal.x
  f4 nab;  // .w = normal.y
  f4 nac;  // .w = normal.z
  f4 aux;  // .x = material id bits, .yzw = m_x1, m_y4, m_y8
};
static_assert(sizeof(DevNode) == 64 && sizeof(DevTri) == 64, "64-B records");
__host__ __device__ inline f3 tri_normal(const f4 &v0, const f4 &nab, const f4 &nac) {
  return (f3){v0.w, nab.w, nac.w};
}
// the three triangle-only minors of cramer_reduced (mcpt_refmath.h): m_x1 =
// fma(b2,c3,-(c2*b3)), m_y4 = fma(b1,c3,-(c1*b3)), m_y8 = fma(b1,c2,-(c1*b2))
__device__ inline void tri_minors(f3 b, f3 c, float &m_x1, float &m_y4, float &m_y8) {
  m_x1 = __builtin_fmaf(b.y, c.z, -(c.y * b.z));
  m_y4 = __builtin_fmaf(b.x, c.z, -(c.x * b.z));
  m_y8 = __builtin_fmaf(b.x, c.y, -(c.x * b.y));
}
// a traced hit carries its triangle as ~index in best_nrm.w (the material is
// read at shading); a cached primary hit (PrimHit) carries the material id
__device__ inline int32_t hit_material(const DevTri *__restrict__ tris, int32_t w) {
  return w >= 0 ? w : as_i(tris[~w].aux.x);
}

// 4-wide node of the EXACT path: the binary HLBVH with every other level
// collapsed.  Slots are the node's grandchildren (or a child that is a leaf)
// in left-to-right order, so visiting passing slots in slot order IS the
// reference's left-first DFS.  Skipping the middle box test is exact: a
// grandchild box lies inside its parent's, and (bb - o) * rcp(d) is monotone
// in bb, so a grandchild's slab interval lies inside its parent's — it can
// only pass if the parent passes.
struct __attribute__((aligned(16))) DevNode4 {
  f4 q[6];          // per slot k: (minx,maxx) (miny,maxy) (minz,maxz) pairs, packed 6 floats/slot
  int32_t link[4];  // >= 0 internal DevNode4, < 0 leaf ~triangle, kEmptySlot unused
  f4 pad;
};
static_assert(sizeof(DevNode4) == 128 && sizeof(DevNode4) == sizeof(mcpt::Node4Rec), "128-B 4-wide node");
// 64-B quantized search-tree node (mcpt::Node4Q): four 16-B loads.  c0 =
// (origin.xyz, scale.x); qb[0..5] = the 24 plane bytes in DevNode4::q order
// (decoded fma(q, s, o): a strictly larger box than the exact one); then
// scale.y, scale.z and the four links.
struct __attribute__((aligned(16))) DevNode4Q {
  f4 c0;
  uint32_t qb[6];
  float sy, sz;
  int32_t link[4];
};
static_assert(sizeof(DevNode4Q) == 64 && sizeof(DevNode4Q) == sizeof(mcpt::Node4Q), "64-B quantized node");
// Triangle record of the quantized path: the raw vertices (so the L phase can
// rebuild the reference leaf's exact box, hlbvh.cpp:97-100) with the three
// triangle-only Cramer minors in .w, then the packed normal / material id.
struct __attribute__((aligned(16))) DevTriQ {
  f4 v0, v1, v2, nrm;
};
static_assert(sizeof(DevTriQ) == 64, "64-B triangle");

constexpr int32_t kDone = INT32_MIN;           // traversal finished
constexpr int32_t kPop = INT32_MIN + 1;        // take the next entry from the stack
constexpr int32_t kEmptySlot = INT32_MIN + 2;  // unused 4-wide slot
static_assert(kEmptySlot == mcpt::kEmptySlot4, "one empty-slot marker");

struct SceneView {
  int32_t n_near4, n_nodes4, n_int;  // record counts (bounds of the MCPT_DEBUG checks)
  int64_t n_tris;
  const DevNode4 *near4;   // EXACT search tree (binned SAH, nearest-first; mcpt_sah.cpp)
  const DevNode4 *nodes4;  // the reference HLBVH collapsed 4-wide (left-first fallback)
  const DevNode *nodes;
  const DevTri *tris;
  const DevNode4Q *near4q;  // near4 quantized (nullptr: the scene keeps the 128-B nodes only)
  const DevTriQ *triq;      // triangles for the quantized path
  const mcpt_material *mats;
  f4 root_min, root_max;
  int32_t root_leaf;  // >= 0: single-triangle scene, root is that leaf
  int32_t n_mats;
  float prune_margin;
};

struct mcpt_scene {
  int device;
  uint64_t uid = 0;  // never reused: keys the context's primary-hit cache
  DevNode4 *near4 = nullptr;
  DevNode4 *nodes4 = nullptr;
  int32_t stack_depth4 = 1;  // EXACT: max of both 4-wide trees' stack needs
  DevNode *nodes = nullptr;
  DevTri *tris = nullptr;
  DevNode4Q *near4q = nullptr;
  DevTriQ *triq = nullptr;
  int64_t near4_bytes = 0;  // the 128-B search tree's size (auto choice of the quantized one)
  mcpt_material *mats = nullptr;
  int64_t n_tris = 0, n_internal = 0;
  int32_t n_mats = 0;
  int32_t stack_depth = 1;
  bool has_glossy = true;  // any GLOSSY material: k_render's glossy-lobe shading path
  SceneView view;
};

constexpr int kQueues = 8;         // k_render work queues (at most): one per XCD (MI355X has 8)
constexpr int kQueueStride = 32;   // u32 words between queue heads: one 128-B line each
constexpr int kDefaultBlockEntries = 8;  // mcpt_tuning.block_entries = 0 (launch plan, below)
constexpr int kHandoffWords = 4;   // seed, mean.xyzw, count in four tagged 8-B granules (two 16-B stores)
constexpr int kMaxBlocksPerLaunch = 255;  // the hand-off tag's 8 bits of block index
constexpr int kStatSlots = 24;
constexpr int64_t kQuantAutoBytes = 32ll << 20;  // 8 XCDs x 4 MiB of L2
// primary-hit pass: k_primary (one ray per lane) for search trees up to this
// size, k_render's PRIM form (batched phases, resident grid) beyond: C3's
// 0.24 MB tree 0.07 vs 0.13 ms, C2's 2.1 MB 0.18 vs 0.15, C5's 435 MB 3.57 vs
// 1.66 (profiles/r02_primary_cache.txt)
constexpr int64_t kPrimSmallTree = 1ll << 20;
// k_render counters (mcpt_stats): kStatSlots words
constexpr int kPhaseSlot = 16;     // MCPT_PHASE_TIMING: shader-clock ticks per phase (fetch, T, L, S)
constexpr int kDebugSlot = 12;     // MCPT_DEBUG: violations of the stack bound, node and triangle indices
constexpr int kWaveLogWords = 8;   // MCPT_PHASE_TIMING wave log (mcpt_get_wave_log)

// -DMCPT_DEBUG (make debug -> lib/libmcpt_hip_debug.so): k_render checks every
// stack push against its capacity and every node / triangle index against
// its array before use, counts violations (mcpt_stats.debug_violations) and
// skips the bad access instead of faulting.  The reference's own traversal
// has an unchecked int stack[64] (objdef.h:247).
// -DMCPT_PHASE_TIMING (make timing -> lib/libmcpt_hip_timing.so): every wave
// adds the shader-clock ticks (s_memtime) it spends in each phase of its loop
// (fetch, T, L, S) to mcpt_stats.phase_ticks: where a wave's time goes,
// latency included.  Diagnostics only; the reads cost time themselves.
#ifdef MCPT_PHASE_TIMING
constexpr bool kTiming = true;
#define MCPT_TICK(k)                                            \
  do {                                                          \
    const uint64_t now_ = __builtin_amdgcn_s_memtime();         \
    ph[k] += now_ - tick;                                       \
    tick = now_;                                                \
  } while (0)
#else
constexpr bool kTiming = false;
#define MCPT_TICK(k) do {} while (0)
#endif

#ifdef MCPT_DEBUG
constexpr bool kDebug = true;
#define MCPT_DCHECK(cond, slot) (__builtin_expect(!(cond), 0) ? (atomicAdd(&A.stats[kDebugSlot + (slot)], 1ull), false) : true)
#else
constexpr bool kDebug = false;
#define MCPT_DCHECK(cond, slot) true
#endif

// The primary hit of a pixel (k_primary): the reference re-shoots the same
// primary ray every frame (rayGenerator.cl has no jitter), so its closest hit
// is the same in every frame; k_render reads it instead of tracing segment 0.
// nrm = the hit triangle's packed normal (material id bits in .w), t = the
// closest-hit distance (kFltMax: miss), ray = the primary ray's per-pixel
// part as gen_ray_px makes it: the direction's xyz (pinhole camera) or the
// origin's xyz (camera_type 1); the rest of the ray is the same for every
// pixel (LdsUniforms::ray_u), so a frame starts without generateRay's
// arithmetic.
struct __attribute__((aligned(16))) PrimHit {
  f4 nrm;
  float t;
  float ray[3];
};
static_assert(sizeof(PrimHit) == 32, "32-B primary hit");
// What a primary-hit cache was computed for: same scene, camera, image,
// stripes and mode give the same hits.
struct PrimKey {
  uint64_t scene_uid;
  mcpt_camera cam;
  int32_t w, h, stripe_rows, stripe_index, stripe_count, mode;
};

struct mcpt_ctx {
  int device;
  int n_cu = 0;
  bool stats_on = false;
  uint32_t *px_segments = nullptr;        // mcpt_set_pixel_segments (stats calls only)
  uint32_t *px_iters = nullptr;
  int64_t px_cap = 0;                     // their capacity in pixels (a larger image collects nothing)
  unsigned long long *d_stats = nullptr;  // segments, nodes, tris, bad, wave T/L/S phases
  uint32_t *d_queue = nullptr;            // k_render work-queue heads, kQueues per launch
  int32_t queue_cap = 0;                  // launches the head array holds
  unsigned long long *d_handoff = nullptr;  // k_render per-pixel block hand-off granules
  int64_t handoff_cap = 0;                // pixels
  uint32_t launch_seq = 0;                // tags hand-off granules with the launch they belong to
  int32_t *d_spill = nullptr;             // k_render WindowStack spill areas
  int64_t spill_cap = 0;
  mcpt_tuning tune;                       // launch-plan knobs (mcpt_set_tuning)
  struct Occ {
    const void *fn;
    size_t lds;
    int per_cu;
  };
  std::vector<Occ> occ;                   // occupancy per (kernel, LDS bytes), queried once
  mcpt_stats last;
  bool last_pending = false;              // the last render call's events/counters not read yet
  bool last_stats = false;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  hipEvent_t ev_prim = nullptr;           // after k_primary, when the call ran it
  PrimHit *d_prim = nullptr;              // primary-hit cache, one record per pixel
  uint32_t *d_prim_cost = nullptr;        // each cached pixel's primary-ray traversal cost (lane-iterations)
  int32_t *d_tile_order = nullptr;        // queue position -> tile, dearest first (from d_prim_cost)
  uint8_t *d_tile_key = nullptr;          // per tile: its cost, saturated to 8 bits
  int64_t tile_cap = 0;
  int32_t tile_order_mode = 0;            // the mcpt_tuning.tile_order value d_tile_order was built with (0: none)
  int64_t prim_cap = 0;                   // pixels
  bool prim_valid = false;
  PrimKey prim_key;                       // what d_prim holds
  bool seen_valid = false;
  PrimKey seen_key;                       // the previous render call's view
  unsigned long long *d_wave_log = nullptr;  // MCPT_PHASE_TIMING: kWaveLogWords per workgroup of the last launch
  int64_t wave_log_cap = 0, wave_log_n = 0;
  uint32_t *d_entry_log = nullptr;        // MCPT_PHASE_TIMING: 3 words per (pixel, block) of the last launch
  int64_t entry_log_cap = 0, entry_log_n = 0;
  int32_t entry_log_blocks = 0;
};

struct mcpt_state {
  int device;
  int32_t width, height;
  uint32_t *seeds = nullptr;
  float *hist = nullptr;
  int32_t *count = nullptr;
};

#define HIP_OK(expr)                                                                        \
  do {                                                                                      \
    hipError_t e_ = (expr);                                                                 \
    if (e_ != hipSuccess) return mcpt::fail(MCPT_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

// ----------------------------------------------------------------- traversal
struct Trace {
  float t;        // closest accepted t (FLT_MAX = miss)
  int32_t tri;    // triangle that set t
  int32_t last;   // last accepted triangle (the reference's Hit.triangleID)
  uint32_t nodes, tests;
};

template <bool LITERAL>
__device__ inline BoxT box_test(f3 bmin, f3 bmax, f3 o, f3 d, f3 rinv) {
  if (LITERAL) {  // objdef.h:227-228 verbatim: (bb - o) / d
    f3 t1 = (bmin - o) / d;
    f3 t2 = (bmax - o) / d;
    BoxT r;
    r.tnear = fmaxf(fmaxf(fminf(t1.x, t2.x), fminf(t1.y, t2.y)), fminf(t1.z, t2.z));
    r.tfar = fminf(fminf(fmaxf(t1.x, t2.x), fmaxf(t1.y, t2.y)), fmaxf(t1.z, t2.z));
    return r;
  }
  return slab(bmin, bmax, o, rinv);
}

// Both child boxes of a node (objdef.h:223-237 twice).  Packed form: the
// (min, max) pair of each axis is one float2, so (bb - o) * rcp(d) is one
// v_pk_add_f32 + one v_pk_mul_f32 per axis and box — the same IEEE operations
// as the scalar form, two lanes at a time.
typedef float f2 __attribute__((ext_vector_type(2)));
__device__ inline BoxT slab_pairs(f2 px, f2 py, f2 pz, f3 o, f3 rinv) {
  f2 tx = (px - o.x) * rinv.x, ty = (py - o.y) * rinv.y, tz = (pz - o.z) * rinv.z;
  BoxT r;
  r.tnear = fmaxf(fmaxf(fminf(tx.x, tx.y), fminf(ty.x, ty.y)), fminf(tz.x, tz.y));
  r.tfar = fminf(fminf(fmaxf(tx.x, tx.y), fmaxf(ty.x, ty.y)), fmaxf(tz.x, tz.y));
  return r;
}
template <bool LITERAL>
__device__ inline void child_boxes(const DevNode &N, f3 o, f3 d, f3 rinv, BoxT &bl, BoxT &br) {
  if (LITERAL) {
    bl = box_test<true>((f3){N.a.x, N.a.z, N.b.x}, (f3){N.a.y, N.a.w, N.b.y}, o, d, rinv);
    br = box_test<true>((f3){N.b.z, N.c.x, N.c.z}, (f3){N.b.w, N.c.y, N.c.w}, o, d, rinv);
  } else {
    bl = slab_pairs(N.a.xy, N.a.zw, N.b.xy, o, rinv);
    br = slab_pairs(N.b.zw, N.c.xy, N.c.zw, o, rinv);
  }
}

// Per-lane traversal stacks.  Plain: every entry in LDS, column-major
// [depth][64] (conflict-free ds_read/write_b32).  Window: only the top K
// entries live in LDS (entry i in slot i mod K); an entry pushed out of the
// window goes to the lane's spill area in global memory and comes back when
// the stack shrinks below it.  Same logical stack, so the same traversal; the
// LDS footprint per wave drops from depth*256 B to K*256 B, which is what
// bounds the waves per CU.
struct PlainStack {
  int32_t *lds;
  int stride;
  __device__ inline void push(int &sp, int32_t v) const { lds[(sp++) * stride] = v; }
  __device__ inline int32_t pop(int &sp) const { return lds[(--sp) * stride]; }
  __device__ inline int32_t peek(int sp) const { return lds[(sp - 1) * stride]; }
};
template <int K>
struct WindowStack {
  static_assert((K & (K - 1)) == 0, "power of two window");
  int32_t *lds;    // lds_stack + lane
  int32_t *spill;  // this lane's entries [0, depth - K)
  __device__ inline void push(int &sp, int32_t v) const {
    int32_t *slot = lds + (sp & (K - 1)) * 64;
    if (sp >= K) spill[sp - K] = *slot;
    *slot = v;
    ++sp;
  }
  __device__ inline int32_t pop(int &sp) const {
    --sp;
    int32_t *slot = lds + (sp & (K - 1)) * 64;
    const int32_t v = *slot;
    if (sp >= K) *slot = spill[sp - K];
    return v;
  }
  __device__ inline int32_t peek(int sp) const { return lds[((sp - 1) & (K - 1)) * 64]; }  // the top is in the window
};

// One 4-wide node: slab test of the 4 slots, then pick the slot to enter.
// NEAREST (the SAH search tree): the passing slot with the smallest entry
// distance, ties to the lower slot; otherwise (the reference tree) the lowest
// passing slot, i.e. the reference's left-first DFS.  The other passing slots
// are pushed so that they pop in slot order.  Returns the slot's link (an
// internal node or ~triangle) or kPop.
template <bool PRUNE, class Stk>
__device__ inline int32_t step4q(f4 q0, f4 q1, f4 q2, f4 q3, f4 q4, f4 q5, int32_t l0, int32_t l1, int32_t l2,
                                 int32_t l3, f3 o, f3 rinv, float tmin, float lim, bool nearest, const Stk &stk, int &sp,
                                 uint32_t &nodes_ctr);
template <bool PRUNE, class Stk>
__device__ inline int32_t step4(const DevNode4 &N, f3 o, f3 rinv, float tmin, float lim, bool nearest, const Stk &stk,
                                int &sp, uint32_t &nodes_ctr) {
  return step4q<PRUNE>(N.q[0], N.q[1], N.q[2], N.q[3], N.q[4], N.q[5], N.link[0], N.link[1], N.link[2], N.link[3], o,
                       rinv, tmin, lim, nearest, stk, sp, nodes_ctr);
}
template <bool PRUNE, class Stk>
__device__ inline int32_t step4q(f4 q0, f4 q1, f4 q2, f4 q3, f4 q4, f4 q5, int32_t l0, int32_t l1, int32_t l2,
                                 int32_t l3, f3 o, f3 rinv, float tmin, float lim, bool nearest, const Stk &stk, int &sp,
                                 uint32_t &nodes_ctr) {
  BoxT b0 = slab_pairs(q0.xy, q0.zw, q1.xy, o, rinv);
  BoxT b1 = slab_pairs(q1.zw, q2.xy, q2.zw, o, rinv);
  BoxT b2 = slab_pairs(q3.xy, q3.zw, q4.xy, o, rinv);
  BoxT b3 = slab_pairs(q4.zw, q5.xy, q5.zw, o, rinv);
  bool h0 = slab_pass(b0, tmin) && l0 != kEmptySlot, h1 = slab_pass(b1, tmin) && l1 != kEmptySlot;
  bool h2 = slab_pass(b2, tmin) && l2 != kEmptySlot, h3 = slab_pass(b3, tmin) && l3 != kEmptySlot;
  if (PRUNE) {
    h0 = h0 && !(b0.tnear > lim);
    h1 = h1 && !(b1.tnear > lim);
    h2 = h2 && !(b2.tnear > lim);
    h3 = h3 && !(b3.tnear > lim);
  }
  nodes_ctr++;
  // left-first: every key 0, so the lowest passing slot wins the <= chain
  const float k0 = nearest ? b0.tnear : 0.0f, k1 = nearest ? b1.tnear : 0.0f;
  const float k2 = nearest ? b2.tnear : 0.0f, k3 = nearest ? b3.tnear : 0.0f;
  int32_t nxt = kPop;
  int sel = 4;
  float kb = __builtin_inff();
  if (h3) kb = k3, nxt = l3, sel = 3;
  if (h2 && !(k2 > kb)) kb = k2, nxt = l2, sel = 2;
  if (h1 && !(k1 > kb)) kb = k1, nxt = l1, sel = 1;
  if (h0 && !(k0 > kb)) nxt = l0, sel = 0;
  if (h3 && sel != 3) stk.push(sp, l3);
  if (h2 && sel != 2) stk.push(sp, l2);
  if (h1 && sel != 1) stk.push(sp, l1);
  if (h0 && sel != 0) stk.push(sp, l0);
  return nxt;
}

// MCPT_POW_LOBE 0: the Phong lobe calls ocml's pow (A/B builds only)
#ifndef MCPT_POW_LOBE
#define MCPT_POW_LOBE 1
#endif

// Result rule of the EXACT search.  The reference keeps the
// first triangle in its DFS order and replaces it only by one at least EPS
// closer (objdef.h:213).  Searching in another order, track the closest
// accepted t1 and the runner-up t2: if every other accepted triangle lies at
// least EPS behind t1 (t2 - t1 >= EPS in the reference's float arithmetic),
// the t1 triangle replaces whatever the reference holds when it reaches it
// and nothing replaces it afterwards, so it IS the reference's answer in any
// order.  Otherwise the ray is re-searched in the reference's own order.
__device__ inline void near_update(float t, float &t1, float &t2) {  // selects, not branches
  const bool lt1 = t < t1, lt2 = t < t2;
  t2 = lt1 ? t1 : (lt2 ? t : t2);
  t1 = lt1 ? t : t1;
}
__device__ inline bool near_ambiguous(float t1, float t2) { return t2 < kFltMax && !(t2 - t1 >= kEps); }

// NOPRUNE: the reference's exhaustive left-first DFS of objdef.h:240-275 on
// its binary tree with the literal division.
//
// SIMT shape ("while-while", Aila & Laine 2009): the inner loop walks internal
// nodes until EVERY lane of the wave holds a leaf (or is done); then all lanes
// with a leaf run the Cramer test together.  Each lane still tests its
// triangles in exactly the reference's DFS order.
__device__ inline Trace traverse_noprune(const SceneView &S, f3 o, f3 d, float tmin, int32_t *stk, int stride) {
  Trace tr;
  tr.t = kFltMax;
  tr.tri = -1;
  tr.last = -1;
  tr.nodes = 0;
  tr.tests = 0;
  f3 rinv;
  rinv.x = __builtin_amdgcn_rcpf(d.x);
  rinv.y = __builtin_amdgcn_rcpf(d.y);
  rinv.z = __builtin_amdgcn_rcpf(d.z);
  int32_t cur;  // >= 0 internal node, kDone, or ~triangle (a leaf waiting for its test)
  if (!slab_pass(box_test<true>(S.root_min.xyz, S.root_max.xyz, o, d, rinv), tmin))
    cur = kDone;
  else
    cur = S.root_leaf >= 0 ? ~S.root_leaf : 0;
  const DevNode *__restrict__ nodes = S.nodes;
  int sp = 0;
  while (cur != kDone) {
    while (cur >= 0) {
      const DevNode N = nodes[cur];
      tr.nodes++;
      BoxT bl, br;
      child_boxes<true>(N, o, d, rinv, bl, br);
      const bool hl = slab_pass(bl, tmin), hr = slab_pass(br, tmin);
      if (hl && hr) stk[(sp++) * stride] = N.right;  // reference: push right, descend left
      cur = hl ? N.left : (hr ? N.right : kPop);
      if (cur == kPop) cur = sp == 0 ? kDone : stk[(--sp) * stride];
    }
    if (cur != kDone) {
      const int32_t id = ~cur;
      const DevTri T = S.tris[id];
      const TriHit h = cramer(d, T.nab.xyz, T.nac.xyz, T.v0.xyz - o, tri_normal(T.v0, T.nab, T.nac), tmin);
      tr.tests++;
      if (h.accept) {
        tr.last = id;
        if (tr.t - h.t >= kEps) {  // objdef.h:213 — first-found wins near-ties
          tr.t = h.t;
          tr.tri = id;
        }
      }
      cur = sp == 0 ? kDone : stk[(--sp) * stride];
    }
  }
  return tr;
}

// EXACT: nearest-first search of the SAH tree under the result rule above;
// a ray whose answer could depend on the order is searched again left-first
// on the reference tree with the reference's rule.  Both searches skip a
// child whose box starts farther than the current hit plus a margin: every
// triangle inside it lies behind the hit.
__device__ inline Trace traverse_exact(const SceneView &S, f3 o, f3 d, float tmin, int32_t *stk, int stride,
                                       uint32_t &fallbacks) {
  Trace tr;
  tr.nodes = 0;
  tr.tests = 0;
  f3 rinv;
  rinv.x = __builtin_amdgcn_rcpf(d.x);
  rinv.y = __builtin_amdgcn_rcpf(d.y);
  rinv.z = __builtin_amdgcn_rcpf(d.z);
  const bool enter = slab_pass(slab(S.root_min.xyz, S.root_max.xyz, o, rinv), tmin);
  for (int pass = 0;; ++pass) {
    const bool ref = pass > 0;
    const DevNode4 *__restrict__ tree = ref ? S.nodes4 : S.near4;
    tr.t = kFltMax;
    tr.tri = -1;
    tr.last = -1;
    float t2 = kFltMax;
    int32_t cur = !enter ? kDone : (S.root_leaf >= 0 ? ~S.root_leaf : 0);
    int sp = 0;
    while (cur != kDone) {
      while (cur >= 0) {
        cur = step4<true>(tree[cur], o, rinv, tmin, tr.t + S.prune_margin, !ref, PlainStack{stk, stride}, sp,
                          tr.nodes);
        if (cur == kPop) cur = sp == 0 ? kDone : stk[(--sp) * stride];
      }
      if (cur != kDone) {
        const int32_t id = ~cur;
        const DevTri T = S.tris[id];
        float m_x1, m_y4, m_y8;
        tri_minors(T.nab.xyz, T.nac.xyz, m_x1, m_y4, m_y8);
        const TriHit h = cramer_reduced(d, T.nab.xyz, T.nac.xyz, T.v0.xyz - o, tri_normal(T.v0, T.nab, T.nac), m_x1,
                                        m_y4, m_y8, tmin);
        tr.tests++;
        if (h.accept) {
          tr.last = id;
          if (ref ? tr.t - h.t >= kEps : h.t < tr.t) tr.tri = id;
          if (ref) {
            if (tr.t - h.t >= kEps) tr.t = h.t;
          } else {
            near_update(h.t, tr.t, t2);
          }
        }
        cur = sp == 0 ? kDone : stk[(--sp) * stride];
      }
    }
    if (ref || !near_ambiguous(tr.t, t2)) break;
    fallbacks++;
  }
  return tr;
}

// --------------------------------------------------------------- generateRay
// rayGenerator.cl:1-31.  The per-launch constants (0.5/tan(arg/2) and W/H,
// identical in every work-item of the reference) are split off so the fused
// kernel can keep them in scalar registers; the arithmetic is unchanged.
struct CamConst {
  float distance, ratio;
};
__device__ inline CamConst cam_const(const mcpt_camera &cam, uint32_t w, uint32_t h) {
  size_t width = w, height = h;  // NDRange {W, H}: get_global_size is a size_t
  CamConst c;
  c.ratio = width * 1.0f / height;
  c.distance = 0.5f / cl_tan(cam.arg / 2);
  return c;
}
__device__ inline void gen_ray_px(const mcpt_camera &cam, CamConst cc, uint32_t idx, uint32_t idy, uint32_t w,
                                  uint32_t h, f4 &o, f4 &dir) {
  size_t width = w, height = h;
  float px = ((float)idx) / width, py = (float)idy / height;
  const f4 cdir = (f4){cam.direction[0], cam.direction[1], cam.direction[2], cam.direction[3]};
  const f4 chor = (f4){cam.horizontal[0], cam.horizontal[1], cam.horizontal[2], cam.horizontal[3]};
  const f4 cup = (f4){cam.up[0], cam.up[1], cam.up[2], cam.up[3]};
  const f4 ccen = (f4){cam.center[0], cam.center[1], cam.center[2], cam.center[3]};
  if (cam.camera_type == 0) {
    float temp1 = px - 0.5f;
    float temp2 = py - 0.5f;
    float distance = cc.distance, ratio = cc.ratio;
    f4 dd = cdir * distance + temp1 * chor * ratio + temp2 * cup;
    o = ccen;
    dir = cl_normalize(dd);
  } else {
    float ratio = cc.ratio;
    o = ccen + (px - 0.5f) * (cam.arg) * (chor)*ratio + (py - 0.5f) * (cam.arg) * (cup);
    dir = cl_normalize(cdir);
  }
  o.w = as_f(0);
  dir.w = as_f((int32_t)(idy * w + idx));
}
__device__ inline void gen_ray(const mcpt_camera &cam, uint32_t idx, uint32_t idy, uint32_t w, uint32_t h,
                               f4 &o, f4 &dir) {
  gen_ray_px(cam, cam_const(cam, w, h), idx, idy, w, h, o, dir);
}

// -------------------------------------------------------------------- shade
struct ShadeIn {
  f4 o, d;       // ray (o.w = term_depth bits, d.w = id bits)
  f4 nrm;        // hit normal (flipped to face the ray)
  f4 pt;         // hit point
  int32_t mat;
};
struct ShadeOut {
  f4 o, d;
  f4 color;
  bool new_ray;  // the reference writes rays[id] = newRay
  bool bad;      // unknown material type (reference prints "Crash!!!")
  bool pending;  // glossy lobe sample below the surface: resample (resample = true)
};

// shade.cl:75-206 for one live ray that hit something, in steps: a glossy
// lobe's rejection loop (shade.cl:130-132, `while (dot(nd, n) <= 0) nd =
// randomDirection(refl)`) runs ONE draw per call.  A call whose draw falls
// below the surface returns pending with `resample` set and no other effect;
// the next call with the same input and seed chain draws again (the lobe's
// coin is not redrawn), so the lane's sequence of draws is the loop's.  The
// fused kernel leaves such a lane in its S phase, where its next draw shares
// the one randomDirection call site with every other lane's first draw
// (diffuse, and glossy either lobe), instead of holding the whole wave in
// the loop.  G = false: a scene without glossy materials (C2's diffuse-only
// override, C5): the diffuse lobe alone, no coin, never pending.
template <bool G = true, class Mat = const mcpt_material>
__device__ inline ShadeOut shade_hit(Mat *__restrict__ mats, const ShadeIn &in, f4 color, uint32_t &seed,
                                     int max_depth, bool &resample) {
  ShadeOut r;
  r.bad = false;
  r.new_ray = true;
  r.pending = false;
  // material fields are read where they are used (the table is in LDS): the
  // draw below keeps fewer values live
  Mat *__restrict__ Mp = mats + in.mat;
  const int32_t type = Mp->type;
  auto kd_of = [&]() { return (f4){Mp->kd[0], Mp->kd[1], Mp->kd[2], Mp->kd[3]}; };
  auto kaks_of = [&]() { return (f4){Mp->ka_ks[0], Mp->ka_ks[1], Mp->ka_ks[2], Mp->ka_ks[3]}; };
  int32_t td = as_i(in.o.w);
  f4 no, nd;
  if (!G && type == MCPT_GLOSSY) goto bad_material;  // excluded by the G = false scene check
  switch (type) {
    case MCPT_DIFFUSE:
    case MCPT_GLOSSY: {
      if constexpr (!G) {
        nd = random_dir(in.nrm, seed);
        no = in.pt + kEps * nd;
        no.w = as_f(td + 1);
        nd.w = in.d.w;
        color = cl_div4(color * kd_of() * cl_dot3(nd.xyz, in.nrm.xyz), (float)(2 * kClPi));
        break;
      }
      // glossy: the lobe coin (shade.cl:115), then the Phong lobe around the
      // mirror direction, else the diffuse lobe (shade.cl:139)
      const bool lobe = resample || (type == MCPT_GLOSSY && (lcg15(seed) & 0x00000001));
      const f4 mir = lobe ? mirror_dir(in.nrm, in.d) : in.nrm;  // the lobe's axis
      nd = random_dir(mir, seed);
      if (lobe && cl_dot3(nd.xyz, in.nrm.xyz) <= 0) {  // rejected: draw again next call
        resample = true;
        r.pending = true;
        return r;
      }
      resample = false;
      no = in.pt + kEps * nd;
      no.w = as_f(td + 1);
      nd.w = in.d.w;
      // diffuse: color * kd * cos / 2pi; glossy: color * ks * pow(cos_r, Ns) * cos / 2pi
      f4 c;
      if (lobe)
#if MCPT_POW_LOBE
        c = color * kaks_of() * cl_pow_lobe(cl_dot3(nd.xyz, mir.xyz), Mp->Ns);
#else
        c = color * kaks_of() * cl_pow(cl_dot3(nd.xyz, mir.xyz), Mp->Ns);
#endif
      else
        c = color * kd_of();
      color = cl_div4(c * cl_dot3(nd.xyz, in.nrm.xyz), (float)(2 * kClPi));
      break;
    }
    case MCPT_LIGHT:
      r.new_ray = false;
      r.o = in.o;
      r.o.w = as_f(td | (int32_t)MCPT_TERMINATED);
      r.d = in.d;
      r.color = color * kaks_of();
      return r;
    case MCPT_TRANSPARENT: {
      const float Ni = Mp->Ni;
      bool inside = (td & 0x00FF0000) != 0;
      float ei = inside ? Ni : 1.0f;
      float et = inside ? 1.0f : Ni;
      if (!transmit_dir(in.nrm, in.d, ei, et, nd)) {  // total internal reflection
        no = in.pt;
        nd = mirror_dir(in.nrm, in.d);
        nd.w = in.d.w;
        no.w = as_f(td + 1);
        break;
      }
      float fr = fresnel(in.nrm, nd, Ni);
      no = in.pt;
      nd.w = in.d.w;
      int32_t ntd = td + 1;
      if (lcg15(seed) * 1.0f * 0x1p-15f >= fr) {  // x / 32768, exact either way
        ntd ^= 0x00FF0000;
      } else {
        nd.xyz = mirror_dir(in.nrm, in.d).xyz;
      }
      no.w = as_f(ntd);
      break;
    }
    default:  // the reference leaves newRay uninitialised here; we end the path
    bad_material:
      r.bad = true;
      r.new_ray = false;
      r.o = in.o;
      r.o.w = as_f(td | (int32_t)MCPT_TERMINATED);
      r.d = in.d;
      r.color = (f4){0.0f, 0.0f, 0.0f, 0.0f};
      return r;
  }
  int32_t ntd = as_i(no.w);
  if ((ntd & 0x0000FFFF) >= max_depth) {
    color = (f4){0.0f, 0.0f, 0.0f, 0.0f};
    no.w = as_f(ntd | (int32_t)MCPT_TERMINATED);
  }
  r.o = no;
  r.d = nd;
  r.color = color;
  return r;
}
// the whole of shade.cl's work for one ray (the wavefront kernel)
__device__ inline ShadeOut shade_hit_full(const mcpt_material *__restrict__ mats, const ShadeIn &in, f4 color,
                                          uint32_t &seed, int max_depth) {
  bool resample = false;
  ShadeOut so;
  do {
    so = shade_hit(mats, in, color, seed, max_depth, resample);
  } while (so.pending);
  return so;
}

// history.cl:3-28 on one pixel; returns the colour the reference shows.
// length(now) == 0 is evaluated as "every component is +-0": with IEEE
// denormals the built-in's rescaling branch makes length() > 0 for any
// non-zero (or NaN) component, so the two tests agree for every input.
__device__ inline f4 accumulate_one(f4 now, f4 &hist, int32_t &cnt, int max_attempt) {
  const bool zero = now.x == 0.0f && now.y == 0.0f && now.z == 0.0f && now.w == 0.0f;
  if (zero || cnt >= max_attempt) return hist;
  now = cl_div4(now + hist * cnt, (float)(cnt + 1));
  hist = now;
  hist.w = 0.0f;
  ++cnt;
  return now;
}

// --------------------------------------------------------- fused hot kernel
// Block hand-off: a pixel's state passes from the lane that ran frame block
// b-1 to the lane that runs block b as four 8-byte granules {tag:16 |
// payload:48} carrying the 192 bits of (seed, mean.xyzw, count), written as
// two 16-B system-coherent stores and read as two 16-B loads
// (global_store/load_dwordx4 sc0 sc1: bypass the CU's L1, coherent across
// the XCDs' L2s; a 16-B sc1 store costs about what an 8-B one does, so this
// halves the hand-off's fabric writes against one store per word).  The
// reader accepts the state only when all four tags name this launch and
// block b, so every 48-bit piece it keeps is the one the writer stored with
// that tag: the protocol needs each aligned 8-B granule untorn, nothing more
// (no flag, no fence; MI355X_MICROARCH.md "handoff-1to1": data-tagged
// granules are the cheapest hand-off).
// The accesses are buffer loads / stores with the sc1 cache bit (aux 16:
// write-through / coherent at agent scope) rather than volatile ones: volatile
// made the compiler wait for each store to complete and each load to land
// before the next memory instruction, a full memory round trip per 16 B.
typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr uint32_t kHandoffMaxBytes = 0x7FFFFFFFu;  // images beyond it run without hand-offs (mcpt_render_frames)
__device__ inline __amdgpu_buffer_rsrc_t handoff_rsrc(unsigned long long *base) {
  return __builtin_amdgcn_make_buffer_rsrc(base, 0, (int)kHandoffMaxBytes, 0x00020000);
}
__device__ inline u64x2 handoff_load2(__amdgpu_buffer_rsrc_t rs, uint32_t off) {
  return __builtin_bit_cast(u64x2, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 16));
}
__device__ inline void handoff_store2(__amdgpu_buffer_rsrc_t rs, uint32_t off, unsigned long long a,
                                      unsigned long long b) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, (u64x2){a, b}), rs, off, 0, 16);
}
// This wave's XCD (0-7).  Picks the home queue: speed only — any placement
// gives the same result, and waves steal from the other queues when theirs
// runs dry (MI355X_MICROARCH.md, "dequeue": one head word saturates at about
// 88 dequeues/us; sharded per XCD the rate scales with the heads).
__device__ inline uint32_t xcc_id() { return __builtin_amdgcn_s_getreg((3 << 11) | 20) & 7u; }  // hwreg(HW_REG_XCC_ID, 0, 4)

// The search tree's top levels in LDS (RenderArgs::top_levels, 0-kMaxTopLevels;
// mcpt_tuning.top_levels): a complete 4-ary layout after the uniforms, node i's
// slot-k child at 4i + 1 + k, 112 B each (six plane quads and the links).  A
// segment descends through them where it begins (the S phase) instead of
// taking one T-phase gather per level: every traced segment starts at the
// root and enters one node per level.
// MCPT_WG_WAVES: waves per k_render workgroup (4 shipped).  A workgroup's
// waves share one copy of the uniforms, the top levels and the materials (each
// wave keeps its own stack), so the LDS per wave shrinks and a fourth level
// (85 nodes, 9.3 KB) fits.  Against one wave per workgroup, both at the
// shipped 4 waves per SIMD: C4 -3.4 %, C5 -1.2 %, the 8-rank shares of C2 / C4
// / C5 -4.3 / -2.5 / -2.7 %, C2 and C3 even (profiles/r06_wg_waves_w4.jsonl).
#ifndef MCPT_WG_WAVES
#define MCPT_WG_WAVES 4
#endif
constexpr int kWgWaves = MCPT_WG_WAVES;
static_assert(kWgWaves == 1 || kWgWaves == 2 || kWgWaves == 4 || kWgWaves == 8, "k_render workgroups of 1-8 waves");
constexpr int kMaxTopLevels = kWgWaves >= 8 ? 5 : (kWgWaves > 1 ? 4 : 3);
__host__ __device__ constexpr int top_nodes(int levels) {
  return levels <= 0 ? 0 : (levels == 1 ? 1 : (levels == 2 ? 5 : (levels == 3 ? 21 : (levels == 4 ? 85 : 341))));
}

// Uniforms of a launch kept in LDS (k_render).  80-B camera + 16 + 32 + 16 B.
struct __attribute__((aligned(16))) LdsUniforms {
  mcpt_camera cam;
  f4 cc;  // generateRay's 0.5 / tan(arg / 2) and W / H (cam_const)
  f4 root_min, root_max;
  f4 ray_u;  // the primary ray's pixel-independent part: the origin (pinhole) or the direction (camera_type 1)
};
static_assert(sizeof(LdsUniforms) == 144, "LDS uniforms");

struct RenderArgs {
  mcpt_camera cam;
  SceneView S;
  uint32_t *seeds;
  f4 *hist;
  int32_t *count;
  unsigned long long *stats;
  int32_t W, H, local_rows, tiles_x;
  int32_t stripe_rows, stripe_index, stripe_count;
  int32_t max_depth, max_attempt, frame_begin, frames;  // frames: of this launch
  int32_t fpl, blocks;         // frames per block, blocks in this launch
  int32_t nb_head, fpl_tail;   // blocks >= nb_head have fpl_tail frames (nb_head = blocks: all fpl)
  unsigned long long *handoff; // per pixel: kHandoffWords tagged granules
  uint32_t tag_base;           // this launch's tag; a granule for block b carries tag_base | b (16 bits)
  int32_t stack_depth;
  int32_t th_leaf, th_shade;  // lanes waiting before the L / S phase runs
  uint32_t *queue;            // n_queues work-queue heads, kQueueStride apart (zeroed before each launch)
  uint32_t n_queues;          // 1..kQueues
  int32_t lds_mats;           // 1: copy the material table to LDS after the stack
  int32_t top_levels;         // EXACT: the search tree's top levels kept in LDS (0-kMaxTopLevels)
  int32_t chunk;              // queue entries a wave claims per atomic (at least)
  int32_t th_fetch;           // lanes needing an entry before the wave claims
  int32_t *spill;             // WindowStack spill areas, one per resident lane
  int32_t spill_stride;       // entries per lane (stack depth - window)
  const PrimHit *prim;        // per-pixel primary hits (k_primary), nullptr: trace segment 0
  PrimHit *prim_out;          // PRIM launches: where each pixel's primary hit goes
  unsigned long long *wave_log;  // MCPT_PHASE_TIMING: 4 words per workgroup (mcpt_get_wave_log), or nullptr
  uint32_t *px_segments;      // STATS: each pixel's segments of the call added here (mcpt_set_pixel_segments), or nullptr
  uint32_t *px_iters;         // STATS: each pixel's busy lane-iterations of the call, or nullptr
  uint32_t *prim_cost;        // PRIM launches: each pixel's primary-ray lane-iterations (its traversal cost)
  const int32_t *tile_order;  // queue position -> 8x8 tile (dearest first, mcpt_tuning.tile_order), or nullptr: image order
  uint32_t *entry_log;        // MCPT_PHASE_TIMING: per (pixel, block) claim / start / end times (mcpt_get_entry_log), or nullptr
  int32_t spread;             // 1: each run of 64 queue slots takes one pixel from each of 64 tiles (mcpt_tuning.pixel_spread)
};

__device__ inline int32_t global_row(int32_t lr, const RenderArgs &A) {
  int32_t s = lr / A.stripe_rows;
  return (s * A.stripe_count + A.stripe_index) * A.stripe_rows + lr % A.stripe_rows;
}

constexpr float kTmin = 0.001f;  // host EPSILON passed as tmin (oclbasic.h:193, scenebuild.cpp:125)

// Queue x of nq holds the 8x8 tiles t with t % nq == x: queue_items pixel
// slots, each entry q = block * items + slot (block-major).
__device__ inline uint32_t queue_items(uint32_t x, uint32_t n_tiles, uint32_t nq) {
  return x < n_tiles ? ((n_tiles - 1u - x) / nq + 1u) * 64u : 0u;
}

// The fused kernel is a persistent per-wave state machine.
//
// Work queues: a launch renders `frames` frames of every pixel of this GPU's
// stripes, in frame blocks.  (pixel, block) entries are handed out in 8x8-tile
// order from n_queues atomic counters, one per XCD (tiles dealt round-robin);
// a wave takes from its own XCD's queue and steals from the others when that
// one runs dry.  A lane owns a pixel for one block of frames (the seed chain
// and the running mean are sequential per pixel), hands the state on when
// done and pulls the next entry, so lanes whose paths were short keep working
// instead of idling until the wave's slowest pixel finishes.
//
// Phases.  Every lane with a pixel is in one of
//   T: walking internal BVH nodes (cur >= 0)
//   L: holding a leaf whose triangle must be tested (cur = ~tri)
//   S: segment traced (cur == kDone): shade, accumulate, start the next segment
// and each loop iteration runs one T step for the T lanes, then the L phase
// and the S phase only when enough lanes wait for them (or nothing else can
// run).  Expensive phases therefore execute with most of the wave active
// instead of once per diverging lane.  Each lane's own
// sequence of operations is exactly the reference's, so results are unchanged.
// PRIM: the primary-hit pass (PrimHit) run by the same machine: one frame,
// no pixel state; a lane traces its pixel's primary ray, stores the closest
// hit at the S phase instead of shading, and takes the next pixel.
template <int MODE, bool STATS, bool WIN, bool PAIR, bool Q, bool PRIM = false, bool G = true>
__global__ void __launch_bounds__(64 * kWgWaves, MCPT_WAVES_PER_SIMD) k_render(RenderArgs A) {
  constexpr bool PRUNE = MODE != MCPT_MODE_NOPRUNE;
  constexpr bool LIT = MODE == MCPT_MODE_NOPRUNE;
  static_assert(!(Q && LIT), "the quantized search tree is an EXACT-mode structure");
  extern __shared__ int32_t lds_stack[];
  const int lane = threadIdx.x & 63;
  const int wv = kWgWaves > 1 ? (int)(threadIdx.x >> 6) : 0;  // this wave in its workgroup
  const size_t gwave = (size_t)blockIdx.x * kWgWaves + wv;      // this wave in the launch
  // the whole stack in LDS, or its top kStackWindow entries (deep trees, where
  // the whole stack would cap the resident waves per CU; chosen at launch);
  // each wave of the workgroup has its own
  using Stack = typename std::conditional<WIN, WindowStack<kStackWindow>, PlainStack>::type;
  Stack stk;
  int32_t *const my_stack = lds_stack + (size_t)wv * A.stack_depth * 64;
  if constexpr (WIN)
    stk = Stack{my_stack + lane, A.spill + (gwave * 64 + lane) * (size_t)A.spill_stride};
  else
    stk = Stack{my_stack + lane, 64};
  const SceneView &S = A.S;
  const int stack_cap = WIN ? kStackWindow + A.spill_stride : A.stack_depth;  // entries (MCPT_DEBUG bound)
  (void)stack_cap;
  // LDS behind the stack: the per-launch uniforms that only segment and frame
  // starts read (camera, generateRay constants, root box: kept out of the
  // SGPRs, the scarce register file of this kernel), then the material table
  // (small tables only)
  LdsUniforms *U = reinterpret_cast<LdsUniforms *>(lds_stack + (size_t)kWgWaves * A.stack_depth * 64);
  if (threadIdx.x == 0) {
    U->cam = A.cam;
    const CamConst c0 = cam_const(A.cam, (uint32_t)A.W, (uint32_t)A.H);
    U->cc = (f4){c0.distance, c0.ratio, 0.0f, 0.0f};
    U->root_min = S.root_min;
    U->root_max = S.root_max;
    f4 o0, d0;  // the pixel-independent part of every primary ray (PrimHit)
    gen_ray_px(A.cam, c0, 0u, 0u, (uint32_t)A.W, (uint32_t)A.H, o0, d0);
    U->ray_u = A.cam.camera_type == 0 ? o0 : d0;
  }
  // the top nodes follow the uniforms, the material table follows them
  f4 *const top4 = reinterpret_cast<f4 *>(U + 1);
  const int n_top = LIT || S.root_leaf >= 0 ? 0 : top_nodes(A.top_levels);
  if (n_top > 0) {
    // the top levels (the 128-B tree's; the quantized tree has the same ids and
    // links): lane-strided over the nodes' 16-B quads, node by node in layout
    // order; a slot's child id comes from its parent's links in global memory
    for (int e = (int)threadIdx.x; e < n_top * 7; e += 64 * kWgWaves) {
      const int i = e / 7, w = e % 7;
      int lv[kMaxTopLevels], nl = 0;  // the slots on the path from the root, deepest first
      for (int up = i; up > 0; up = (up - 1) >> 2) lv[nl++] = (up - 1) & 3;
      int32_t id = 0;  // layout node i's id, or < 0 (a leaf or an empty slot on the path)
      for (int t = nl - 1; t >= 0 && id >= 0; --t) id = S.near4[id].link[lv[t]];
      if (id >= 0) top4[i * 7 + w] = reinterpret_cast<const f4 *>(S.near4 + id)[w];
    }
  }
  typedef const __attribute__((address_space(3))) mcpt_material LdsMaterial;
  LdsMaterial *const lds_mat_table = (LdsMaterial *)reinterpret_cast<mcpt_material *>(top4 + n_top * 7);
  if (A.lds_mats) {
    mcpt_material *lm = reinterpret_cast<mcpt_material *>(top4 + n_top * 7);
    for (int k = (int)threadIdx.x; k < S.n_mats; k += 64 * kWgWaves) lm[k] = S.mats[k];
  }
  __syncthreads();

  unsigned long long n_seg = 0, n_nodes = 0, n_tests = 0, n_bad = 0;
  unsigned long long w_t = 0, w_l = 0, w_s = 0, n_fb = 0;
  unsigned long long w_it = 0, n_wait = 0, n_idle = 0, n_rej = 0;
  uint32_t px_seg = 0, px_it = 0;  // STATS: segments / busy iterations of the lane's current entry (A.px_*)
  // pixel state.  lst: this lane's role in the queue protocol, one small
  // int (one VGPR; kept out of lane-mask SGPR pairs on purpose, SGPRs are
  // the scarce register file of this kernel)
  // kRes: busy, its glossy lobe sample rejected; it stays in S and draws again
  constexpr int32_t kRes = -1, kBusy = 0, kNeed = 1, kPend = 2, kDead = 3;
  int32_t lst = kNeed;
  int32_t f = 0, cnt = 0;
  uint32_t seed = 0, pxy = 0;  // pxy = x | y << 16 (the pending entry's pixel while kPend)
  int32_t blk = 0;             // frame block of the pixel (the pending entry's block while kPend)
  f4 hist = (f4){0.0f, 0.0f, 0.0f, 0.0f};
  f4 o = hist, d = hist, color = hist;
  auto primary = [&]() __attribute__((always_inline)) {  // no jitter: every frame re-shoots the same primary ray
    const f4 c4 = U->cc;
    CamConst cc;
    cc.distance = c4.x;
    cc.ratio = c4.y;
    gen_ray_px(U->cam, cc, pxy & 0xFFFFu, pxy >> 16, (uint32_t)A.W, (uint32_t)A.H, o, d);
  };
  // path / traversal state (declared with the pixel state below)
  f3 rinv = (f3){0.0f, 0.0f, 0.0f};
  float best_t = kFltMax;
  int32_t cur = kDone, sp = 0;
  f4 best_nrm = (f4){0.0f, 0.0f, 0.0f, 0.0f};  // hit triangle's packed normal, kept from the L phase
  // EXACT: ref = searching the reference tree left-first (the fallback of
  // traverse_exact); t2 = runner-up t of the nearest-first search
  bool ref = LIT;
  float t2 = kFltMax;
  const Stack &sk = stk;
  auto pop_next = [&]() __attribute__((always_inline)) -> int32_t { return sp == 0 ? kDone : sk.pop(sp); };
  auto begin_segment = [&]() __attribute__((always_inline)) {
    rinv.x = __builtin_amdgcn_rcpf(d.x);
    rinv.y = __builtin_amdgcn_rcpf(d.y);
    rinv.z = __builtin_amdgcn_rcpf(d.z);
    best_t = kFltMax;
    t2 = kFltMax;
    ref = LIT;
    sp = 0;
    if (!slab_pass(box_test<LIT>(U->root_min.xyz, U->root_max.xyz, o.xyz, d.xyz, rinv), kTmin)) {
      cur = kDone;
    } else if (S.root_leaf >= 0) {
      cur = ~S.root_leaf;
    } else if (!LIT && n_top > 0) {
      // the top levels from LDS (ds_read_b128; at the root the same address in
      // every lane): the exact 128-B nodes also for the quantized tree, whose
      // node ids and links are the 128-B tree's -- exact boxes are the
      // union-of-leaf boxes the candidate-set argument needs
      typedef const __attribute__((address_space(3))) f4 LdsF4;
      uint32_t ctr = 0;
      int ti = 0;  // layout index of the node to step
      cur = 0;
#pragma unroll
      for (int lvl = 0; lvl < kMaxTopLevels; ++lvl) {
        if (lvl >= A.top_levels) break;
        LdsF4 *rq = (LdsF4 *)(top4 + ti * 7);
        const f4 q0 = rq[0], q1 = rq[1], q2 = rq[2], q3 = rq[3], q4 = rq[4], q5 = rq[5], lk = rq[6];
        cur = step4q<PRUNE>(q0, q1, q2, q3, q4, q5, as_i(lk.x), as_i(lk.y), as_i(lk.z), as_i(lk.w), o.xyz, rinv, kTmin,
                            best_t + S.prune_margin, true, sk, sp, ctr);
        // the entered slot's child, when it is internal: the next level's node
        const int k = cur < 0 ? -1 : (cur == as_i(lk.x) ? 0 : (cur == as_i(lk.y) ? 1 : (cur == as_i(lk.z) ? 2 : 3)));
        ti = k < 0 ? -1 : 4 * ti + 1 + k;
        if (ti < 0) break;
      }
      if (STATS) n_nodes += ctr;
      if (cur == kPop) cur = pop_next();
    } else {
      cur = 0;
    }
  };
  // a frame's first segment: the primary ray and its hit are the same every
  // frame (the primary-hit pass computed them once), so the lane takes both
  // from the pixel's record and goes straight to S
  auto begin_frame = [&]() __attribute__((always_inline)) {
    color = (f4){1.0f, 1.0f, 1.0f, 1.0f};
    if (A.prim) {
      const uint32_t pid = (pxy >> 16) * (uint32_t)A.W + (pxy & 0xFFFFu);
      const f4 *ph = reinterpret_cast<const f4 *>(A.prim + pid);
      const f4 h0 = ph[0], h1 = ph[1];  // nrm | t, ray xyz
      const f4 u = U->ray_u;
      const f4 v = (f4){h1.y, h1.z, h1.w, 0.0f};
      const bool pin = U->cam.camera_type == 0;
      o = pin ? u : v;
      d = pin ? v : u;
      o.w = as_f(0);
      d.w = as_f((int32_t)pid);  // gen_ray_px: idy * w + idx
      best_nrm = h0;
      best_t = h1.x;
      t2 = kFltMax;
      ref = LIT;
      sp = 0;
      cur = kDone;
    } else {
      primary();
      begin_segment();
    }
  };
  // Queue entry q of queue x = block * items + slot: frame block q / items of
  // pixel slot q % items of that queue's tiles.  Blocks of one pixel run in
  // order: the lane that takes (p, b > 0) waits until the lane that ran
  // (p, b - 1) has published its granules with tag (tag_base | b).
  // No deadlock: every entry waits only for an entry of the same queue with
  // a lower index, entries are claimed in index order, and a wave starts all
  // its claimed entries before it claims more.
  const uint32_t n_tiles = (uint32_t)A.tiles_x * (uint32_t)((A.local_rows + 7) >> 3);
  const uint32_t nq = A.n_queues;
  // wave-uniform queue state, packed into one SGPR: bits 0-3 the queue claims
  // go to, 4-7 the queue of the pool, 8-11 queues found dry, bit 12 "the
  // claim queue ran dry: the next claim moves on"
  uint32_t qs = (xcc_id() % nq) * 0x11u;
  uint32_t pool = 0, pool_left = 0;  // wave-uniform: claimed, unassigned entries of queue (qs >> 4) & 15

#ifdef MCPT_PHASE_TIMING
  uint64_t ph[4] = {0, 0, 0, 0};
  uint64_t tick = __builtin_amdgcn_s_memtime();
  // the wave's timeline (mcpt_get_wave_log): start, the first iteration a
  // lane found every queue dry, end (s_memrealtime, 100 MHz, chip-wide),
  // entries started
  const uint64_t rt_start = __builtin_amdgcn_s_memrealtime();
  uint64_t rt_dry = 0, n_started = 0, w_it_log = 0, rt_last = 0, pend_it = 0;
#endif
  for (;;) {
    // ---- fetch: lanes without work take the next queue entries, from the
    // wave's pool of claimed entries; one atomic claims max(chunk, shortfall)
    {
      // lanes that need an entry start together once th_fetch of them wait
      // (their state loads then share one wait), or when no lane is busy
      const unsigned long long mn = __ballot(lst == kNeed);
      if (mn && (__popcll(mn) >= A.th_fetch || !__ballot(G ? lst <= kBusy : lst == kBusy))) {
        const uint32_t n_need = (uint32_t)__popcll(mn);
        const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(mn >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mn, 0));
        uint32_t q = pool + rank, qx = (qs >> 4) & 15u;
        bool got = rank < pool_left;
        if (n_need <= pool_left) {
          pool += n_need;
          pool_left -= n_need;
        } else {
          if (qs & 0x1000u) {  // steal: the next queue round the ring
            const uint32_t nxt = (qs & 15u) + 1u == nq ? 0u : (qs & 15u) + 1u;
            qs = (qs & 0x0F0u) + 0x100u * (((qs >> 8) & 15u) + 1u) + nxt;
          }
          const uint32_t qid = qs & 15u;
          const uint32_t shortfall = n_need - pool_left;
          if (((qs >> 8) & 15u) < nq) {
            const uint32_t claim = max((uint32_t)A.chunk, shortfall);
            const uint32_t total = queue_items(qid, n_tiles, nq) * (uint32_t)A.blocks;
            const int leader = __builtin_ctzll(mn);
            uint32_t base = 0;
            if (lane == leader) base = atomicAdd(A.queue + qid * kQueueStride, claim);
            base = __builtin_amdgcn_readfirstlane(__shfl(base, leader));
            if (!got) {
              q = base + (rank - pool_left);
              qx = qid;
              got = q < total;
            }
            pool = base + shortfall;
            pool_left = claim - shortfall;
            qs = (qs & ~0xF0u) | (qid << 4);
            if (base + claim >= total) {  // the queue is dry after this claim
              qs |= 0x1000u;
              pool_left = pool < total ? min(pool_left, total - pool) : 0u;
            }
          } else {
            pool_left = 0;
          }
        }
        if (lst == kNeed) {
          if (got) {
            const uint32_t items = queue_items(qx, n_tiles, nq);
            const uint32_t b = q / items, j = q - b * items;
            uint32_t u = j >> 6, kk = j & 63u;  // the queue's tile u, its pixel kk
            if (A.spread) {
              // spread: slot j of the group of (up to) 64 tiles g0.. is pixel
              // i / gs of tile g0 + i % gs, i = its index in the group, so a
              // wave's 64 consecutive slots come from 64 tiles and the dear
              // pixels of one tile run in different waves.  A bijection on the
              // group's slots, the same for every block of the pixel.
              const uint32_t g0 = u & ~63u, gs = min(64u, (items >> 6) - g0), i = ((u - g0) << 6) + kk;
              u = g0 + i % gs;
              kk = i / gs;
            }
            const int32_t tpos = (int32_t)(u * nq + qx), k = (int32_t)kk;
            const int32_t tile = A.tile_order ? A.tile_order[tpos] : tpos;
            const int32_t x = (tile % A.tiles_x) * 8 + (k & 7);
            const int32_t lr = (tile / A.tiles_x) * 8 + (k >> 3);
            const int32_t y = lr < A.local_rows ? global_row(lr, A) : A.H;
            if (x < A.W && y < A.H) {  // else an edge-tile hole: fetch again
              lst = kPend;
              blk = (int32_t)b;
              pxy = (uint32_t)x | ((uint32_t)y << 16);
#ifdef MCPT_PHASE_TIMING
              if (A.entry_log)
                A.entry_log[((size_t)(y * A.W + x) * A.blocks + b) * 3] = (uint32_t)__builtin_amdgcn_s_memrealtime();
#endif
            }
          } else if (((qs >> 8) & 15u) >= nq) {
            lst = kDead;  // every queue is dry
          }
#ifdef MCPT_PHASE_TIMING
          if (lst == kDead && rt_dry == 0) rt_dry = __builtin_amdgcn_s_memrealtime();
#endif
        }
      }
      if (lst == kPend) {  // start the entry once its pixel's previous block is published
        const int32_t pp = (int32_t)(pxy >> 16) * A.W + (int32_t)(pxy & 0xFFFFu);
        bool ready = true;
        if (PRIM) {  // no pixel state: only the primary ray
        } else if (blk == 0) {  // state from before this launch
          seed = A.seeds[pp];
          hist = A.hist[pp];
          cnt = A.count[pp];
        } else {  // published by another lane, any XCD
          const __amdgpu_buffer_rsrc_t hr = handoff_rsrc(A.handoff);
          const uint32_t go = (uint32_t)pp * (uint32_t)(kHandoffWords * 8);
          asm volatile("" ::: "memory");  // a poll: the granules are read again every iteration
          const u64x2 h0 = handoff_load2(hr, go), h1 = handoff_load2(hr, go + 16);
          const unsigned long long want = (unsigned long long)(A.tag_base | (uint32_t)blk);
          ready = (h0.x >> 48) == want && (h0.y >> 48) == want && (h1.x >> 48) == want && (h1.y >> 48) == want;
          // 192 payload bits, 48 per granule: seed | mean.x | mean.y | mean.z | mean.w | count
          seed = (uint32_t)h0.x;
          hist = (f4){as_f((int32_t)(((uint32_t)(h0.x >> 32) & 0xFFFFu) | ((uint32_t)h0.y << 16))),
                      as_f((int32_t)(uint32_t)(h0.y >> 16)), as_f((int32_t)(uint32_t)h1.x),
                      as_f((int32_t)(((uint32_t)(h1.x >> 32) & 0xFFFFu) | ((uint32_t)h1.y << 16)))};
          cnt = (int32_t)(uint32_t)(h1.y >> 16);
        }
        if (ready) {
          lst = kBusy;
          f = 0;
          begin_frame();
        }
#ifdef MCPT_PHASE_TIMING
        if (ready) {
          n_started++, rt_last = __builtin_amdgcn_s_memrealtime();
          if (A.entry_log) A.entry_log[((size_t)pp * A.blocks + blk) * 3 + 1] = (uint32_t)rt_last;
        } else {
          pend_it++;
        }
#endif
      }
    }
    MCPT_TICK(0);
    if (!__ballot(lst != kDead)) break;
#ifdef MCPT_PHASE_TIMING
    ++w_it_log;
#endif
    const bool live = G ? lst <= kBusy : lst == kBusy;  // (kRes only with glossy materials)
    if (STATS || PRIM) px_it += live;
    // phase thresholds scaled to the wave's live lanes: a wave with few pixels
    // (a launch's tail, a strong-scaled rank) does not wait for lane counts
    // only a full wave reaches (C2 -3 %, C5 -4 %, C2 4- and 8-rank shares
    // -16 % / -19 %; profiles/r02_shares_calls.txt)
    const int n_live = __popcll(__ballot(live));
    const int th_leaf = max(1, (A.th_leaf * n_live + 63) >> 6), th_shade = max(1, (A.th_shade * n_live + 63) >> 6);
    if (STATS) {
      if (lane == __builtin_ctzll(__ballot(1))) w_it++;
      n_wait += lst == kPend;
      n_idle += lst == kNeed || lst == kDead;  // no claim yet, an edge hole, or out of work (tail)
    }
    // one triangle test with the reference's arithmetic and result rule (the
    // L phase)
    using Tri = typename std::conditional<Q, DevTriQ, DevTri>::type;
    auto test = [&](const Tri &X, int32_t xi) {
      TriHit h;
      if constexpr (Q) {
        // the reference leaf's own box (hlbvh.cpp:97-100: min/max of the
        // vertices; equal to the stored box, checked at upload), tested with
        // the reference's arithmetic: the search tree's quantized boxes only
        // ever let MORE leaves through, this restores exactly its set
        const f2 bx = (f2){fminf(fminf(X.v0.x, X.v1.x), X.v2.x), fmaxf(fmaxf(X.v0.x, X.v1.x), X.v2.x)};
        const f2 by = (f2){fminf(fminf(X.v0.y, X.v1.y), X.v2.y), fmaxf(fmaxf(X.v0.y, X.v1.y), X.v2.y)};
        const f2 bz = (f2){fminf(fminf(X.v0.z, X.v1.z), X.v2.z), fmaxf(fmaxf(X.v0.z, X.v1.z), X.v2.z)};
        const bool leaf = slab_pass(slab_pairs(bx, by, bz, o.xyz, rinv), kTmin);
        // objdef.h:190-199: AB = v1 - v0, AC = v2 - v0, matrix rows -AB, -AC
        const f3 nab = -(X.v1.xyz - X.v0.xyz), nac = -(X.v2.xyz - X.v0.xyz);
        h = cramer_reduced(d.xyz, nab, nac, X.v0.xyz - o.xyz, X.nrm.xyz, X.v0.w, X.v1.w, X.v2.w, kTmin);
        h.accept = h.accept && leaf;
        if (STATS) n_rej += !leaf;
      } else {
        const f3 xn = tri_normal(X.v0, X.nab, X.nac);
        if (LIT) {
          h = cramer(d.xyz, X.nab.xyz, X.nac.xyz, X.v0.xyz - o.xyz, xn, kTmin);
        } else {
          float m_x1, m_y4, m_y8;
          tri_minors(X.nab.xyz, X.nac.xyz, m_x1, m_y4, m_y8);
          h = cramer_reduced(d.xyz, X.nab.xyz, X.nac.xyz, X.v0.xyz - o.xyz, xn, m_x1, m_y4, m_y8, kTmin);
        }
      }
      if (STATS) n_tests++;
      if (h.accept) {
        if (ref ? best_t - h.t >= kEps : h.t < best_t) {  // objdef.h:213
          if constexpr (Q)
            best_nrm = X.nrm;
          else
            best_nrm = (f4){X.v0.w, X.nab.w, X.nac.w, as_f(~xi)};  // the material is read at shading
        }
        if (ref) {
          if (best_t - h.t >= kEps) best_t = h.t;
        } else {
          near_update(h.t, best_t, t2);
        }
      }
    };
    // ---- T: one node step (objdef.h:252-273 with child boxes)
    const bool in_t = live && cur >= 0;
    if (__ballot(in_t)) {
      if (STATS && lane == __builtin_ctzll(__ballot(1))) w_t++;
      if (in_t) {
        if (Q) {  // EXACT, quantized SAH tree nearest-first (4 loads), or the reference tree left-first
          uint32_t ctr = 0;
          if (MCPT_DCHECK(cur < (ref ? S.n_nodes4 : S.n_near4), 1)) {
            f4 q0, q1, q2, q3, q4, q5;
            int32_t l0, l1, l2, l3;
            if (!ref) {
              const f4 *p = reinterpret_cast<const f4 *>(S.near4q + cur);
              const f4 c0 = p[0], c1 = p[1], c2 = p[2], c3 = p[3];
              const float ox = c0.x, oy = c0.y, oz = c0.z, sx = c0.w, sy = c2.z, sz = c2.w;
              // plane byte k of a word, decoded as fma(q, s, o) (v_cvt_f32_ubyte + fma)
              auto dec = [](uint32_t w, float sa, float oa, float sb, float ob) -> f4 {
                return (f4){__builtin_fmaf((float)(w & 0xFFu), sa, oa), __builtin_fmaf((float)((w >> 8) & 0xFFu), sa, oa),
                            __builtin_fmaf((float)((w >> 16) & 0xFFu), sb, ob), __builtin_fmaf((float)(w >> 24), sb, ob)};
              };
              q0 = dec(as_u(c1.x), sx, ox, sy, oy);  // slot 0: x x y y
              q1 = dec(as_u(c1.y), sz, oz, sx, ox);  // slot 0: z z | slot 1: x x
              q2 = dec(as_u(c1.z), sy, oy, sz, oz);  // slot 1: y y z z
              q3 = dec(as_u(c1.w), sx, ox, sy, oy);  // slot 2: x x y y
              q4 = dec(as_u(c2.x), sz, oz, sx, ox);  // slot 2: z z | slot 3: x x
              q5 = dec(as_u(c2.y), sy, oy, sz, oz);  // slot 3: y y z z
              l0 = as_i(c3.x), l1 = as_i(c3.y), l2 = as_i(c3.z), l3 = as_i(c3.w);
            } else {
              const DevNode4 &N = S.nodes4[cur];
              q0 = N.q[0], q1 = N.q[1], q2 = N.q[2], q3 = N.q[3], q4 = N.q[4], q5 = N.q[5];
              l0 = N.link[0], l1 = N.link[1], l2 = N.link[2], l3 = N.link[3];
            }
            cur = step4q<PRUNE>(q0, q1, q2, q3, q4, q5, l0, l1, l2, l3, o.xyz, rinv, kTmin, best_t + S.prune_margin,
                                !ref, sk, sp, ctr);
            if (!MCPT_DCHECK(sp <= stack_cap, 0)) sp = stack_cap;
          } else {
            cur = kPop;
          }
          if (STATS) n_nodes += ctr;
        } else if (!LIT) {  // EXACT: SAH tree nearest-first, or the reference tree left-first
          uint32_t ctr = 0;
          const DevNode4 *__restrict__ tree = ref ? S.nodes4 : S.near4;
          if (MCPT_DCHECK(cur < (ref ? S.n_nodes4 : S.n_near4), 1)) {
            cur = step4<PRUNE>(tree[cur], o.xyz, rinv, kTmin, best_t + S.prune_margin, !ref, sk, sp, ctr);
            if (!MCPT_DCHECK(sp <= stack_cap, 0)) sp = stack_cap;
          } else {
            cur = kPop;
          }
          if (STATS) n_nodes += ctr;
        } else {  // NOPRUNE: the reference's binary tree, literal division
          const DevNode N = S.nodes[MCPT_DCHECK(cur < S.n_int, 1) ? cur : 0];
          if (STATS) n_nodes++;
          BoxT bl, br;
          child_boxes<LIT>(N, o.xyz, d.xyz, rinv, bl, br);
          bool hl = slab_pass(bl, kTmin), hr = slab_pass(br, kTmin);
          if (PRUNE) {
            const float lim = best_t + S.prune_margin;
            hl = hl && !(bl.tnear > lim);
            hr = hr && !(br.tnear > lim);
          }
          if (hl && hr) sk.push(sp, N.right);  // push right, descend left
          cur = hl ? N.left : (hr ? N.right : kPop);
          if (!MCPT_DCHECK(sp <= stack_cap, 0)) sp = stack_cap;
        }
        if (cur == kPop) cur = pop_next();
      }
    }
    MCPT_TICK(1);
    // ---- L: triangle tests, batched
    const bool in_l = live && cur < 0 && cur != kDone;
    const unsigned long long ml = __ballot(in_l);
    if (ml && (__popcll(ml) >= th_leaf || !__ballot(live && cur >= 0))) {
      if (STATS && lane == __builtin_ctzll(__ballot(1))) w_l++;
      if (in_l) {
        // PAIR (MCPT_SCHED_PAIRED): when the next stack entry is a leaf too,
        // its triangle is fetched with this one and tested right after it;
        // the lane's sequence of tests is unchanged, one phase serves two leaves
        const int32_t nx = !PAIR || sp == 0 ? kDone : sk.peek(sp);
        const bool two = PAIR && nx < 0 && nx != kDone;
        const Tri *tri_arr;
        if constexpr (Q)
          tri_arr = S.triq;
        else
          tri_arr = S.tris;
        const int32_t ti = MCPT_DCHECK(~cur < S.n_tris, 2) ? ~cur : 0;
        const Tri T = tri_arr[ti];
        Tri T2;
        int32_t ti2 = 0;
        if (two) {
          ti2 = MCPT_DCHECK(~nx < S.n_tris, 2) ? ~nx : 0;
          T2 = tri_arr[ti2];
        }
        test(T, ti);
        if (two) {
          (void)sk.pop(sp);
          test(T2, ti2);
        }
        cur = pop_next();
      }
    }
    MCPT_TICK(2);
    // ---- S: finish the segment (shade.cl), accumulate (history.cl), next segment
    const bool in_s = live && cur == kDone;
    const unsigned long long ms = __ballot(in_s);
    if (ms && (__popcll(ms) >= th_shade || !__ballot(live && cur != kDone))) {
      if (STATS && lane == __builtin_ctzll(__ballot(1))) w_s++;
      if (in_s && !ref && near_ambiguous(best_t, t2)) {  // order could matter: search again left-first
        if (STATS) n_fb++;
        ref = true;
        best_t = kFltMax;
        sp = 0;
        cur = S.root_leaf >= 0 ? ~S.root_leaf : 0;  // the root box passed: there were hits
      } else if (PRIM && in_s) {
        PrimHit h;
        h.nrm = (f4){0.0f, 0.0f, 0.0f, 0.0f};
        if (best_t < kFltMax) {
          h.nrm = best_nrm;
          if (!Q) h.nrm.w = as_f(hit_material(S.tris, as_i(best_nrm.w)));  // the record carries the material
        }
        h.t = best_t;
        const f4 v = U->cam.camera_type == 0 ? d : o;
        h.ray[0] = v.x, h.ray[1] = v.y, h.ray[2] = v.z;
        A.prim_out[(size_t)(pxy >> 16) * (size_t)A.W + (pxy & 0xFFFFu)] = h;
        A.prim_cost[(size_t)(pxy >> 16) * (size_t)A.W + (pxy & 0xFFFFu)] = px_it;
        px_it = 0;
        lst = kNeed;
      } else if (in_s) {
        if (STATS && lst == kBusy) n_seg++, px_seg++;
        bool done = false, fresh = false, pending = false;
        if (best_t >= kFltMax) {  // shade.cl:92-96 — miss: black, terminate
          color = (f4){0.0f, 0.0f, 0.0f, 0.0f};
          done = true;
        } else {
          const f4 tn = best_nrm;
          ShadeIn in;
          in.o = o;
          in.d = d;
          in.nrm = (f4){tn.x, tn.y, tn.z, 0.0f};
          if (cl_dot3(d.xyz, in.nrm.xyz) > 0) in.nrm = -in.nrm;  // intersect.cl:23-25
          in.pt = o + best_t * d;                                  // objdef.h:218
          in.mat = Q ? as_i(tn.w) : hit_material(S.tris, as_i(tn.w));
          bool rs = G && lst == kRes;
          ShadeOut so;
          if (A.lds_mats)  // LDS-typed reads (ds_read, no flat access waiting on vector memory)
            so = shade_hit<G>(lds_mat_table, in, color, seed, A.max_depth, rs);
          else
            so = shade_hit<G>(S.mats, in, color, seed, A.max_depth, rs);
          pending = so.pending;
          lst = pending ? kRes : kBusy;
          if (!pending) {
            if (STATS) n_bad += so.bad;
            color = so.color;
            o = so.o;
            d = so.d;
            done = (as_i(o.w) & (int32_t)MCPT_TERMINATED) != 0;
          }
        }
        if (done) {
          // ColorOut: history runs while attemptCount <= MAX_ATTEMPT (colorout.cpp:56)
          const bool head = blk < A.nb_head;
          const int32_t f0 = head ? blk * A.fpl : A.nb_head * A.fpl + (blk - A.nb_head) * A.fpl_tail;
          if (A.frame_begin + f0 + f <= A.max_attempt) (void)accumulate_one(color, hist, cnt, A.max_attempt);
          ++f;
          const int32_t fend = min(head ? A.fpl : A.fpl_tail, A.frames - f0);
          fresh = f < fend;
          if (f == fend) {  // block complete: write back, fetch another next iteration
            const int32_t pid = (int32_t)(pxy >> 16) * A.W + (int32_t)(pxy & 0xFFFFu);
            if (blk + 1 < A.blocks) {  // publish for the lane that takes the next block
              const unsigned long long tag = (unsigned long long)(A.tag_base | (uint32_t)(blk + 1)) << 48;
              const uint32_t w1 = (uint32_t)as_i(hist.x), w2 = (uint32_t)as_i(hist.y);
              const uint32_t w3 = (uint32_t)as_i(hist.z), w4 = (uint32_t)as_i(hist.w);
              const __amdgpu_buffer_rsrc_t hr = handoff_rsrc(A.handoff);
              const uint32_t go = (uint32_t)pid * (uint32_t)(kHandoffWords * 8);
              handoff_store2(hr, go, tag | seed | (unsigned long long)(w1 & 0xFFFFu) << 32,
                             tag | (w1 >> 16) | (unsigned long long)w2 << 16);
              handoff_store2(hr, go + 16, tag | w3 | (unsigned long long)(w4 & 0xFFFFu) << 32,
                             tag | (w4 >> 16) | (unsigned long long)(uint32_t)cnt << 16);
            } else {
              A.seeds[pid] = seed;
              A.hist[pid] = hist;
              A.count[pid] = cnt;
            }
            if (STATS && A.px_segments) atomicAdd(A.px_segments + pid, px_seg);
            if (STATS && A.px_iters) atomicAdd(A.px_iters + pid, px_it);
            if (STATS) px_it = 0;
#ifdef MCPT_PHASE_TIMING
            if (A.entry_log) A.entry_log[((size_t)pid * A.blocks + blk) * 3 + 2] = (uint32_t)__builtin_amdgcn_s_memrealtime();
#endif
            if (STATS) px_seg = 0;
            lst = kNeed;
          }
        }
        if (lst == kBusy) {
          if (fresh)
            begin_frame();
          else
            begin_segment();
        }
      }
    }
    MCPT_TICK(3);
  }
#ifdef MCPT_PHASE_TIMING
  if (lane == 0)
    for (int k = 0; k < 4; ++k) atomicAdd(&A.stats[kPhaseSlot + k], (unsigned long long)ph[k]);
  {
    // wave reductions of the lanes' records: earliest dry time, latest
    // entry start, entries started, iterations spent waiting for a block
    auto red = [&](uint64_t v, int op) {  // 0 min, 1 max, 2 sum
      for (int off = 32; off > 0; off >>= 1) {
        const uint64_t o2 = ((uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), off) << 32) |
                            (uint32_t)__shfl_xor((int)(uint32_t)v, off);
        v = op == 0 ? (o2 < v ? o2 : v) : (op == 1 ? (o2 > v ? o2 : v) : v + o2);
      }
      return v;
    };
    const uint64_t dry = red(rt_dry ? rt_dry : ~0ull, 0);
    const uint64_t last = red(rt_last, 1), started = red(n_started, 2), pend = red(pend_it, 2);
    const uint64_t rt_end = __builtin_amdgcn_s_memrealtime();
    if (A.wave_log && lane == 0) {
      unsigned long long *w = A.wave_log + gwave * kWaveLogWords;
      w[0] = rt_start;
      w[1] = dry == ~0ull ? rt_end : dry;
      w[2] = rt_end;
      w[3] = w_it_log;
      w[4] = started;
      w[5] = last ? last : rt_start;
      w[6] = pend;
      w[7] = xcc_id();
    }
  }
#endif
  if (STATS) {
    atomicAdd(&A.stats[0], n_seg);
    atomicAdd(&A.stats[1], n_nodes);
    atomicAdd(&A.stats[2], n_tests);
    if (n_bad) atomicAdd(&A.stats[3], n_bad);
    if (n_fb) atomicAdd(&A.stats[7], n_fb);
    if (w_t | w_l | w_s) {
      atomicAdd(&A.stats[4], w_t);
      atomicAdd(&A.stats[5], w_l);
      atomicAdd(&A.stats[6], w_s);
    }
    if (w_it) atomicAdd(&A.stats[8], w_it);
    if (n_wait) atomicAdd(&A.stats[9], n_wait);
    if (n_idle) atomicAdd(&A.stats[10], n_idle);
    if (n_rej) atomicAdd(&A.stats[11], n_rej);
  }
}

// ------------------------------------------------------ wavefront kernels
__global__ void k_generate(mcpt_camera cam, uint32_t w, uint32_t h, mcpt_ray *rays) {
  uint32_t x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
  if (x >= w || y >= h) return;
  f4 o, d;
  gen_ray(cam, x, y, w, h, o, d);
  mcpt_ray &r = rays[(size_t)y * w + x];
  *(f4 *)r.origin = o;
  *(f4 *)r.direction = d;
}

template <int MODE>
__global__ void __launch_bounds__(64) k_intersect(SceneView S, const mcpt_ray *rays, int64_t n, mcpt_hit *hits,
                                                  float tmin) {
  extern __shared__ int32_t lds_stack[];
  int64_t id = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (id >= n) return;
  const f4 o = *(const f4 *)rays[id].origin;
  const f4 d = *(const f4 *)rays[id].direction;
  if (as_i(o.w) & (int32_t)0xFF000000) return;  // intersect.cl:16-18 (hit left untouched)
  uint32_t fallbacks = 0;
  Trace tr = MODE == MCPT_MODE_NOPRUNE ? traverse_noprune(S, o.xyz, d.xyz, tmin, lds_stack + threadIdx.x, 64)
                                       : traverse_exact(S, o.xyz, d.xyz, tmin, lds_stack + threadIdx.x, 64, fallbacks);
  mcpt_hit h;
  f4 nrm = (f4){0.0f, 0.0f, 0.0f, 0.0f}, pt = (f4){0.0f, 0.0f, 0.0f, 0.0f};
  h.t = tr.t;
  h.triangle_id = 0;
  h.material_id = 0;
  h.pad = 0;
  if (tr.tri >= 0) {
    const DevTri &T = S.tris[tr.tri];
    nrm = (f4){T.v0.w, T.nab.w, T.nac.w, 0.0f};
    pt = o + tr.t * d;
    h.material_id = (uint32_t)as_i(T.aux.x);
  }
  if (tr.last >= 0) {
    h.triangle_id = (uint32_t)(MODE == MCPT_MODE_NOPRUNE ? tr.last : tr.tri);
    if (cl_dot3(d.xyz, nrm.xyz) > 0) nrm = -nrm;
  }
  *(f4 *)h.normal = nrm;
  *(f4 *)h.point = pt;
  hits[id] = h;
}

// The primary hit of every pixel of this rank's stripes (the cache k_render
// reads at each frame start, PrimHit): the frame's first ray (gen_ray_px, as
// k_render's frame start makes it) traced with the same traversal k_intersect
// uses, which is the reference's closest hit (EXACT: the order-free search
// with its fallback; NOPRUNE: the reference tree itself).
template <int MODE>
__global__ void __launch_bounds__(64) k_primary(RenderArgs A, PrimHit *out) {
  extern __shared__ int32_t lds_stack[];
  // one 8x8 tile of the rank's rows per wave: neighbouring primary rays walk
  // the same nodes, so the wave's gathers share lines
  const int32_t tile = (int32_t)blockIdx.x;
  const int32_t x = (tile % A.tiles_x) * 8 + (int32_t)(threadIdx.x & 7u);
  const int32_t lr = (tile / A.tiles_x) * 8 + (int32_t)(threadIdx.x >> 3);
  if (x >= A.W || lr >= A.local_rows) return;
  const int32_t y = global_row(lr, A);
  f4 o, d;
  gen_ray_px(A.cam, cam_const(A.cam, (uint32_t)A.W, (uint32_t)A.H), (uint32_t)x, (uint32_t)y, (uint32_t)A.W,
             (uint32_t)A.H, o, d);
  uint32_t fallbacks = 0;
  const Trace tr = MODE == MCPT_MODE_NOPRUNE ? traverse_noprune(A.S, o.xyz, d.xyz, kTmin, lds_stack + threadIdx.x, 64)
                                             : traverse_exact(A.S, o.xyz, d.xyz, kTmin, lds_stack + threadIdx.x, 64,
                                                              fallbacks);
  PrimHit h;
  h.nrm = (f4){0.0f, 0.0f, 0.0f, 0.0f};
  if (tr.tri >= 0) {
    const DevTri &T = A.S.tris[tr.tri];
    h.nrm = (f4){T.v0.w, T.nab.w, T.nac.w, T.aux.x};
  }
  h.t = tr.t;
  const f4 v = A.cam.camera_type == 0 ? d : o;
  h.ray[0] = v.x, h.ray[1] = v.y, h.ray[2] = v.z;
  out[(size_t)y * A.W + x] = h;
  A.prim_cost[(size_t)y * A.W + x] = tr.nodes + tr.tests;
}

// The dearest-first tile order (mcpt_tuning.tile_order): each 8x8 tile of
// the rank's rows keyed by its pixels' primary-ray traversal cost (the
// costliest pixel, or the sum), counting-sorted descending (k_tile_sort), so the tiles
// whose pixel chains take longest are claimed first.  Speed only: which lane
// runs which entry when never changes a bit.
constexpr int kTileBuckets = 256;  // tile-order keys: the cost saturated to 8 bits
__global__ void __launch_bounds__(64) k_tile_keys(RenderArgs A, const uint32_t *cost, int32_t n_tiles, int sum,
                                                  uint8_t *keys) {
  // one wave per tile, one lane per pixel
  const int32_t t = (int32_t)blockIdx.x;
  const int k = (int)threadIdx.x;
  const int32_t x = (t % A.tiles_x) * 8 + (k & 7), lr = (t / A.tiles_x) * 8 + (k >> 3);
  uint32_t c = x < A.W && lr < A.local_rows ? cost[(size_t)global_row(lr, A) * A.W + x] : 0u;
  for (int off = 32; off > 0; off >>= 1) {
    const uint32_t o = (uint32_t)__shfl_xor((int)c, off);
    c = sum ? c + o : max(c, o);
  }
  if (sum) c = (c + 7u) >> 3;  // the summed cost in units of 8
  if (k == 0) keys[t] = (uint8_t)min(c, (uint32_t)(kTileBuckets - 1));
}
// Counting sort of the tile keys, dearest first, in one workgroup (tiles in
// a bucket keep no particular order: speed only).
__global__ void __launch_bounds__(1024) k_tile_sort(const uint8_t *keys, int32_t n_tiles, int32_t *order) {
  __shared__ uint32_t hist[kTileBuckets];
  for (int b = threadIdx.x; b < kTileBuckets; b += blockDim.x) hist[b] = 0;
  __syncthreads();
  for (int32_t t = threadIdx.x; t < n_tiles; t += blockDim.x) atomicAdd(&hist[kTileBuckets - 1 - keys[t]], 1u);
  __syncthreads();
  if (threadIdx.x == 0) {  // exclusive scan of 256 counters
    uint32_t run = 0;
    for (int b = 0; b < kTileBuckets; ++b) {
      const uint32_t c = hist[b];
      hist[b] = run;
      run += c;
    }
  }
  __syncthreads();
  for (int32_t t = threadIdx.x; t < n_tiles; t += blockDim.x) order[atomicAdd(&hist[kTileBuckets - 1 - keys[t]], 1u)] = t;
}

__global__ void k_shade(const mcpt_material *mats, mcpt_ray *rays, const mcpt_hit *hits, f4 *colors,
                        uint32_t *seeds, int64_t n, int max_depth) {
  int64_t id = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= n) return;
  mcpt_ray &R = rays[id];
  const mcpt_hit &H = hits[id];
  f4 o = *(f4 *)R.origin;
  if (as_i(o.w) & (int32_t)0xFF000000) return;  // shade.cl:86-88
  if (H.t >= kFltMax) {                          // shade.cl:89-93
    colors[id] = (f4){0.0f, 0.0f, 0.0f, 0.0f};
    R.origin[3] = as_f(as_i(o.w) | (int32_t)0xFF000000);
    return;
  }
  ShadeIn in;
  in.o = o;
  in.d = *(f4 *)R.direction;
  in.nrm = *(const f4 *)H.normal;
  in.pt = *(const f4 *)H.point;
  in.mat = (int32_t)H.material_id;
  uint32_t seed = seeds[id];
  ShadeOut so = shade_hit_full(mats, in, colors[id], seed, max_depth);
  colors[id] = so.color;
  seeds[id] = seed;
  if (so.new_ray) {
    *(f4 *)R.origin = so.o;
    *(f4 *)R.direction = so.d;
    *(f4 *)R.ratio = (f4){0.0f, 0.0f, 0.0f, 0.0f};
  } else {
    R.origin[3] = so.o.w;
  }
}

__global__ void k_accumulate(f4 *colors, f4 *hist, int32_t *count, int64_t n, int max_attempt) {
  int64_t id = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= n) return;
  f4 h = hist[id];
  int32_t c = count[id];
  colors[id] = accumulate_one(colors[id], h, c, max_attempt);
  hist[id] = h;
  count[id] = c;
}

// testkernel.cl func (the GL display of ColorOut::outputColorCL,
// colorout.cpp:58-70): per pixel (pow(r, 1/2.2f), pow(g, ..), pow(b, ..), 0)
// into the display's RGBA32F texture (openglapp.cpp:84).  Headless here: the
// texture is a float4 buffer.  `1/2.2f` is the reference's constant (int 1 /
// float 2.2f, folded at compile time); pow is OpenCL's, i.e. ocml's.
__global__ void k_gamma_preview(const f4 *color, f4 *out, int64_t n) {  // out may be color (in place)
  const int64_t id = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= n) return;
  constexpr float kInvGamma = 1 / 2.2f;
  const f4 c = color[id];
  out[id] = (f4){cl_pow(c.x, kInvGamma), cl_pow(c.y, kInvGamma), cl_pow(c.z, kInvGamma), 0.0f};
}

// =================================================================== ABI
extern "C" {

int32_t mcpt_abi_version(void) { return MCPT_ABI_VERSION; }

const char *mcpt_version(void) {
  return kDebug ? "mcpt-mi355x 0.3 (gfx950, MCPT_DEBUG)"
                : (kTiming ? "mcpt-mi355x 0.3 (gfx950, MCPT_PHASE_TIMING)" : "mcpt-mi355x 0.3 (gfx950)");
}

int mcpt_device_count(int32_t *count) {
  if (!count) return mcpt::fail(MCPT_ERR_ARG, "device_count: null");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  *count = e == hipSuccess ? n : 0;
  return MCPT_OK;
}

int mcpt_ctx_create(int32_t device, mcpt_ctx **out) {
  if (!out) return mcpt::fail(MCPT_ERR_ARG, "ctx_create: null out");
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return mcpt::fail(MCPT_ERR_NOGPU, "ctx_create: no HIP device");
  if (device < 0 || device >= n) return mcpt::fail(MCPT_ERR_NOGPU, "ctx_create: device index out of range");
  HIP_OK(hipSetDevice(device));
  mcpt_ctx *c = new mcpt_ctx();
  c->device = device;
  std::memset(&c->last, 0, sizeof(c->last));
  std::memset(&c->tune, 0, sizeof(c->tune));
  if (hipDeviceGetAttribute(&c->n_cu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess ||
      hipMalloc(&c->d_stats, kStatSlots * sizeof(unsigned long long)) != hipSuccess ||
      hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess ||
      hipEventCreate(&c->ev_prim) != hipSuccess) {
    delete c;
    return mcpt::fail(MCPT_ERR_HIP, "ctx_create: allocation failed");
  }
  *out = c;
  return MCPT_OK;
}

int mcpt_ctx_destroy(mcpt_ctx *c) {
  if (!c) return MCPT_OK;
  (void)hipSetDevice(c->device);
  if (c->d_stats) (void)hipFree(c->d_stats);
  if (c->last_pending && c->ev1) (void)hipEventSynchronize(c->ev1);  // the last render may still use the buffers
  if (c->d_queue) (void)hipFree(c->d_queue);
  if (c->d_handoff) (void)hipFree(c->d_handoff);
  if (c->d_spill) (void)hipFree(c->d_spill);
  if (c->d_prim) (void)hipFree(c->d_prim);
  if (c->d_prim_cost) (void)hipFree(c->d_prim_cost);
  if (c->d_tile_order) (void)hipFree(c->d_tile_order);
  if (c->d_tile_key) (void)hipFree(c->d_tile_key);
  if (c->d_wave_log) (void)hipFree(c->d_wave_log);
  if (c->d_entry_log) (void)hipFree(c->d_entry_log);
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  if (c->ev_prim) (void)hipEventDestroy(c->ev_prim);
  delete c;
  return MCPT_OK;
}

// sincos_small vs the ocml calls, bit for bit (mcpt_selfcheck_trig).
__global__ void k_selfcheck_trig(uint32_t n, int angles, unsigned long long *bad) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float x = angles ? random_phi(i) : __builtin_bit_cast(float, i);
  float s, c;
  sincos_small(x, s, c);
  const bool ok = __builtin_bit_cast(uint32_t, s) == __builtin_bit_cast(uint32_t, cl_sin(x)) &&
                  __builtin_bit_cast(uint32_t, c) == __builtin_bit_cast(uint32_t, cl_cos(x));
  if (!ok) atomicAdd(bad, 1ull);
}

// The self-checks count mismatches in a scratch allocation of their own (not
// ctx->d_stats, which holds the last stats render's counters until
// mcpt_get_stats reads them), freed on every exit path.
struct DevScratch {
  void *p = nullptr;
  ~DevScratch() {
    if (p) (void)hipFree(p);
  }
};

int mcpt_selfcheck_trig(mcpt_ctx *c, int64_t *angle_bad, int64_t *range_bad) {
  if (!c || !angle_bad || !range_bad) return mcpt::fail(MCPT_ERR_ARG, "selfcheck_trig: null");
  HIP_OK(hipSetDevice(c->device));
  DevScratch scr;
  HIP_OK(hipMalloc(&scr.p, 2 * sizeof(unsigned long long)));
  unsigned long long *bad = (unsigned long long *)scr.p;
  HIP_OK(hipMemset(bad, 0, 2 * sizeof(unsigned long long)));
  const uint32_t n_range = 0x41000000u;  // bit patterns of [0, 8.0f)
  hipLaunchKernelGGL(k_selfcheck_trig, dim3(32768 / 256), dim3(256), 0, 0, 32768u, 1, bad);
  hipLaunchKernelGGL(k_selfcheck_trig, dim3((n_range + 255) / 256), dim3(256), 0, 0, n_range, 0, bad + 1);
  HIP_OK(hipGetLastError());
  unsigned long long h[2];
  HIP_OK(hipMemcpy(h, bad, sizeof(h), hipMemcpyDeviceToHost));
  *angle_bad = (int64_t)h[0];
  *range_bad = (int64_t)h[1];
  return MCPT_OK;
}

// cl_pow_lobe vs __ocml_pow_f32, bit for bit, over every float x of the
// restatement's domain (0, 1 + 2^-10] for each exponent (mcpt_selfcheck_pow)
__global__ void __launch_bounds__(256) k_selfcheck_pow(const float *ys, int32_t ny, unsigned long long *bad) {
  constexpr uint32_t kLast = 0x3F802000u;  // 1 + 2^-10
  unsigned long long n_bad = 0;
  for (uint32_t b = blockIdx.x * 256u + threadIdx.x + 1u; b <= kLast; b += gridDim.x * 256u) {
    const float x = __builtin_bit_cast(float, b);
    for (int k = 0; k < ny; ++k) {
      const float y = ys[k];
      n_bad += __builtin_bit_cast(uint32_t, cl_pow_lobe(x, y)) != __builtin_bit_cast(uint32_t, __ocml_pow_f32(x, y));
    }
  }
  if (n_bad) atomicAdd(bad, n_bad);
}

int mcpt_selfcheck_pow(mcpt_ctx *c, const float *ys, int32_t n, int64_t *mismatches) {
  if (!c || !ys || n <= 0 || n > 4096 || !mismatches) return mcpt::fail(MCPT_ERR_ARG, "selfcheck_pow: bad argument");
  HIP_OK(hipSetDevice(c->device));
  DevScratch scr;  // the counter, then the exponents
  HIP_OK(hipMalloc(&scr.p, 16 + (size_t)n * sizeof(float)));
  unsigned long long *bad = (unsigned long long *)scr.p;
  float *dy = (float *)((char *)scr.p + 16);
  HIP_OK(hipMemcpy(dy, ys, (size_t)n * sizeof(float), hipMemcpyHostToDevice));
  HIP_OK(hipMemset(bad, 0, sizeof(unsigned long long)));
  hipLaunchKernelGGL(k_selfcheck_pow, dim3((unsigned)(c->n_cu * 16)), dim3(256), 0, 0, dy, n, bad);
  HIP_OK(hipGetLastError());
  unsigned long long h = 0;
  HIP_OK(hipMemcpy(&h, bad, sizeof(h), hipMemcpyDeviceToHost));
  *mismatches = (int64_t)h;
  return MCPT_OK;
}

// Streaming read of n float4 (grid-stride, 16 B per lane per load), one
// partial sum per block so nothing is optimised away (mcpt_measure_read_bw).
__global__ void __launch_bounds__(256) k_stream_read(const f4 *__restrict__ src, int64_t n, float *sink) {
  f4 acc = (f4){0.0f, 0.0f, 0.0f, 0.0f};
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) acc += __builtin_nontemporal_load(&src[i]);
  const float v = acc.x + acc.y + acc.z + acc.w;
  if (v == 12345.678f) sink[blockIdx.x] = v;  // never true for the zeroed buffer
}

int mcpt_measure_read_bw(mcpt_ctx *c, int64_t bytes, double *gbps) {
  if (!c || !gbps || bytes < (1 << 20)) return mcpt::fail(MCPT_ERR_ARG, "measure_read_bw: bad argument");
  HIP_OK(hipSetDevice(c->device));
  const int64_t n = bytes / 16;
  void *buf = nullptr;
  float *sink = nullptr;
  if (hipMalloc(&buf, (size_t)n * 16) != hipSuccess) return mcpt::fail(MCPT_ERR_HIP, "measure_read_bw: hipMalloc");
  int n_cu = 0;
  (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, c->device);
  const int grid = std::max(1, n_cu) * 32;
  if (hipMalloc(&sink, grid * sizeof(float)) != hipSuccess || hipMemset(buf, 0, (size_t)n * 16) != hipSuccess) {
    (void)hipFree(buf);
    if (sink) (void)hipFree(sink);
    return mcpt::fail(MCPT_ERR_HIP, "measure_read_bw: setup");
  }
  float best = 1e30f;
  for (int rep = 0; rep < 6; ++rep) {
    (void)hipEventRecord(c->ev0, 0);
    hipLaunchKernelGGL(k_stream_read, dim3(grid), dim3(256), 0, 0, (const f4 *)buf, n, sink);
    (void)hipEventRecord(c->ev1, 0);
    (void)hipEventSynchronize(c->ev1);
    float ms = 0.0f;
    (void)hipEventElapsedTime(&ms, c->ev0, c->ev1);
    if (rep > 0) best = std::min(best, ms);  // rep 0 warms up
  }
  (void)hipFree(buf);
  (void)hipFree(sink);
  HIP_OK(hipGetLastError());
  *gbps = (double)n * 16.0 / (best * 1e-3) / 1e9;
  return MCPT_OK;
}

// Calibration of the memory-side byte counters (rocprofv3 FETCH_SIZE) for
// k_render's access shape: each lane gathers whole records of 4 or 8 float4
// (64-B triangles, 128-B nodes) with one dwordx4 load per 16 B, at scrambled
// record indices, every record of the table exactly once
// (mcpt_gather_probe).
__global__ void __launch_bounds__(256) k_gather_probe(const f4 *__restrict__ tab, uint64_t n_rec, int words,
                                                      float *sink) {
  f4 acc = (f4){0.0f, 0.0f, 0.0f, 0.0f};
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n_rec; i += stride) {
    const uint64_t r = (i * 0x9E3779B97F4A7C15ull) & (n_rec - 1);  // odd multiplier: a bijection mod 2^k
    const f4 *p = tab + r * (uint64_t)words;
    if (words == 8) {
      acc += p[0] + p[1] + p[2] + p[3] + p[4] + p[5] + p[6] + p[7];
    } else {
      acc += p[0] + p[1] + p[2] + p[3];
    }
  }
  const float v = acc.x + acc.y + acc.z + acc.w;
  if (v == 12345.678f) sink[blockIdx.x] = v;  // never true for the zeroed table
}

int mcpt_gather_probe(mcpt_ctx *c, int32_t record_bytes, int64_t table_bytes, double *ms_out) {
  if (!c || !ms_out || (record_bytes != 64 && record_bytes != 128) || table_bytes < (1 << 20) ||
      (table_bytes & (table_bytes - 1)) != 0)
    return mcpt::fail(MCPT_ERR_ARG, "gather_probe: record 64/128 B, table a power of two >= 1 MiB");
  HIP_OK(hipSetDevice(c->device));
  void *tab = nullptr, *flush = nullptr;
  float *sink = nullptr;
  const size_t flush_bytes = (size_t)1 << 30;  // evicts the table from the 256 MiB Infinity Cache after the fill
  if (hipMalloc(&tab, (size_t)table_bytes) != hipSuccess || hipMalloc(&flush, flush_bytes) != hipSuccess ||
      hipMalloc(&sink, (size_t)c->n_cu * 32 * sizeof(float)) != hipSuccess ||
      hipMemset(tab, 0, (size_t)table_bytes) != hipSuccess || hipMemset(flush, 1, flush_bytes) != hipSuccess ||
      hipDeviceSynchronize() != hipSuccess) {
    if (tab) (void)hipFree(tab);
    if (flush) (void)hipFree(flush);
    if (sink) (void)hipFree(sink);
    return mcpt::fail(MCPT_ERR_HIP, "gather_probe: setup");
  }
  const uint64_t n_rec = (uint64_t)table_bytes / (uint64_t)record_bytes;
  (void)hipEventRecord(c->ev0, 0);
  hipLaunchKernelGGL(k_gather_probe, dim3(std::max(1, c->n_cu) * 32), dim3(256), 0, 0, (const f4 *)tab, n_rec,
                     record_bytes / 16, sink);
  (void)hipEventRecord(c->ev1, 0);
  (void)hipEventSynchronize(c->ev1);
  float ms = 0.0f;
  (void)hipEventElapsedTime(&ms, c->ev0, c->ev1);
  (void)hipFree(tab);
  (void)hipFree(flush);
  (void)hipFree(sink);
  HIP_OK(hipGetLastError());
  *ms_out = ms;
  return MCPT_OK;
}

int mcpt_set_stats(mcpt_ctx *c, int32_t on) {
  if (!c) return mcpt::fail(MCPT_ERR_ARG, "set_stats: null ctx");
  c->stats_on = on != 0;
  return MCPT_OK;
}

int mcpt_set_pixel_segments(mcpt_ctx *c, uint32_t *counts_dev, uint32_t *iters_dev, int64_t n_pixels) {
  if (!c) return mcpt::fail(MCPT_ERR_ARG, "set_pixel_segments: null ctx");
  if ((counts_dev || iters_dev) && n_pixels <= 0) return mcpt::fail(MCPT_ERR_ARG, "set_pixel_segments: no capacity");
  c->px_segments = counts_dev;
  c->px_iters = iters_dev;
  c->px_cap = (counts_dev || iters_dev) ? n_pixels : 0;
  return MCPT_OK;
}

int mcpt_get_primary_cost(mcpt_ctx *c, uint32_t *out, int64_t cap, int64_t *n) {
  if (!c || !n) return mcpt::fail(MCPT_ERR_ARG, "get_primary_cost: null");
  *n = c->prim_valid ? (int64_t)c->prim_key.w * c->prim_key.h : 0;
  if (!out || *n == 0) return MCPT_OK;
  if (cap < *n) return mcpt::fail(MCPT_ERR_ARG, "get_primary_cost: buffer too small");
  HIP_OK(hipSetDevice(c->device));
  if (c->last_pending) HIP_OK(hipEventSynchronize(c->ev1));
  HIP_OK(hipMemcpy(out, c->d_prim_cost, (size_t)*n * sizeof(uint32_t), hipMemcpyDeviceToHost));
  return MCPT_OK;
}

int mcpt_get_stats(mcpt_ctx *c, mcpt_stats *out) {
  if (!c || !out) return mcpt::fail(MCPT_ERR_ARG, "get_stats: null");
  if (c->last_pending) {  // the last render call was enqueued asynchronously: wait for it, then read
    HIP_OK(hipSetDevice(c->device));
    c->last_pending = false;
    HIP_OK(hipEventSynchronize(c->ev1));
    float ms = 0.0f;
    HIP_OK(hipEventElapsedTime(&ms, c->ev0, c->ev1));
    c->last.kernel_ms = ms;
    if (c->last.primary_cache == 2) {  // the primary-hit pass's share of kernel_ms
      HIP_OK(hipEventElapsedTime(&ms, c->ev0, c->ev_prim));
      c->last.primary_ms = ms;
    }
    if (c->last_stats) {
      unsigned long long h[kStatSlots];
      HIP_OK(hipMemcpy(h, c->d_stats, sizeof(h), hipMemcpyDeviceToHost));
      c->last.segments = h[0];
      c->last.node_visits = h[1];
      c->last.tri_tests = h[2];
      c->last.bad_material = h[3];
      c->last.wave_node_phases = h[4];
      c->last.wave_leaf_phases = h[5];
      c->last.wave_shade_phases = h[6];
      c->last.order_fallbacks = h[7];
      c->last.wave_iterations = h[8];
      c->last.lane_waiting = h[9];
      c->last.lane_idle = h[10];
      c->last.leaf_rejects = h[11];
      c->last.debug_violations = h[kDebugSlot] + h[kDebugSlot + 1] + h[kDebugSlot + 2];
      for (int k = 0; k < 4; ++k) c->last.phase_ticks[k] = h[kPhaseSlot + k];
    }
  }
  *out = c->last;
  return MCPT_OK;
}

int mcpt_get_wave_log(mcpt_ctx *c, uint64_t *out, int64_t cap_workgroups, int64_t *n_workgroups) {
  if (!c || !n_workgroups) return mcpt::fail(MCPT_ERR_ARG, "get_wave_log: null");
  *n_workgroups = c->wave_log_n;
  if (!out || c->wave_log_n == 0) return MCPT_OK;
  if (cap_workgroups < c->wave_log_n) return mcpt::fail(MCPT_ERR_ARG, "get_wave_log: buffer too small");
  HIP_OK(hipSetDevice(c->device));
  if (c->last_pending) HIP_OK(hipEventSynchronize(c->ev1));
  HIP_OK(hipMemcpy(out, c->d_wave_log, (size_t)c->wave_log_n * kWaveLogWords * sizeof(uint64_t), hipMemcpyDeviceToHost));
  return MCPT_OK;
}

int mcpt_get_entry_log(mcpt_ctx *c, uint32_t *out, int64_t cap_entries, int64_t *n_entries, int32_t *blocks) {
  if (!c || !n_entries) return mcpt::fail(MCPT_ERR_ARG, "get_entry_log: null");
  *n_entries = c->entry_log_n;
  if (blocks) *blocks = c->entry_log_blocks;
  if (!out || c->entry_log_n == 0) return MCPT_OK;
  if (cap_entries < c->entry_log_n) return mcpt::fail(MCPT_ERR_ARG, "get_entry_log: buffer too small");
  HIP_OK(hipSetDevice(c->device));
  if (c->last_pending) HIP_OK(hipEventSynchronize(c->ev1));
  HIP_OK(hipMemcpy(out, c->d_entry_log, (size_t)c->entry_log_n * 3 * sizeof(uint32_t), hipMemcpyDeviceToHost));
  return MCPT_OK;
}

int mcpt_set_tuning(mcpt_ctx *c, const mcpt_tuning *t) {
  if (!c) return mcpt::fail(MCPT_ERR_ARG, "set_tuning: null ctx");
  if (t && (t->stack_window < 0 || t->stack_window > 2 || t->quantized < 0 || t->quantized > 2 ||
            t->primary_cache < 0 || t->primary_cache > 2 || t->lds_pad < 0 || t->lds_pad > 65536 ||
            t->queue_chunk > 4096 || t->leaf_threshold > 64 || t->shade_threshold > 64 || t->fetch_threshold > 64 ||
            t->last_block_frames < -1 || t->tile_order < 0 || t->tile_order > 2 || t->pixel_spread < 0 ||
            t->pixel_spread > 2 || t->top_levels < -1 || t->top_levels > kMaxTopLevels))
    return mcpt::fail(MCPT_ERR_ARG, "set_tuning: value out of range");
  if (t)
    c->tune = *t;
  else
    std::memset(&c->tune, 0, sizeof(c->tune));
  return MCPT_OK;
}

int mcpt_drop_caches(mcpt_ctx *c) {
  if (!c) return mcpt::fail(MCPT_ERR_ARG, "drop_caches: null ctx");
  c->prim_valid = false;
  c->seen_valid = false;
  return MCPT_OK;
}

int mcpt_get_tuning(mcpt_ctx *c, mcpt_tuning *out) {
  if (!c || !out) return mcpt::fail(MCPT_ERR_ARG, "get_tuning: null");
  *out = c->tune;
  return MCPT_OK;
}

int mcpt_state_create(mcpt_ctx *c, int32_t w, int32_t h, const uint32_t *seeds, mcpt_state **out) {
  if (!c || !seeds || !out || w <= 0 || h <= 0 || (int64_t)w * h > (int64_t)INT32_MAX)
    return mcpt::fail(MCPT_ERR_ARG, "state_create: bad argument");
  HIP_OK(hipSetDevice(c->device));
  const size_t n = (size_t)w * h;
  mcpt_state *s = new mcpt_state();
  s->device = c->device;
  s->width = w;
  s->height = h;
  if (hipMalloc(&s->seeds, n * 4) != hipSuccess || hipMalloc(&s->hist, n * 16) != hipSuccess ||
      hipMalloc(&s->count, n * 4) != hipSuccess || hipMemcpy(s->seeds, seeds, n * 4, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemset(s->hist, 0, n * 16) != hipSuccess || hipMemset(s->count, 0, n * 4) != hipSuccess) {
    mcpt_state_destroy(s);
    return mcpt::fail(MCPT_ERR_HIP, "state_create: allocation or copy failed");
  }
  *out = s;
  return MCPT_OK;
}

int mcpt_state_buffers(mcpt_state *s, uint32_t **seeds, float **hist, int32_t **count) {
  if (!s) return mcpt::fail(MCPT_ERR_ARG, "state_buffers: null state");
  if (seeds) *seeds = s->seeds;
  if (hist) *hist = s->hist;
  if (count) *count = s->count;
  return MCPT_OK;
}

int mcpt_download(mcpt_ctx *c, const mcpt_state *s, float *hist, int32_t *count, uint32_t *seeds, void *stream) {
  if (!c || !s || s->device != c->device) return mcpt::fail(MCPT_ERR_ARG, "download: bad argument");
  HIP_OK(hipSetDevice(c->device));
  hipStream_t st = (hipStream_t)stream;
  const size_t n = (size_t)s->width * s->height;
  if (hist) HIP_OK(hipMemcpyAsync(hist, s->hist, n * 16, hipMemcpyDeviceToHost, st));
  if (count) HIP_OK(hipMemcpyAsync(count, s->count, n * 4, hipMemcpyDeviceToHost, st));
  if (seeds) HIP_OK(hipMemcpyAsync(seeds, s->seeds, n * 4, hipMemcpyDeviceToHost, st));
  HIP_OK(hipStreamSynchronize(st));
  return MCPT_OK;
}

int mcpt_upload(mcpt_ctx *c, mcpt_state *s, const float *hist, const int32_t *count, const uint32_t *seeds,
                void *stream) {
  if (!c || !s || s->device != c->device) return mcpt::fail(MCPT_ERR_ARG, "upload: bad argument");
  HIP_OK(hipSetDevice(c->device));
  hipStream_t st = (hipStream_t)stream;
  const size_t n = (size_t)s->width * s->height;
  if (hist) HIP_OK(hipMemcpyAsync(s->hist, hist, n * 16, hipMemcpyHostToDevice, st));
  if (count) HIP_OK(hipMemcpyAsync(s->count, count, n * 4, hipMemcpyHostToDevice, st));
  if (seeds) HIP_OK(hipMemcpyAsync(s->seeds, seeds, n * 4, hipMemcpyHostToDevice, st));
  HIP_OK(hipStreamSynchronize(st));  // the host arrays may be reused on return
  return MCPT_OK;
}

int mcpt_state_destroy(mcpt_state *s) {
  if (!s) return MCPT_OK;
  (void)hipSetDevice(s->device);
  (void)hipDeviceSynchronize();  // work enqueued on the state may still be running
  if (s->seeds) (void)hipFree(s->seeds);
  if (s->hist) (void)hipFree(s->hist);
  if (s->count) (void)hipFree(s->count);
  delete s;
  return MCPT_OK;
}

int mcpt_scene_upload(mcpt_ctx *ctx, const mcpt_triangle *tris, int64_t n_tris, const mcpt_bvh_node *nodes,
                      int64_t n_nodes, const mcpt_material *mats, int32_t n_mats, mcpt_scene **out) {
  if (!ctx || !tris || !nodes || !mats || !out || n_tris <= 0 || n_mats <= 0)
    return mcpt::fail(MCPT_ERR_ARG, "scene_upload: bad argument");
  if (n_nodes != 2 * n_tris - 1) return mcpt::fail(MCPT_ERR_ARG, "scene_upload: expected 2n-1 BVH nodes");
  int32_t depth = 0;
  int rc = mcpt_bvh_stack_depth(nodes, n_nodes, &depth);
  if (rc) return rc;
  if (depth > 64) return mcpt::fail(MCPT_ERR_LIMIT, "scene_upload: BVH deeper than the reference's 64-entry stack");
  const int64_t n = n_tris;
  // validate links and material ids before anything reaches the GPU
  for (int64_t i = 0; i < n_nodes; ++i) {
    const mcpt_bvh_node &b = nodes[i];
    if (b.left < 0 || b.right < 0) return mcpt::fail(MCPT_ERR_ARG, "scene_upload: negative child index");
    if (b.left == b.right) {
      if (b.left >= n) return mcpt::fail(MCPT_ERR_ARG, "scene_upload: leaf triangle index out of range");
    } else if (b.left >= n_nodes || b.right >= n_nodes) {
      return mcpt::fail(MCPT_ERR_ARG, "scene_upload: child index out of range");
    }
  }
  for (int64_t i = 0; i < n; ++i) {
    int32_t m;
    std::memcpy(&m, &tris[i].normal[3], 4);
    if (m < 0 || m >= n_mats) return mcpt::fail(MCPT_ERR_ARG, "scene_upload: triangle material id out of range");
    for (int k = 0; k < 3; ++k)
      for (int j = 0; j < 3; ++j)
        if (!std::isfinite(tris[i].v[k][j]))
          return mcpt::fail(MCPT_ERR_ARG, "scene_upload: non-finite vertex coordinate");
  }
  // reference node index -> device index: internal nodes keep their index in
  // a compacted array (the HLBVH puts them at [0, n-2]); leaves become ~tri.
  std::vector<int32_t> remap(n_nodes, -1);
  int64_t n_int = 0;
  for (int64_t i = 0; i < n_nodes; ++i)
    if (nodes[i].left != nodes[i].right) remap[i] = (int32_t)n_int++;
  auto child = [&](int32_t c) -> int32_t { return nodes[c].left == nodes[c].right ? ~nodes[c].left : remap[c]; };
  std::vector<DevNode> dn(std::max<int64_t>(n_int, 1));
  std::memset(dn.data(), 0, dn.size() * sizeof(DevNode));
  for (int64_t i = 0; i < n_nodes; ++i) {
    if (remap[i] < 0) continue;
    const mcpt_bvh_node &b = nodes[i], &L = nodes[b.left], &R = nodes[b.right];
    DevNode &d = dn[remap[i]];
    d.a = (f4){L.bbmin[0], L.bbmax[0], L.bbmin[1], L.bbmax[1]};
    d.b = (f4){L.bbmin[2], L.bbmax[2], R.bbmin[0], R.bbmax[0]};
    d.c = (f4){R.bbmin[1], R.bbmax[1], R.bbmin[2], R.bbmax[2]};
    d.left = child(b.left);
    d.right = child(b.right);
  }
  if (n_int > 0 && remap[0] != 0) return mcpt::fail(MCPT_ERR_ARG, "scene_upload: root must be node 0");
  // 4-wide collapse (DevNode4): breadth-first over the binary internal nodes
  // that start a 4-wide node (the root and every internal grandchild).
  std::vector<DevNode4> dn4;
  int32_t depth4 = 1;
  if (n_int > 0) {
    std::vector<int32_t> order(1, 0);  // binary ids of 4-wide nodes, index = DevNode4 id
    std::vector<int32_t> need;         // stack entries needed below each 4-wide node
    for (size_t k = 0; k < order.size(); ++k) {
      const mcpt_bvh_node &b = nodes[order[k]];
      DevNode4 q;
      std::memset(&q, 0, sizeof(q));
      int slot = 0;
      auto put = [&](int32_t c) {
        const mcpt_bvh_node &x = nodes[c];
        float v[6] = {x.bbmin[0], x.bbmax[0], x.bbmin[1], x.bbmax[1], x.bbmin[2], x.bbmax[2]};
        float *qf = reinterpret_cast<float *>(q.q);
        std::memcpy(qf + 6 * slot, v, sizeof(v));
        if (x.left == x.right) {
          q.link[slot] = ~x.left;
        } else {
          q.link[slot] = (int32_t)order.size();
          order.push_back(c);
        }
        ++slot;
      };
      for (int32_t c : {b.left, b.right}) {
        const mcpt_bvh_node &x = nodes[c];
        if (x.left == x.right) {
          put(c);
        } else {
          put(x.left);
          put(x.right);
        }
      }
      for (; slot < 4; ++slot) q.link[slot] = kEmptySlot;
      dn4.push_back(q);
    }
    // stack need: visiting slot i of a k-slot node leaves k-1-i entries pending
    need.assign(dn4.size(), 0);
    for (int64_t k = (int64_t)dn4.size() - 1; k >= 0; --k) {  // children have larger ids
      int ns = 0;
      while (ns < 4 && dn4[k].link[ns] != kEmptySlot) ++ns;
      int best = ns - 1;
      for (int i = 0; i < ns; ++i)
        if (dn4[k].link[i] >= 0) best = std::max(best, ns - 1 - i + need[dn4[k].link[i]]);
      need[k] = best;
    }
    depth4 = std::max(need[0], 1);
  } else {
    dn4.resize(1);
    std::memset(dn4.data(), 0, sizeof(DevNode4));
  }
  // the EXACT search tree over the reference's own leaves (their boxes as stored)
  std::vector<mcpt::LeafRef> leaves;
  leaves.reserve((size_t)n);
  for (int64_t i = 0; i < n_nodes; ++i) {
    const mcpt_bvh_node &b = nodes[i];
    if (b.left != b.right) continue;
    mcpt::LeafRef L;
    const float bx[6] = {b.bbmin[0], b.bbmax[0], b.bbmin[1], b.bbmax[1], b.bbmin[2], b.bbmax[2]};
    std::memcpy(L.box, bx, sizeof(bx));
    L.tri = b.left;
    leaves.push_back(L);
  }
  std::vector<mcpt::Node4Rec> near;
  int32_t depth_near = 1;
  if (n_int > 0) {
    const unsigned hw = std::thread::hardware_concurrency();
    if (mcpt::build_sah4(leaves, near, &depth_near, (int)std::min(16u, std::max(1u, hw))) != 0)
      return mcpt::fail(MCPT_ERR_ARG, "scene_upload: no leaves");
  } else {
    near.resize(1);
    std::memset(near.data(), 0, sizeof(mcpt::Node4Rec));
  }
  depth4 = std::max(depth4, depth_near);
  if (depth4 > 192) return mcpt::fail(MCPT_ERR_LIMIT, "scene_upload: 4-wide stack too deep");
  std::vector<DevTri> dt(n);
  for (int64_t i = 0; i < n; ++i) {
    const mcpt_triangle &t = tris[i];
    DevTri &d = dt[i];
    // objdef.h:190-199: AB = (v1 - v0).s012, AC = (v2 - v0).s012, matrix rows -AB, -AC
    const float b1 = -(t.v[1][0] - t.v[0][0]), b2 = -(t.v[1][1] - t.v[0][1]), b3 = -(t.v[1][2] - t.v[0][2]);
    const float c1 = -(t.v[2][0] - t.v[0][0]), c2 = -(t.v[2][1] - t.v[0][1]), c3 = -(t.v[2][2] - t.v[0][2]);
    // triangle-only minors of cramer_reduced (std::fma = the device's fused v_fma_f32)
    d.v0 = (f4){t.v[0][0], t.v[0][1], t.v[0][2], t.normal[0]};
    d.nab = (f4){b1, b2, b3, t.normal[1]};
    d.nac = (f4){c1, c2, c3, t.normal[2]};
    d.aux = (f4){t.normal[3], std::fma(b2, c3, -(c2 * b3)), std::fma(b1, c3, -(c1 * b3)), std::fma(b1, c2, -(c1 * b2))};
  }
  // The quantized search tree: 64-B nodes whose decoded
  // boxes strictly contain the exact ones, so every box test is a superset of
  // the exact one, and the L phase re-tests the reference leaf's own box,
  // rebuilt from the triangle's vertices -- valid when every reference leaf's
  // box IS min/max of its vertices (hlbvh.cpp:97-100; a foreign tree may differ,
  // and then keeps the 128-B path).
  std::vector<DevNode4Q> nq;
  std::vector<DevTriQ> tq;
  bool quant = n_int > 0;
  for (int64_t i = 0; quant && i < n_nodes; ++i) {
    const mcpt_bvh_node &b = nodes[i];
    if (b.left != b.right) continue;
    const mcpt_triangle &t = tris[b.left];
    for (int a = 0; a < 3; ++a) {
      const float lo = std::min(std::min(t.v[0][a], t.v[1][a]), t.v[2][a]);
      const float hi = std::max(std::max(t.v[0][a], t.v[1][a]), t.v[2][a]);
      if (!(b.bbmin[a] == lo && b.bbmax[a] == hi)) quant = false;
    }
  }
  if (quant) {
    nq.resize(near.size());
    for (size_t k = 0; quant && k < near.size(); ++k)
      quant = mcpt::quantize_node4(near[k], *reinterpret_cast<mcpt::Node4Q *>(&nq[k])) == 0;
  }
  if (quant) {
    tq.resize(n);
    for (int64_t i = 0; i < n; ++i) {
      const mcpt_triangle &t = tris[i];
      tq[i].v0 = (f4){t.v[0][0], t.v[0][1], t.v[0][2], dt[i].aux.y};
      tq[i].v1 = (f4){t.v[1][0], t.v[1][1], t.v[1][2], dt[i].aux.z};
      tq[i].v2 = (f4){t.v[2][0], t.v[2][1], t.v[2][2], dt[i].aux.w};
      tq[i].nrm = (f4){t.normal[0], t.normal[1], t.normal[2], t.normal[3]};
    }
  } else {
    nq.clear();
  }
  // pruning margin: 2^-10 of the scene diagonal
  const mcpt_bvh_node &root = nodes[0];
  float dx = root.bbmax[0] - root.bbmin[0], dy = root.bbmax[1] - root.bbmin[1], dz = root.bbmax[2] - root.bbmin[2];
  float diag = std::sqrt(dx * dx + dy * dy + dz * dz);

  HIP_OK(hipSetDevice(ctx->device));
  static std::atomic<uint64_t> scene_uids{0};
  mcpt_scene *s = new mcpt_scene();
  s->uid = ++scene_uids;
  s->device = ctx->device;
  if (hipMalloc(&s->near4, near.size() * sizeof(DevNode4)) != hipSuccess ||
      hipMalloc(&s->nodes4, dn4.size() * sizeof(DevNode4)) != hipSuccess ||
      hipMalloc(&s->nodes, dn.size() * sizeof(DevNode)) != hipSuccess ||
      hipMalloc(&s->tris, dt.size() * sizeof(DevTri)) != hipSuccess ||
      hipMalloc(&s->mats, n_mats * sizeof(mcpt_material)) != hipSuccess) {
    mcpt_scene_destroy(s);
    return mcpt::fail(MCPT_ERR_HIP, "scene_upload: hipMalloc failed");
  }
  if (hipMemcpy(s->near4, near.data(), near.size() * sizeof(DevNode4), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(s->nodes4, dn4.data(), dn4.size() * sizeof(DevNode4), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(s->nodes, dn.data(), dn.size() * sizeof(DevNode), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(s->tris, dt.data(), dt.size() * sizeof(DevTri), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(s->mats, mats, n_mats * sizeof(mcpt_material), hipMemcpyHostToDevice) != hipSuccess) {
    mcpt_scene_destroy(s);
    return mcpt::fail(MCPT_ERR_HIP, "scene_upload: hipMemcpy failed");
  }
  if (quant && (hipMalloc(&s->near4q, nq.size() * sizeof(DevNode4Q)) != hipSuccess ||
                hipMalloc(&s->triq, tq.size() * sizeof(DevTriQ)) != hipSuccess ||
                hipMemcpy(s->near4q, nq.data(), nq.size() * sizeof(DevNode4Q), hipMemcpyHostToDevice) != hipSuccess ||
                hipMemcpy(s->triq, tq.data(), tq.size() * sizeof(DevTriQ), hipMemcpyHostToDevice) != hipSuccess)) {
    mcpt_scene_destroy(s);
    return mcpt::fail(MCPT_ERR_HIP, "scene_upload: quantized tree upload failed");
  }
  s->n_tris = n;
  s->near4_bytes = (int64_t)(near.size() * sizeof(DevNode4));
  s->n_internal = n_int;
  s->n_mats = n_mats;
  s->has_glossy = false;
  for (int32_t k = 0; k < n_mats; ++k) s->has_glossy |= mats[k].type == MCPT_GLOSSY;
  s->stack_depth = std::max(depth, 1);
  s->stack_depth4 = depth4;
  SceneView &v = s->view;
  v.n_near4 = (int32_t)near.size();
  v.n_nodes4 = (int32_t)dn4.size();
  v.n_int = (int32_t)dn.size();
  v.n_tris = n;
  v.nodes = s->nodes;
  v.nodes4 = s->nodes4;
  v.near4 = s->near4;
  v.tris = s->tris;
  v.near4q = s->near4q;
  v.triq = s->triq;
  v.mats = s->mats;
  v.root_min = (f4){root.bbmin[0], root.bbmin[1], root.bbmin[2], root.bbmin[3]};
  v.root_max = (f4){root.bbmax[0], root.bbmax[1], root.bbmax[2], root.bbmax[3]};
  v.root_leaf = root.left == root.right ? root.left : -1;
  v.n_mats = n_mats;
  v.prune_margin = std::isfinite(diag) ? std::ldexp(diag, -10) : __builtin_inff();
  *out = s;
  return MCPT_OK;
}

// SceneBuild::buildScene with the scene already in HBM: every device
// structure of mcpt_scene_upload, built on the GPU (mcpt_upload.hip), the
// same bytes.
int mcpt_scene_upload_device(mcpt_ctx *ctx, const mcpt_triangle *tris_dev, int64_t n_tris,
                             const mcpt_bvh_node *nodes_dev, int64_t n_nodes, const mcpt_material *mats,
                             int32_t n_mats, void *stream, mcpt_scene **out) {
  if (!ctx || !tris_dev || !nodes_dev || !mats || !out || n_tris <= 0 || n_mats <= 0)
    return mcpt::fail(MCPT_ERR_ARG, "scene_upload_device: bad argument");
  if (n_nodes != 2 * n_tris - 1) return mcpt::fail(MCPT_ERR_ARG, "scene_upload_device: expected 2n-1 BVH nodes");
  HIP_OK(hipSetDevice(ctx->device));
  mcpt::DeviceScene D;
  int rc = mcpt::build_scene_device(tris_dev, n_tris, nodes_dev, n_mats, (hipStream_t)stream, &D);
  auto free_d = [&]() {
    for (void *p : {D.near4, D.near4q, D.nodes4, D.nodes, D.tris, D.triq})
      if (p) (void)hipFree(p);
  };
  if (rc != MCPT_OK) {
    free_d();
    return rc;
  }
  static std::atomic<uint64_t> scene_uids_d{1ull << 62};  // distinct from mcpt_scene_upload's
  mcpt_scene *s = new mcpt_scene();
  s->uid = ++scene_uids_d;
  s->device = ctx->device;
  s->near4 = (DevNode4 *)D.near4;
  s->near4q = (DevNode4Q *)D.near4q;
  s->nodes4 = (DevNode4 *)D.nodes4;
  s->nodes = (DevNode *)D.nodes;
  s->tris = (DevTri *)D.tris;
  s->triq = (DevTriQ *)D.triq;
  if (hipMalloc(&s->mats, n_mats * sizeof(mcpt_material)) != hipSuccess ||
      hipMemcpy(s->mats, mats, n_mats * sizeof(mcpt_material), hipMemcpyHostToDevice) != hipSuccess) {
    mcpt_scene_destroy(s);
    return mcpt::fail(MCPT_ERR_HIP, "scene_upload_device: material upload failed");
  }
  const mcpt_bvh_node &root = D.root;
  s->n_tris = n_tris;
  s->near4_bytes = D.n_near4 * (int64_t)sizeof(DevNode4);
  s->n_internal = D.n_int;
  s->n_mats = n_mats;
  s->has_glossy = false;
  for (int32_t k = 0; k < n_mats; ++k) s->has_glossy |= mats[k].type == MCPT_GLOSSY;
  s->stack_depth = std::max(D.stack_depth, 1);
  s->stack_depth4 = D.depth4;
  float dx = root.bbmax[0] - root.bbmin[0], dy = root.bbmax[1] - root.bbmin[1], dz = root.bbmax[2] - root.bbmin[2];
  float diag = std::sqrt(dx * dx + dy * dy + dz * dz);
  SceneView &v = s->view;
  v.n_near4 = (int32_t)D.n_near4;
  v.n_nodes4 = (int32_t)D.n_nodes4;
  v.n_int = (int32_t)std::max<int64_t>(D.n_int, 1);
  v.n_tris = n_tris;
  v.nodes = s->nodes;
  v.nodes4 = s->nodes4;
  v.near4 = s->near4;
  v.tris = s->tris;
  v.near4q = s->near4q;
  v.triq = s->triq;
  v.mats = s->mats;
  v.root_min = (f4){root.bbmin[0], root.bbmin[1], root.bbmin[2], root.bbmin[3]};
  v.root_max = (f4){root.bbmax[0], root.bbmax[1], root.bbmax[2], root.bbmax[3]};
  v.root_leaf = root.left == root.right ? root.left : -1;
  v.n_mats = n_mats;
  v.prune_margin = std::isfinite(diag) ? std::ldexp(diag, -10) : __builtin_inff();
  *out = s;
  return MCPT_OK;
}

// A scene's device arrays, copied to the host (introspection: tests compare
// the two upload paths byte for byte).  which: 0 near4, 1 near4q, 2 nodes4,
// 3 nodes, 4 tris, 5 triq, 6 int32[4] {stack_depth, stack_depth4, quantized,
// n_internal}.  *bytes = the array's size; host may be NULL to ask for it.
int mcpt_scene_read(const mcpt_scene *s, int32_t which, void *host, int64_t cap, int64_t *bytes) {
  if (!s || !bytes) return mcpt::fail(MCPT_ERR_ARG, "scene_read: bad argument");
  const void *src = nullptr;
  int64_t n = 0;
  int32_t meta[4] = {s->stack_depth, s->stack_depth4, s->near4q ? 1 : 0, (int32_t)s->n_internal};
  switch (which) {
    case 0: src = s->near4, n = (int64_t)s->view.n_near4 * (int64_t)sizeof(DevNode4); break;
    case 1: src = s->near4q, n = s->near4q ? (int64_t)s->view.n_near4 * (int64_t)sizeof(DevNode4Q) : 0; break;
    case 2: src = s->nodes4, n = (int64_t)s->view.n_nodes4 * (int64_t)sizeof(DevNode4); break;
    case 3: src = s->nodes, n = (int64_t)s->view.n_int * (int64_t)sizeof(DevNode); break;
    case 4: src = s->tris, n = s->n_tris * (int64_t)sizeof(DevTri); break;
    case 5: src = s->triq, n = s->triq ? s->n_tris * (int64_t)sizeof(DevTriQ) : 0; break;
    case 6: n = sizeof(meta); break;
    default: return mcpt::fail(MCPT_ERR_ARG, "scene_read: unknown array");
  }
  *bytes = n;
  if (!host) return MCPT_OK;
  if (cap < n) return mcpt::fail(MCPT_ERR_ARG, "scene_read: buffer too small");
  if (which == 6) {
    std::memcpy(host, meta, sizeof(meta));
    return MCPT_OK;
  }
  HIP_OK(hipSetDevice(s->device));
  if (n) HIP_OK(hipMemcpy(host, src, (size_t)n, hipMemcpyDeviceToHost));
  return MCPT_OK;
}

int mcpt_scene_destroy(mcpt_scene *s) {
  if (!s) return MCPT_OK;
  (void)hipSetDevice(s->device);
  if (s->nodes) (void)hipFree(s->nodes);
  if (s->nodes4) (void)hipFree(s->nodes4);
  if (s->near4) (void)hipFree(s->near4);
  if (s->tris) (void)hipFree(s->tris);
  if (s->near4q) (void)hipFree(s->near4q);
  if (s->triq) (void)hipFree(s->triq);
  if (s->mats) (void)hipFree(s->mats);
  delete s;
  return MCPT_OK;
}

// Resident workgroups (kWgWaves waves each) per CU of a k_render
// instantiation at an LDS size, asked once per (kernel, size) and kept in the
// context.
static int occupancy(mcpt_ctx *ctx, const void *fn, size_t lds, int *out) {
  for (const auto &e : ctx->occ)
    if (e.fn == fn && e.lds == lds) {
      *out = e.per_cu;
      return MCPT_OK;
    }
  int n = 0;
  HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, 64 * kWgWaves, lds));
  ctx->occ.push_back({fn, lds, n});
  *out = n;
  return MCPT_OK;
}

static int check_render(const mcpt_render_params *p) {
  if (p->width <= 0 || p->height <= 0 || p->max_depth <= 0 || p->max_depth > 0xFFFF || p->frames < 0 ||
      p->frame_begin < 0 || p->stripe_count <= 0 || p->stripe_rows <= 0 || p->stripe_index < 0 ||
      p->stripe_index >= p->stripe_count || p->width > 65535 || p->height > 65535 ||
      (int64_t)p->width * p->height > (int64_t)INT32_MAX)
    return mcpt::fail(MCPT_ERR_ARG, "render: bad parameters");
  if (p->mode != MCPT_MODE_EXACT && p->mode != MCPT_MODE_NOPRUNE) return mcpt::fail(MCPT_ERR_ARG, "render: bad mode");
  if (p->schedule != MCPT_SCHED_SINGLE && p->schedule != MCPT_SCHED_PAIRED)
    return mcpt::fail(MCPT_ERR_ARG, "render: bad schedule");
  return MCPT_OK;
}

int mcpt_render_frames(mcpt_ctx *ctx, const mcpt_scene *scene, const mcpt_camera *cam, const mcpt_render_params *p,
                       uint32_t *seeds, float *hist, int32_t *count, void *stream) {
  if (!ctx || !scene || !cam || !p || !seeds || !hist || !count) return mcpt::fail(MCPT_ERR_ARG, "render: null argument");
  int rc = check_render(p);
  if (rc) return rc;
  HIP_OK(hipSetDevice(ctx->device));
  hipStream_t st = (hipStream_t)stream;
  RenderArgs A;
  A.cam = *cam;
  A.S = scene->view;
  A.seeds = seeds;
  A.hist = (f4 *)hist;
  A.count = count;
  A.stats = ctx->d_stats;
  A.W = p->width;
  A.H = p->height;
  A.stripe_rows = p->stripe_rows;
  A.stripe_index = p->stripe_index;
  A.stripe_count = p->stripe_count;
  // rows owned by this stripe residue
  int32_t full = p->height / (p->stripe_rows * p->stripe_count);
  int32_t rem = p->height - full * p->stripe_rows * p->stripe_count;
  int32_t extra = std::min(std::max(rem - p->stripe_index * p->stripe_rows, 0), p->stripe_rows);
  A.local_rows = full * p->stripe_rows + extra;
  A.tiles_x = (p->width + 7) / 8;
  A.max_depth = p->max_depth;
  A.max_attempt = p->max_attempt;
  A.stack_depth = scene->stack_depth;
  // tuned (tools/sweep.py, tools/ab.py): leaf phase at >= 4 lanes
  // (single-leaf schedule) or >= 16 (paired), shade at >= 32
  const mcpt_tuning &T = ctx->tune;
  const bool pair = p->schedule == MCPT_SCHED_PAIRED;
  A.th_leaf = T.leaf_threshold > 0 ? T.leaf_threshold : (pair ? 16 : 4);
  A.th_shade = T.shade_threshold > 0 ? T.shade_threshold : 32;
  A.chunk = T.queue_chunk > 0 ? T.queue_chunk : 4;  // queue entries per atomic (at least)
  A.th_fetch = T.fetch_threshold > 0 ? T.fetch_threshold : 1;
  A.n_queues = T.queues > 0 ? (uint32_t)std::min(T.queues, kQueues) : (uint32_t)kQueues;
  const int64_t tiles = (int64_t)A.tiles_x * ((A.local_rows + 7) / 8);
  const int depth_entries = p->mode == MCPT_MODE_NOPRUNE ? scene->stack_depth : scene->stack_depth4;
  A.lds_mats = scene->n_mats <= 256 ? 1 : 0;
  const size_t lds_mats = A.lds_mats ? scene->n_mats * sizeof(mcpt_material) : 0;
  // persistent grid: as many kWgWaves-wave workgroups as can be resident at once.
  // The stack lives in LDS; when the whole stack would allow fewer resident
  // workgroups than a kStackWindow window does, the windowed kernel runs.
  const bool noprune = p->mode == MCPT_MODE_NOPRUNE;
  // [kind: 0 EXACT 128-B nodes, 1 NOPRUNE, 2 EXACT quantized][stats][window][pair][glossy materials]
#define MCPT_KG(M, ST, W, P, QN) {(const void *)k_render<M, ST, W, P, QN, false, false>, \
                                  (const void *)k_render<M, ST, W, P, QN, false, true>}
#define MCPT_KR(M, ST, W, QN) {MCPT_KG(M, ST, W, false, QN), MCPT_KG(M, ST, W, true, QN)}
#define MCPT_KK(M, QN) {{MCPT_KR(M, false, false, QN), MCPT_KR(M, false, true, QN)}, \
                        {MCPT_KR(M, true, false, QN), MCPT_KR(M, true, true, QN)}}
  static const void *const kfns[3][2][2][2][2] = {MCPT_KK(MCPT_MODE_EXACT, false), MCPT_KK(MCPT_MODE_NOPRUNE, false),
                                                  MCPT_KK(MCPT_MODE_EXACT, true)};
  // the primary-hit pass: [kind][window][pair], no stats
#define MCPT_KP(M, W, QN) {(const void *)k_render<M, false, W, false, QN, true, false>, \
                           (const void *)k_render<M, false, W, true, QN, true, false>}
  static const void *const kpfns[3][2][2] = {{MCPT_KP(MCPT_MODE_EXACT, false, false), MCPT_KP(MCPT_MODE_EXACT, true, false)},
                                             {MCPT_KP(MCPT_MODE_NOPRUNE, false, false), MCPT_KP(MCPT_MODE_NOPRUNE, true, false)},
                                             {MCPT_KP(MCPT_MODE_EXACT, false, true), MCPT_KP(MCPT_MODE_EXACT, true, true)}};
#undef MCPT_KP
#undef MCPT_KK
#undef MCPT_KR
#undef MCPT_KG
  // quantized search tree: forced on (1) or off (2), or auto (0): on when the
  // 128-B tree outgrows the GPU's aggregate L2, where its halved node bytes and
  // gathers pay (C5 -6 %); on cache-resident trees its looser boxes cost more
  // node steps and leaf tests than the saved gathers (C2 +6 %, C3 +11 %;
  // profiles/r02_quant_ab.txt)
  const bool quant = scene->near4q && (T.quantized == 1 || (T.quantized == 0 && scene->near4_bytes > kQuantAutoBytes));
  const int kind = noprune ? 1 : (quant ? 2 : 0);
  const int glossy = scene->has_glossy ? 1 : 0;  // the shading instantiation (speed only: same bits)
  const size_t pad = (size_t)std::max(0, T.lds_pad);
  // the search tree's top levels in LDS, stepped where a segment begins
  // (EXACT; k_render): auto 2, kMaxTopLevels (4) on trees over 4 MiB
  // (against none, C2 -2.7 %, C3 -5.8 %, C4 -7.6 % with 2 and
  // -12.4 % with 3, where C2 and C3 lose 3-5 % with 3; 4-wave workgroups: C4 a
  // further -4.2 % with 4 against 3, C5 -0.6 %)
  A.top_levels = noprune || scene->view.root_leaf >= 0 ? 0
               : (T.top_levels < 0 ? 0 : (T.top_levels > 0 ? std::min(T.top_levels, kMaxTopLevels)
                                                              : (scene->near4_bytes > (4ll << 20) ? kMaxTopLevels : 2)));
  const size_t lds_top = (size_t)top_nodes(A.top_levels) * 7 * sizeof(f4);
  // a stack per wave; one copy of the uniforms, top levels and materials per workgroup
  const size_t lds_plain = (((size_t)kWgWaves * depth_entries * 64 * sizeof(int32_t) + sizeof(LdsUniforms) + lds_top +
                             lds_mats + 15) & ~(size_t)15) + pad;
  const size_t lds_win = (((size_t)kWgWaves * kStackWindow * 64 * sizeof(int32_t) + sizeof(LdsUniforms) + lds_top +
                           lds_mats + 15) & ~(size_t)15) + pad;
  bool win = false;
  int per_cu = 0;
  if (T.stack_window == 1) {  // forced (tests, experiments): the window even when the whole stack fits in it
    win = true;
    rc = occupancy(ctx, kfns[kind][ctx->stats_on][1][pair][glossy], lds_win, &per_cu);
    if (rc) return rc;
  } else if (depth_entries > kStackWindow && T.stack_window != 2) {
    int per_cu_plain = 0, per_cu_win = 0;
    rc = occupancy(ctx, kfns[kind][ctx->stats_on][0][pair][glossy], lds_plain, &per_cu_plain);
    if (rc) return rc;
    rc = occupancy(ctx, kfns[kind][ctx->stats_on][1][pair][glossy], lds_win, &per_cu_win);
    if (rc) return rc;
    win = per_cu_win > per_cu_plain;
    per_cu = win ? per_cu_win : per_cu_plain;
  } else {
    rc = occupancy(ctx, kfns[kind][ctx->stats_on][0][pair][glossy], lds_plain, &per_cu);
    if (rc) return rc;
  }
  const size_t lds = win ? lds_win : lds_plain;
  const void *kfn = kfns[kind][ctx->stats_on][win][pair][glossy];
  A.stack_depth = win ? kStackWindow : depth_entries;  // the uniforms and material table follow the stack in LDS
  A.spill_stride = win ? std::max(0, depth_entries - kStackWindow) : 0;
  // grid_wg workgroups of kWgWaves waves: `grid` waves (a tile per wave at most)
  const int64_t grid_wg = std::max<int64_t>(
      1, std::min<int64_t>((tiles + kWgWaves - 1) / kWgWaves, (int64_t)std::max(per_cu, 1) * ctx->n_cu));
  const int64_t grid = grid_wg * kWgWaves;
  const int64_t spill_need = win ? grid * 64 * (int64_t)A.spill_stride : 0;
  if (win && spill_need > ctx->spill_cap) {
    if (ctx->d_spill) HIP_OK(hipFree(ctx->d_spill));
    ctx->d_spill = nullptr;
    ctx->spill_cap = 0;
    HIP_OK(hipMalloc(&ctx->d_spill, (size_t)spill_need * sizeof(int32_t)));
    ctx->spill_cap = spill_need;
  }
  // frames_per_launch = frames per BLOCK: a lane runs one pixel for one block
  // of frames, then hands the pixel's state to whichever lane takes its next
  // block.  One launch runs many blocks of every pixel, block-major, so lanes
  // stay busy until the last block (no per-block drain of the GPU).
  // frames_per_launch <= 0: auto.  Blocks let the launch's tail shrink: the
  // fewest blocks (at least 2) that give every resident lane `block_entries`
  // queue entries (so the tail, where lanes run dry, is about
  // 1/block_entries of the launch), frames split evenly over them, at most
  // max_block_frames each.  Each block boundary costs a hand-off per pixel;
  // with the packed hand-off, 8 entries and 2-3 blocks per call measured best
  // (20-frame calls: C2 -2 %, C3 -11 %, C4 -1 %, C5 even against 32 entries;
  // one block loses 2-7 % to the tail; profiles/r03_blocks.txt).
  // That needs several entries per lane in each block (>= 4): a pixel's next
  // block is then claimed long after its previous one started.  With fewer
  // (small images, strong-scaled ranks: about one pixel per lane) every block
  // boundary becomes a wait for the slowest pixel of the previous block, so
  // blocks there keep at least 4 frames (measured on C2 and C4 shares of 2,
  // 4 and 8 ranks, tools/sweep.py --stripes).
  const uint32_t n_items = (uint32_t)A.tiles_x * (uint32_t)((A.local_rows + 7) / 8) * 64u;
  const int cap = T.max_block_frames > 0 ? T.max_block_frames : 32;  // frames per block at most (auto plans)
  int fpl = p->frames_per_launch;
  bool tail_ok = false;  // auto plan with several entries per lane: a short last block may apply
  double slots_per_px = 0;  // pixels per resident lane (auto plans)
  const double px_per_lane =
      (double)n_items / ((double)std::max(per_cu, 1) * ctx->n_cu * 64 * kWgWaves);  // vs resident lanes
  if (fpl <= 0) {
    const int frames = std::max(p->frames, 1);
    const double per_block = (double)n_items / (double)(grid * 64);  // entries per lane per block
    const int want = T.block_entries > 0 ? T.block_entries : kDefaultBlockEntries;
    int nb = std::max(2, (int)std::ceil(want / std::max(per_block, 1e-9)));
    nb = std::max(1, std::min(nb, frames));
    fpl = (frames + nb - 1) / nb;
    if (per_block < 4.0) fpl = std::max(fpl, 4);
    // at most a few pixels per lane (strong-scaled ranks): little left to
    // balance but the pixels' own chains, so one block per pixel below 0.75
    // pixels per lane and two up to 2.5 (C2 shares of 4 and 8 ranks, C4 of 8:
    // 1-12 % faster than 4-frame blocks; the C5 8-rank share, 2 pixels per
    // lane: 4 % faster than 5-frame blocks; tools/sweep.py --stripes --fpl)
    const double per_slot = px_per_lane;
    slots_per_px = per_slot;
    if (per_slot < 0.75)
      fpl = frames;
    else if (per_slot <= 2.5)
      fpl = std::max(fpl, (frames + 1) / 2);
    else
      tail_ok = true;
    fpl = std::max(1, std::min({fpl, cap, frames}));
  }
  // the hand-off area is addressed with 32-bit byte offsets below 2^31
  // (handoff_rsrc): a larger image runs ONE block per launch, at most `cap`
  // frames (no hand-off; launches chain through the state arrays, so every
  // launch stays bounded: ~67 M+ pixels x 32 frames)
  const bool no_handoff = (int64_t)p->width * p->height * kHandoffWords * 8 > (int64_t)kHandoffMaxBytes;
  if (no_handoff) fpl = std::max(1, std::min(p->frames_per_launch > 0 ? p->frames_per_launch : std::max(p->frames, 1), cap));
  // blocks per launch: the hand-off tag holds 8 bits of block index, and
  // one launch covers at most ~4096 frames
  const int64_t max_blocks = no_handoff ? 1 : std::max<int64_t>(
      1, std::min<int64_t>({(int64_t)INT32_MAX / std::max<uint32_t>(n_items, 1), 4096 / fpl + 1,
                            (int64_t)kMaxBlocksPerLaunch}));
  const int64_t n_blocks_all = (p->frames + fpl - 1) / fpl;
  const int n_launch = (int)((n_blocks_all + max_blocks - 1) / max_blocks);
  // a short last block (last_block_frames, auto plans of one launch with
  // several entries per lane): the first nb-1 blocks share frames - L evenly
  // and the last takes the remainder (<= L).  Entries are block-major, so the
  // last block's entries are the launch's tail; shorter ones leave lanes idle
  // for less time at its end.  Same blocks, same hand-offs, same bits.
  // Auto: ceil(frames / 8) frames once a lane has at least 6 pixels (20-frame
  // C3 -2 %, 16-frame C4 -2 %, 8-frame C5 -3 %); between 2.5 and 6 a longer
  // one, ceil(frames / 4) (below); Renderer.tune tries equal blocks and both.
  int fpl_head = fpl;
  A.nb_head = INT32_MAX;  // every block fpl frames
  A.fpl_tail = fpl;
  // Auto: ceil(frames / 8) from 6 pixels per lane; from 2.5, on a whole image (one
  // stripe set), ceil(frames / 4): C2 and C3 at 4 pixels per lane, 20 frames: 9.00 /
  // 2.98 ms against equal blocks' 9.34 / 3.08 (and (17, 3) 9.24 / 3.02); a strong-scaled
  // share keeps equal blocks (the C5 4-rank share: 43.1 ms with (15, 5), 40.4 equal;
  // profiles/r04_last_block_auto.jsonl)
  const bool tail_auto = T.last_block_frames == 0 && (slots_per_px >= 6.0 || p->stripe_count == 1);
  if (tail_ok && n_launch == 1 && n_blocks_all >= 2 && (T.last_block_frames > 0 || tail_auto)) {
    const int nb = (int)n_blocks_all;
    const int L = T.last_block_frames > 0 ? T.last_block_frames
                                          : (slots_per_px >= 6.0 ? (p->frames + 7) / 8 : (p->frames + 3) / 4);
    if (L < fpl) {
      const int head = (p->frames - L + nb - 2) / (nb - 1);
      const int last = p->frames - (nb - 1) * head;
      if (last >= 1 && last <= L && head <= cap) {  // the head blocks keep the block cap
        fpl_head = head;
        A.nb_head = nb - 1;
        A.fpl_tail = last;
      }
    }
  }
  if (n_launch + 1 > ctx->queue_cap) {  // kQueues heads per launch (+ the primary pass), zeroed by memsets
    if (ctx->d_queue) HIP_OK(hipFree(ctx->d_queue));
    ctx->d_queue = nullptr;
    ctx->queue_cap = 0;
    const int cap = std::max(n_launch + 1, 64);
    HIP_OK(hipMalloc(&ctx->d_queue, (size_t)cap * kQueues * kQueueStride * sizeof(uint32_t)));
    ctx->queue_cap = cap;
  }
  const int64_t n_px = (int64_t)p->width * p->height;
  if (max_blocks > 1 && n_blocks_all > 1 && n_px > ctx->handoff_cap) {
    if (ctx->d_handoff) HIP_OK(hipFree(ctx->d_handoff));
    ctx->d_handoff = nullptr;
    ctx->handoff_cap = 0;
    const size_t bytes = (size_t)n_px * kHandoffWords * sizeof(unsigned long long);
    HIP_OK(hipMalloc(&ctx->d_handoff, bytes));
    HIP_OK(hipMemsetAsync(ctx->d_handoff, 0, bytes, st));  // tag 0 never matches (blocks >= 1)
    ctx->handoff_cap = n_px;
  }
  A.fpl = fpl_head;
  A.handoff = ctx->d_handoff;
  A.spill = ctx->d_spill;
  A.wave_log = nullptr;
  const bool px_fit = ctx->stats_on && n_px <= ctx->px_cap;  // never past the caller's buffers
  A.px_segments = px_fit ? ctx->px_segments : nullptr;
  A.px_iters = px_fit ? ctx->px_iters : nullptr;
  A.prim_cost = nullptr;  // set where the primary-hit pass runs
  ctx->wave_log_n = 0;
  if (kTiming) {  // diagnostics: each launch's workgroups log their timeline (the last launch's remain)
    if (grid > ctx->wave_log_cap) {
      if (ctx->d_wave_log) HIP_OK(hipFree(ctx->d_wave_log));
      ctx->d_wave_log = nullptr;
      ctx->wave_log_cap = 0;
      HIP_OK(hipMalloc(&ctx->d_wave_log, (size_t)grid * kWaveLogWords * sizeof(unsigned long long)));
      ctx->wave_log_cap = grid;
    }
    A.wave_log = ctx->d_wave_log;
    ctx->wave_log_n = grid;
  }
  // pixel_spread auto: spread slots up to 2.5 pixels per resident lane, where
  // each pixel's own chain sets the time (an N-rank share).  Tile-major slots
  // put one tile's dear pixels (C2: the pitcher's inside, ~29 loop iterations
  // per segment) in one wave, whose iterations then run the union of their
  // phases; spread, they share waves with cheap pixels that finish early.
  // Slowest share of 8 ranks: C2 5.83 -> 4.20 ms, C4 (64 frames) 58.1 -> 50.9;
  // 4 ranks: C2 6.51 -> 5.22, C4 76.7 -> 73.0; whole images even (C2, C3, C4,
  // C5 within 0.7 %; profiles/r04_spread.jsonl).
  A.spread = T.pixel_spread == 2 || (T.pixel_spread == 0 && px_per_lane <= 2.5) ? 1 : 0;
  A.entry_log = nullptr;
  ctx->entry_log_n = 0;
  if (kTiming && n_launch == 1 && (int64_t)p->width * p->height * n_blocks_all <= (16ll << 20)) {
    const int64_t need = (int64_t)p->width * p->height * n_blocks_all;
    if (need > ctx->entry_log_cap) {
      if (ctx->d_entry_log) HIP_OK(hipFree(ctx->d_entry_log));
      ctx->d_entry_log = nullptr;
      ctx->entry_log_cap = 0;
      HIP_OK(hipMalloc(&ctx->d_entry_log, (size_t)need * 3 * sizeof(uint32_t)));
      ctx->entry_log_cap = need;
    }
    HIP_OK(hipMemsetAsync(ctx->d_entry_log, 0, (size_t)need * 3 * sizeof(uint32_t), st));
    A.entry_log = ctx->d_entry_log;
    ctx->entry_log_n = need;
    ctx->entry_log_blocks = (int32_t)n_blocks_all;
  }
  if (ctx->stats_on || kDebug || kTiming)
    HIP_OK(hipMemsetAsync(ctx->d_stats, 0, kStatSlots * sizeof(unsigned long long), st));
  HIP_OK(hipEventRecord(ctx->ev0, st));
  // primary-hit cache (PrimHit): computed once per (scene, camera, image,
  // stripes, mode) and kept across calls; auto (0) computes it for a call of
  // two or more frames, or for a one-frame call of the same view as the
  // previous call (the reference's one frame per update()); 1 always, 2
  // never.  Speed only: the same bits either way.
  A.prim = nullptr;
  A.prim_out = nullptr;
  A.tile_order = nullptr;
  int prim_state = 0;
  if (T.primary_cache != 2 && tiles > 0 && p->frames > 0) {
    PrimKey key;
    std::memset(&key, 0, sizeof key);
    key.scene_uid = scene->uid;
    std::memcpy(&key.cam, cam, sizeof key.cam);
    key.w = p->width;
    key.h = p->height;
    key.stripe_rows = p->stripe_rows;
    key.stripe_index = p->stripe_index;
    key.stripe_count = p->stripe_count;
    key.mode = p->mode;
    const bool have = ctx->prim_valid && std::memcmp(&key, &ctx->prim_key, sizeof key) == 0;
    const bool again = ctx->seen_valid && std::memcmp(&key, &ctx->seen_key, sizeof key) == 0;
    ctx->seen_key = key;
    ctx->seen_valid = true;
    if (have || T.primary_cache == 1 || p->frames >= 2 || again) {
      if (!have) {
        const int64_t n_px = (int64_t)p->width * p->height;
        if (n_px > ctx->prim_cap) {
          ctx->prim_valid = false;
          if (ctx->d_prim) HIP_OK(hipFree(ctx->d_prim));
          if (ctx->d_prim_cost) HIP_OK(hipFree(ctx->d_prim_cost));
          ctx->d_prim = nullptr;
          ctx->d_prim_cost = nullptr;
          ctx->prim_cap = 0;
          HIP_OK(hipMalloc(&ctx->d_prim, (size_t)n_px * sizeof(PrimHit)));
          HIP_OK(hipMalloc(&ctx->d_prim_cost, (size_t)n_px * sizeof(uint32_t)));
          ctx->prim_cap = n_px;
        }
        A.prim_cost = ctx->d_prim_cost;
        // the pass writes its own stripes' costs only: zero the others, so
        // the tile keys and mcpt_get_primary_cost never read stale words
        if (p->stripe_count > 1) HIP_OK(hipMemsetAsync(ctx->d_prim_cost, 0, (size_t)n_px * sizeof(uint32_t), st));
        if (scene->near4_bytes <= kPrimSmallTree) {
          // small trees: one ray per lane, one 8x8 tile per workgroup
          const size_t lds_p = (size_t)depth_entries * 64 * sizeof(int32_t);
          const dim3 g((unsigned)tiles);
          if (noprune)
            hipLaunchKernelGGL(k_primary<MCPT_MODE_NOPRUNE>, g, dim3(64), lds_p, st, A, ctx->d_prim);
          else
            hipLaunchKernelGGL(k_primary<MCPT_MODE_EXACT>, g, dim3(64), lds_p, st, A, ctx->d_prim);
          HIP_OK(hipGetLastError());
        } else {
          // the same persistent machine in its PRIM form: one frame, no state;
          // its own queue heads (the slot after the render launches')
          RenderArgs Ap = A;
          Ap.frame_begin = 0;
          Ap.frames = 1;
          Ap.fpl = 1;
          Ap.blocks = 1;
          Ap.nb_head = INT32_MAX;
          Ap.fpl_tail = 1;
          Ap.prim = nullptr;
          Ap.prim_out = ctx->d_prim;
          Ap.wave_log = nullptr;
          Ap.px_segments = nullptr;
          Ap.px_iters = nullptr;
          Ap.entry_log = nullptr;
          Ap.spread = 0;  // coherent primary rays: tile-major slots (spread measured slower here)
          Ap.queue = ctx->d_queue + (size_t)n_launch * kQueues * kQueueStride;
          HIP_OK(hipMemsetAsync(Ap.queue, 0, (size_t)kQueues * kQueueStride * sizeof(uint32_t), st));
          // its own resident grid: the PRIM form needs fewer registers
          const void *pfn = kpfns[kind][win][pair];
          int per_cu_p = 0;
          rc = occupancy(ctx, pfn, lds, &per_cu_p);
          if (rc) return rc;
          const int64_t grid_pwg = std::max<int64_t>(
              1, std::min<int64_t>((tiles + kWgWaves - 1) / kWgWaves, (int64_t)std::max(per_cu_p, 1) * ctx->n_cu));
          const int64_t spill_p = win ? grid_pwg * kWgWaves * 64 * (int64_t)A.spill_stride : 0;
          if (spill_p > ctx->spill_cap) {
            if (ctx->d_spill) HIP_OK(hipFree(ctx->d_spill));
            ctx->d_spill = nullptr;
            ctx->spill_cap = 0;
            HIP_OK(hipMalloc(&ctx->d_spill, (size_t)spill_p * sizeof(int32_t)));
            ctx->spill_cap = spill_p;
            A.spill = ctx->d_spill;
          }
          Ap.spill = ctx->d_spill;
          void *pargs[] = {&Ap};
          HIP_OK(hipLaunchKernel(pfn, dim3((unsigned)grid_pwg), dim3(64 * kWgWaves), pargs, lds, st));
        }
        HIP_OK(hipEventRecord(ctx->ev_prim, st));
        ctx->prim_key = key;
        ctx->tile_order_mode = 0;  // a new cache: the tile order is rebuilt from its costs
        ctx->prim_valid = true;
      }
      A.prim = ctx->d_prim;
      prim_state = have ? 1 : 2;
      // the dearest-first tile order, built from the pass's per-pixel costs
      // once per primary-hit cache (and order mode)
      const int32_t mode = T.tile_order == 0 ? 1 : T.tile_order;  // 1 max, 2 sum (tuning value 1: off)
      if (T.tile_order != 1) {
        if (!have || ctx->tile_order_mode != mode) {
          if (tiles > ctx->tile_cap) {
            if (ctx->d_tile_order) HIP_OK(hipFree(ctx->d_tile_order));
            if (ctx->d_tile_key) HIP_OK(hipFree(ctx->d_tile_key));
            ctx->d_tile_order = nullptr;
            ctx->d_tile_key = nullptr;
            ctx->tile_cap = 0;
            HIP_OK(hipMalloc(&ctx->d_tile_order, (size_t)tiles * sizeof(int32_t)));
            HIP_OK(hipMalloc(&ctx->d_tile_key, (size_t)tiles));
            ctx->tile_cap = tiles;
          }
          hipLaunchKernelGGL(k_tile_keys, dim3((unsigned)tiles), dim3(64), 0, st, A, ctx->d_prim_cost, (int32_t)tiles,
                             mode == 2 ? 1 : 0, ctx->d_tile_key);
          hipLaunchKernelGGL(k_tile_sort, dim3(1), dim3(1024), 0, st, ctx->d_tile_key, (int32_t)tiles,
                             ctx->d_tile_order);
          HIP_OK(hipGetLastError());
          ctx->tile_order_mode = mode;
        }
        A.tile_order = ctx->d_tile_order;
      }
    }
  }
  int launches = 0;
  if (tiles > 0 && p->frames > 0) {
    HIP_OK(hipMemsetAsync(ctx->d_queue, 0, (size_t)n_launch * kQueues * kQueueStride * sizeof(uint32_t), st));
    for (int64_t f0 = 0; f0 < p->frames; f0 += max_blocks * fpl) {
      A.frame_begin = p->frame_begin + (int32_t)f0;
      A.frames = (int32_t)std::min<int64_t>(max_blocks * fpl, p->frames - f0);
      A.blocks = (A.frames + fpl - 1) / fpl;
      A.queue = ctx->d_queue + (size_t)launches * kQueues * kQueueStride;
      // a fresh tag per launch: granules of earlier launches never match.
      // After 255 launches the 8-bit launch tags wrap; the granules are
      // cleared then (stream-ordered before this launch), so every granule in
      // the area was written during the current cycle of tags.
      if (((++ctx->launch_seq) & 0xFFu) == 0) {
        ++ctx->launch_seq;
        if (ctx->d_handoff)
          HIP_OK(hipMemsetAsync(ctx->d_handoff, 0, (size_t)ctx->handoff_cap * kHandoffWords * 8, st));
      }
      A.tag_base = (ctx->launch_seq & 0xFFu) << 8;
      void *kargs[] = {&A};
      HIP_OK(hipLaunchKernel(kfn, dim3((unsigned)grid_wg), dim3(64 * kWgWaves), kargs, lds, st));
      ++launches;
    }
  }
  HIP_OK(hipEventRecord(ctx->ev1, st));
  // asynchronous: mcpt_get_stats waits for ev1 and reads the time and counters
  std::memset(&ctx->last, 0, sizeof(ctx->last));
  ctx->last.launches = launches;
  ctx->last.frames_per_block = fpl_head;
  ctx->last.stack_window = win ? 1 : 0;
  ctx->last.quantized = kind == 2 ? 1 : 0;
  ctx->last.top_levels = A.top_levels;
  ctx->last.workgroups = (int32_t)grid;
  ctx->last.primary_cache = prim_state;
  ctx->last_pending = true;
  ctx->last_stats = ctx->stats_on || kDebug || kTiming;
  return MCPT_OK;
}

int mcpt_generate_rays(mcpt_ctx *ctx, const mcpt_camera *cam, int32_t w, int32_t h, mcpt_ray *rays, void *stream) {
  if (!ctx || !cam || !rays || w <= 0 || h <= 0) return mcpt::fail(MCPT_ERR_ARG, "generate_rays: bad argument");
  HIP_OK(hipSetDevice(ctx->device));
  hipLaunchKernelGGL(k_generate, dim3((w + 63) / 64, h), dim3(64), 0, (hipStream_t)stream, *cam, (uint32_t)w,
                     (uint32_t)h, rays);
  HIP_OK(hipGetLastError());
  return MCPT_OK;
}

int mcpt_intersect(mcpt_ctx *ctx, const mcpt_scene *scene, const mcpt_ray *rays, int64_t n, mcpt_hit *hits,
                   float tmin, int32_t mode, void *stream) {
  if (!ctx || !scene || !rays || !hits || n < 0) return mcpt::fail(MCPT_ERR_ARG, "intersect: bad argument");
  if (n == 0) return MCPT_OK;
  HIP_OK(hipSetDevice(ctx->device));
  size_t lds = (size_t)(mode == MCPT_MODE_NOPRUNE ? scene->stack_depth : scene->stack_depth4) * 64 * sizeof(int32_t);
  dim3 g((unsigned)((n + 63) / 64));
  if (mode == MCPT_MODE_NOPRUNE)
    hipLaunchKernelGGL(k_intersect<MCPT_MODE_NOPRUNE>, g, dim3(64), lds, (hipStream_t)stream, scene->view, rays, n,
                       hits, tmin);
  else
    hipLaunchKernelGGL(k_intersect<MCPT_MODE_EXACT>, g, dim3(64), lds, (hipStream_t)stream, scene->view, rays, n,
                       hits, tmin);
  HIP_OK(hipGetLastError());
  return MCPT_OK;
}

int mcpt_shade(mcpt_ctx *ctx, const mcpt_scene *scene, mcpt_ray *rays, const mcpt_hit *hits, float *color,
               uint32_t *seeds, int64_t n, int32_t max_depth, void *stream) {
  if (!ctx || !scene || !rays || !hits || !color || !seeds || n < 0 || max_depth <= 0)
    return mcpt::fail(MCPT_ERR_ARG, "shade: bad argument");
  if (n == 0) return MCPT_OK;
  HIP_OK(hipSetDevice(ctx->device));
  hipLaunchKernelGGL(k_shade, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, scene->mats, rays,
                     hits, (f4 *)color, seeds, n, max_depth);
  HIP_OK(hipGetLastError());
  return MCPT_OK;
}

int mcpt_accumulate(mcpt_ctx *ctx, float *color, float *hist, int32_t *count, int64_t n, int32_t max_attempt,
                    void *stream) {
  if (!ctx || !color || !hist || !count || n < 0) return mcpt::fail(MCPT_ERR_ARG, "accumulate: bad argument");
  if (n == 0) return MCPT_OK;
  HIP_OK(hipSetDevice(ctx->device));
  hipLaunchKernelGGL(k_accumulate, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, (f4 *)color,
                     (f4 *)hist, count, n, max_attempt);
  HIP_OK(hipGetLastError());
  return MCPT_OK;
}

int mcpt_gamma_preview(mcpt_ctx *ctx, const float *color, float *out, int64_t n, void *stream) {
  if (!ctx || !color || !out || n < 0) return mcpt::fail(MCPT_ERR_ARG, "gamma_preview: bad argument");
  if (n == 0) return MCPT_OK;
  HIP_OK(hipSetDevice(ctx->device));
  hipLaunchKernelGGL(k_gamma_preview, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     (const f4 *)color, (f4 *)out, n);
  HIP_OK(hipGetLastError());
  return MCPT_OK;
}

}  // extern "C"
