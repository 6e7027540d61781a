/* mcpt_oracle.c — TEST INFRASTRUCTURE ONLY: CPU restatement of the reference
 * path-tracing hot path (see mcpt_oracle.h).  Compiled with -ffp-contract=off;
 * every fused multiply-add below is an explicit fmaf() placed where clang's
 * OpenCL FP_CONTRACT ON fuses the reference expression (LHS product first,
 * then RHS product; x - y*z fuses as fma(-y, z, x)).
 */
#include "mcpt_oracle.h"

#include <float.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef struct {
  float x, y, z, w;
} f4;

static inline f4 mk(float x, float y, float z, float w) {
  f4 r = {x, y, z, w};
  return r;
}
static inline f4 ld4(const float *p) { return mk(p[0], p[1], p[2], p[3]); }
static inline void st4(float *p, f4 v) {
  p[0] = v.x, p[1] = v.y, p[2] = v.z, p[3] = v.w;
}
static inline float asf(int32_t i) {
  float f;
  memcpy(&f, &i, 4);
  return f;
}
static inline int32_t asi(float f) {
  int32_t i;
  memcpy(&i, &f, 4);
  return i;
}

#define DEV_EPS 1e-5f /* objdef.h:16 */
#define CL_PI 3.14159265358979323846 /* OpenCL M_PI, a double */
#define HOST_PI 3.14159265358       /* oclbasic.h:192 */

/* ------------------------------------------------ OpenCL built-ins (CPU) */
static inline float dot3(f4 a, f4 b) { return fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)); }
static inline float dot4(f4 a, f4 b) { return fmaf(a.w, b.w, fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x))); }
static inline f4 cross4(f4 a, f4 b) {
  return mk(fmaf(a.y, b.z, b.y * -a.z), fmaf(a.z, b.x, b.z * -a.x), fmaf(a.x, b.y, b.x * -a.y), 0.0f);
}
static inline f4 scale(f4 a, float s) { return mk(a.x * s, a.y * s, a.z * s, a.w * s); }
static inline float rsq(float x) { return (float)(1.0 / sqrt((double)x)); }
static f4 normalize4(f4 p) {
  if (p.x == 0.0f && p.y == 0.0f && p.z == 0.0f && p.w == 0.0f) return p;
  float l2 = dot4(p, p);
  f4 q = p;
  if (l2 < FLT_MIN) {
    q = scale(p, 0x1p86f);
    l2 = dot4(q, q);
  } else if (isinf(l2)) {
    q = scale(p, 0x1p-66f);
    l2 = dot4(q, q);
    if (isinf(l2)) {
      q = mk(copysignf(isinf(q.x) ? 1.0f : 0.0f, q.x), copysignf(isinf(q.y) ? 1.0f : 0.0f, q.y),
             copysignf(isinf(q.z) ? 1.0f : 0.0f, q.z), copysignf(isinf(q.w) ? 1.0f : 0.0f, q.w));
      l2 = dot4(q, q);
    }
  }
  return scale(q, rsq(l2));
}
static inline int is_zero4(f4 c) { return c.x == 0.0f && c.y == 0.0f && c.z == 0.0f && c.w == 0.0f; }

/* ----------------------------------------------------- host-side pieces */
static f4 hsub(f4 a, f4 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w); }
static f4 hcross(f4 a, f4 b) { /* oclbasic.h:119-127 */
  return mk(a.y * b.z - a.z * b.y, -a.x * b.z + a.z * b.x, a.x * b.y - a.y * b.x, 0.0f);
}
static f4 hnormalize(f4 a) { /* oclbasic.h:139-147 */
  float s = 0.0f;
  s += a.x * a.x;
  s += a.y * a.y;
  s += a.z * a.z;
  s += a.w * a.w;
  s = sqrtf(s);
  return mk(a.x / s, a.y / s, a.z / s, a.w / s);
}

int oracle_parse_camera(const double pos[3], const double look[3], const double up[3], double fov, mcpt_camera *out) {
  /* Auxiliary::parseCamera, auxiliary.cpp:20-71 (perspective branch) */
  memset(out, 0, sizeof(*out));
  f4 c = mk((float)pos[0], (float)pos[1], (float)pos[2], 0.0f);
  f4 l = mk((float)look[0], (float)look[1], (float)look[2], 0.0f);
  f4 u = mk((float)up[0], (float)up[1], (float)up[2], 0.0f);
  f4 d = hsub(l, c);
  d.w = 0.0f;
  out->arg = (float)((double)(float)fov * HOST_PI / 180.0f);
  f4 hz = hcross(d, u);
  u = hcross(hz, d);
  out->tmin = 0.0f;
  st4(out->center, c);
  st4(out->direction, hnormalize(d));
  st4(out->up, hnormalize(u));
  st4(out->horizontal, hnormalize(hz));
  out->camera_type = 0;
  return 0;
}

int oracle_pack_triangles(mcpt_triangle *t, const int32_t *mi, int64_t n) {
  /* SceneCL::SceneCL, scenebuild.cpp:58-62 */
  for (int64_t i = 0; i < n; ++i) {
    f4 v0 = ld4(t[i].v[0]), v1 = ld4(t[i].v[1]), v2 = ld4(t[i].v[2]);
    f4 nn = hnormalize(hcross(hsub(v1, v0), hsub(v2, v0)));
    st4(t[i].normal, nn);
    memcpy(&t[i].normal[3], &mi[i], 4);
  }
  return 0;
}

/* HLBVH<CPU>::build, hlbvh.cpp:92-200 */
typedef struct {
  int id, code;
} prim_t;

static uint32_t lshift3(uint32_t x) { /* hlbvh.cpp:12-23 */
  if (x == (1u << 10)) --x;
  x = (x | (x << 16)) & 0x030000FFu;
  x = (x | (x << 8)) & 0x0300F00Fu;
  x = (x | (x << 4)) & 0x030C30C3u;
  x = (x | (x << 2)) & 0x09249249u;
  return x;
}
static int clz_ref(int a) {
  if (a == 0) return 32;
  int n = 0;
  uint32_t u = (uint32_t)a;
  while ((int32_t)u > 0) u <<= 1, ++n;
  return n;
}
static uint32_t round_to_u32_msvc(float x) {
  float r = roundf(x); /* NaN / out of range -> cvttss2si(64) -> low word 0 */
  if (!(r > -9.2233720368547758e18f && r < 9.2233720368547758e18f)) return 0u;
  return (uint32_t)(int64_t)r;
}
static f4 vminf4(f4 a, f4 b) { /* std::min(a, b) = (b < a) ? b : a per lane */
  return mk(b.x < a.x ? b.x : a.x, b.y < a.y ? b.y : a.y, b.z < a.z ? b.z : a.z, b.w < a.w ? b.w : a.w);
}
static f4 vmaxf4(f4 a, f4 b) { /* std::max(a, b) = (a < b) ? b : a */
  return mk(a.x < b.x ? b.x : a.x, a.y < b.y ? b.y : a.y, a.z < b.z ? b.z : a.z, a.w < b.w ? b.w : a.w);
}

static int64_t find_split(const prim_t *p, int64_t left, int64_t right) {
  int target = clz_ref(p[left].code ^ p[right].code);
  if (target == 32) return (right + left) >> 1;
  do {
    int64_t mid = (right + left) >> 1;
    if (clz_ref(p[left].code ^ p[mid].code) > target)
      left = mid;
    else
      right = mid;
  } while (right > left + 1);
  return left;
}

static void refit(mcpt_bvh_node *nodes, int64_t root) {
  /* recursiveBuildNode (hlbvh.cpp:64-76), post-order with an explicit stack */
  int64_t cap = 64, sp = 0;
  int64_t *st = malloc(sizeof(int64_t) * cap);
  int *phase = malloc(sizeof(int) * cap);
  st[sp] = root, phase[sp++] = 0;
  while (sp) {
    int64_t id = st[sp - 1];
    mcpt_bvh_node *nd = &nodes[id];
    if (nd->left == nd->right) {
      --sp;
      continue;
    }
    if (sp + 2 > cap) {
      cap *= 2;
      st = realloc(st, sizeof(int64_t) * cap);
      phase = realloc(phase, sizeof(int) * cap);
    }
    if (phase[sp - 1] == 0) {
      phase[sp - 1] = 1;
      st[sp] = nd->left, phase[sp++] = 0;
    } else if (phase[sp - 1] == 1) {
      phase[sp - 1] = 2;
      st[sp] = nd->right, phase[sp++] = 0;
    } else {
      const mcpt_bvh_node *L = &nodes[nd->left], *R = &nodes[nd->right];
      st4(nd->bbmin, vminf4(ld4(L->bbmin), ld4(R->bbmin)));
      st4(nd->bbmax, vmaxf4(ld4(L->bbmax), ld4(R->bbmax)));
      --sp;
    }
  }
  free(st);
  free(phase);
}

int oracle_build_hlbvh(const mcpt_triangle *t, int64_t n, mcpt_bvh_node *nodes) {
  if (n <= 0) return -1;
  f4 *bmin = malloc(sizeof(f4) * n), *bmax = malloc(sizeof(f4) * n), *cen = malloc(sizeof(f4) * n);
  for (int64_t i = 0; i < n; ++i) {
    f4 a = ld4(t[i].v[0]), b = ld4(t[i].v[1]), c = ld4(t[i].v[2]);
    a.w = b.w = c.w = 0.0f;
    bmin[i] = vminf4(vminf4(a, b), c);
    bmax[i] = vmaxf4(vmaxf4(a, b), c);
    f4 s = mk(bmin[i].x + bmax[i].x, bmin[i].y + bmax[i].y, bmin[i].z + bmax[i].z, bmin[i].w + bmax[i].w);
    cen[i] = scale(s, 0.5f);
  }
  f4 gmin = mk(FLT_MAX, FLT_MAX, FLT_MAX, FLT_MAX), gmax = mk(-FLT_MAX, -FLT_MAX, -FLT_MAX, -FLT_MAX);
  for (int64_t i = 0; i < n; ++i) gmin = vminf4(gmin, cen[i]), gmax = vmaxf4(gmax, cen[i]);
  f4 gs = hsub(gmax, gmin);
  prim_t *p = malloc(sizeof(prim_t) * n), *tmp = malloc(sizeof(prim_t) * n);
  for (int64_t i = 0; i < n; ++i) {
    f4 d = hsub(cen[i], gmin);
    float q[3] = {d.x, d.y, d.z}, g[3] = {gs.x, gs.y, gs.z};
    uint32_t u[3];
    for (int k = 0; k < 3; ++k) {
      q[k] /= g[k];
      q[k] *= 1024.0f;
      u[k] = round_to_u32_msvc(q[k]);
    }
    p[i].id = (int)i;
    p[i].code = (int)((lshift3(u[2]) << 2) | (lshift3(u[1]) << 1) | lshift3(u[0]));
  }
  /* radixSort: 5 LSD passes of 6 bits (hlbvh.cpp:27-63) */
  for (int pass = 0; pass < 5; ++pass) {
    prim_t *in = (pass & 1) ? tmp : p, *out = (pass & 1) ? p : tmp;
    int cnt[64] = {0}, off[64];
    int lo = pass * 6;
    for (int64_t i = 0; i < n; ++i) cnt[(in[i].code >> lo) & 63]++;
    off[0] = 0;
    for (int b = 1; b < 64; ++b) off[b] = off[b - 1] + cnt[b - 1];
    for (int64_t i = 0; i < n; ++i) out[off[(in[i].code >> lo) & 63]++] = in[i];
  }
  prim_t *sorted = tmp; /* odd number of passes: result in the temp vector */
  int64_t nn = 2 * n - 1;
  memset(nodes, 0, sizeof(mcpt_bvh_node) * nn);
  nodes[0].parent = -1;
  if (n > 1) {
    int64_t *q = malloc(sizeof(int64_t) * 3 * n), qh = 0, qt = 0;
    q[qt++] = 0, q[qt++] = n - 1, q[qt++] = 0;
    while (qh < qt) {
      int64_t lo = q[qh++], hi = q[qh++], nd = q[qh++];
      int64_t s = find_split(sorted, lo, hi);
      int64_t li = (s != lo) ? s : s + n - 1;
      int64_t ri = (s + 1 != hi) ? s + 1 : s + n;
      nodes[nd].left = (int32_t)li, nodes[li].parent = (int32_t)nd;
      nodes[nd].right = (int32_t)ri, nodes[ri].parent = (int32_t)nd;
      if (li == s) q[qt++] = lo, q[qt++] = s, q[qt++] = s;
      if (ri == s + 1) q[qt++] = s + 1, q[qt++] = hi, q[qt++] = s + 1;
    }
    free(q);
  }
  for (int64_t i = n - 1; i < nn; ++i) {
    int id = sorted[i - (n - 1)].id;
    nodes[i].left = nodes[i].right = id;
    st4(nodes[i].bbmin, bmin[id]);
    st4(nodes[i].bbmax, bmax[id]);
  }
  if (n > 1) refit(nodes, 0);
  free(bmin), free(bmax), free(cen), free(p), free(tmp);
  return 0;
}

/* ------------------------------------------------------ device kernels */
static void gen_one(const mcpt_camera *cam, uint32_t x, uint32_t y, uint32_t w, uint32_t h, f4 *o, f4 *d) {
  /* rayGenerator.cl:1-31 */
  float px = (float)x / (float)w, py = (float)y / (float)h;
  float ratio = (float)w * 1.0f / (float)h;
  f4 dir = ld4(cam->direction), hor = ld4(cam->horizontal), up = ld4(cam->up);
  float t1 = px - 0.5f, t2 = py - 0.5f;
  float dist = 0.5f / tanf(cam->arg / 2);
  f4 dd;
  dd.x = fmaf(t2, up.x, fmaf(dir.x, dist, (t1 * hor.x) * ratio));
  dd.y = fmaf(t2, up.y, fmaf(dir.y, dist, (t1 * hor.y) * ratio));
  dd.z = fmaf(t2, up.z, fmaf(dir.z, dist, (t1 * hor.z) * ratio));
  dd.w = fmaf(t2, up.w, fmaf(dir.w, dist, (t1 * hor.w) * ratio));
  *o = ld4(cam->center);
  *d = normalize4(dd);
  o->w = asf(0);
  d->w = asf((int32_t)(y * w + x));
}

void oracle_generate(const mcpt_camera *cam, int32_t w, int32_t h, mcpt_ray *rays) {
  for (int32_t y = 0; y < h; ++y)
    for (int32_t x = 0; x < w; ++x) {
      f4 o, d;
      gen_one(cam, (uint32_t)x, (uint32_t)y, (uint32_t)w, (uint32_t)h, &o, &d);
      mcpt_ray *r = &rays[(int64_t)y * w + x];
      st4(r->origin, o);
      st4(r->direction, d);
      memset(r->ratio, 0, 16);
    }
}

/* objdef.h:102-124, contracted as clang contracts them */
static inline float det2(float a, float b, float c, float d) { return fmaf(a, d, -(b * c)); }
static inline float det3(float a1, float a2, float a3, float b1, float b2, float b3, float c1, float c2, float c3) {
  return fmaf(c1, det2(a2, a3, b2, b3), fmaf(a1, det2(b2, b3, c2, c3), -(b1 * det2(a2, a3, c2, c3))));
}

typedef struct {
  float t;
  int32_t tri, last;
  uint32_t nodes, tests;
} trace_t;

/* intersectTriangle, objdef.h:178-221 (4x4 Cramer inverse) */
static int tri_test(const mcpt_triangle *T, f4 o, f4 d, float tmin, float *t_out) {
  f4 N = ld4(T->normal);
  if (fabsf(dot3(N, d)) < DEV_EPS) return 0;
  f4 v0 = ld4(T->v[0]), v1 = ld4(T->v[1]), v2 = ld4(T->v[2]);
  float a1 = d.x, a2 = d.y, a3 = d.z, a4 = 0.0f;
  float b1 = -(v1.x - v0.x), b2 = -(v1.y - v0.y), b3 = -(v1.z - v0.z), b4 = 0.0f;
  float c1 = -(v2.x - v0.x), c2 = -(v2.y - v0.y), c3 = -(v2.z - v0.z), c4 = 0.0f;
  float d1 = 0.0f, d2 = 0.0f, d3 = 0.0f, d4 = 1.0f;
  f4 aro = mk(v0.x - o.x, v0.y - o.y, v0.z - o.z, 0.0f);
  float X1 = det3(b2, b3, b4, c2, c3, c4, d2, d3, d4), X2 = det3(a2, a3, a4, c2, c3, c4, d2, d3, d4);
  float X3 = det3(a2, a3, a4, b2, b3, b4, d2, d3, d4), X4 = det3(a2, a3, a4, b2, b3, b4, c2, c3, c4);
  float det = fmaf(-d1, X4, fmaf(c1, X3, fmaf(a1, X1, -(b1 * X2))));
  if (fabsf(det) < DEV_EPS) return 0;
  float s0 = X1 / det, s1 = -X2 / det, s2 = X3 / det;
  float s4 = -det3(b1, b3, b4, c1, c3, c4, d1, d3, d4) / det;
  float s5 = det3(a1, a3, a4, c1, c3, c4, d1, d3, d4) / det;
  float s6 = -det3(a1, a3, a4, b1, b3, b4, d1, d3, d4) / det;
  float s8 = det3(b1, b2, b4, c1, c2, c4, d1, d2, d4) / det;
  float s9 = -det3(a1, a2, a4, c1, c2, c4, d1, d2, d4) / det;
  float sa = det3(a1, a2, a4, b1, b2, b4, d1, d2, d4) / det;
  if (s0 == FLT_MAX) return 0;
  float t = dot3(aro, mk(s0, s4, s8, 0)), b = dot3(aro, mk(s1, s5, s9, 0)), c = dot3(aro, mk(s2, s6, sa, 0));
  if (b < 0 || c < 0 || b + c > 1 || t <= tmin) return 0;
  *t_out = t;
  return 1;
}

static int g_prune = 0; /* counting mode only: skip boxes beyond the current hit */
void oracle_set_prune(int on) { g_prune = on; }

/* intersectAABB, objdef.h:223-237 */
static int box_test(const float *bmin, const float *bmax, f4 o, f4 d, float tmin, float *tnear) {
  float t1x = (bmin[0] - o.x) / d.x, t1y = (bmin[1] - o.y) / d.y, t1z = (bmin[2] - o.z) / d.z;
  float t2x = (bmax[0] - o.x) / d.x, t2y = (bmax[1] - o.y) / d.y, t2z = (bmax[2] - o.z) / d.z;
  float tn = fmaxf(fmaxf(fminf(t1x, t2x), fminf(t1y, t2y)), fminf(t1z, t2z));
  float tf = fminf(fminf(fmaxf(t1x, t2x), fmaxf(t1y, t2y)), fmaxf(t1z, t2z));
  *tnear = tn;
  return !(tf < tn || tf < tmin);
}

/* intersectObjects, objdef.h:240-275: exhaustive left-first DFS, stack[64] */
static trace_t traverse_nearest(const mcpt_triangle *tris, const mcpt_bvh_node *nodes, f4 o, f4 d, float tmin);

static trace_t traverse(const mcpt_triangle *tris, const mcpt_bvh_node *nodes, f4 o, f4 d, float tmin) {
  trace_t tr = {FLT_MAX, -1, -1, 0, 0};
  if (g_prune == 2) return traverse_nearest(tris, nodes, o, d, tmin);
  int32_t stack[64];
  int sp = 1;
  stack[0] = 0;
  while (sp > 0) {
    int32_t cur = stack[--sp];
    for (;;) {
      const mcpt_bvh_node *N = &nodes[cur];
      float tn;
      tr.nodes++;
      if (!box_test(N->bbmin, N->bbmax, o, d, tmin, &tn)) break;
      if (g_prune && tn > tr.t) break; /* t-pruned variant (E_node/E_tri) */
      if (N->left == N->right) {
        float t;
        tr.tests++;
        if (tri_test(&tris[N->left], o, d, tmin, &t)) {
          tr.last = N->left;
          if (tr.t - t >= DEV_EPS) tr.t = t, tr.tri = N->left;
        }
        break;
      }
      if (sp >= 64) { /* the reference overflows silently here; stop loudly */
        fprintf(stderr, "oracle: BVH deeper than the reference's 64-entry stack\n");
        abort();
      }
      stack[sp++] = N->right;
      cur = N->left;
    }
  }
  return tr;
}

/* Counting mode 2 only (not the reference's order): nearest-child-first
 * traversal with t-pruning, the box-test / triangle-test counts an
 * order-free closest-hit search would need. Same box-test unit as the
 * DFS above (one test per node entered). */
static trace_t traverse_nearest(const mcpt_triangle *tris, const mcpt_bvh_node *nodes, f4 o, f4 d, float tmin) {
  trace_t tr = {FLT_MAX, -1, -1, 0, 0};
  int32_t stack[64];
  float stack_t[64];
  int sp = 0;
  float tn0;
  tr.nodes++;
  if (!box_test(nodes[0].bbmin, nodes[0].bbmax, o, d, tmin, &tn0)) return tr;
  int32_t cur = 0;
  for (;;) {
    const mcpt_bvh_node *N = &nodes[cur];
    if (N->left == N->right) {
      float t;
      tr.tests++;
      if (tri_test(&tris[N->left], o, d, tmin, &t) && t < tr.t) tr.t = t, tr.tri = N->left, tr.last = N->left;
      cur = -1;
    } else {
      float tl, tq;
      tr.nodes += 2;
      int hl = box_test(nodes[N->left].bbmin, nodes[N->left].bbmax, o, d, tmin, &tl) && !(tl > tr.t);
      int hr = box_test(nodes[N->right].bbmin, nodes[N->right].bbmax, o, d, tmin, &tq) && !(tq > tr.t);
      if (hl && hr) {
        int near_left = tl <= tq;
        stack[sp] = near_left ? N->right : N->left;
        stack_t[sp++] = near_left ? tq : tl;
        cur = near_left ? N->left : N->right;
      } else {
        cur = hl ? N->left : (hr ? N->right : -1);
      }
    }
    while (cur < 0 && sp > 0) {
      --sp;
      if (!(stack_t[sp] > tr.t)) cur = stack[sp];
    }
    if (cur < 0) break;
  }
  return tr;
}

static void make_hit(const mcpt_triangle *tris, const trace_t *tr, f4 o, f4 d, mcpt_hit *h) {
  /* intersect.cl:9-27 */
  memset(h, 0, sizeof(*h));
  h->t = tr->t;
  f4 nrm = mk(0, 0, 0, 0), pt = mk(0, 0, 0, 0);
  if (tr->tri >= 0) {
    const mcpt_triangle *T = &tris[tr->tri];
    nrm = mk(T->normal[0], T->normal[1], T->normal[2], 0.0f);
    pt = mk(fmaf(tr->t, d.x, o.x), fmaf(tr->t, d.y, o.y), fmaf(tr->t, d.z, o.z), fmaf(tr->t, d.w, o.w));
    memcpy(&h->material_id, &T->normal[3], 4);
  }
  if (tr->last >= 0) {
    h->triangle_id = (uint32_t)tr->last;
    if (dot3(d, nrm) > 0) nrm = mk(-nrm.x, -nrm.y, -nrm.z, -nrm.w);
  }
  st4(h->normal, nrm);
  st4(h->point, pt);
}

void oracle_intersect(const mcpt_triangle *tris, const mcpt_bvh_node *nodes, const mcpt_ray *rays, int64_t n,
                      mcpt_hit *hits, float tmin) {
  for (int64_t i = 0; i < n; ++i) {
    f4 o = ld4(rays[i].origin), d = ld4(rays[i].direction);
    if (asi(o.w) & (int32_t)0xFF000000) continue;
    trace_t tr = traverse(tris, nodes, o, d, tmin);
    make_hit(tris, &tr, o, d, &hits[i]);
  }
}

/* ------------------------------------------------------------- shade.cl */
static inline uint32_t lcg15(uint32_t *s) { /* shade.cl:1-6 */
  *s = *s * 1103515245u + 12345u;
  return (*s >> 16) & 0x7FFFu;
}
static f4 mirror_dir(f4 n, f4 in) { /* shade.cl:19-25 */
  n.w = 0, in.w = 0;
  float k = 2 * dot4(n, in);
  f4 r = mk(fmaf(-k, n.x, in.x), fmaf(-k, n.y, in.y), fmaf(-k, n.z, in.z), 0.0f);
  return normalize4(r);
}
static int transmit_dir(f4 n, f4 in, float ei, float et, f4 *out) { /* shade.cl:27-38 */
  n.w = 0, in.w = 0;
  float eta = ei / et;
  float ci = -dot4(n, in);
  float k = fmaf(-(eta * eta), fmaf(-ci, ci, 1), 1.0f);
  if (k < 0.0f) return 0;
  float a = fmaf(eta, ci, -sqrtf(k));
  *out = normalize4(mk(fmaf(a, n.x, eta * in.x), fmaf(a, n.y, eta * in.y), fmaf(a, n.z, eta * in.z),
                       fmaf(a, n.w, eta * in.w)));
  return 1;
}
static f4 random_dir(f4 n, uint32_t *seed) { /* shade.cl:40-59 */
  n.w = 0;
  float phi = (float)(2 * CL_PI / 32768 * (double)lcg15(seed));
  float u = (float)lcg15(seed) * 1.0f / 32768;
  float s = sqrtf(u);
  f4 a1 = (n.z == 0) ? mk(0, 0, 1.0f, 0) : mk(1, 0, 0, 0);
  f4 a2 = normalize4(cross4(a1, n));
  a1 = normalize4(cross4(a2, n));
  float cs = cosf(phi) * s, sn = sinf(phi) * s, m = 1 - u;
  f4 r = mk(fmaf(m, n.x, fmaf(cs, a1.x, sn * a2.x)), fmaf(m, n.y, fmaf(cs, a1.y, sn * a2.y)),
            fmaf(m, n.z, fmaf(cs, a1.z, sn * a2.z)), fmaf(m, n.w, fmaf(cs, a1.w, sn * a2.w)));
  return normalize4(r);
}
static float fresnel(f4 n, f4 d, float ior) { /* shade.cl:69-73 */
  float k = powf((ior - 1) / (ior + 1), 2.0f);
  return fmaf(1 - k, powf(1 - fabsf(dot3(n, d)), 5.0f), k);
}

/* One live ray that hit something (shade.cl:98-206).  Returns 1 if a new
 * ray record is written, 0 if only the terminate flag changes. */
static int shade_hit(const mcpt_material *mats, f4 o, f4 d, f4 nrm, f4 pt, int32_t mat, f4 *color, uint32_t *seed,
                     int max_depth, f4 *no_out, f4 *nd_out, int *bad) {
  const mcpt_material *M = &mats[mat];
  f4 kd = ld4(M->kd), ks = ld4(M->ka_ks), c = *color;
  int32_t td = asi(o.w);
  f4 no, nd;
  const float twopi = (float)(2 * CL_PI);
  *bad = 0;
  int type = M->type;
  if (type == MCPT_GLOSSY) {
    if (lcg15(seed) & 1) {
      f4 refl = mirror_dir(nrm, d);
      nd = random_dir(refl, seed);
      while (dot3(nd, nrm) <= 0) nd = random_dir(refl, seed);
      no = mk(fmaf(DEV_EPS, nd.x, pt.x), fmaf(DEV_EPS, nd.y, pt.y), fmaf(DEV_EPS, nd.z, pt.z), 0);
      no.w = asf(td + 1);
      nd.w = d.w;
      float p = powf(dot3(nd, refl), M->Ns), cn = dot3(nd, nrm);
      c = mk(c.x * ks.x * p * cn / twopi, c.y * ks.y * p * cn / twopi, c.z * ks.z * p * cn / twopi,
             c.w * ks.w * p * cn / twopi);
      goto tail;
    }
    type = MCPT_DIFFUSE; /* diffuse lobe */
  }
  switch (type) {
    case MCPT_DIFFUSE: {
      nd = random_dir(nrm, seed);
      no = mk(fmaf(DEV_EPS, nd.x, pt.x), fmaf(DEV_EPS, nd.y, pt.y), fmaf(DEV_EPS, nd.z, pt.z), 0);
      no.w = asf(td + 1);
      nd.w = d.w;
      float cn = dot3(nd, nrm);
      c = mk(c.x * kd.x * cn / twopi, c.y * kd.y * cn / twopi, c.z * kd.z * cn / twopi, c.w * kd.w * cn / twopi);
      break;
    }
    case MCPT_LIGHT:
      *color = mk(c.x * ks.x, c.y * ks.y, c.z * ks.z, c.w * ks.w);
      *no_out = o;
      no_out->w = asf(td | (int32_t)0xFF000000);
      *nd_out = d;
      return 0;
    case MCPT_TRANSPARENT: {
      int inside = (td & 0x00FF0000) != 0;
      float ei = inside ? M->Ni : 1.0f, et = inside ? 1.0f : M->Ni;
      if (!transmit_dir(nrm, d, ei, et, &nd)) {
        no = pt;
        nd = mirror_dir(nrm, d);
        nd.w = d.w;
        no.w = asf(td + 1);
        break;
      }
      float fr = fresnel(nrm, nd, M->Ni);
      no = pt;
      nd.w = d.w;
      int32_t ntd = td + 1;
      if (((float)lcg15(seed) * 1.0f / 32768) >= fr) {
        ntd ^= 0x00FF0000;
      } else {
        f4 m = mirror_dir(nrm, d);
        nd.x = m.x, nd.y = m.y, nd.z = m.z;
      }
      no.w = asf(ntd);
      break;
    }
    default:
      *bad = 1;
      *color = mk(0, 0, 0, 0);
      *no_out = o;
      no_out->w = asf(td | (int32_t)0xFF000000);
      *nd_out = d;
      return 0;
  }
tail:;
  int32_t ntd = asi(no.w);
  if ((ntd & 0xFFFF) >= max_depth) {
    c = mk(0, 0, 0, 0);
    no.w = asf(ntd | (int32_t)0xFF000000);
  }
  *color = c;
  *no_out = no;
  *nd_out = nd;
  return 1;
}

void oracle_shade(const mcpt_material *mats, mcpt_ray *rays, const mcpt_hit *hits, float *colors, uint32_t *seeds,
                  int64_t n, int32_t max_depth) {
  for (int64_t i = 0; i < n; ++i) {
    f4 o = ld4(rays[i].origin);
    if (asi(o.w) & (int32_t)0xFF000000) continue;
    if (hits[i].t >= FLT_MAX) {
      st4(colors + 4 * i, mk(0, 0, 0, 0));
      rays[i].origin[3] = asf(asi(o.w) | (int32_t)0xFF000000);
      continue;
    }
    f4 c = ld4(colors + 4 * i), no, nd;
    int bad;
    int wr = shade_hit(mats, o, ld4(rays[i].direction), ld4(hits[i].normal), ld4(hits[i].point),
                       (int32_t)hits[i].material_id, &c, &seeds[i], max_depth, &no, &nd, &bad);
    st4(colors + 4 * i, c);
    if (wr) {
      st4(rays[i].origin, no);
      st4(rays[i].direction, nd);
      memset(rays[i].ratio, 0, 16);
    } else {
      rays[i].origin[3] = no.w;
    }
  }
}

/* history.cl:3-28 on one pixel */
static f4 accum_one(f4 now, f4 *hist, int32_t *cnt, int max_attempt) {
  if (is_zero4(now) || *cnt >= max_attempt) return *hist;
  float n = (float)*cnt, n1 = (float)(*cnt + 1);
  f4 h = *hist;
  now = mk(fmaf(h.x, n, now.x) / n1, fmaf(h.y, n, now.y) / n1, fmaf(h.z, n, now.z) / n1, fmaf(h.w, n, now.w) / n1);
  *hist = now;
  hist->w = 0.0f;
  ++*cnt;
  return now;
}

void oracle_accumulate(float *colors, float *hist, int32_t *count, int64_t n, int32_t max_attempt) {
  for (int64_t i = 0; i < n; ++i) {
    f4 h = ld4(hist + 4 * i);
    f4 out = accum_one(ld4(colors + 4 * i), &h, &count[i], max_attempt);
    st4(hist + 4 * i, h);
    st4(colors + 4 * i, out);
  }
}

/* ---------------------------------------------------- whole frame loop */
static void render_pixel(const mcpt_camera *cam, const mcpt_triangle *tris, const mcpt_bvh_node *nodes,
                         const mcpt_material *mats, int32_t w, int32_t h, int32_t pid, int32_t max_depth,
                         int32_t frame_begin, int32_t frames, int32_t max_attempt, uint32_t *seeds, float *hist,
                         int32_t *count, uint64_t *st) {
  f4 o0, d0;
  gen_one(cam, (uint32_t)(pid % w), (uint32_t)(pid / w), (uint32_t)w, (uint32_t)h, &o0, &d0);
  uint32_t seed = seeds[pid];
  f4 hh = ld4(hist + 4 * pid);
  int32_t cnt = count[pid];
  for (int32_t f = 0; f < frames; ++f) {
    f4 o = o0, d = d0, c = mk(1, 1, 1, 1);
    for (int b = 0; b < max_depth; ++b) {
      trace_t tr = traverse(tris, nodes, o, d, 0.001f);
      st[0]++, st[1] += tr.nodes, st[2] += tr.tests;
      if (tr.t >= FLT_MAX) {
        c = mk(0, 0, 0, 0);
        break;
      }
      mcpt_hit hit;
      make_hit(tris, &tr, o, d, &hit);
      f4 no, nd;
      int bad;
      shade_hit(mats, o, d, ld4(hit.normal), ld4(hit.point), (int32_t)hit.material_id, &c, &seed, max_depth, &no,
                &nd, &bad);
      st[3] += bad;
      o = no, d = nd;
      if (asi(o.w) & (int32_t)0xFF000000) break;
    }
    if (frame_begin + f <= max_attempt) accum_one(c, &hh, &cnt, max_attempt);
  }
  seeds[pid] = seed;
  st4(hist + 4 * pid, hh);
  count[pid] = cnt;
}

void oracle_render_pixels(const mcpt_camera *cam, const mcpt_triangle *tris, const mcpt_bvh_node *nodes,
                          const mcpt_material *mats, int32_t w, int32_t h, const int32_t *pixels, int64_t npix,
                          int32_t max_depth, int32_t frame_begin, int32_t frames, int32_t max_attempt,
                          uint32_t *seeds, float *hist, int32_t *count, int32_t threads, uint64_t *stats) {
  uint64_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;
#ifdef _OPENMP
  if (threads <= 0) threads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 64) num_threads(threads) reduction(+ : s0, s1, s2, s3)
#endif
  for (int64_t k = 0; k < npix; ++k) {
    uint64_t st[4] = {0, 0, 0, 0};
    int32_t pid = pixels ? pixels[k] : (int32_t)k;
    render_pixel(cam, tris, nodes, mats, w, h, pid, max_depth, frame_begin, frames, max_attempt, seeds, hist, count,
                 st);
    s0 += st[0], s1 += st[1], s2 += st[2], s3 += st[3];
  }
  if (stats) stats[0] = s0, stats[1] = s1, stats[2] = s2, stats[3] = s3;
}

void oracle_render(const mcpt_camera *cam, const mcpt_triangle *tris, const mcpt_bvh_node *nodes,
                   const mcpt_material *mats, int32_t w, int32_t h, int32_t max_depth, int32_t frame_begin,
                   int32_t frames, int32_t max_attempt, uint32_t *seeds, float *hist, int32_t *count, int32_t threads,
                   uint64_t *stats) {
  oracle_render_pixels(cam, tris, nodes, mats, w, h, NULL, (int64_t)w * h, max_depth, frame_begin, frames,
                       max_attempt, seeds, hist, count, threads, stats);
}

/* ------------------------------------------- stb_image_write RGBE (v1.13) */
typedef struct {
  uint8_t *buf;
  int64_t cap, n;
} sink_t;
static void put(sink_t *s, const void *p, int64_t len) {
  if (s->buf && s->n + len <= s->cap) memcpy(s->buf + s->n, p, (size_t)len);
  s->n += len;
}
static void rgbe(uint8_t *o, const float *l) { /* stb_image_write.h:579-593 */
  float m = l[0] > (l[1] > l[2] ? l[1] : l[2]) ? l[0] : (l[1] > l[2] ? l[1] : l[2]);
  if (m < 1e-32f) {
    o[0] = o[1] = o[2] = o[3] = 0;
    return;
  }
  int e;
  float nm = frexpf(m, &e) * 256.0f / m;
  o[0] = (uint8_t)(int)(l[0] * nm);
  o[1] = (uint8_t)(int)(l[1] * nm);
  o[2] = (uint8_t)(int)(l[2] * nm);
  o[3] = (uint8_t)(e + 128);
}
int64_t oracle_encode_hdr(int32_t w, int32_t h, const float *rgba, int32_t flip, uint8_t *out, int64_t cap) {
  sink_t s = {out, cap, 0};
  const char *hd = "#?RADIANCE\n# Written by stb_image_write.h\nFORMAT=32-bit_rle_rgbe\n";
  put(&s, hd, (int64_t)strlen(hd));
  char b[128];
  int len = snprintf(b, sizeof b, "EXPOSURE=          1.0000000000000\n\n-Y %d +X %d\n", h, w);
  put(&s, b, len);
  uint8_t *scr = malloc((size_t)w * 4), px[4];
  for (int32_t i = 0; i < h; ++i) {
    const float *row = rgba + (int64_t)4 * w * (flip ? h - 1 - i : i);
    if (w < 8 || w >= 32768) {
      for (int32_t x = 0; x < w; ++x) rgbe(px, row + 4 * x), put(&s, px, 4);
      continue;
    }
    for (int32_t x = 0; x < w; ++x) {
      rgbe(px, row + 4 * x);
      for (int c = 0; c < 4; ++c) scr[x + w * c] = px[c];
    }
    uint8_t sh[4] = {2, 2, (uint8_t)((w & 0xff00) >> 8), (uint8_t)(w & 0xff)};
    put(&s, sh, 4);
    for (int c = 0; c < 4; ++c) {
      const uint8_t *cp = scr + (size_t)w * c;
      int x = 0;
      while (x < w) {
        int r = x;
        while (r + 2 < w && !(cp[r] == cp[r + 1] && cp[r] == cp[r + 2])) ++r;
        if (r + 2 >= w) r = w;
        while (x < r) {
          int l = r - x > 128 ? 128 : r - x;
          uint8_t lb = (uint8_t)l;
          put(&s, &lb, 1);
          put(&s, cp + x, l);
          x += l;
        }
        if (r + 2 < w) {
          while (r < w && cp[r] == cp[x]) ++r;
          while (x < r) {
            int l = r - x > 127 ? 127 : r - x;
            uint8_t rb[2] = {(uint8_t)(l + 128), cp[x]};
            put(&s, rb, 2);
            x += l;
          }
        }
      }
    }
  }
  free(scr);
  return s.n;
}

/* ----------------------------------------------- BVH metrics (testbvh) */
static float host_area(const mcpt_bvh_node *b) { /* auxiliary.cpp:15-18 */
  float x = b->bbmax[0] - b->bbmin[0], y = b->bbmax[1] - b->bbmin[1], z = b->bbmax[2] - b->bbmin[2];
  return 2.0f * (x * y + x * z + y * z);
}

float oracle_bvh_sah(const mcpt_bvh_node *node, int64_t size) { /* bvhtest.cpp:97-108 */
  double sahAns = 0.0f;
  for (int64_t i = 0; i < (size >> 1); ++i) sahAns += 1.2f * host_area(&node[i]);
  for (int64_t i = (size >> 1); i < size; ++i) sahAns += 1.0f * host_area(&node[i]);
  sahAns /= host_area(&node[0]);
  return (float)sahAns;
}

/* LCV (bvhtest.cpp:324-444), literally: rays pushed i (width) outer, j inner;
 * cl_float4 host operators; intersectBox with std::min/std::max. */
static int lcv_box(const float *o, const float *d, const mcpt_bvh_node *b) { /* bvhtest.cpp:23-34 */
  float mn[3], mx[3];
  for (int a = 0; a < 3; ++a) {
    float off1 = (b->bbmin[a] - o[a]) / d[a];
    float off2 = (b->bbmax[a] - o[a]) / d[a];
    mn[a] = (off2 < off1) ? off2 : off1;
    mx[a] = (off1 < off2) ? off2 : off1;
  }
  float t0 = (mn[1] < mn[0]) ? mn[0] : mn[1]; /* std::max(a, b) = (a < b) ? b : a */
  t0 = (t0 < mn[2]) ? mn[2] : t0;
  float t1 = (mx[1] < mx[0]) ? mx[1] : mx[0]; /* std::min(a, b) = (b < a) ? b : a */
  t1 = (mx[2] < t1) ? mx[2] : t1;
  return !(t1 < t0 || t1 < 0.001f);
}

float oracle_bvh_lcv(const mcpt_bvh_node *node, int64_t n_nodes, const mcpt_camera *cam, int32_t W, int32_t H,
                     uint32_t *counts) {
  int32_t *stack = malloc(sizeof(int32_t) * (size_t)(n_nodes + 1));
  double En = 0.0, En2 = 0.0;
  const float distance = 0.5f / tanf(cam->arg / 2);
  for (int32_t i = 0; i < W; ++i) {
    for (int32_t j = 0; j < H; ++j) {
      float temp1 = (i + 0.5f) / W - 0.5f;
      float temp2 = (j + 0.5f) / H - 0.5f;
      float o[3], d[3];
      for (int a = 0; a < 3; ++a) {
        o[a] = cam->center[a];
        d[a] = distance * cam->direction[a] + temp1 * cam->horizontal[a] + temp2 * cam->up[a];
      }
      uint64_t ans = 0;
      int64_t sp = 0;
      int32_t pt = 0;
      for (;;) {
        if (lcv_box(o, d, &node[pt])) {
          if (node[pt].left == node[pt].right) {
            ++ans;
          } else {
            stack[sp++] = node[pt].right;
            pt = node[pt].left;
            continue;
          }
        }
        if (sp == 0) break;
        pt = stack[--sp];
      }
      if (counts) counts[(int64_t)i * H + j] = (uint32_t)ans;
      En += (double)ans;
      En2 += (double)(ans * ans);
    }
  }
  free(stack);
  En /= (double)W * H;
  En2 /= (double)W * H;
  return (float)sqrt(En2 - En * En);
}

/* EPO.cl:1-197 calculateEPO on the CPU: fmaf where OpenCL contracts, libm
 * sqrtf and IEEE '/' for the GPU's 3-ulp sqrt / 2.5-ulp division (so values
 * agree to a few ulp, not bit for bit: tests state the tolerance). */
typedef struct {
  float s[3];
} v3_t;
static float o_len3(const float *a) {
  float l2 = fmaf(a[2], a[2], fmaf(a[1], a[1], a[0] * a[0]));
  if (l2 < FLT_MIN) {
    float q[3] = {a[0] * 0x1p86f, a[1] * 0x1p86f, a[2] * 0x1p86f};
    return sqrtf(fmaf(q[2], q[2], fmaf(q[1], q[1], q[0] * q[0]))) * 0x1p-86f;
  }
  if (isinf(l2)) {
    float q[3] = {a[0] * 0x1p-66f, a[1] * 0x1p-66f, a[2] * 0x1p-66f};
    return sqrtf(fmaf(q[2], q[2], fmaf(q[1], q[1], q[0] * q[0]))) * 0x1p66f;
  }
  return sqrtf(l2);
}
static float o_cross_len(const float *a, const float *b) {
  float c[3] = {fmaf(a[1], b[2], b[1] * -a[2]), fmaf(a[2], b[0], b[2] * -a[0]), fmaf(a[0], b[1], b[0] * -a[1])};
  return o_len3(c);
}
static void o_round_tr(v3_t *pts, int *size, int axis, float pos, int arg) {
  if (*size == 0) return;
  v3_t buf[32];
  int bs = *size, ins[32], n = 0;
  for (int i = 0; i < bs; ++i) buf[i] = pts[i];
  for (int i = 0; i < bs; ++i) ins[i] = arg > 0 ? (buf[i].s[axis] >= pos) : (buf[i].s[axis] <= pos);
  for (int i = 0; i < bs; ++i) {
    int i1 = (i + 1 == bs) ? 0 : i + 1;
    if (!ins[i] && !ins[i1]) continue;
    if (ins[i] && ins[i1]) {
      if (n < 32) pts[n] = buf[i];
      ++n;
      continue;
    }
    if (ins[i]) {
      if (n < 32) pts[n] = buf[i];
      ++n;
    }
    float dir[3] = {buf[i1].s[0] - buf[i].s[0], buf[i1].s[1] - buf[i].s[1], buf[i1].s[2] - buf[i].s[2]};
    float t = (pos - buf[i].s[axis]) / dir[axis];
    v3_t p = {{fmaf(t, dir[0], buf[i].s[0]), fmaf(t, dir[1], buf[i].s[1]), fmaf(t, dir[2], buf[i].s[2])}};
    if (n < 32) pts[n] = p;
    ++n;
  }
  *size = n < 32 ? n : 32;
}
static float o_intersect(const mcpt_triangle *tr, const float *mn, const float *mx) {
  int in[3];
  for (int k = 0; k < 3; ++k) {
    const float *p = tr->v[k];
    in[k] = p[0] >= mn[0] && p[0] <= mx[0] && p[1] >= mn[1] && p[1] <= mx[1] && p[2] >= mn[2] && p[2] <= mx[2];
  }
  if (in[0] && in[1] && in[2]) {
    float e1[3], e2[3];
    for (int a = 0; a < 3; ++a) e1[a] = tr->v[1][a] - tr->v[0][a], e2[a] = tr->v[2][a] - tr->v[0][a];
    return o_cross_len(e1, e2) * 0.5f;
  }
  v3_t pts[32];
  int n = 3;
  for (int k = 0; k < 3; ++k)
    for (int a = 0; a < 3; ++a) pts[k].s[a] = tr->v[k][a];
  for (int a = 0; a < 3; ++a) o_round_tr(pts, &n, a, mn[a], 1);
  for (int a = 0; a < 3; ++a) o_round_tr(pts, &n, a, mx[a], -1);
  float ans = 0.0f;
  if (n < 2) return ans;
  for (int i = 1; i < n - 1; ++i) {
    float x1[3], x2[3];
    for (int a = 0; a < 3; ++a) x1[a] = pts[i].s[a] - pts[0].s[a], x2[a] = pts[i + 1].s[a] - pts[0].s[a];
    ans = fmaf(o_cross_len(x1, x2), 0.5f, ans);
  }
  return ans;
}

void oracle_bvh_epo(const mcpt_bvh_node *bvh, const mcpt_triangle *tris, int64_t num, float *epo, float *area) {
#pragma omp parallel for schedule(dynamic, 64)
  for (int64_t gid = 0; gid < num; ++gid) {
    int64_t my = gid + num - 1;
    const mcpt_triangle *tr = &tris[bvh[my].left];
    float e = 0.0f;
    int anc[256], an = 1, stk[256], sp = 1;
    anc[0] = (int)my;
    for (int p = bvh[my].parent; p != -1 && an < 256; p = bvh[p].parent) anc[an++] = p;
    stk[0] = 0;
    while (sp > 0) {
      int now = stk[--sp], skip = 0;
      const mcpt_bvh_node *b = &bvh[now];
      for (int i = 0; i < an; ++i)
        if (now == anc[i]) {
          if (b->left != b->right && sp + 2 <= 256) stk[sp++] = b->right, stk[sp++] = b->left;
          skip = 1;
          break;
        }
      if (skip) continue;
      float ta = o_intersect(tr, b->bbmin, b->bbmax);
      if (ta > 0) {
        e = fmaf(ta, (now >= num - 1) ? 1.0f : 1.2f, e);
        if (b->left != b->right && sp + 2 <= 256) stk[sp++] = b->right, stk[sp++] = b->left;
      }
    }
    epo[gid] = e;
    float e1[3], e2[3];
    for (int a = 0; a < 3; ++a) e1[a] = tr->v[1][a] - tr->v[0][a], e2[a] = tr->v[2][a] - tr->v[0][a];
    area[gid] = o_cross_len(e1, e2) * 0.5f;
  }
}
