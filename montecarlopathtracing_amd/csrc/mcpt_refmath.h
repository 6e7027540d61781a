// mcpt_refmath.h — device-side arithmetic of the reference's OpenCL kernels,
// restated for gfx950 HIP so that the HIP path computes the SAME IEEE
// operations the reference kernels do when compiled for this GPU.
//
// How bit-exactness is obtained:
//  * the translation unit is compiled with -ffp-contract=on (OpenCL's default
//    FP_CONTRACT ON: a*b+c inside ONE expression becomes llvm.fmuladd, which
//    gfx950 always fuses) and -fno-hip-fp32-correctly-rounded-divide-sqrt
//    (OpenCL's default 2.5-ulp '/' and 3-ulp sqrt: !fpmath metadata);
//  * vectors are clang ext_vector_type, exactly OpenCL's float4/float3, so
//    every expression below has the reference's expression tree;
//  * the OpenCL built-ins are restated from ROCm's opencl.bc / ocml.bc
//    (dot = fma chain, cross = fma, normalize = p * rsqrt(dot) with the
//    denormal/overflow rescaling branches) and the transcendental ones call
//    the very same __ocml_* entry points the OpenCL library calls.
// LLVM applies no value-changing rewrite without fast-math flags, so equal
// expression trees give equal bits, whatever the control flow around them.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mcpt {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f3 __attribute__((ext_vector_type(3)));

constexpr float kEps = 1e-5f;          // objdef.h:16 (device EPSILON)
constexpr float kFltMax = 3.402823466e+38f;
constexpr double kClPi = 3.141592653589793115997963468544185161590576171875;  // OpenCL M_PI (double)

__device__ inline float as_f(int32_t i) { return __builtin_bit_cast(float, i); }
__device__ inline int32_t as_i(float f) { return __builtin_bit_cast(int32_t, f); }
__device__ inline uint32_t as_u(float f) { return __builtin_bit_cast(uint32_t, f); }

// ------------------------------------------------------------ built-ins
// dot(float3)/dot(float4): opencl.bc _Z3dotDv3_fS_/_Z3dotDv4_fS_
__device__ inline float cl_dot3(f3 a, f3 b) {
  return __builtin_fmaf(a.z, b.z, __builtin_fmaf(a.y, b.y, a.x * b.x));
}
__device__ inline float cl_dot4(f4 a, f4 b) {
  return __builtin_fmaf(a.w, b.w, __builtin_fmaf(a.z, b.z, __builtin_fmaf(a.y, b.y, a.x * b.x)));
}
// cross(float4): opencl.bc _Z5crossDv4_fS_ (w = 0)
__device__ inline f4 cl_cross(f4 a, f4 b) {
  f4 r;
  r.x = __builtin_fmaf(a.y, b.z, b.y * -a.z);
  r.y = __builtin_fmaf(a.z, b.x, b.z * -a.x);
  r.z = __builtin_fmaf(a.x, b.y, b.x * -a.y);
  r.w = 0.0f;
  return r;
}
// normalize(float4): opencl.bc _Z9normalizeDv4_f, with two steps reordered
// for fewer instructions on the common path, same value for every input:
//  * the all-zero test (return p) moved inside the small-l2 branch: an
//    all-zero p has l2 = +0 and reaches it, any other p returns from the
//    same arithmetic either way;
//  * ocml's rsqrt scales an argument below 2^-126 before v_rsq_f32; l2 is
//    never below 2^-126 there (a non-zero p rescaled by 2^86 has a
//    component of at least 2^-63, the inf branch ends at >= 1 or NaN), so
//    its v_rsq_f32 is taken directly.
__device__ inline f4 cl_normalize(f4 p) {
  float l2 = cl_dot4(p, p);
  f4 q = p;
  if (l2 < 0x1p-126f) {
    if (p.x == 0.0f && p.y == 0.0f && p.z == 0.0f && p.w == 0.0f) return p;
    q = p * 0x1p86f;
    l2 = cl_dot4(q, q);
  } else if (l2 == __builtin_inff()) {
    q = p * 0x1p-66f;
    l2 = cl_dot4(q, q);
    if (l2 == __builtin_inff()) {
      f4 one;
      one.x = __builtin_isinf(q.x) ? 1.0f : 0.0f;
      one.y = __builtin_isinf(q.y) ? 1.0f : 0.0f;
      one.z = __builtin_isinf(q.z) ? 1.0f : 0.0f;
      one.w = __builtin_isinf(q.w) ? 1.0f : 0.0f;
      q = __builtin_elementwise_copysign(one, q);
      l2 = cl_dot4(q, q);
    }
  }
  return q * __builtin_amdgcn_rsqf(l2);
}
// OpenCL's default sqrt: llvm.sqrt with !fpmath 3.0, which gfx950 lowers to
// v_sqrt_f32 with denormal range scaling (x < 2^-126: sqrt(x * 2^32) * 2^-16).
// Written out with the raw instruction because LLVM drops !fpmath when it
// hoists or speculates a sqrt, and then emits the correctly rounded sequence.
__device__ inline float cl_sqrt(float x) {
  const bool s = x < 0x1p-126f;
  const float r = __builtin_amdgcn_sqrtf(__builtin_amdgcn_ldexpf(x, s ? 32 : 0));
  return __builtin_amdgcn_ldexpf(r, s ? -16 : 0);
}
// OpenCL's default 2.5-ulp x / y as ROCm's compiler lowers it for gfx950 —
// the form of every division in the reference's shade.cl and history.cl
// objects (oracle/_ref: no v_div_scale there): ldexp(frexp_mant(x) *
// rcp(frexp_mant(y)), ex - ey).  A constant y's rcp folds at compile time
// exactly as it does there.  Written out for the same reason as cl_sqrt: a
// '/' that LLVM hoists or speculates loses its !fpmath and becomes the
// correctly rounded v_div_scale sequence (it did in the restructured shade).
__device__ inline float cl_div(float x, float y) {
  return __builtin_amdgcn_ldexpf(__builtin_amdgcn_frexp_mantf(x) * __builtin_amdgcn_rcpf(__builtin_amdgcn_frexp_mantf(y)),
                                 __builtin_amdgcn_frexp_expf(x) - __builtin_amdgcn_frexp_expf(y));
}
__device__ inline f4 cl_div4(f4 x, float y) {
  return (f4){cl_div(x.x, y), cl_div(x.y, y), cl_div(x.z, y), cl_div(x.w, y)};
}
// length(float4): opencl.bc _Z6lengthDv4_f
__device__ inline float cl_length4(f4 p) {
  float l2 = cl_dot4(p, p);
  if (l2 < 0x1p-126f) {
    f4 q = p * 0x1p86f;
    return cl_sqrt(cl_dot4(q, q)) * 0x1p-86f;
  }
  if (l2 == __builtin_inff()) {
    f4 q = p * 0x1p-66f;
    return cl_sqrt(cl_dot4(q, q)) * 0x1p66f;
  }
  return cl_sqrt(l2);
}
__device__ inline float cl_pow(float x, float y) { return __ocml_pow_f32(x, y); }
// shade.cl:139's pow(cos_r, Ns) for the ranges the Phong lobe reaches: ocml's
// pow_f32 (ROCm device libs, gfx950: the fma forms, no unsafe math) is an
// extended-precision log (__ocmlpriv_epln_f32), y x log in double-float,
// exp with a correction (__ocmlpriv_expep_f32), then ~40 instructions of
// special cases (zero, negative, infinite, NaN operands, odd-integer
// exponents, overflow).  For x in (0, 1 + 2^-10] and y in [0, 65536] none of
// those cases applies: y x log(x) <= 64 stays finite and below expep's 88.72
// threshold, exp and the result are finite and >= +0, so ocml returns the
// core's value unchanged.  The same operations on that domain: the same bits
// (mcpt_selfcheck_pow compares every float of the domain, for the scenes'
// exponents, against __ocml_pow_f32); outside it, ocml itself.
typedef float f2v_ __attribute__((ext_vector_type(2)));
extern "C" __device__ f2v_ __ocmlpriv_epln_f32(float);
__device__ inline float cl_pow_lobe(float x, float y) {
  if (!(x > 0.0f && x <= 0x1.004p0f && y >= 0.0f && y <= 65536.0f)) return __ocml_pow_f32(x, y);
  const float yy = x == 1.0f ? 1.0f : y;   // ocml: pow(1, y) takes y = 1
  const float xx = yy == 0.0f ? 1.0f : x;  // and pow(x, 0) takes x = 1
  const f2v_ e = __ocmlpriv_epln_f32(xx);  // log(xx) as hi (.y) + lo (.x)
  const float hi = yy * e.y;
  const float lo = __builtin_fmaf(yy, e.x, __builtin_fmaf(yy, e.y, -hi));
  const float s = hi + lo;
  const float rlo = lo - (s - hi);
  const float ex = __ocml_exp_f32(s);  // expep: exp(hi), then fma(e, lo, e)
  return __builtin_fmaf(ex, rlo, ex);
}
__device__ inline float cl_cos(float x) { return __ocml_cos_f32(x); }
__device__ inline float cl_sin(float x) { return __ocml_sin_f32(x); }
__device__ inline float cl_tan(float x) { return __ocml_tan_f32(x); }

// ------------------------------------------------------------- shade.cl
// random(): shade.cl:1-6 — 32-bit LCG, 15-bit output
__device__ inline uint32_t lcg15(uint32_t &s) {
  s = s * 1103515245u + 12345u;
  return (s >> 16) & 0x00007FFFu;
}
// mirrorDirection: shade.cl:19-25
__device__ inline f4 mirror_dir(f4 n, f4 in) {
  n.w = 0.0f;
  in.w = 0.0f;
  f4 r = in - 2 * cl_dot4(n, in) * n;
  r.w = 0.0f;
  return cl_normalize(r);
}
// transmittedDirection: shade.cl:27-38
__device__ inline bool transmit_dir(f4 n, f4 in, float eta_i, float eta_t, f4 &out) {
  n.w = 0.0f;
  in.w = 0.0f;
  float eta = cl_div(eta_i, eta_t);
  float cos_i = -cl_dot4(n, in);
  float k = 1.0f - eta * eta * (1 - cos_i * cos_i);
  if (k < 0.0f) return false;
  out = cl_normalize((eta * cos_i - cl_sqrt(k)) * n + eta * in);
  return true;
}
// sin and cos of 0 <= x < 131072, bit-identical to __ocml_sin_f32 /
// __ocml_cos_f32 there: the gfx9 branch of ocml's __ocmlpriv_trigredsmall_f32
// (3-term Cody-Waite reduction by pi/2, quadrant = rint(x*2/pi) & 3) and
// __ocmlpriv_sincosred_f32's two minimax polynomials (its llvm.fmuladd calls
// are the a*b+c forms below under -ffp-contract=on). ocml selects the
// Payne-Hanek reduction for |x| >= 131072; randomDirection's angle is always
// below 2*pi, so keeping that branch out of the kernel drops its 64-bit
// multiply chain and the registers it holds. Checked exhaustively over all
// 32768 angles against the ocml calls by mcpt_selfcheck_trig.
__device__ inline void sincos_small(float x, float &s, float &c) {
  const float t = __builtin_rintf(x * 0x1.45f306p-1f);
  float r = __builtin_fmaf(t, -0x1.921fb4p+0f, x);
  r = __builtin_fmaf(t, -0x1.4442d0p-24f, r);
  r = __builtin_fmaf(t, -0x1.846988p-48f, r);
  const int q = (int)t & 3;
  const float r2 = r * r;
  float p = r2 * -0x1.983304p-13f + 0x1.110388p-7f;
  p = r2 * p + -0x1.55553ap-3f;
  const float sr = r * (r2 * p) + r;
  float k = r2 * 0x1.aea668p-16f + -0x1.6c9e76p-10f;
  k = r2 * k + 0x1.5557eep-5f;
  k = r2 * k + -0x1.000008p-1f;
  const float cr = r2 * k + 1.0f;
  const uint32_t flip = q > 1 ? 0x80000000u : 0u;
  s = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, (q & 1) ? cr : sr) ^ flip);
  c = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, (q & 1) ? -sr : cr) ^ flip);
}
// randomDirection's angle for a 15-bit draw: formed in double (OpenCL M_PI
// is a double constant), then rounded to float (shade.cl:40-59).
__device__ inline float random_phi(uint32_t r) { return (float)(2 * kClPi / 32768 * (double)r); }

// randomDirection: shade.cl:40-59 — the angle is formed in double, the radius
// in float.
__device__ inline f4 random_dir(f4 n, uint32_t &seed) {
  n.w = 0;
  float phi = random_phi(lcg15(seed));
  float u = lcg15(seed) * 1.0f * 0x1p-15f;  // = the 2.5-ulp x / 32768: both exact for x < 2^24
  float s = __builtin_amdgcn_sqrtf(u);        // = cl_sqrt(u): u is 0 or >= 2^-15, never scaled
  float sin_phi, cos_phi;
  sincos_small(phi, sin_phi, cos_phi);
  f4 a1, a2;
  if (n.z == 0) {
    a1 = (f4){0, 0, 1.0f, 0};
  } else {
    a1 = (f4){1, 0, 0, 0};
  }
  a2 = cl_normalize(cl_cross(a1, n));
  a1 = cl_normalize(cl_cross(a2, n));
  return cl_normalize(cos_phi * s * a1 + sin_phi * s * a2 + (1 - u) * n);
}
// calcFresnel: shade.cl:69-73 (Schlick on the transmitted direction)
__device__ inline float fresnel(f4 n, f4 d, float ior) {
  float k = cl_pow(cl_div(ior - 1, ior + 1), 2.0f);
  return k + (1 - k) * cl_pow(1 - __builtin_fabsf(cl_dot3(n.xyz, d.xyz)), 5.0f);
}

// --------------------------------------------------------- objdef.h tests
// Cramer's rule on the 4x4 system of intersectTriangle (objdef.h:102-221).
// The minors are written with the reference's expression shapes; only the
// nine cofactors t/b/c need are evaluated, in an early-out order.
__device__ inline float m2(float a, float b, float c, float d) { return a * d - b * c; }
__device__ inline float m3(float a1, float a2, float a3, float b1, float b2, float b3, float c1,
                           float c2, float c3) {
  return a1 * m2(b2, b3, c2, c3) - b1 * m2(a2, a3, c2, c3) + c1 * m2(a2, a3, b2, b3);
}

struct TriHit {
  float t;
  bool accept;  // passed every test (the reference's "return true")
};

// rd: ray direction, nab = -(v1 - v0), nac = -(v2 - v0), aro = v0 - origin,
// realn: triangle normal.  Row layout of the reference matrix:
//   a = (rd, 0)  b = (nab, 0)  c = (nac, 0)  d = (0, 0, 0, 1)
__device__ inline TriHit cramer(f3 rd, f3 nab, f3 nac, f3 aro, f3 realn, float tmin) {
  TriHit r;
  r.accept = false;
  r.t = 0.0f;
  if (__builtin_fabsf(cl_dot3(realn, rd)) < kEps) return r;
  const float a1 = rd.x, a2 = rd.y, a3 = rd.z, a4 = 0.0f;
  const float b1 = nab.x, b2 = nab.y, b3 = nab.z, b4 = 0.0f;
  const float c1 = nac.x, c2 = nac.y, c3 = nac.z, c4 = 0.0f;
  const float d1 = 0.0f, d2 = 0.0f, d3 = 0.0f, d4 = 1.0f;
  float det = a1 * m3(b2, b3, b4, c2, c3, c4, d2, d3, d4) - b1 * m3(a2, a3, a4, c2, c3, c4, d2, d3, d4) +
              c1 * m3(a2, a3, a4, b2, b3, b4, d2, d3, d4) - d1 * m3(a2, a3, a4, b2, b3, b4, c2, c3, c4);
  if (__builtin_fabsf(det) < kEps) return r;
  // b = dot(A_Ro, (s1, s5, s9))
  float s1 = -m3(a2, a3, a4, c2, c3, c4, d2, d3, d4) / det;
  float s5 = m3(a1, a3, a4, c1, c3, c4, d1, d3, d4) / det;
  float s9 = -m3(a1, a2, a4, c1, c2, c4, d1, d2, d4) / det;
  float bb = cl_dot3(aro, (f3){s1, s5, s9});
  if (bb < 0) return r;
  // c = dot(A_Ro, (s2, s6, s10))
  float s2 = m3(a2, a3, a4, b2, b3, b4, d2, d3, d4) / det;
  float s6 = -m3(a1, a3, a4, b1, b3, b4, d1, d3, d4) / det;
  float sa = m3(a1, a2, a4, b1, b2, b4, d1, d2, d4) / det;
  float cc = cl_dot3(aro, (f3){s2, s6, sa});
  if (cc < 0 || bb + cc > 1) return r;
  // t = dot(A_Ro, (s0, s4, s8)); s0 == FLT_MAX is the reference's singular flag
  float s0 = m3(b2, b3, b4, c2, c3, c4, d2, d3, d4) / det;
  if (s0 == kFltMax) return r;
  float s4 = -m3(b1, b3, b4, c1, c3, c4, d1, d3, d4) / det;
  float s8 = m3(b1, b2, b4, c1, c2, c4, d1, d2, d4) / det;
  float t = cl_dot3(aro, (f3){s0, s4, s8});
  if (t <= tmin) return r;
  r.t = t;
  r.accept = true;
  return r;
}

// The same test with the reference matrix's constant entries eliminated.
// Row a = (rd, 0), b = (-(v1-v0), 0), c = (-(v2-v0), 0), d = (0, 0, 0, 1):
// every minor above then reduces to ONE contracted 2x2 term, e.g.
//   m3(b2,b3,0, c2,c3,0, 0,0,1) = fma(0, +-0, fma(b2, m2(c3,0,0,1), -(c2*m2(b3,0,0,1))))
//                              = fma(b2, c3, -(c2*b3))            (exactly)
// because x*1 = x, y + (+-0) = y and x*0 = +-0 for finite x (vertices are
// checked finite at upload); only the sign of an exactly-zero intermediate can
// differ, and a zero b/c/t/det compares identically with either sign.  The
// three triangle-only minors come precomputed (same fma, on the host):
//   m_x1 = fma(b2,c3,-(c2*b3)), m_y4 = fma(b1,c3,-(c1*b3)), m_y8 = fma(b1,c2,-(c1*b2)).
// The nine quotients use x * rcp(det) for the reference's 2.5-ulp x / det
// (= ldexp(mant(x)*rcp(mant(det)), ex-edet)): identical whenever the quotient
// is a normal float, i.e. unless a cofactor quotient falls below 2^-126.
__device__ inline TriHit cramer_reduced(f3 rd, f3 nab, f3 nac, f3 aro, f3 realn, float m_x1, float m_y4,
                                        float m_y8, float tmin) {
  TriHit r;
  r.accept = false;
  r.t = 0.0f;
  if (__builtin_fabsf(cl_dot3(realn, rd)) < kEps) return r;
  const float a1 = rd.x, a2 = rd.y, a3 = rd.z;
  const float b1 = nab.x, b2 = nab.y, b3 = nab.z;
  const float c1 = nac.x, c2 = nac.y, c3 = nac.z;
  const float x2 = __builtin_fmaf(a2, c3, -(c2 * a3));
  const float x3 = __builtin_fmaf(a2, b3, -(b2 * a3));
  const float det = __builtin_fmaf(c1, x3, __builtin_fmaf(a1, m_x1, -(b1 * x2)));
  if (__builtin_fabsf(det) < kEps) return r;
  const float rdet = __builtin_amdgcn_rcpf(det);
  // b = dot(A_Ro, (s1, s5, s9))
  const float s1 = -x2 * rdet;
  const float s5 = __builtin_fmaf(a1, c3, -(c1 * a3)) * rdet;
  const float s9 = -__builtin_fmaf(a1, c2, -(c1 * a2)) * rdet;
  const float bb = cl_dot3(aro, (f3){s1, s5, s9});
  if (bb < 0) return r;
  // c = dot(A_Ro, (s2, s6, s10))
  const float s2 = x3 * rdet;
  const float s6 = -__builtin_fmaf(a1, b3, -(b1 * a3)) * rdet;
  const float sa = __builtin_fmaf(a1, b2, -(b1 * a2)) * rdet;
  const float cc = cl_dot3(aro, (f3){s2, s6, sa});
  if (cc < 0 || bb + cc > 1) return r;
  const float s0 = m_x1 * rdet;
  if (s0 == kFltMax) return r;
  const float s4 = -m_y4 * rdet;
  const float s8 = m_y8 * rdet;
  const float t = cl_dot3(aro, (f3){s0, s4, s8});
  if (t <= tmin) return r;
  r.t = t;
  r.accept = true;
  return r;
}

// intersectAABB (objdef.h:223-237).  (bb - o) / d under the 2.5-ulp OpenCL
// division is ldexp(mant(x) * rcp(mant(d)), ex - ed) == x * rcp(d) for every
// normal-range quotient; rcp(d) is hoisted per ray (verified on the GPU
// against the literal division, tests/test_gpu_parity.py).
struct BoxT {
  float tnear, tfar;
};
__device__ inline BoxT slab(f3 bmin, f3 bmax, f3 o, f3 rinv) {
  f3 t1 = (bmin - o) * rinv;
  f3 t2 = (bmax - o) * rinv;
  BoxT r;
  r.tnear = fmaxf(fmaxf(fminf(t1.x, t2.x), fminf(t1.y, t2.y)), fminf(t1.z, t2.z));
  r.tfar = fminf(fminf(fmaxf(t1.x, t2.x), fmaxf(t1.y, t2.y)), fmaxf(t1.z, t2.z));
  return r;
}
__device__ inline bool slab_pass(BoxT b, float tmin) { return !(b.tfar < b.tnear || b.tfar < tmin); }

}  // namespace mcpt
