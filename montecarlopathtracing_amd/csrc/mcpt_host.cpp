// mcpt_host.cpp — host half of libmcpt_hip.so: the scene-side code the
// reference runs on the CPU before/after the per-sample loop.
//
//   parseCamera            MCPT/auxiliary.cpp:20-71
//   material classification MCPT/thirdpartywrapper.cpp:65-97
//   OBJ/MTL loading        MCPT/thirdpartywrapper.cpp:25-63 (+ tinyobjloader 2.0.0rc number
//                          parsing, MCPT/tiny_obj_loader.h:805-954)
//   triangle packing       MCPT/scenebuild.cpp:58-62
//   HLBVH build            MCPT/BVH/hlbvh.cpp:12-200
//   RGBE (.hdr) writer     MCPT/thirdpartywrapper.cpp:14-23 -> stb_image_write v1.13 (:579-724)
//
// Host arithmetic follows the reference host build: IEEE binary32, no FMA
// contraction (MSVC /fp:precise on SSE2), so this file is compiled with
// -ffp-contract=off.
#include "../../include/mcpt_hip.h"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

namespace mcpt {
// thread-local last error shared with the device half (mcpt_device.hip)
thread_local std::string g_last_error;
int fail(int code, const std::string &msg) {
  g_last_error = msg;
  return code;
}
}  // namespace mcpt

using mcpt::fail;

namespace {

// host float4 helpers with the reference host semantics (MCPT/oclbasic.h:119-237):
// component loops over all 4 lanes, plain IEEE ops, std::min/std::max.
struct V4 {
  float s[4];
};
inline V4 v4(const float *p) { return V4{{p[0], p[1], p[2], p[3]}}; }
inline V4 sub(const V4 &a, const V4 &b) {
  V4 r;
  for (int i = 0; i < 4; ++i) r.s[i] = a.s[i] - b.s[i];
  return r;
}
inline V4 add(const V4 &a, const V4 &b) {
  V4 r;
  for (int i = 0; i < 4; ++i) r.s[i] = a.s[i] + b.s[i];
  return r;
}
inline V4 vmin(const V4 &a, const V4 &b) {
  V4 r;
  for (int i = 0; i < 4; ++i) r.s[i] = std::min(a.s[i], b.s[i]);
  return r;
}
inline V4 vmax(const V4 &a, const V4 &b) {
  V4 r;
  for (int i = 0; i < 4; ++i) r.s[i] = std::max(a.s[i], b.s[i]);
  return r;
}
inline V4 cross_host(const V4 &a, const V4 &b) {  // oclbasic.h:119-127 (w = 0)
  V4 r{{0, 0, 0, 0}};
  r.s[0] = a.s[1] * b.s[2] - a.s[2] * b.s[1];
  r.s[1] = -a.s[0] * b.s[2] + a.s[2] * b.s[0];
  r.s[2] = a.s[0] * b.s[1] - a.s[1] * b.s[0];
  return r;
}
inline float dot_host(const V4 &a, const V4 &b) {  // oclbasic.h:129-137: float sum from 0
  float acc = 0.0f;
  for (int i = 0; i < 4; ++i) acc += a.s[i] * b.s[i];
  return acc;
}
inline V4 normalize_host(const V4 &a) {  // oclbasic.h:139-147: divide by sqrtf(dot)
  float len = std::sqrt(dot_host(a, a));
  V4 r = a;
  for (int i = 0; i < 4; ++i) r.s[i] /= len;
  return r;
}
inline void store(float *dst, const V4 &v) { std::memcpy(dst, v.s, 16); }

// The reference host's pi (oclbasic.h:192) — deliberately short.
constexpr double kRefPi = 3.14159265358;

}  // namespace

extern "C" {

const char *mcpt_last_error(void) { return mcpt::g_last_error.c_str(); }

int mcpt_parse_camera(const double position[3], const double lookat[3], const double up[3],
                      double fov_deg, mcpt_camera *out) {
  if (!position || !lookat || !up || !out) return fail(MCPT_ERR_ARG, "parse_camera: null argument");
  mcpt_camera c;
  std::memset(&c, 0, sizeof(c));
  V4 center{{0, 0, 0, 0}}, look{{0, 0, 0, 0}}, upv{{0, 0, 0, 0}};
  for (int i = 0; i < 3; ++i) {
    center.s[i] = (float)position[i];
    look.s[i] = (float)lookat[i];
    upv.s[i] = (float)up[i];
  }
  V4 dir = sub(look, center);
  dir.s[3] = 0.0f;
  // fov: float(json) * M_PI / 180.0f evaluated in double, stored as float
  c.arg = (float)((double)(float)fov_deg * kRefPi / 180.0f);
  V4 horizontal = cross_host(dir, upv);
  V4 realup = cross_host(horizontal, dir);
  c.tmin = 0.0f;
  c.camera_type = 0;  // always perspective (auxiliary.cpp:22)
  store(c.center, center);
  store(c.direction, normalize_host(dir));
  store(c.up, normalize_host(realup));
  store(c.horizontal, normalize_host(horizontal));
  *out = c;
  return MCPT_OK;
}

int mcpt_classify_material(float ior, const float ambient[3], const float diffuse[3],
                           const float specular[3], float shininess, mcpt_material *out) {
  if (!ambient || !diffuse || !specular || !out) return fail(MCPT_ERR_ARG, "classify_material: null argument");
  mcpt_material m;
  std::memset(&m, 0, sizeof(m));
  if (ior != 1.0f) {
    m.type = MCPT_TRANSPARENT;
    m.Ni = ior;
  } else if (ambient[0] > 0.0f || ambient[1] > 0.0f || ambient[2] > 0.0f) {
    m.type = MCPT_LIGHT;
    for (int i = 0; i < 3; ++i) m.ka_ks[i] = ambient[i];
  } else if (shininess != 1.0f) {
    m.type = MCPT_GLOSSY;
    m.Ns = shininess;
    // (Ns + 2) * (2.0 / M_PI) * ks: scalar deduced as double, per-lane double product
    double sc = (double)(shininess + 2) * (2.0 / kRefPi);
    for (int i = 0; i < 3; ++i) m.ka_ks[i] = (float)(sc * (double)specular[i]);
    for (int i = 0; i < 3; ++i) m.kd[i] = (float)((1.0 / kRefPi) * (double)diffuse[i]);
  } else {
    m.type = MCPT_DIFFUSE;
    for (int i = 0; i < 3; ++i) m.kd[i] = (float)((1.0 / kRefPi) * (double)diffuse[i]);
  }
  *out = m;
  return MCPT_OK;
}

}  // extern "C"

// ------------------------------------------------------------------ OBJ / MTL
namespace {

// tinyobjloader's number reader: digits accumulated in double, fraction digits
// weighted by 10^-k, exponent applied as ldexp(m * 5^e, e); result cast to float.
bool parse_number(const char *s, const char *end, double *out) {
  if (s >= end) return false;
  const char *p = s;
  double mant = 0.0;
  int exponent = 0, ndig = 0;
  char sign = '+', esign = '+';
  bool leading_dot = false;
  if (*p == '+' || *p == '-') {
    sign = *p++;
    if (p != end && *p == '.') leading_dot = true;
  } else if (*p >= '0' && *p <= '9') {
  } else if (*p == '.') {
    leading_dot = true;
  } else {
    return false;
  }
  bool more = p != end;
  if (!leading_dot) {
    while (more && *p >= '0' && *p <= '9') {
      mant *= 10;
      mant += (int)(*p - '0');
      ++p, ++ndig;
      more = p != end;
    }
    if (ndig == 0) return false;
  }
  if (!more) goto done;
  if (*p == '.') {
    ++p;
    int k = 1;
    more = p != end;
    static const double lut[] = {1.0, 0.1, 0.01, 0.001, 0.0001, 0.00001, 0.000001, 0.0000001};
    while (more && *p >= '0' && *p <= '9') {
      mant += (int)(*p - '0') * (k < 8 ? lut[k] : std::pow(10.0, -k));
      ++k, ++p;
      more = p != end;
    }
  } else if (*p == 'e' || *p == 'E') {
  } else {
    goto done;
  }
  if (!more) goto done;
  if (*p == 'e' || *p == 'E') {
    ++p;
    more = p != end;
    if (more && (*p == '+' || *p == '-')) {
      esign = *p++;
    } else if (!(more && *p >= '0' && *p <= '9')) {
      return false;
    }
    int nexp = 0;
    more = p != end;
    while (more && *p >= '0' && *p <= '9') {
      exponent = exponent * 10 + (int)(*p - '0');
      ++p, ++nexp;
      more = p != end;
    }
    exponent *= (esign == '+' ? 1 : -1);
    if (nexp == 0) return false;
  }
done:
  *out = (sign == '+' ? 1 : -1) * (exponent ? std::ldexp(mant * std::pow(5.0, exponent), exponent) : mant);
  return true;
}

struct Tok {
  const char *p, *e;
};
Tok next_token(const char *&p, const char *end) {
  while (p < end && (*p == ' ' || *p == '\t')) ++p;
  const char *b = p;
  while (p < end && *p != ' ' && *p != '\t' && *p != '\r' && *p != '\n') ++p;
  return Tok{b, p};
}
float read_float(const char *&p, const char *end, double dflt) {
  Tok t = next_token(p, end);
  double v = dflt;
  parse_number(t.p, t.e, &v);
  return (float)v;
}

struct MtlRec {
  std::string name;
  float ka[3] = {0, 0, 0}, kd[3] = {0, 0, 0}, ks[3] = {0, 0, 0};
  float ns = 1.0f, ni = 1.0f;  // tinyobj defaults (tiny_obj_loader.h:1297-1298)
};

bool read_file(const std::string &path, std::string *out) {
  std::ifstream f(path, std::ios::binary);
  if (!f) return false;
  std::stringstream ss;
  ss << f.rdbuf();
  *out = ss.str();
  return true;
}

void parse_mtl(const std::string &text, std::vector<MtlRec> *mats, std::map<std::string, int> *index) {
  const char *p = text.data(), *end = p + text.size();
  MtlRec cur;
  bool have = false;
  auto flush = [&]() {
    if (have) {
      if (!index->count(cur.name)) (*index)[cur.name] = (int)mats->size();
      mats->push_back(cur);
    }
  };
  while (p < end) {
    const char *eol = (const char *)std::memchr(p, '\n', end - p);
    if (!eol) eol = end;
    const char *q = p;
    while (q < eol && (*q == ' ' || *q == '\t')) ++q;
    Tok key = next_token(q, eol);
    std::string k(key.p, key.e);
    auto rgb = [&](float *dst) {
      dst[0] = read_float(q, eol, 0.0);
      dst[1] = read_float(q, eol, 0.0);
      dst[2] = read_float(q, eol, 0.0);
    };
    if (k == "newmtl") {
      flush();
      cur = MtlRec();
      have = true;
      while (q < eol && (*q == ' ' || *q == '\t')) ++q;
      const char *ne = eol;
      while (ne > q && (ne[-1] == '\r' || ne[-1] == ' ' || ne[-1] == '\t')) --ne;
      cur.name.assign(q, ne);
    } else if (k == "Ka") {
      rgb(cur.ka);
    } else if (k == "Kd") {
      rgb(cur.kd);
    } else if (k == "Ks") {
      rgb(cur.ks);
    } else if (k == "Ns") {
      cur.ns = read_float(q, eol, 0.0);
    } else if (k == "Ni") {
      cur.ni = read_float(q, eol, 0.0);
    }
    p = eol + 1;
  }
  flush();
}

// fan/ear triangulation: convex polygons give (0,1,2), (0,2,3), ... which is
// what tinyobj's ear clipper (tiny_obj_loader.h:1359-1500) emits for them.
struct Face {
  int v[3];
  int mat;
};

}  // namespace

extern "C" int mcpt_load_obj(const char *directory, const char *objname, mcpt_triangle *tris,
                             int32_t *mat_index, int64_t *n_tris, mcpt_material *mats, int32_t *n_mats) {
  if (!directory || !objname || !n_tris || !n_mats) return fail(MCPT_ERR_ARG, "load_obj: null argument");
  std::string dir(directory), text;
  if (!read_file(dir + objname, &text)) return fail(MCPT_ERR_IO, "load_obj: cannot read " + dir + objname);
  std::vector<float> verts;
  std::vector<Face> faces;
  std::vector<MtlRec> mtl;
  std::map<std::string, int> mtl_index;
  int cur_mat = -1;
  const char *p = text.data(), *end = p + text.size();
  std::vector<int> poly;
  while (p < end) {
    const char *eol = (const char *)std::memchr(p, '\n', end - p);
    if (!eol) eol = end;
    const char *q = p;
    while (q < eol && (*q == ' ' || *q == '\t')) ++q;
    if (q + 1 < eol && q[0] == 'v' && (q[1] == ' ' || q[1] == '\t')) {
      q += 2;
      float x = read_float(q, eol, 0.0), y = read_float(q, eol, 0.0), z = read_float(q, eol, 0.0);
      verts.push_back(x), verts.push_back(y), verts.push_back(z);
    } else if (q + 1 < eol && q[0] == 'f' && (q[1] == ' ' || q[1] == '\t')) {
      q += 2;
      poly.clear();
      int nv = (int)(verts.size() / 3);
      for (;;) {
        Tok t = next_token(q, eol);
        if (t.p == t.e) break;
        int idx = std::atoi(std::string(t.p, t.e).c_str());  // "v", "v/vt", "v//vn", "v/vt/vn"
        if (idx == 0) return fail(MCPT_ERR_PARSE, "load_obj: bad face index");
        poly.push_back(idx > 0 ? idx - 1 : nv + idx);
      }
      if (poly.size() < 3) continue;  // tinyobj drops faces with < 3 vertices
      for (size_t k = 1; k + 1 < poly.size(); ++k) faces.push_back(Face{{poly[0], poly[k], poly[k + 1]}, cur_mat});
    } else if (eol - q >= 6 && std::strncmp(q, "usemtl", 6) == 0 && (q[6] == ' ' || q[6] == '\t')) {
      q += 7;
      while (q < eol && (*q == ' ' || *q == '\t')) ++q;
      const char *ne = eol;
      while (ne > q && (ne[-1] == '\r' || ne[-1] == ' ' || ne[-1] == '\t')) --ne;
      auto it = mtl_index.find(std::string(q, ne));
      cur_mat = it == mtl_index.end() ? -1 : it->second;
    } else if (eol - q >= 6 && std::strncmp(q, "mtllib", 6) == 0 && (q[6] == ' ' || q[6] == '\t')) {
      q += 7;
      for (;;) {
        Tok t = next_token(q, eol);
        if (t.p == t.e) break;
        std::string mt;
        if (read_file(dir + std::string(t.p, t.e), &mt)) {
          parse_mtl(mt, &mtl, &mtl_index);
          break;  // tinyobj uses the first library that loads
        }
      }
    }
    p = eol + 1;
  }
  for (const Face &f : faces)
    for (int k = 0; k < 3; ++k)
      if (f.v[k] < 0 || (size_t)(3 * f.v[k] + 2) >= verts.size()) return fail(MCPT_ERR_PARSE, "load_obj: face index out of range");
  if (tris) {
    if (*n_tris < (int64_t)faces.size()) return fail(MCPT_ERR_ARG, "load_obj: triangle buffer too small");
    for (size_t i = 0; i < faces.size(); ++i) {
      mcpt_triangle t;
      std::memset(&t, 0, sizeof(t));
      for (int k = 0; k < 3; ++k)
        for (int j = 0; j < 3; ++j) t.v[k][j] = verts[3 * faces[i].v[k] + j];
      tris[i] = t;
      if (mat_index) mat_index[i] = faces[i].mat;
    }
  }
  if (mats) {
    if (*n_mats < (int32_t)mtl.size()) return fail(MCPT_ERR_ARG, "load_obj: material buffer too small");
    for (size_t i = 0; i < mtl.size(); ++i)
      mcpt_classify_material(mtl[i].ni, mtl[i].ka, mtl[i].kd, mtl[i].ks, mtl[i].ns, &mats[i]);
  }
  *n_tris = (int64_t)faces.size();
  *n_mats = (int32_t)mtl.size();
  return MCPT_OK;
}

// --------------------------------------------------------- triangle packing
extern "C" int mcpt_pack_triangles(mcpt_triangle *tris, const int32_t *mat_index, int64_t n) {
  if (n < 0 || (n > 0 && (!tris || !mat_index))) return fail(MCPT_ERR_ARG, "pack_triangles: bad argument");
  for (int64_t i = 0; i < n; ++i) {
    V4 a = v4(tris[i].v[0]), b = v4(tris[i].v[1]), c = v4(tris[i].v[2]);
    V4 nrm = normalize_host(cross_host(sub(b, a), sub(c, a)));
    store(tris[i].normal, nrm);
    std::memcpy(&tris[i].normal[3], &mat_index[i], 4);
  }
  return MCPT_OK;
}

// -------------------------------------------------------------------- HLBVH
namespace {

inline uint32_t spread_bits10(uint32_t x) {  // hlbvh.cpp:12-23 (1024 clamps to 1023)
  if (x == (1u << 10)) --x;
  x = (x | (x << 16)) & 0x030000FFu;
  x = (x | (x << 8)) & 0x0300F00Fu;
  x = (x | (x << 4)) & 0x030C30C3u;
  x = (x | (x << 2)) & 0x09249249u;
  return x;
}

// (cl_uint)roundf(v) as the reference's MSVC x64 build evaluates it: the
// conversion goes through a 64-bit cvttss2si, so NaN (0/0 on a flat axis)
// and out-of-range values keep the low 32 bits of 0x8000000000000000 = 0.
inline uint32_t to_uint_like_msvc(float v) {
  float r = std::round(v);
  if (!(r > -9.2233720368547758e18f && r < 9.2233720368547758e18f)) return 0u;
  return (uint32_t)(int64_t)r;
}

inline int clz_ref(int a) {  // hlbvh.cpp:138-146
  if (a == 0) return 32;
  int n = 0;
  uint32_t u = (uint32_t)a;
  while ((int32_t)u > 0) {
    u <<= 1;
    ++n;
  }
  return n;
}

struct Prim {
  int id;
  int code;
};

}  // namespace

extern "C" int mcpt_build_hlbvh(const mcpt_triangle *tris, int64_t n, mcpt_bvh_node *nodes) {
  if (n <= 0 || !tris || !nodes) return fail(MCPT_ERR_ARG, "build_hlbvh: empty scene or null pointer");
  if (n > (int64_t)0x3FFFFFFF) return fail(MCPT_ERR_LIMIT, "build_hlbvh: too many triangles");
  std::vector<V4> bmin(n), bmax(n), cen(n);
  for (int64_t i = 0; i < n; ++i) {
    V4 a = v4(tris[i].v[0]), b = v4(tris[i].v[1]), c = v4(tris[i].v[2]);
    a.s[3] = b.s[3] = c.s[3] = 0.0f;  // packFloat zero-initialises .w (thirdpartywrapper.cpp:38)
    bmin[i] = vmin(vmin(a, b), c);
    bmax[i] = vmax(vmax(a, b), c);
    V4 s = add(bmin[i], bmax[i]);
    for (int k = 0; k < 4; ++k) cen[i].s[k] = 0.5f * s.s[k];
  }
  V4 gmin{{FLT_MAX, FLT_MAX, FLT_MAX, FLT_MAX}}, gmax{{-FLT_MAX, -FLT_MAX, -FLT_MAX, -FLT_MAX}};
  for (int64_t i = 0; i < n; ++i) {
    gmin = vmin(gmin, cen[i]);
    gmax = vmax(gmax, cen[i]);
  }
  V4 gsize = sub(gmax, gmin);
  std::vector<Prim> prims(n);
  for (int64_t i = 0; i < n; ++i) {
    V4 d = sub(cen[i], gmin);
    uint32_t q[3];
    for (int k = 0; k < 3; ++k) {
      float x = d.s[k] / gsize.s[k];
      x *= 1024.0f;
      q[k] = to_uint_like_msvc(x);
    }
    uint32_t code = (spread_bits10(q[2]) << 2) | (spread_bits10(q[1]) << 1) | spread_bits10(q[0]);
    prims[i] = Prim{(int)i, (int)code};
  }
  // 5 stable LSD passes of 6 bits over the 30-bit code == a stable sort on the code
  std::stable_sort(prims.begin(), prims.end(), [](const Prim &a, const Prim &b) {
    return (uint32_t)(a.code & 0x3FFFFFFF) < (uint32_t)(b.code & 0x3FFFFFFF);
  });
  const int64_t nn = 2 * n - 1;
  std::memset(nodes, 0, sizeof(mcpt_bvh_node) * (size_t)nn);
  nodes[0].parent = -1;
  auto delta = [&](int64_t a, int64_t b) { return clz_ref(prims[a].code ^ prims[b].code); };
  auto split = [&](int64_t left, int64_t right) -> int64_t {  // hlbvh.cpp:152-161
    int target = delta(left, right);
    if (target == 32) return (right + left) >> 1;
    do {
      int64_t mid = (right + left) >> 1;
      if (delta(left, mid) > target)
        left = mid;
      else
        right = mid;
    } while (right > left + 1);
    return left;
  };
  if (n > 1) {
    struct Range {
      int64_t lo, hi, node;
    };
    std::deque<Range> work;  // breadth-first, hlbvh.cpp:165-188
    work.push_back(Range{0, n - 1, 0});
    while (!work.empty()) {
      Range r = work.front();
      work.pop_front();
      int64_t s = split(r.lo, r.hi);
      int64_t li = (s != r.lo) ? s : s + n - 1;
      int64_t ri = (s + 1 != r.hi) ? s + 1 : s + n;
      nodes[r.node].left = (int32_t)li;
      nodes[li].parent = (int32_t)r.node;
      nodes[r.node].right = (int32_t)ri;
      nodes[ri].parent = (int32_t)r.node;
      if (li == s) work.push_back(Range{r.lo, s, s});
      if (ri == s + 1) work.push_back(Range{s + 1, r.hi, s + 1});
    }
  }
  for (int64_t i = n - 1; i < nn; ++i) {
    int id = prims[i - (n - 1)].id;
    nodes[i].left = nodes[i].right = id;
    store(nodes[i].bbmin, bmin[id]);
    store(nodes[i].bbmax, bmax[id]);
  }
  if (n == 1) return MCPT_OK;  // the reference indexes past its 1-node array here (hlbvh.cpp:176-181)
  // refit (hlbvh.cpp:64-76), iterative post-order so deep trees cannot blow the C stack
  std::vector<std::pair<int64_t, int>> st;
  st.push_back({0, 0});
  while (!st.empty()) {
    auto &top = st.back();
    int64_t id = top.first;
    mcpt_bvh_node &nd = nodes[id];
    if (nd.left == nd.right) {
      st.pop_back();
      continue;
    }
    if (top.second == 0) {
      top.second = 1;
      st.push_back({nd.left, 0});
    } else if (top.second == 1) {
      top.second = 2;
      st.push_back({nd.right, 0});
    } else {
      V4 lmin = v4(nodes[nd.left].bbmin), lmax = v4(nodes[nd.left].bbmax);
      V4 rmin = v4(nodes[nd.right].bbmin), rmax = v4(nodes[nd.right].bbmax);
      store(nd.bbmin, vmin(lmin, rmin));
      store(nd.bbmax, vmax(lmax, rmax));
      st.pop_back();
    }
  }
  return MCPT_OK;
}

extern "C" int mcpt_bvh_stack_depth(const mcpt_bvh_node *nodes, int64_t n_nodes, int32_t *depth) {
  if (!nodes || n_nodes <= 0 || !depth) return fail(MCPT_ERR_ARG, "bvh_stack_depth: bad argument");
  // left-first DFS pushes the right child at every internal node it descends
  // through; the stack holds at most (#internal ancestors) entries.
  int32_t best = 1;
  std::vector<std::pair<int32_t, int32_t>> st;  // node, pushes so far
  st.push_back({0, 0});
  while (!st.empty()) {
    auto [id, d] = st.back();
    st.pop_back();
    if (id < 0 || id >= n_nodes) return fail(MCPT_ERR_ARG, "bvh_stack_depth: child index out of range");
    const mcpt_bvh_node &nd = nodes[id];
    best = std::max(best, d + 1);
    if (nd.left == nd.right) continue;
    if ((int64_t)st.size() > 4 * n_nodes) return fail(MCPT_ERR_ARG, "bvh_stack_depth: cyclic tree");
    st.push_back({nd.left, d + 1});
    st.push_back({nd.right, d});
  }
  *depth = best;
  return MCPT_OK;
}

// BVH::TEST::SAH (bvhtest.cpp:97-108): float products summed in double,
// Cinn for nodes [0, size/2), Ctri for the rest, over the root's area.
extern "C" int mcpt_bvh_sah(const mcpt_bvh_node *nodes, int64_t n_nodes, double *out) {
  if (!nodes || n_nodes <= 0 || !out) return fail(MCPT_ERR_ARG, "bvh_sah: bad argument");
  auto area = [](const mcpt_bvh_node &b) {  // auxiliary.cpp:15-18
    const float x = b.bbmax[0] - b.bbmin[0], y = b.bbmax[1] - b.bbmin[1], z = b.bbmax[2] - b.bbmin[2];
    return 2.0f * (x * y + x * z + y * z);
  };
  const float cinn = 1.2f, ctri = 1.0f;  // auxiliary.h:9-11
  double sah = 0.0f;
  const size_t size = (size_t)n_nodes;
  for (size_t i = 0; i < (size >> 1); ++i) sah += cinn * area(nodes[i]);
  for (size_t i = (size >> 1); i < size; ++i) sah += ctri * area(nodes[i]);
  sah /= area(nodes[0]);
  *out = (double)(float)sah;  // SAH returns float
  return MCPT_OK;
}

// ---------------------------------------------------------------------- HDR
namespace {

void rgbe_pixel(uint8_t *o, const float *lin) {  // stb_image_write.h:579-593
  auto mx = [](float a, float b) { return a > b ? a : b; };
  float maxcomp = mx(lin[0], mx(lin[1], lin[2]));
  if (maxcomp < 1e-32f) {
    o[0] = o[1] = o[2] = o[3] = 0;
    return;
  }
  int e;
  float norm = (float)std::frexp(maxcomp, &e) * 256.0f / maxcomp;
  for (int i = 0; i < 3; ++i) o[i] = (uint8_t)(int)(lin[i] * norm);
  o[3] = (uint8_t)(e + 128);
}

struct Sink {
  uint8_t *buf;
  int64_t cap, n;
  void put(const void *p, int64_t len) {
    if (buf && n + len <= cap) std::memcpy(buf + n, p, (size_t)len);
    n += len;
  }
  void byte(uint8_t b) { put(&b, 1); }
};

void scanline(Sink &s, int w, const float *row, std::vector<uint8_t> &scr) {
  uint8_t rgbe[4];
  if (w < 8 || w >= 32768) {  // no RLE
    for (int x = 0; x < w; ++x) {
      rgbe_pixel(rgbe, row + 4 * x);
      s.put(rgbe, 4);
    }
    return;
  }
  for (int x = 0; x < w; ++x) {
    rgbe_pixel(rgbe, row + 4 * x);
    for (int c = 0; c < 4; ++c) scr[x + w * c] = rgbe[c];
  }
  uint8_t hdr[4] = {2, 2, (uint8_t)((w & 0xff00) >> 8), (uint8_t)(w & 0xff)};
  s.put(hdr, 4);
  for (int c = 0; c < 4; ++c) {  // per-component RLE (stb_image_write.h:650-690)
    const uint8_t *comp = &scr[(size_t)w * c];
    int x = 0;
    while (x < w) {
      int r = x;
      while (r + 2 < w && !(comp[r] == comp[r + 1] && comp[r] == comp[r + 2])) ++r;
      if (r + 2 >= w) r = w;
      while (x < r) {
        int len = std::min(r - x, 128);
        s.byte((uint8_t)len);
        s.put(comp + x, len);
        x += len;
      }
      if (r + 2 < w) {
        while (r < w && comp[r] == comp[x]) ++r;
        while (x < r) {
          int len = std::min(r - x, 127);
          s.byte((uint8_t)(len + 128));
          s.byte(comp[x]);
          x += len;
        }
      }
    }
  }
}

int64_t encode_hdr(Sink &s, int w, int h, const float *rgba, int flip) {
  static const char head[] = "#?RADIANCE\n# Written by stb_image_write.h\nFORMAT=32-bit_rle_rgbe\n";
  s.put(head, sizeof(head) - 1);
  char buf[128];
  int len = std::snprintf(buf, sizeof(buf), "EXPOSURE=          1.0000000000000\n\n-Y %d +X %d\n", h, w);
  s.put(buf, len);
  std::vector<uint8_t> scr((size_t)w * 4);
  for (int i = 0; i < h; ++i) scanline(s, w, rgba + (size_t)4 * w * (flip ? h - 1 - i : i), scr);
  return s.n;
}

}  // namespace

extern "C" int64_t mcpt_encode_hdr(int32_t width, int32_t height, const float *rgba, int32_t flip,
                                   uint8_t *out, int64_t cap) {
  if (width <= 0 || height <= 0 || !rgba) return fail(MCPT_ERR_ARG, "encode_hdr: bad argument");
  Sink s{out, cap, 0};
  const int64_t n = encode_hdr(s, width, height, rgba, flip);
  if (out && n > cap) return fail(MCPT_ERR_ARG, "encode_hdr: output buffer too small");
  return n;
}

extern "C" int mcpt_write_hdr(const char *path, int32_t width, int32_t height, const float *rgba,
                              int32_t flip) {
  if (!path) return fail(MCPT_ERR_ARG, "write_hdr: null path");
  int64_t n = mcpt_encode_hdr(width, height, rgba, flip, nullptr, 0);
  if (n < 0) return (int)n;
  std::vector<uint8_t> bytes((size_t)n);
  mcpt_encode_hdr(width, height, rgba, flip, bytes.data(), n);
  FILE *f = std::fopen(path, "wb");
  if (!f) return fail(MCPT_ERR_IO, std::string("write_hdr: cannot open ") + path);
  size_t wr = std::fwrite(bytes.data(), 1, bytes.size(), f);
  std::fclose(f);
  if (wr != bytes.size()) return fail(MCPT_ERR_IO, "write_hdr: short write");
  return MCPT_OK;
}
