// abi_host.cpp — the reference's application loop as a C++ consumer of the C ABI
// (include/mcpt_hip.h): the binding INTEGRATION.md shows for
// MonteCarloPathTracing/OpenCLApp.cpp:36-82 (OpenCL::init/update) and
// colorout.cpp:55-68 (the .hdr dump), compiled and linked against
// libmcpt_hip.so only — no HIP headers, no torch, no Python.  Test
// infrastructure (tests/test_gpu_abi_host.py drives it).
//
//   abi_host <config.json> <configid> <seeds.u32|-> <out_dir> [--frames-per-update F] [--updates U]
//            [--resume-at K]   (before update K: mcpt_download, a new state, mcpt_upload)
//
// init: Config::CONFIG (config.cpp:70-124, '#' comments), loadObject
// (thirdpartywrapper.cpp:25-99), SceneCL packing + HLBVH<CPU>
// (scenebuild.cpp:50-101), parseCamera (auxiliary.cpp:20-71), the image state
// (randBuffer / frameBuffer / sampleCount).  update: mcpt_render_frames with
// F frames (default 1, as OpenCL::update renders one frame per call); after
// attempt+1 frames the .hdr is written once (colorout.cpp:55-68).  Writes
// <out_dir>/state.bin (hist f32x4, count i32, seeds u32 per pixel) and prints
// one JSON line with the update timing.
#include <chrono>
#include <cctype>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/mcpt_hip.h"

#define OK(x)                                                                                      \
  do {                                                                                             \
    int rc_ = (x);                                                                                 \
    if (rc_ < 0) throw std::runtime_error(std::string(#x) + ": " + mcpt_last_error());             \
  } while (0)

// ------------------------------------------------------------ tiny JSON
// Enough of JSON for config.json: objects, arrays, numbers, strings, bools,
// null, and the reference's '#' line comments (its patched json.hpp:3037).
struct Json {
  enum Kind { NUL, BOOL, NUM, STR, ARR, OBJ } kind = NUL;
  bool b = false;
  double num = 0.0;
  std::string str;
  std::vector<Json> arr;
  std::map<std::string, Json> obj;
  const Json &operator[](const std::string &k) const {
    auto it = obj.find(k);
    if (it == obj.end()) throw std::runtime_error("config: missing key " + k);
    return it->second;
  }
  bool has(const std::string &k) const { return kind == OBJ && obj.count(k); }
  const Json &operator[](size_t i) const { return arr.at(i); }
};

struct Parser {
  const std::string &s;
  size_t i = 0;
  void ws() {
    for (;;) {
      while (i < s.size() && std::isspace((unsigned char)s[i])) ++i;
      if (i < s.size() && s[i] == '#') {
        while (i < s.size() && s[i] != '\n') ++i;
        continue;
      }
      return;
    }
  }
  char peek() {
    ws();
    if (i >= s.size()) throw std::runtime_error("config: unexpected end");
    return s[i];
  }
  void expect(char c) {
    if (peek() != c) throw std::runtime_error(std::string("config: expected ") + c);
    ++i;
  }
  std::string string_() {
    expect('"');
    std::string out;
    while (i < s.size() && s[i] != '"') {
      if (s[i] == '\\' && i + 1 < s.size()) ++i;
      out += s[i++];
    }
    ++i;
    return out;
  }
  Json value() {
    Json j;
    const char c = peek();
    if (c == '{') {
      j.kind = Json::OBJ;
      ++i;
      if (peek() == '}') return ++i, j;
      for (;;) {
        std::string k = string_();
        expect(':');
        j.obj[k] = value();
        if (peek() == ',') {
          ++i;
          continue;
        }
        expect('}');
        return j;
      }
    }
    if (c == '[') {
      j.kind = Json::ARR;
      ++i;
      if (peek() == ']') return ++i, j;
      for (;;) {
        j.arr.push_back(value());
        if (peek() == ',') {
          ++i;
          continue;
        }
        expect(']');
        return j;
      }
    }
    if (c == '"') {
      j.kind = Json::STR;
      j.str = string_();
      return j;
    }
    if (s.compare(i, 4, "true") == 0) return i += 4, j.kind = Json::BOOL, j.b = true, j;
    if (s.compare(i, 5, "false") == 0) return i += 5, j.kind = Json::BOOL, j;
    if (s.compare(i, 4, "null") == 0) return i += 4, j;
    char *end = nullptr;
    j.num = std::strtod(s.c_str() + i, &end);
    if (end == s.c_str() + i) throw std::runtime_error("config: bad value");
    i = end - s.c_str();
    j.kind = Json::NUM;
    return j;
  }
};

static std::string slurp(const std::string &path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("cannot read " + path);
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

// ------------------------------------------------------------ the app
struct App {
  mcpt_ctx *ctx = nullptr;
  mcpt_scene *scene = nullptr;
  mcpt_state *state = nullptr;
  mcpt_camera cam{};
  int32_t width = 0, height = 0, max_depth = 0, max_attempt = 0;
  int attempt_count = 0;
  std::string objname, out_dir, dumped;

  // OpenCL::init (OpenCLApp.cpp:36-55)
  void init(const Json &c, const std::string &root, const std::vector<uint32_t> *seeds_in) {
    width = (int32_t)c["width"].num;  // read as double, stored as int (config.cpp:103-104)
    height = (int32_t)c["height"].num;
    max_depth = (int32_t)c["maxdepth"].num;
    max_attempt = (int32_t)c["attempt"].num;
    objname = c["objname"].str;
    const std::string bvhtype = c.has("bvhtype") ? c["bvhtype"].str : "hlbvh";
    if (bvhtype != "hlbvh" && bvhtype != "treelet" && bvhtype != "treeletGPU")
      throw std::runtime_error("BVH Not Implemented");  // scenebuild.cpp:77-79
    const Json &jc = c["camera"];
    if (jc.has("resolution") && ((int32_t)jc["resolution"][0].num != width || (int32_t)jc["resolution"][1].num != height))
      throw std::runtime_error("camera.resolution must equal width/height");
    if (mcpt_abi_version() != MCPT_ABI_VERSION)  // a library built from another header: refuse it
      throw std::runtime_error("libmcpt_hip.so ABI mismatch");
    OK(mcpt_ctx_create(0, &ctx));
    // ThirdPartyWrapper::loadObject, two-call sizing
    std::string dir = root + "/" + c["directory"].str;
    int64_t n = 0;
    int32_t nm = 0;
    OK(mcpt_load_obj(dir.c_str(), objname.c_str(), nullptr, nullptr, &n, nullptr, &nm));
    std::vector<mcpt_triangle> tris(n);
    std::vector<int32_t> mat_id(n);
    std::vector<mcpt_material> mats(nm);
    OK(mcpt_load_obj(dir.c_str(), objname.c_str(), tris.data(), mat_id.data(), &n, mats.data(), &nm));
    if (c.has("materials") && c["materials"].str == "diffuse_only")  // BASELINE C2's override
      for (auto &m : mats)
        if (m.type != MCPT_LIGHT) m.type = MCPT_DIFFUSE;
    // SceneCL ctor: pack normals + material ids, then (every bvhtype falls
    // through into the GPUBVH block, scenebuild.cpp:87-95) a fresh HLBVH<CPU>
    // restructured by TreeletBVH<GPU>, upload
    OK(mcpt_pack_triangles(tris.data(), mat_id.data(), n));
    std::vector<mcpt_bvh_node> nodes(2 * n - 1);
    OK(mcpt_build_hlbvh(tris.data(), n, nodes.data()));
    OK(mcpt_treelet_gpu(nodes.data(), (int64_t)nodes.size()));
    OK(mcpt_scene_upload(ctx, tris.data(), n, nodes.data(), (int64_t)nodes.size(), mats.data(), nm, &scene));
    // Auxiliary::parseCamera
    double p[3], l[3], u[3];
    for (int k = 0; k < 3; ++k) p[k] = jc["position"][k].num, l[k] = jc["lookat"][k].num, u[k] = jc["up"][k].num;
    OK(mcpt_parse_camera(p, l, u, jc["fov"].num, &cam));
    // randBuffer (scenebuild.cpp:113-120 draws srand(time); rand(): parity runs pass seeds)
    std::vector<uint32_t> seeds((size_t)width * height);
    if (seeds_in) {
      if (seeds_in->size() != seeds.size()) throw std::runtime_error("seed file has the wrong pixel count");
      seeds = *seeds_in;
    } else {
      std::srand(1);
      for (auto &x : seeds) x = (uint32_t)std::rand() & 0x7FFFu;  // MSVC rand(): 15 bits
    }
    OK(mcpt_state_create(ctx, width, height, seeds.data(), &state));
  }

  // OpenCL::update (OpenCLApp.cpp:57-82) + ColorOut::outputColorCL (colorout.cpp:40-73)
  void update(int frames) {
    uint32_t *d_seeds;
    float *d_hist;
    int32_t *d_count;
    OK(mcpt_state_buffers(state, &d_seeds, &d_hist, &d_count));
    mcpt_render_params rp{};
    rp.width = width;
    rp.height = height;
    rp.max_depth = max_depth;
    rp.max_attempt = max_attempt;
    rp.frame_begin = attempt_count;
    rp.frames = frames;
    rp.stripe_rows = 16;
    rp.stripe_index = 0;
    rp.stripe_count = 1;
    rp.mode = MCPT_MODE_EXACT;
    rp.schedule = MCPT_SCHED_PAIRED;
    OK(mcpt_render_frames(ctx, scene, &cam, &rp, d_seeds, d_hist, d_count, nullptr));
    const int before = attempt_count;
    attempt_count += frames;
    if (before <= max_attempt && attempt_count > max_attempt && dumped.empty()) {  // frame attempt+1: dump once
      std::vector<float> img((size_t)width * height * 4);
      OK(mcpt_download(ctx, state, img.data(), nullptr, nullptr, nullptr));
      dumped = out_dir + "/" + objname + ".hdr";
      OK(mcpt_write_hdr(dumped.c_str(), width, height, img.data(), 1));  // outputPicture: vertically flipped
    }
  }

  // checkpoint / resume: the image state saved to host arrays, the state
  // destroyed, a new one created and the saved arrays uploaded into it
  void checkpoint_resume() {
    const size_t n = (size_t)width * height;
    std::vector<float> hist(n * 4);
    std::vector<int32_t> count(n);
    std::vector<uint32_t> seeds(n);
    OK(mcpt_download(ctx, state, hist.data(), count.data(), seeds.data(), nullptr));
    OK(mcpt_state_destroy(state));
    state = nullptr;
    std::vector<uint32_t> zero(n, 0u);
    OK(mcpt_state_create(ctx, width, height, zero.data(), &state));
    OK(mcpt_upload(ctx, state, hist.data(), count.data(), seeds.data(), nullptr));
  }

  void save_state(const std::string &path) {
    const size_t n = (size_t)width * height;
    std::vector<float> hist(n * 4);
    std::vector<int32_t> count(n);
    std::vector<uint32_t> seeds(n);
    OK(mcpt_download(ctx, state, hist.data(), count.data(), seeds.data(), nullptr));
    FILE *f = std::fopen(path.c_str(), "wb");
    if (!f) throw std::runtime_error("cannot write " + path);
    std::fwrite(hist.data(), 4, hist.size(), f);
    std::fwrite(count.data(), 4, count.size(), f);
    std::fwrite(seeds.data(), 4, seeds.size(), f);
    std::fclose(f);
  }

  ~App() {
    mcpt_state_destroy(state);
    mcpt_scene_destroy(scene);
    mcpt_ctx_destroy(ctx);
  }
};

int main(int argc, char **argv) {
  if (argc < 5) {
    std::fprintf(stderr, "usage: %s config.json configid seeds.u32|- out_dir [--frames-per-update F] [--updates U]\n",
                 argv[0]);
    return 2;
  }
  try {
    const std::string cfg_path = argv[1];
    const int configid = std::atoi(argv[2]);
    int fpu = 1, updates = -1, resume_at = -1;
    for (int k = 5; k + 1 < argc; k += 2) {
      if (!std::strcmp(argv[k], "--frames-per-update")) fpu = std::atoi(argv[k + 1]);
      else if (!std::strcmp(argv[k], "--updates")) updates = std::atoi(argv[k + 1]);
      else if (!std::strcmp(argv[k], "--resume-at")) resume_at = std::atoi(argv[k + 1]);
    }
    const std::string text = slurp(cfg_path);
    Parser ps{text};
    const Json root = ps.value();
    const Json &c = root["config"][(size_t)configid];
    std::string base = cfg_path.substr(0, cfg_path.find_last_of('/') == std::string::npos ? 0 : cfg_path.find_last_of('/'));
    if (base.empty()) base = ".";
    std::unique_ptr<std::vector<uint32_t>> seeds;
    if (std::strcmp(argv[3], "-") != 0) {
      const std::string raw = slurp(argv[3]);
      seeds.reset(new std::vector<uint32_t>(raw.size() / 4));
      std::memcpy(seeds->data(), raw.data(), seeds->size() * 4);
    }
    App app;
    app.out_dir = argv[4];
    app.init(c, base, seeds.get());
    if (updates < 0) updates = (app.max_attempt + 1 + fpu - 1) / fpu;  // attempt+1 frames: history, then the dump
    mcpt_stats st{};
    app.update(fpu);  // the first update outside the clock (lazy allocations)
    OK(mcpt_get_stats(app.ctx, &st));
    const auto t0 = std::chrono::steady_clock::now();
    for (int k = 1; k < updates; ++k) {
      if (k == resume_at) app.checkpoint_resume();
      app.update(fpu);
    }
    OK(mcpt_get_stats(app.ctx, &st));  // waits for the last update
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    app.save_state(app.out_dir + "/state.bin");
    const double frames = (double)(updates - 1) * fpu;
    std::printf("{\"width\": %d, \"height\": %d, \"max_depth\": %d, \"frames_per_update\": %d, \"updates\": %d, "
                "\"frames_done\": %d, \"dumped\": \"%s\", \"timed_frames\": %.0f, \"ms_per_frame\": %.4f, "
                "\"Msamples_per_s\": %.2f}\n",
                app.width, app.height, app.max_depth, fpu, updates, app.attempt_count, app.dumped.c_str(), frames,
                frames > 0 ? s * 1e3 / frames : 0.0,
                frames > 0 ? (double)app.width * app.height * frames * app.max_depth / s / 1e6 : 0.0);
    return 0;
  } catch (const std::exception &e) {
    std::fprintf(stderr, "abi_host: %s\n", e.what());
    return 1;
  }
}
