// Host ASan + UBSan harness ("Race detection / sanitizers":
// host ASan/UBSan builds of the CPU restatement).  The reference relies on Zig's
// ReleaseSafe checks (build.zig:12); the host half of this repository is C/C++, so
// its equivalent is a sanitizer build of every host source that touches scene
// data, driven through the same C ABI the GPU path uses:
//
//   scene_io.cpp   zrt_scene_load (scenes.zig / obj_reader.zig), zrt_scene_write/read
//   image_io.cpp   zrt_image_read_png / write_png / write_ppm (png_image.zig)
//   bvh_build.cpp  zrt_bvh_build (bvh.zig:62-185)
//   accel_build.cpp  the wide tree over the reference leaves (render.hip's FAST layout)
//   oracle/        oracle_render (both RNG modes), oracle_render_scanlines,
//                  oracle_trace, oracle_bvh_build
//
// Device code is not built here (GPU sanitizers are not available on the pool);
// build_bvh_device is stubbed to "not available", which is what the host build
// path does without a GPU.  Any sanitizer report aborts with a non-zero status
// (-fno-sanitize-recover=all); tests/test_sanitizers.py builds and runs this.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/zrt.h"
#include "../../oracle/oracle.h"
#include "../../zraytrace_amd/csrc/accel_build.hpp"
#include "../../zraytrace_amd/csrc/bvh_build.hpp"

namespace zrt {
bool build_bvh_device(const zrt_prim*, uint32_t, int, BuiltBvh*) { return false; }
}  // namespace zrt
// the C++ scene API's render() (zrt.hpp) forwards here; nothing in this harness calls it
extern "C" int zrt_render(const zrt_scene*, const zrt_camera*, const zrt_params*, float*, zrt_stats*) {
  return ZRT_E_NODEVICE;
}

static int g_fail = 0;
#define CHECK(cond, ...)                         \
  do {                                           \
    if (!(cond)) {                               \
      std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      std::fprintf(stderr, __VA_ARGS__);         \
      std::fprintf(stderr, "\n");                \
      ++g_fail;                                  \
    }                                            \
  } while (0)

static zrt_params params(uint32_t w, uint32_t h, uint32_t spp, uint32_t depth, uint32_t rng) {
  zrt_params p;
  std::memset(&p, 0, sizeof p);
  p.width = w;
  p.height = h;
  p.samples_per_pixel = spp;
  p.max_depth = depth;
  p.bounded_volume_hierarchy = 1;
  p.rng_mode = rng;
  p.seed = 42;
  p.world_size = 1;
  p.sample_chunk = 3;
  return p;
}

// the reference BVH's leaves in DFS order, as render.hip's flatten_scene hands
// them to build_wide_bvh (refs are placeholders: the builder only carries them)
static uint32_t wide_tree(const zrt::BuiltBvh& bvh) {
  std::vector<zrt::RefLeaf> leaves;
  for (const zrt::BuildNode& b : bvh.nodes) {
    if (b.left >= 0) continue;
    zrt::RefLeaf L;
    for (int k = 0; k < 3; ++k) {
      L.mn[k] = b.mn[k];
      L.mx[k] = b.mx[k];
    }
    L.prim_a = b.left;
    L.prim_b = b.right;
    leaves.push_back(L);
  }
  const zrt::WideBvh w = zrt::build_wide_bvh(leaves);
  return w.n_nodes;
}

static void one_scene(uint32_t index, const std::string& assets, const std::string& tmp) {
  zrt_scene_data* data = nullptr;
  zrt_camera cam;
  int rc = zrt_scene_load(index, assets.c_str(), &data, &cam);
  CHECK(rc == ZRT_OK, "scene %u: %s", index, zrt_last_error());
  if (rc) return;
  const zrt_scene* s = zrt_scene_view(data);

  // host BVH build (bvh.zig:62-185) == the oracle's comparison-sort build
  zrt_bvh_node* nodes = nullptr;
  uint32_t n_nodes = 0, depth = 0;
  rc = zrt_bvh_build(s, &nodes, &n_nodes, &depth);
  CHECK(rc == ZRT_OK, "scene %u bvh: %s", index, zrt_last_error());
  zrt_bvh_node* onodes = nullptr;
  uint32_t on = 0, od = 0;
  if (s->n_prims > 10) {
    rc = oracle_bvh_build(s, &onodes, &on, &od);
    CHECK(rc == 0 && on == n_nodes && od == depth && std::memcmp(nodes, onodes, sizeof(zrt_bvh_node) * on) == 0,
          "scene %u: host BVH differs from the oracle's", index);
    const zrt::BuiltBvh built = zrt::build_bvh(s->prims, s->n_prims);
    CHECK(built.nodes.size() == n_nodes, "scene %u: build_bvh node count", index);
    CHECK(wide_tree(built) > 0, "scene %u: empty wide tree", index);
  }
  zrt_free(nodes);
  oracle_free(onodes);

  // oracle renders: counter mode (the GPU's partner) and the reference stream
  for (uint32_t rng : {uint32_t(ZRT_RNG_COUNTER), uint32_t(ZRT_RNG_REFERENCE_STREAM)}) {
    const zrt_params p = params(12, 9, 3, 6, rng);
    std::vector<float> img(size_t(p.width) * p.height * 3);
    zrt_stats st;
    rc = oracle_render(s, &cam, &p, img.data(), &st);
    CHECK(rc == 0 && st.pixels_processed > 0 && st.samples_processed == st.pixels_processed * p.samples_per_pixel,
          "scene %u rng %u: oracle_render rc %d", index, rng, rc);
    std::vector<zrt_scanline> rows(p.height);
    rc = oracle_render_scanlines(s, &cam, &p, img.data(), &st, rows.data());
    CHECK(rc == 0, "scene %u rng %u: oracle_render_scanlines rc %d", index, rng, rc);
  }

  // closest-hit queries through both of the oracle's surface structures
  std::vector<float> rays;
  for (int i = 0; i < 64; ++i) {
    const float a = 0.1f * float(i);
    const float r[6] = {cam.origin.x, cam.origin.y, cam.origin.z, std::sin(a) * 0.3f, std::cos(a) * 0.2f - 0.1f, -1.f};
    rays.insert(rays.end(), r, r + 6);
  }
  std::vector<float> t(64);
  std::vector<int32_t> surf(64);
  for (int bvh = 0; bvh < 2; ++bvh) {
    rc = oracle_trace(s, bvh, rays.data(), 64, t.data(), surf.data());
    CHECK(rc == 0, "scene %u: oracle_trace(bvh=%d) rc %d", index, bvh, rc);
  }

  // binary scene file round trip
  const std::string path = tmp + "/scene" + std::to_string(index) + ".zrts";
  rc = zrt_scene_write(s, &cam, path.c_str());
  CHECK(rc == ZRT_OK, "scene %u write: %s", index, zrt_last_error());
  zrt_scene_data* back = nullptr;
  zrt_camera cam2;
  rc = zrt_scene_read(path.c_str(), &back, &cam2);
  CHECK(rc == ZRT_OK, "scene %u read: %s", index, zrt_last_error());
  if (!rc) {
    const zrt_scene* b = zrt_scene_view(back);
    CHECK(b->n_prims == s->n_prims && std::memcmp(b->prims, s->prims, sizeof(zrt_prim) * s->n_prims) == 0,
          "scene %u: prims differ after the round trip", index);
    CHECK(std::memcmp(&cam, &cam2, sizeof cam) == 0, "scene %u: camera differs after the round trip", index);
    zrt_scene_free(back);
  }
  zrt_scene_free(data);
}

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: %s ASSETS_DIR TMP_DIR\n", argv[0]);
    return 2;
  }
  const std::string assets = argv[1], tmp = argv[2];
  for (uint32_t i : {0u, 1u, 2u, 3u, 4u}) one_scene(i, assets, tmp);

  // error paths: unknown scene index, missing files, a truncated binary scene
  zrt_scene_data* d = nullptr;
  zrt_camera cam;
  CHECK(zrt_scene_load(99, assets.c_str(), &d, &cam) == ZRT_E_INVALID, "scene 99 accepted");
  CHECK(zrt_scene_read((tmp + "/missing.zrts").c_str(), &d, &cam) != ZRT_OK, "missing scene file accepted");
  {
    const std::string trunc = tmp + "/trunc.zrts";
    FILE* in = std::fopen((tmp + "/scene2.zrts").c_str(), "rb");
    FILE* out = std::fopen(trunc.c_str(), "wb");
    if (in && out) {
      std::vector<char> buf(4096);
      const size_t n = std::fread(buf.data(), 1, buf.size(), in);
      std::fwrite(buf.data(), 1, n / 2, out);
    }
    if (in) std::fclose(in);
    if (out) std::fclose(out);
    CHECK(zrt_scene_read(trunc.c_str(), &d, &cam) != ZRT_OK, "truncated scene file accepted");
  }
  zrt_prim* prims = nullptr;
  uint32_t n = 0;
  CHECK(zrt_obj_read((tmp + "/missing.obj").c_str(), 0, &prims, &n) != ZRT_OK, "missing OBJ accepted");
  CHECK(zrt_obj_read((assets + "/teapot.obj").c_str(), 0, &prims, &n) == ZRT_OK && n > 6000, "teapot.obj: %s",
        zrt_last_error());
  zrt_free(prims);

  // PNG codec: the reference's textures in, PNG / PPM out, read back
  for (const char* name : {"earthmap.png", "nitor-logo-25.png"}) {
    uint32_t w = 0, h = 0;
    float* px = nullptr;
    int rc = zrt_image_read_png((assets + "/" + name).c_str(), &w, &h, &px);
    CHECK(rc == ZRT_OK && w > 0 && h > 0, "%s: %s", name, zrt_last_error());
    if (rc) continue;
    const std::string png = tmp + "/out.png", ppm = tmp + "/out.ppm";
    CHECK(zrt_image_write_png(png.c_str(), px, w, h) == ZRT_OK, "write png: %s", zrt_last_error());
    CHECK(zrt_image_write_ppm(ppm.c_str(), px, w, h) == ZRT_OK, "write ppm: %s", zrt_last_error());
    uint32_t w2 = 0, h2 = 0;
    float* back = nullptr;
    CHECK(zrt_image_read_png(png.c_str(), &w2, &h2, &back) == ZRT_OK && w2 == w && h2 == h &&
              std::memcmp(back, px, sizeof(float) * 3 * w * h) == 0,
          "%s: PNG round trip differs", name);
    zrt_free(back);
    zrt_free(px);
  }
  uint32_t w = 0, h = 0;
  float* px = nullptr;
  CHECK(zrt_image_read_png((assets + "/teapot.obj").c_str(), &w, &h, &px) != ZRT_OK, "an OBJ decoded as PNG");

  if (g_fail) {
    std::fprintf(stderr, "%d check(s) failed\n", g_fail);
    return 1;
  }
  std::printf("sanitized host run ok\n");
  return 0;
}
