// cli.cpp — `zrt-raytrace`: main.zig's command line on the HIP path.
//
//   zrt-raytrace width height samples depth scene_index filename
//
// A plain client of libzrt.so's C ABI (as a Zig host would be): builds the
// scene (scenes.zig:267-277 via zrt_scene_load), renders it with zrt_render
// (raytrace.zig:136-203: BVH on, DefaultPrng seed 42 -> counter RNG), prints
// the reference's start, per-scanline and summary lines on stderr
// (raytrace.zig:143-159, 37-50 + 184, 191-201) and writes the PNG (main.zig:33,
// png_image.zig:96-148).  The scanline lines carry each row's counters as the
// reference counts them (ZRT_FLAG_SCANLINES, zrt_render_progress); they are
// printed when the frame is done (it is one launch), and their Pixels/s is the
// frame's rate, since rows are not rendered one after another.  Assets come from $ZRT_ASSETS, else <exe dir>/../assets;
// $ZRT_DEVICE picks the GPU, $ZRT_DEVICES="0,1,..." renders over several
// (zrt_render_multi: tiles round-robin, one RCCL gather).
#include <unistd.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/zrt.h"

namespace {

// std.fmt.parseInt(u16, s, 10)
bool parse_u16(const char* s, uint16_t* out, const char** err) {
  if (!s) {
    *err = "missing argument";
    return false;
  }
  const char* p = s;
  if (*p == '+') ++p;
  if (!*p) {
    *err = "InvalidCharacter";
    return false;
  }
  uint32_t v = 0;
  for (; *p; ++p) {
    if (*p < '0' || *p > '9') {
      *err = "InvalidCharacter";
      return false;
    }
    v = v * 10 + uint32_t(*p - '0');
    if (v > 0xffff) {
      *err = "Overflow";
      return false;
    }
  }
  *out = uint16_t(v);
  return true;
}

std::string default_assets() {
  if (const char* env = std::getenv("ZRT_ASSETS")) return env;
  char buf[4096];
  const ssize_t n = readlink("/proc/self/exe", buf, sizeof(buf) - 1);
  if (n <= 0) return "assets";
  buf[n] = 0;
  std::string exe(buf);
  return exe.substr(0, exe.rfind('/')) + "/../assets";
}

const char* scene_title(unsigned index) {  // the scene constructors' first line
  switch (index) {
    case 0: return "Rendering scene Man and a big ball";            // scenes.zig:27
    case 1: return "Rendering scene Three balls";                   // scenes.zig:55
    case 2: return "Rendering scene Bunny and a big ball";          // scenes.zig:103
    case 3: return "Rendering scene Bunny and a big ball";          // scenes.zig:207 (sic)
    case 4: return "Rendering scene Bunny and a circle of balls";   // scenes.zig:169 (sic)
    case 6: return "Rendering scene Textured teapot (config C5 substitute)";
    default: return nullptr;                                        // goat prints none
  }
}

double seconds_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

}  // namespace

int main(int argc, char** argv) {
  std::fprintf(stderr, "raytrace\nUSAGE;\nraytrace width heigth samples depth scene_index filename\n");
  uint16_t width = 0, height = 0, samples = 0, depth = 0, scene_index = 0;
  const char* err = nullptr;
  uint16_t* fields[5] = {&width, &height, &samples, &depth, &scene_index};
  for (int i = 0; i < 5; ++i) {
    if (!parse_u16(i + 1 < argc ? argv[i + 1] : nullptr, fields[i], &err)) {
      std::fprintf(stderr, "error: %s\n", err);
      return 1;
    }
  }
  if (argc < 7) {
    std::fprintf(stderr, "error: missing argument\n");
    return 1;
  }
  const char* filename = argv[6];

  const auto t_start = std::chrono::steady_clock::now();
  if (const char* title = scene_title(scene_index)) std::fprintf(stderr, "%s\n", title);
  zrt_scene_data* data = nullptr;
  zrt_camera camera;
  int rc = zrt_scene_load(scene_index, default_assets().c_str(), &data, &camera);
  if (rc != ZRT_OK) {
    std::fprintf(stderr, "error: %s\n", zrt_last_error());
    return 1;
  }
  const zrt_scene* scene = zrt_scene_view(data);

  zrt_params params;
  std::memset(&params, 0, sizeof(params));
  params.width = width;
  params.height = height;
  params.samples_per_pixel = samples;
  params.max_depth = depth;
  params.bounded_volume_hierarchy = 1;  // main.zig:28
  params.rng_mode = ZRT_RNG_COUNTER;
  params.prng = ZRT_PRNG_XOROSHIRO128;
  params.traversal = ZRT_TRAVERSAL_FAST;
  params.seed = 42;  // DefaultPrng.init(42) in every scene
  params.world_size = 1;
  if (const char* dev = std::getenv("ZRT_DEVICE")) params.device = uint32_t(std::atoi(dev));
  // $ZRT_DEVICES="0,1,...,7": tiles over those GPUs, one RCCL gather (zrt_render_multi)
  std::vector<uint32_t> devices;
  if (const char* list = std::getenv("ZRT_DEVICES")) {
    for (const char* q = list; *q;) {
      char* end = nullptr;
      const unsigned long d = std::strtoul(q, &end, 10);
      if (end == q) break;
      devices.push_back(uint32_t(d));
      q = *end == ',' ? end + 1 : end;
    }
  }

  std::fprintf(stderr, "Raytrace start\n");
  std::fprintf(stderr, " - Surfaces:                 %u\n", scene->n_prims);
  std::fprintf(stderr, " - Pixels:                   %ux%u\n", unsigned(width), unsigned(height));
  std::fprintf(stderr, " - Samples per pixel:        %u\n", unsigned(samples));
  std::fprintf(stderr, " - Recursion depth:          %u\n", unsigned(depth));
  std::fprintf(stderr, " - Bounded volume hierarchy: true\n");
  std::fprintf(stderr, scene->n_prims > 10 ? "Using Bounded Volume Hierarchy\n" : "Using surface list\n");

  std::vector<float> image(size_t(width) * height * 3, 0.0f);
  std::vector<zrt_scanline> rows(height);
  zrt_stats stats;
  const auto t_render = std::chrono::steady_clock::now();
  if (devices.empty()) {
    rc = zrt_render_progress(scene, &camera, &params, image.data(), &stats, rows.data());
  } else {
    params.flags |= ZRT_FLAG_SCANLINES;
    zrt_multi* multi = nullptr;
    rc = zrt_multi_create(scene, &params, devices.data(), uint32_t(devices.size()), &multi);
    if (rc == ZRT_OK) rc = zrt_multi_render(multi, &camera, &params, image.data(), &stats);
    if (rc == ZRT_OK) rc = zrt_multi_scanlines(multi, rows.data(), height);
    const std::string msg = zrt_last_error();
    zrt_multi_destroy(multi);
    if (rc != ZRT_OK) std::fprintf(stderr, "error: %s\n", msg.c_str());
  }
  if (rc != ZRT_OK) {
    if (devices.empty()) std::fprintf(stderr, "error: %s\n", zrt_last_error());
    zrt_scene_free(data);
    return 1;
  }
  const double runtime = seconds_since(t_start);
  const double call = seconds_since(t_render);
  const double render_runtime = stats.render_ms / 1000.0;  // the sampling loop itself
  std::fprintf(stderr, "Preprocess time: %.2f seconds\n", runtime - render_runtime);
  // printProgress after every scanline (raytrace.zig:37-50, 184)
  const double pixels_per_second = double(stats.pixels_processed) / render_runtime;
  unsigned long long pixels = 0, samples_sum = 0, rays = 0;
  for (uint32_t y = 0; y < height; ++y) {
    pixels += rows[y].pixels;
    samples_sum += rows[y].samples;
    rays += rows[y].rays;
    std::fprintf(stderr,
                 "Scanline: %u/%u Pixels: %llu Samples: %llu Rays: %llu Recursion limit: %llu Reflections: %llu "
                 "Background hits: %llu Pixels/s: %.1f\n",
                 y + 1, unsigned(height), pixels, samples_sum, rays,
                 (unsigned long long)rows[y].recursion_depth_hits, (unsigned long long)rows[y].reflections,
                 (unsigned long long)rows[y].background_hits, pixels_per_second);
  }
  std::fprintf(stderr, "Rendering ready\n");
  std::fprintf(stderr, "  Total reflections:     %llu\n", (unsigned long long)stats.reflections);
  std::fprintf(stderr, "  Total background hits: %llu\n", (unsigned long long)stats.background_hits);
  std::fprintf(stderr, "  Total pixels:          %llu\n", (unsigned long long)stats.pixels_processed);
  std::fprintf(stderr, "  Total samples:         %llu\n", (unsigned long long)stats.samples_processed);
  std::fprintf(stderr, "  Total rays:            %llu\n", (unsigned long long)stats.rays_processed);
  std::fprintf(stderr, "  Total reflections:     %llu\n", (unsigned long long)stats.reflections);
  std::fprintf(stderr, "  Pixels per second:     %.2f pixels/s\n", double(stats.pixels_processed) / runtime);
  std::fprintf(stderr, "  Total runtime:         %.2f seconds\n", runtime);
  std::fprintf(stderr, "    Prepare runtime:     %.2f seconds\n", runtime - render_runtime);
  std::fprintf(stderr, "    Render runtime:      %.2f seconds\n", render_runtime);
  std::fprintf(stderr, "  Mrays/s (render):      %.2f  (zrt_render call %.2f s, %u GPU)\n",
               double(stats.rays_processed) / render_runtime / 1e6, call, stats.n_gpus);

  rc = zrt_image_write_png(filename, image.data(), width, height);
  zrt_scene_free(data);
  if (rc != ZRT_OK) {
    std::fprintf(stderr, "error: %s\n", zrt_last_error());
    return 1;
  }
  return 0;
}
