// zrt.hpp — C++ host mirror of the reference's scene/render API.
//
// The reference host is Zig (no Zig toolchain exists in this image), so the
// host side above the C ABI (include/zrt.h) is this C++ layer.  It keeps the
// reference's names, argument meaning and error behaviour:
//
//   Vec3           vector.zig:22-139          Camera     camera.zig:11-52
//   Color, Image   image.zig:9-103             Texture    texture.zig:7-74
//   Material       material.zig:16-52          Surface    surface.zig:12-60
//   RenderParams   raytrace.zig:102-108        render     raytrace.zig:136-203
//   DefaultPrng    std.rand.DefaultPrng (the *Random every scene threads through)
//
// `render` flattens the surface list and the materials/textures/images they
// point at into the C-ABI arrays and calls zrt_render (the HIP path).  Errors
// surface as zrt::Error (the Zig error union's counterpart).
#pragma once

#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/zrt.h"

namespace zrt {

struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& msg) : std::runtime_error(msg), code(c) {}
};

struct Vec3 {
  float x, y, z;
  static Vec3 init(float x, float y, float z) { return Vec3{x, y, z}; }
  static const Vec3 origin, x_unit, y_unit, z_unit;
  Vec3 plus(Vec3 o) const { return {x + o.x, y + o.y, z + o.z}; }
  Vec3 minus(Vec3 o) const { return {x - o.x, y - o.y, z - o.z}; }
  Vec3 scale(float s) const { return {x * s, y * s, z * s}; }
};

struct Color {
  float r, g, b;
  static Color init(float r, float g, float b) { return Color{r, g, b}; }
  static const Color black, white, gold, silver, red, green, blue;  // image.zig:16-22
};

// image.zig:74-103: width*height Colors, row 0 = bottom.
struct Image {
  uint32_t width = 0, height = 0;
  std::vector<float> pixels;  // RGB f32
  static std::unique_ptr<Image> init(uint32_t width, uint32_t height);
};

// png_image.zig:19-94 for the textures the scenes load; the assets are the
// same 8-bit samples stored as P6 (tools/prepare_assets.py).  Rows are flipped
// and scaled c/255 in f32 as png_image.zig:86 does.
std::unique_ptr<Image> readImageFile(const std::string& path);
// png_image.zig:19-94 on the bytes of a PNG file (image_io.cpp)
std::unique_ptr<Image> decode_png(const std::string& path, const std::vector<uint8_t>& bytes);

// DefaultPrng.init(seed): the random source render() and the materials share.
struct DefaultPrng {
  uint64_t seed;
  explicit DefaultPrng(uint64_t s) : seed(s) {}
  DefaultPrng* random() { return this; }
};
using Random = DefaultPrng;

struct Texture {
  uint32_t kind = ZRT_TEX_COLOR;
  Color color{0, 0, 0};
  const Image* image = nullptr;
  float u_offset = 0, v_offset = 0;
  static Texture initColor(Color c);
  static Texture initImage(const Image* img);  // offsets 0.19, 0.1 (texture.zig:14-16)
  static Texture initImageOpts(const Image* img, float u_offset, float v_offset);
};

struct Material {
  uint32_t kind = ZRT_MAT_METAL;
  Texture texture;
  float index_of_refraction = 0;
  Random* random = nullptr;  // Lambertian / Dielectric hold the scene's *Random
  static Material initLambertian(Random* random, Texture t);
  static Material initMetal(Texture t);
  static Material initDielectric(Random* random, float index_of_refraction);
  static Material greenMatte(Random* random);  // material.zig:23-25
  static const Material black_metal, silver_metal, blue_metal, green_metal;  // :18-21
};

struct Surface {
  uint32_t kind = ZRT_PRIM_SPHERE;
  Vec3 center{0, 0, 0};
  float radius = 0;
  Vec3 a{0, 0, 0}, b{0, 0, 0}, c{0, 0, 0};
  const Material* material = nullptr;
  static Surface initSphere(Vec3 center, float radius, const Material* m);
  static Surface initTriangle(Vec3 a, Vec3 b, Vec3 c, const Material* m);
};

struct Camera {
  Vec3 origin, lower_left_corner, horizontal, vertical;
  static Camera init(Vec3 look_from, Vec3 look_at, Vec3 vup, float vfov, float aspect_ratio);
  zrt_camera abi() const;
};

struct RenderParams {
  uint16_t width, height, samples_per_pixel, max_depth;
  bool bounded_volume_hierarchy = true;
};

// obj_reader.zig:114-198: triangles of every face, all with `material`.
std::vector<Surface> readObjFile(const std::string& path, const Material* material);

// Flattened view of a surface list (what crosses the C ABI).
struct FlatScene {
  std::vector<zrt_prim> prims;
  std::vector<zrt_material> materials;
  std::vector<zrt_texture> textures;
  std::vector<zrt_image> images;
  zrt_scene view{};
  void finalize();
};
FlatScene flatten(const std::vector<Surface>& surfaces);

// raytrace.zig:136-203 on the GPU.
std::unique_ptr<Image> render(Random* random, const Camera& camera,
                              const std::vector<Surface>& surfaces,
                              const RenderParams& params, zrt_stats* stats = nullptr,
                              uint32_t device = 0);

// A scene of scenes.zig: the owned materials/images, the surface list, camera.
struct SceneData {
  std::unique_ptr<DefaultPrng> prng;
  std::vector<std::unique_ptr<Image>> images;
  std::vector<std::unique_ptr<Material>> materials;
  std::vector<Surface> surfaces;
  Camera camera;
  FlatScene flat;
};
// scenes.zig:267-277 render_scene's scene table (0..5).
std::unique_ptr<SceneData> buildScene(uint32_t scene_index, const std::string& assets_dir);

// thread-local error slot behind zrt_last_error()
void set_error(const std::string& msg);
int fail(int code, const std::string& msg);

}  // namespace zrt
