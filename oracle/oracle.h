/*
 * ORACLE — test infrastructure only.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load liboracle.so; the product library
 * (zraytrace_amd/libzrt.so) neither links nor calls it.
 *
 * oracle.h — single-threaded CPU restatement of the reference's hot path
 * (jsyrjala/zraytrace, Zig), used as the parity checker of the HIP path and as
 * the reported CPU baseline ("kind": "port").  It consumes the same flat scene
 * description as the product boundary (include/zrt.h) and restates:
 *
 *   raytrace.zig:53-100, 111-203   rayColor / backgroundColor / render loops
 *   camera.zig:17-52               Camera.init / getRay
 *   ray.zig:11-16                  Ray.init (normalizes) / rayAt
 *   vector.zig:65-139              Vec3 arithmetic
 *   aabb.zig:16-127                AABB construction, pseudo surface area, slab test
 *   bvh.zig:38-205                 BVH build (stable sort, n/4 n/2 3n/4 splits) + traversal
 *   sphere.zig:24-71, triangle.zig:32-70, hit_record.zig:28-41
 *   material.zig:43-129            Lambertian / Metal / Dielectric scatter
 *   sample.zig:47-61               randomHemisphere / randomUnitVector
 *   texture.zig:11-74              color / image texture lookup (V-wrap bug kept)
 *
 * Two RNG modes:
 *   ZRT_RNG_REFERENCE_STREAM: one DefaultPrng.init(seed) stream for the whole
 *     render, consumed in the reference's order (pixel jitter x then y, then
 *     every scatter draw) — the reference algorithm as written.
 *   ZRT_RNG_COUNTER: the same arithmetic, but every (pixel, sample) starts its
 *     own stream, DefaultPrng.init(((y*width+x) << 16 | sample) + seed*0x9E3779B97F4A7C15).
 *     The per-pixel sum is taken in chunks of params->sample_chunk samples
 *     (zrt.h), the kernel's unit of work.  This is the bit-for-bit partner of
 *     the GPU kernel.
 */
#ifndef ZRT_ORACLE_H
#define ZRT_ORACLE_H

#include "../include/zrt.h"

#ifdef __cplusplus
extern "C" {
#endif

int oracle_render(const zrt_scene* scene, const zrt_camera* camera,
                  const zrt_params* params, float* out_rgb, zrt_stats* stats);

/* Render only rows [y0, y1) (same per-pixel results as the full render in
 * counter mode; reference-stream mode requires y0 == 0). */
int oracle_render_rows(const zrt_scene* scene, const zrt_camera* camera,
                       const zrt_params* params, uint32_t y0, uint32_t y1,
                       float* out_rgb, zrt_stats* stats);

/* The whole frame plus, per scanline y, the Progress deltas printProgress
 * reports after it (raytrace.zig:37-50, 184-186; rows: height entries). */
int oracle_render_scanlines(const zrt_scene* scene, const zrt_camera* camera,
                            const zrt_params* params, float* out_rgb, zrt_stats* stats,
                            zrt_scanline* rows);

/* BVH built exactly as bvh.zig:62-185, exported in zrt_bvh_node form
 * (pre-order, left first; child < 0 = prim -(c+1)).  Free with oracle_free. */
int oracle_bvh_build(const zrt_scene* scene, zrt_bvh_node** nodes,
                     uint32_t* n_nodes, uint32_t* max_depth);

/* One rayColor closest-hit query (raytrace.zig:71-81 over preprocessSufraces'
 * top-level list, BVHNode.hit bvh.zig:187-205 under BVH) per ray: rays are
 * n x {origin, direction} (Ray.init normalises), t_min 0.001.  out_t = +inf and
 * out_prim = -1 on a miss, else the hit t and the surface's list index. */
int oracle_trace(const zrt_scene* scene, int use_bvh, const float* rays, uint32_t n,
                 float* out_t, int32_t* out_prim);

/* The data of the reference's own BVH test (bvh.zig:234-247 createSurfaces and
 * bvh.zig:277-282): one DefaultPrng(seed) stream draws n_spheres spheres
 * {x, y, z, radius} and then n_rays rays {randomUnitVector * 100,
 * randomUnitVector}. */
void oracle_bvh_test_data(uint32_t prng, uint64_t seed, uint32_t n_spheres, uint32_t n_rays,
                          float* spheres, float* rays);

/* Camera.init (camera.zig:17-35). */
void oracle_camera_init(const float from[3], const float at[3], const float vup[3],
                        float vfov, float aspect, zrt_camera* out);

/* ---- known-answer hooks (reference unit tests) -------------------------- */
void oracle_prng_u64(uint32_t prng, uint64_t seed, uint64_t* out, int n);
void oracle_prng_f32(uint32_t prng, uint64_t seed, float* out, int n);
/* which: 0 randomVector, 1 randomVectorInUnitSphere, 2 randomUnitVector_old,
 * 3 randomUnitVector (sample.zig:9-61), starting from DefaultPrng.init(seed). */
void oracle_sample_vector(uint32_t prng, uint64_t seed, int which, float out[3]);
float oracle_math1(int fn, float x);          /* 0 sin 1 cos 2 acos 3 atan 4 sqrt */
float oracle_math2(int fn, float y, float x);  /* 0 atan2(y,x) 1 pow(y,x) */
void oracle_ray_at(const float o[3], const float d[3], float t, float out[3]);
void oracle_unit_vector(const float v[3], float out[3]);
/* Triangle.hit: returns 1 on hit; out: location[3], normal[3], t, front_face, u, v */
int oracle_triangle_hit(const float a[3], const float b[3], const float c[3],
                        const float o[3], const float d[3], float t_min, float t_max,
                        float out[9]);
/* Sphere.hit: returns 1 on hit; out as above (u, v = spherical texture coords) */
int oracle_sphere_hit(const float center[3], float radius, const float o[3],
                      const float d[3], float t_min, float t_max, float out[9]);
int oracle_aabb_hit(const float c1[3], const float c2[3], const float o[3],
                    const float d[3], float t_min, float t_max);
float oracle_aabb_surface_area(const float c1[3], const float c2[3]);
void oracle_texture_albedo(const zrt_image* img, float u_off, float v_off,
                           float u, float v, float out[3]);

void oracle_free(void* p);

#ifdef __cplusplus
}
#endif
#endif
