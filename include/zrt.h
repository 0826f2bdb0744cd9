/*
 * zrt.h — C ABI of the MI355X path tracer (libzrt.so).
 *
 * This is the drop-in boundary for the reference's per-pixel Monte-Carlo
 * sampling loop.  The reference seam is
 *
 *     pub fn render(allocator: *Allocator, random: *Random,
 *                   camera: Camera, surfaces: ArrayList(Surface),
 *                   render_params: RenderParams) !*Image
 *                                              (src/raytrace.zig:136-138)
 *
 * A Zig caller flattens `ArrayList(Surface)` (src/surface.zig:12-16), the
 * `*const Material` pointers (src/material.zig:16-52), the `Texture` values
 * (src/texture.zig:7-28) and the `*Image` pointers they reference into the flat
 * arrays of `zrt_scene`, keeping the reference list order, and calls
 * `zrt_render`.  See INTEGRATION.md for the `@cImport` adapter.
 *
 * Conventions (all from the reference):
 *   - f32 everywhere (src/base.zig:2).
 *   - Framebuffer: width*height RGB f32, row-major, row 0 = bottom of the image
 *     (src/raytrace.zig:164-182, src/image.zig:74-78).
 *   - Texture images: same layout, already flipped and scaled by 1/255 as
 *     src/png_image.zig:76-89 produces them.
 *   - Camera: the four vectors `Camera.init` computes (src/camera.zig:17-35);
 *     `zrt_camera_init` restates `Camera.init` on the host (tan stays on host).
 *
 * Errors: every entry point returns ZRT_OK (0) or a negative ZRT_E_* code and
 * leaves a message in a thread-local buffer read by `zrt_last_error()`.  This
 * maps 1:1 onto a Zig error union (`!*Image`).  No C++ exception crosses the ABI.
 *
 * Ownership: the library copies every input during the call and keeps no
 * pointer into caller memory after it returns.  `out_rgb` is caller-allocated.
 * Device memory is owned by the library (zrt_render) or by a zrt_ctx handle.
 * The library is not reentrant on one zrt_ctx; distinct contexts may be used
 * from distinct threads.
 */
#ifndef ZRT_H
#define ZRT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: zrt_stats gained sampling_loop (its size changed) and zrt_build_id was added;
 * a client built against version 1 must not pass its smaller zrt_stats. */
#define ZRT_ABI_VERSION 2

/* ---- status codes ------------------------------------------------------- */
enum {
  ZRT_OK = 0,
  ZRT_E_INVALID = -1,     /* bad argument (e.g. unknown kind, index out of range) */
  ZRT_E_NOMEM = -2,       /* host or device allocation failed (Zig: OutOfMemory) */
  ZRT_E_HIP = -3,         /* HIP runtime error */
  ZRT_E_UNSUPPORTED = -4, /* valid for the reference, not provided by this path */
  ZRT_E_NODEVICE = -5,    /* no usable MI355X (gfx950) device */
  ZRT_E_IO = -6,          /* asset file missing / unreadable */
  ZRT_E_PARSE = -7        /* OBJ parse error (obj_reader.zig ParseError) */
};

/* ---- scene description (flattened ArrayList(Surface)) ------------------- */
enum { ZRT_PRIM_SPHERE = 0, ZRT_PRIM_TRIANGLE = 1 };          /* surface.zig:12-16 */
enum { ZRT_MAT_LAMBERTIAN = 0, ZRT_MAT_METAL = 1, ZRT_MAT_DIELECTRIC = 2 }; /* material.zig:27-29 */
enum { ZRT_TEX_COLOR = 0, ZRT_TEX_IMAGE = 1 };                /* texture.zig:7-9 */

typedef struct zrt_vec3 { float x, y, z; } zrt_vec3;          /* vector.zig:22-25 */

/* Camera.{origin, lower_left_corner, horizontal, vertical} (camera.zig:11-15). */
typedef struct zrt_camera {
  zrt_vec3 origin;
  zrt_vec3 lower_left_corner;
  zrt_vec3 horizontal;
  zrt_vec3 vertical;
} zrt_camera;

/* One element of ArrayList(Surface).  kind selects the union member:
 *   SPHERE:   center, radius            (Sphere.init, sphere.zig:24-29)
 *   TRIANGLE: a, b, c (vertex order kept: Triangle.init, triangle.zig:32-44)
 * `material` indexes zrt_scene.materials (the deduplicated *const Material). */
typedef struct zrt_prim {
  uint32_t kind;
  uint32_t material;
  zrt_vec3 center;
  float radius;
  zrt_vec3 a, b, c;
} zrt_prim;

/* Material union (material.zig:16-52).  `texture` indexes zrt_scene.textures
 * and is used by LAMBERTIAN and METAL; `index_of_refraction` by DIELECTRIC. */
typedef struct zrt_material {
  uint32_t kind;
  uint32_t texture;
  float index_of_refraction;
} zrt_material;

/* Texture union (texture.zig:7-28): COLOR uses `color`; IMAGE uses `image`
 * (index into zrt_scene.images), `u_offset`, `v_offset` (Texture.initImage
 * passes 0.19, 0.1: texture.zig:14-16). */
typedef struct zrt_texture {
  uint32_t kind;
  uint32_t image;
  zrt_vec3 color;
  float u_offset;
  float v_offset;
} zrt_texture;

/* Image (image.zig:74-78): width*height RGB f32, row 0 = bottom. */
typedef struct zrt_image {
  uint32_t width;
  uint32_t height;
  const float* pixels;
} zrt_image;

typedef struct zrt_scene {
  const zrt_prim* prims;         /* reference list order (scenes.zig append order) */
  uint32_t n_prims;
  uint32_t n_materials;
  const zrt_material* materials;
  const zrt_texture* textures;
  uint32_t n_textures;
  uint32_t n_images;
  const zrt_image* images;
} zrt_scene;

/* ---- render parameters (RenderParams, raytrace.zig:102-108) ------------- */
enum {
  ZRT_RNG_COUNTER = 0,          /* per-(pixel,sample) stream; the GPU mode */
  ZRT_RNG_REFERENCE_STREAM = 1  /* one sequential stream as the reference; CPU oracle only */
};
enum { ZRT_PRNG_XOROSHIRO128 = 0, ZRT_PRNG_XOSHIRO256 = 1 };
enum {
  /* FAST: a 4-wide SAH tree built over the reference BVH's leaves culls with
   * the narrowed slab test; every leaf reached is put through the reference's
   * own slab test; equal-t ties go to the earlier leaf in the reference's DFS
   * order.  Same answers as REFERENCE. */
  ZRT_TRAVERSAL_FAST = 0,
  ZRT_TRAVERSAL_REFERENCE = 1,  /* left-first DFS with exactly bvh.zig:187-205's tests */
  ZRT_TRAVERSAL_BINARY = 2      /* near-first over the reference BVH itself, narrowed + loose tests */
};

typedef struct zrt_params {
  uint32_t width;                    /* RenderParams.width (u16 in the reference) */
  uint32_t height;                   /* RenderParams.height */
  uint32_t samples_per_pixel;        /* RenderParams.samples_per_pixel */
  uint32_t max_depth;                /* RenderParams.max_depth */
  uint32_t bounded_volume_hierarchy; /* RenderParams.bounded_volume_hierarchy (BVH iff also n>10) */
  uint32_t rng_mode;                 /* ZRT_RNG_* */
  uint32_t prng;                     /* ZRT_PRNG_* (DefaultPrng variant) */
  uint32_t traversal;                /* ZRT_TRAVERSAL_* */
  uint64_t seed;                     /* DefaultPrng.init(seed); the scenes use 42 */
  uint32_t rank;                     /* image-tile partition: this rank ... */
  uint32_t world_size;               /* ... of world_size (1 = whole frame) */
  uint32_t device;                   /* HIP device ordinal */
  /* COUNTER mode: a pixel's samples are summed in chunks of sample_chunk
   * consecutive samples (each chunk sequentially, as raytrace.zig:177 does),
   * and the chunk sums are then added in chunk order.  0 selects 32
   * (ZRT_DEFAULT_SAMPLE_CHUNK).  With sample_chunk >= samples_per_pixel this is
   * the reference's single sequential sum.  A chunk is the kernel's unit of
   * work: shorter units end a launch sooner. */
  uint32_t sample_chunk;
  uint32_t flags;                    /* ZRT_FLAG_* */
  uint32_t reserved;
} zrt_params;

/* flags: ZRT_FLAG_STATS launches the diagnostic flavour of the kernel that also
 * counts BVH node visits, primitive tests, shaded hits and texel fetches
 * (zrt_stats).  Images are identical; the default flavour counts only the
 * Progress counters (raytrace.zig:20-34). */
enum { ZRT_FLAG_STATS = 1u, ZRT_FLAG_NO_SCHEDULE = 2u, ZRT_FLAG_SCANLINES = 4u, ZRT_FLAG_GUARD = 8u };
enum { ZRT_DEFAULT_SAMPLE_CHUNK = 32u };
/* Scheduling (FAST traversal, spp >= 128, unless ZRT_FLAG_NO_SCHEDULE): a probe
 * launch renders 1 sample per pixel of every tile (results discarded) and
 * records each tile's cost; the tiles are radix-sorted by descending cost on
 * the device and the render launch hands out units costliest first, so no long
 * unit starts at the end of the launch.  Images do not depend on it. */

/* ZRT_FLAG_GUARD (FAST traversal): the grazing-triangle guard (DESIGN.md
 * section 3 "Triangles"): every box is widened by the reach of the rounded
 * triangle test (triangle.zig:48-70) for rays nearly parallel to a triangle,
 * whose accepted hits can lie outside their leaf's box.  zrt_trace always uses
 * it; a render uses it (in the path-pool loop) when this flag is set - the
 * reference's scenes render bit for bit the same frames without it, at a third
 * more speed on the teapot.  zrt_stats.guard reports the coefficient used. */

/* ZRT_FLAG_SCANLINES: the launch also counts the recursion-limit hits,
 * reflections and background hits of every frame row (the deltas that
 * printProgress prints after each scanline, raytrace.zig:37-50, 184), read
 * back with zrt_ctx_scanlines / zrt_multi_scanlines / zrt_render_progress.
 * Images and totals are unchanged; the counts are added per finished work
 * unit (a few atomics per 8x8 tile x sample chunk), so the flag costs little
 * but is off in the timed bench. */

/* Progress counters (raytrace.zig:20-34) + timings. */
typedef struct zrt_stats {
  uint64_t recursion_depth_hits;
  uint64_t reflections;
  uint64_t background_hits;
  uint64_t pixels_processed;
  uint64_t samples_processed;
  uint64_t rays_processed;
  uint64_t node_visits;   /* BVH nodes whose box was tested (diagnostic) */
  uint64_t prim_tests;    /* primitive intersection tests, triangles + spheres */
  uint64_t sphere_tests;  /* ... of which spheres */
  uint64_t shade_fetches; /* closest hits shaded (hit record + material reads) */
  uint64_t texel_fetches; /* image-texture lookups */
  uint64_t leaf_visits;   /* FAST traversal: reference leaf boxes tested (node_visits = wide nodes) */
  double preprocess_ms;   /* BVH build + flatten (raytrace.zig:150) */
  double upload_ms;
  double render_ms;       /* device time of the sampling loop: schedule probe + sort + render kernel */
  double gather_ms;
  uint32_t used_bvh;      /* preprocessSufraces decision (raytrace.zig:124-133) */
  uint32_t bvh_nodes;
  uint32_t bvh_max_depth; /* Tracking.max_depth (bvh.zig:23-30) */
  uint32_t n_gpus;
  uint32_t node_bytes;    /* bytes of one node record of the traversal used (32 or 128) */
  uint32_t wide_nodes;    /* FAST traversal: 4-wide nodes over the reference leaves */
  uint32_t texel_bytes;   /* bytes per texel on the device: 4 when every image is exact 8-bit
                             (c == k/255, png_image.zig:76-89), else 12 (f32 RGB); 0: no images */
  float schedule_ms;       /* probe + sort before the render launch (included in render_ms) */
  uint64_t order_replays;  /* FAST: rays re-traced the reference's way for an order hazard (diagnostic) */
  /* REFERENCE traversal + ZRT_FLAG_STATS (diagnostic, DESIGN.md §3 "Exactness"):
   * over every primitive of every leaf the reference opens, the largest
   * max(E/t - 1, t/X - 1) of its hit t (t_max = inf) against the leaf box's
   * loose entry E and exit X - how far rounded hits lie outside their own
   * box - per primitive kind, and how many hits lie out by more than 2^-14. */
  float box_excess_max_triangle;
  float box_excess_max_sphere;
  uint64_t box_excess_hits;
  /* the sampling loop of the last launch: 0 surface list, 1
   * binary / 2 reference BVH traversal, FAST traversal: 3 lockstep, 4 wavefront,
   * 5 path pool; 6 surface list with per-lane work items */
  uint32_t sampling_loop;
  /* the grazing-triangle guard's coefficient of the launch (0: off; ZRT_FLAG_GUARD) */
  float guard;
} zrt_stats;

/* One frame row's share of the Progress counters (raytrace.zig:20-34): what
 * raytrace.zig:184's printProgress(y + 1, ...) reports for scanline y as
 * deltas (recursion limit, reflections, background hits) and as running sums
 * (pixels, samples, rays: add rows 0..y).  rays = samples + reflections -
 * recursion_depth_hits (every rayColor call with depth > 0, raytrace.zig:69). */
typedef struct zrt_scanline {
  uint64_t recursion_depth_hits;
  uint64_t reflections;
  uint64_t background_hits;
  uint64_t pixels;
  uint64_t samples;
  uint64_t rays;
} zrt_scanline;

/* ---- entry points -------------------------------------------------------- */

/* Replaces raytrace.render (raytrace.zig:136-203): render the whole frame on
 * one GPU (params->device).  out_rgb: width*height*3 f32, caller-allocated.
 * rng_mode must be ZRT_RNG_COUNTER.  stats may be NULL. */
int zrt_render(const zrt_scene* scene, const zrt_camera* camera,
               const zrt_params* params, float* out_rgb, zrt_stats* stats);

/* zrt_render that also returns the per-scanline counters of raytrace.zig:184
 * (scanlines: params->height entries, row 0 = bottom, as the reference's y). */
int zrt_render_progress(const zrt_scene* scene, const zrt_camera* camera,
                        const zrt_params* params, float* out_rgb, zrt_stats* stats,
                        zrt_scanline* scanlines);

/* raytrace.render (raytrace.zig:136-203) over several GPUs of one node, from one
 * host thread: the frame's 8x8 tiles are dealt round-robin
 * over devices[0..n_devices) (tile t -> rank t % n_devices), every GPU holds its
 * own copy of the scene and renders its tiles concurrently, and ONE RCCL gather
 * (ncclGather over xGMI, ncclCommInitAll communicators) collects them on
 * devices[0], where they are assembled and copied to out_rgb.  The image is
 * bit-identical to zrt_render's for any device list.  A device listed more
 * than once runs several ranks (tests on one GPU); RCCL takes one rank per
 * device, so such a list gathers with device-to-device copies instead.  RCCL
 * (librccl.so.1) is opened on first use.  params->rank / world_size / device
 * are ignored.  stats: counters summed over ranks, render_ms = the slowest
 * rank's, gather_ms = gather + assemble, n_gpus = distinct devices. */
int zrt_render_multi(const zrt_scene* scene, const zrt_camera* camera,
                     const zrt_params* params, const uint32_t* devices,
                     uint32_t n_devices, float* out_rgb, zrt_stats* stats);

/* zrt_render_multi split into a persistent multi-GPU context (a Zig host
 * rendering many frames of one scene): zrt_multi_create builds the BVH once,
 * uploads the scene to every device of the list and creates the RCCL
 * communicators once (one rank per distinct device, >= 2 devices; otherwise
 * the tiles move by device copies and RCCL is not loaded).
 * zrt_multi_render renders one frame as zrt_render_multi does (same image,
 * same stats); params->rank / world_size / device are ignored and
 * params->bounded_volume_hierarchy must imply the create-time BVH decision.
 * out_rgb may be NULL: the assembled frame then stays in devices[0]'s HBM
 * (a frame loop that times the GPUs, not the PCIe copy) and zrt_multi_frame
 * copies it out later. */
typedef struct zrt_multi zrt_multi;
int zrt_multi_create(const zrt_scene* scene, const zrt_params* params,
                     const uint32_t* devices, uint32_t n_devices, zrt_multi** out);
int zrt_multi_render(zrt_multi* multi, const zrt_camera* camera,
                     const zrt_params* params, float* out_rgb, zrt_stats* stats);
int zrt_multi_destroy(zrt_multi* multi);
/* The last zrt_multi_render's frame (n_floats = width * height * 3, row 0 =
 * bottom) copied from devices[0] to out_rgb. */
int zrt_multi_frame(zrt_multi* multi, float* out_rgb, uint64_t n_floats);
/* The last zrt_multi_render's render-kernel time of each rank in ms (HIP
 * events around its launch; n = n_devices of zrt_multi_create). */
int zrt_multi_rank_ms(zrt_multi* multi, double* kernel_ms, uint32_t n);
/* Per-scanline counters of the last zrt_multi_render made with
 * ZRT_FLAG_SCANLINES, summed over the ranks (height = params->height). */
int zrt_multi_scanlines(zrt_multi* multi, zrt_scanline* out, uint32_t height);

/* The closest-hit query of one rayColor step (raytrace.zig:71-81: the top-level
 * surfaces tested with t_min = 0.001 and a shrinking t_max; under BVH that is
 * BVHNode.hit, bvh.zig:187-205) for a batch of rays on params->device, through
 * the render loop's own traversal (params->traversal).  rays: n_rays x {origin
 * xyz, direction xyz}, directions normalised as Ray.init does (ray.zig:11-13).
 * out_t: the hit's t (+inf on a miss); out_prim: the index of the surface hit
 * in scene->prims (-1 on a miss).  One-shot like zrt_render. */
int zrt_trace(const zrt_scene* scene, const zrt_params* params, const float* rays,
              uint32_t n_rays, float* out_t, int32_t* out_prim);

/* Restates Camera.init (camera.zig:17-35).  look_from/look_at/vup: float[3]. */
int zrt_camera_init(const float look_from[3], const float look_at[3],
                    const float vup[3], float vfov_deg, float aspect_ratio,
                    zrt_camera* out);

/* Thread-local message for the last error on this thread ("" if none). */
const char* zrt_last_error(void);

/* ABI version (ZRT_ABI_VERSION) and build identity string. */
int zrt_abi_version(void);
const char* zrt_build_info(void);
/* What the kernels of this library were built from: sha1 of the device and
 * tree-layout sources + zrt.h (16 hex digits) - sha1 of the device compile
 * flags (8).  Performance-counter records are keyed by it (bench.py). */
const char* zrt_build_id(void);

/* ---- device-resident context (bench / multi-GPU) ------------------------ *
 * zrt_ctx_create does preprocessSufraces (BVH build, raytrace.zig:124-133),
 * flattens the scene and uploads it once to params->device.  zrt_ctx_render
 * then runs only the sampling loop, reading the resident scene and writing a
 * device buffer, so a timed region sees no host<->device traffic.           */
typedef struct zrt_ctx zrt_ctx;

int zrt_ctx_create(const zrt_scene* scene, const zrt_params* params, zrt_ctx** out);
int zrt_ctx_destroy(zrt_ctx* ctx);

/* Number of 8x8 tiles this (rank, world_size) owns; its tile buffer holds
 * n_tiles*64*3 floats.  Tiles are dealt round-robin: tile t -> rank t % world.
 * Tiles cover x in [0, height) (raytrace.zig:168's bound) by y in [0, height).
 * Host-only: ctx may be NULL. */
int zrt_ctx_tile_count(const zrt_ctx* ctx, const zrt_params* params, uint32_t* n_tiles);

/* Render this rank's tiles into dev_tiles (device pointer, tile-major,
 * n_tiles*64*3 f32) on `hip_stream` (a hipStream_t; NULL = the context's own
 * stream, a blocking stream, so work the caller later enqueues on the legacy
 * default stream waits for it).  Asynchronous: returns after enqueueing.
 * zrt_ctx_sync / zrt_ctx_stats / zrt_ctx_last_kernel_ms wait for the launch
 * (on whichever stream it ran) and return ZRT_E_UNSUPPORTED if the device
 * reported an error (a traversal stack overflow); such a launch also writes
 * NaN to every pixel of dev_tiles, and the next zrt_ctx_render_tiles on the
 * context returns the error if the launch has finished by then.
 * params->device must be the context's device, and params->
 * bounded_volume_hierarchy must imply the BVH decision the context was built
 * with (ZRT_E_INVALID otherwise). */
int zrt_ctx_render_tiles(zrt_ctx* ctx, const zrt_camera* camera,
                         const zrt_params* params, float* dev_tiles,
                         void* hip_stream);

/* This rank's per-scanline counters of the last launch, which must have been
 * made with ZRT_FLAG_SCANLINES (ZRT_E_INVALID otherwise); out: height entries
 * (rows of the frame; rows this rank owns no tiles of stay zero). Waits. */
int zrt_ctx_scanlines(zrt_ctx* ctx, zrt_scanline* out, uint32_t height);

/* Wait for the context's last launch; ZRT_OK, or ZRT_E_UNSUPPORTED when the
 * device reported an error during it (see zrt_ctx_render_tiles). */
int zrt_ctx_sync(zrt_ctx* ctx);

/* Scatter gathered tiles of all ranks (rank-major: rank r's n_tiles(r) tiles
 * follow rank r-1's) into the framebuffer layout of raytrace.zig:182.
 * dev_gathered / dev_frame are device pointers; runs on hip_stream. */
int zrt_ctx_assemble(zrt_ctx* ctx, const zrt_params* params,
                     const float* dev_gathered, float* dev_frame, void* hip_stream);

/* The same from the layout a gather of equal per-rank counts produces: rank r's
 * tiles start at tile r * stride_tiles (stride_tiles >= every rank's count;
 * the tiles past a rank's count are padding and are not read). */
int zrt_ctx_assemble_padded(zrt_ctx* ctx, const zrt_params* params,
                            const float* dev_gathered, uint32_t stride_tiles,
                            float* dev_frame, void* hip_stream);

/* Counters of the last zrt_ctx_render_tiles (waits for that launch). */
int zrt_ctx_stats(zrt_ctx* ctx, zrt_stats* out);

/* Raw device counter slots of the last launch (diagnostics; n <= 32):
 * [0..9] progress/traffic counters, [14] work counter, [15] error flag,
 * [16..20] per-section cycle sums of ZRT_PROFILE builds. */
int zrt_ctx_debug_counters(zrt_ctx* ctx, uint64_t* out, uint32_t n);

/* The last launch's schedule (diagnostics): per local tile, the probe's cost
 * (loop iterations its wave spent on ZRT_PROBE_SPP samples per pixel), and the tile order
 * the render launch used.  *n_tiles = 0 when the launch was not scheduled. */
int zrt_ctx_debug_schedule(zrt_ctx* ctx, uint32_t* costs, uint32_t* order, uint32_t cap, uint32_t* n_tiles);

/* ZRT_PROFILE builds only (diagnostics): {start, end} s_memrealtime stamps
 * (100 MHz) of every wave of the last render launch; *n_waves = 0 otherwise. */
int zrt_ctx_debug_wave_times(zrt_ctx* ctx, uint64_t* out, uint32_t cap, uint32_t* n_waves);

/* Duration in ms of the last zrt_ctx_render_tiles' kernel (HIP events on the
 * launch stream; synchronises). */
int zrt_ctx_last_kernel_ms(zrt_ctx* ctx, double* ms);

/* ---- host-side scene ingestion (the caller side of the seam) ------------- *
 * Restatement of scenes.zig / obj_reader.zig / png_image.zig texture loading
 * so tests and bench can build the reference's scenes without Zig.  Assets are
 * read from `assets_dir` (OBJ files and P6 PPM textures, tools/prepare_assets.py). */
typedef struct zrt_scene_data zrt_scene_data;

/* Build scene `scene_index` as scenes.zig:267-277 does (0 man+ball, 1 seven
 * spheres, 2 bunny+ball, 3 teapot+ball, 4 teapot+ball circle, 5 goat - needs
 * high_poly_goat.obj, which the reference does not ship: ZRT_E_IO without it),
 * plus 6: the textured, subdivided teapot that stands in for config C5
 * (DESIGN.md section 4).  The camera is returned in *camera; the scene view
 * stays valid until zrt_scene_free.  Unknown index -> ZRT_E_INVALID
 * (SceneError.UnkownSceneIndex). */
int zrt_scene_load(uint32_t scene_index, const char* assets_dir,
                   zrt_scene_data** out, zrt_camera* camera);
const zrt_scene* zrt_scene_view(const zrt_scene_data* data);
void zrt_scene_free(zrt_scene_data* data);

/* Binary scene files: a loaded (or any caller-built) scene and its camera
 * written as the flat arrays above, so a million-triangle mesh (the C5
 * substitute: 1.6 M triangles) is read back in a fraction of the OBJ parse +
 * subdivision time.  zrt_scene_read returns the same opaque handle as
 * zrt_scene_load (zrt_scene_view / zrt_scene_free).  ZRT_E_IO on an
 * unopenable / truncated file, ZRT_E_PARSE on a foreign or inconsistent one. */
int zrt_scene_write(const zrt_scene* scene, const zrt_camera* camera, const char* path);
int zrt_scene_read(const char* path, zrt_scene_data** out, zrt_camera* camera);

/* Parse an OBJ file into triangles (obj_reader.zig:114-198), all with material
 * `material`.  *out_prims is malloc'd; free with zrt_free. */
int zrt_obj_read(const char* path, uint32_t material, zrt_prim** out_prims, uint32_t* n_prims);
void zrt_free(void* p);

/* ---- image output (the caller side: main.zig:33 writes the rendered image) -- *
 * `rgb` is a framebuffer as zrt_render returns it (row 0 = bottom).
 * PNG: png_image.zig:96-148 - 8-bit RGB, top row first,
 *      u8(std.math.clamp(255.999 * c, 0, 255)) per channel.
 * PPM: ppm_image.zig - plain P3 text, u32(c * 255.999) clamped to [0, 255].
 * Unopenable path -> ZRT_E_IO (PngError.FailedToOpenFile). */
/* png_image.readFile (png_image.zig:19-94): an 8-bit RGB or RGBA PNG (other
 * color types and depths: ZRT_E_UNSUPPORTED, the reference's
 * UnsupportedPngFeature) as width*height RGB f32, row 0 = bottom, c/255, alpha
 * dropped.  Also reads 8-bit binary PPM (P6).  *out_pixels: free with zrt_free. */
int zrt_image_read_png(const char* path, uint32_t* width, uint32_t* height, float** out_pixels);
int zrt_image_write_png(const char* path, const float* rgb, uint32_t width, uint32_t height);
int zrt_image_write_ppm(const char* path, const float* rgb, uint32_t width, uint32_t height);

/* ---- BVH export (parity of bvh.zig:62-185 against the oracle) ------------- *
 * Node i: box min/max and two children.  A child c >= 0 is a node index; a
 * child c < 0 is primitive (-c - 1) in reference list order.  Leaves are
 * exactly the reference's (one prim on both sides, or s[1], s[0]).  The root
 * is node 0; nodes are in depth-first (left-first) pre-order. */
typedef struct zrt_bvh_node {
  zrt_vec3 min;
  int32_t left;
  zrt_vec3 max;
  int32_t right;
} zrt_bvh_node;

int zrt_bvh_build(const zrt_scene* scene, zrt_bvh_node** out_nodes,
                  uint32_t* n_nodes, uint32_t* max_depth);

/* The same tree built on GPU `device` (bvh.zig:62-185 level by level: each
 * level's stable axis sorts as segmented radix sorts, the split scores as
 * one wave per segment).  Node for node equal to zrt_bvh_build.
 * The context entry points use it for scenes of >= 65536 primitives.
 * ZRT_E_UNSUPPORTED for < 3 primitives or NaN midpoints (the host build
 * handles those). */
int zrt_bvh_build_device(const zrt_scene* scene, uint32_t device, zrt_bvh_node** out_nodes,
                         uint32_t* n_nodes, uint32_t* max_depth);

/* ---- device parity probes ------------------------------------------------ *
 * Evaluate the kernel's own device functions on inputs, for bit-exact
 * comparison with the oracle's restatements:
 *   fn 0 sin, 1 cos (std.math, Go/Cephes), 2 acos, 3 atan (musl), 4 sqrt,
 *   5 atan2(x[i], y[i]), 6 pow(x[i], 5.0), 7 x[i] / y[i] (HIP's IEEE `/`),
 *   8 1 / x[i] and 9 x[i] / y[i] through the kernel's short correctly rounded
 *   sequences (rcp_rn / div_rn, device_math.hpp).
 * zrt_debug_rng writes n outputs of DefaultPrng.init(key).next() computed on
 * the device.  zrt_debug_division runs the device self-check of those short
 * sequences against IEEE `/` and sqrtf (counts[5]: mismatches of the reciprocal
 * and the square root over all 2^32 inputs, of division, unit(), 1/d and the jitter quotient over n hashed
 * inputs each; all zero on a correct build).  All run on `device` and synchronise. */
int zrt_debug_math(int fn, const float* x, const float* y, float* out, uint32_t n, uint32_t device);
int zrt_debug_rng(uint32_t prng, uint64_t key, uint64_t* out, uint32_t n, uint32_t device);
int zrt_debug_division(uint64_t n, uint64_t* counts, uint32_t device);
/* Host-side check of the kernels' LDS layouts for this scene (no device
 * needed): the scene is flattened as zrt_ctx_create does, then every plan the
 * launch code can make - each sampling loop, stack width, PRNG and a range of
 * max depths - is checked region by region (stack rows, top wide nodes, pool
 * queues, lane state, attenuation rows, materials: in the block's LDS, disjoint,
 * float4 regions 16-B aligned; the lockstep loop's plan within its 6-block
 * share).  n_checked: the number of plans checked.  ZRT_E_UNSUPPORTED names the
 * first violation. */
int zrt_debug_lds_plans(const zrt_scene* scene, uint32_t* n_checked);
/* Host-side check of the global buffers the launches of a FAST frame share (no
 * device needed): for every sampling loop, stack width, PRNG, node format, a
 * range of max depths and grid sizes, zrt_render's sizing of the attenuation
 * rows and stack overflow rows (the render launch's need, grown to its
 * scheduling probe's) is checked against what each of the two launches needs
 * (zrt::buffer_need; the same check guards every launch, ZRT_E_UNSUPPORTED
 * instead of a device fault).  legacy = 1 applies the sizing before the round-5
 * fix (the probe shared the render's attenuation rows without growing them):
 * it must fail where a loop keeps more rows in LDS than the probe's 4.
 * n_checked: configurations checked. */
int zrt_debug_buffer_plans(const zrt_scene* scene, uint32_t legacy, uint32_t* n_checked);
/* Host-side check of the compressed wide nodes built for this scene (no device
 * needed): every plane of every node's eight octant copies decodes exactly to
 * an f32, every slot's decoded box contains the full node's box of that slot,
 * near / far bytes are the full node's min / max in the octant's order, and
 * every leaf slot's record holds the full node's leaf box and primitive refs bit
 * for bit.  n_checked: the slots checked.  ZRT_E_UNSUPPORTED names the first
 * violation (or a tree the encoder refused). */
int zrt_debug_qnodes(const zrt_scene* scene, uint64_t* n_checked);

#ifdef __cplusplus
}
#endif
#endif /* ZRT_H */
