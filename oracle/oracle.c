/*
 * ORACLE — test infrastructure only (see oracle.h for scope and citations).
 * Deliberately written like the reference: recursive rayColor, pointer-based
 * BVH of "Surface" unions, per-call HitRecord values.  Compiled with
 * -ffp-contract=off so each f32 operation rounds once, in source order.
 */
#include "oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "zig_std.h"

/* ---- vector.zig --------------------------------------------------------- */
typedef struct { float x, y, z; } V3;
typedef struct { float u, v; } V2;

static inline V3 v3(float x, float y, float z) { V3 r = {x, y, z}; return r; }
static inline float v_elem(V3 v, int i) { return i == 0 ? v.x : (i == 1 ? v.y : v.z); }
/* vector.zig:65-67 dot */
static inline float v_dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
/* vector.zig:70-74 cross */
static inline V3 v_cross(V3 u, V3 v) {
  return v3(u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x);
}
static inline float v_len2(V3 v) { return v.x * v.x + v.y * v.y + v.z * v.z; }
static inline float v_len(V3 v) { return zs_sqrt(v_len2(v)); }
/* vector.zig:88-92 unitVector: divide by the length (zero -> NaN) */
static inline V3 v_unit(V3 v) { const float l = v_len(v); return v3(v.x / l, v.y / l, v.z / l); }
static inline V3 v_neg(V3 v) { return v3(-v.x, -v.y, -v.z); }
static inline V3 v_add(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline V3 v_sub(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline V3 v_scale(V3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
/* vector.zig:127-129 reflect: v - n*(2*(v.n)) */
static inline V3 v_reflect(V3 v, V3 n) { return v_sub(v, v_scale(n, 2.0f * v_dot(v, n))); }
/* vector.zig:132-137 refract */
static inline V3 v_refract(V3 v, V3 n, float ratio) {
  const float cos_theta = zs_min(v_dot(v_neg(v), n), 1.0f);
  const V3 r_out_perp = v_scale(v_add(v, v_scale(n, cos_theta)), ratio);
  const V3 r_out_parallel = v_scale(n, -zs_sqrt(fabsf(1.0f - v_len2(r_out_perp))));
  return v_add(r_out_perp, r_out_parallel);
}
static inline V3 c_mul(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }

/* ---- ray.zig ------------------------------------------------------------ */
typedef struct { V3 origin, direction; } Ray;
/* ray.zig:11-13: Ray.init always normalizes the direction */
static inline Ray ray_init(V3 o, V3 d) { Ray r; r.origin = o; r.direction = v_unit(d); return r; }
/* ray.zig:14-16 */
static inline V3 ray_at(const Ray* r, float t) { return v_add(r->origin, v_scale(r->direction, t)); }

/* ---- aabb.zig ----------------------------------------------------------- */
typedef struct { V3 min, max, midpoint; } AABB;
static inline V3 min_vec(V3 a, V3 b) { return v3(zs_min(a.x, b.x), zs_min(a.y, b.y), zs_min(a.z, b.z)); }
static inline V3 max_vec(V3 a, V3 b) { return v3(zs_max(a.x, b.x), zs_max(a.y, b.y), zs_max(a.z, b.z)); }
static inline V3 mid_vec(V3 a, V3 b) { return v3((a.x + b.x) / 2.0f, (a.y + b.y) / 2.0f, (a.z + b.z) / 2.0f); }
/* aabb.zig:37-41 */
static AABB aabb_min_max(V3 c1, V3 c2) {
  AABB b; b.min = min_vec(c1, c2); b.max = max_vec(c1, c2); b.midpoint = mid_vec(c1, c2); return b;
}
/* aabb.zig:68-71 */
static AABB aabb_union(AABB a, AABB b) { return aabb_min_max(min_vec(a.min, b.min), max_vec(a.max, b.max)); }
/* aabb.zig:99-105: "surface area" is 2*(dx^2+dy^2+dz^2) */
static float aabb_area(AABB b) {
  const V3 d = v_sub(b.min, b.max);
  const float dx = fabsf(d.x), dy = fabsf(d.y), dz = fabsf(d.z);
  return 2.0f * (dx * dx + dy * dy + dz * dz);
}

typedef struct { uint64_t node_visits, prim_tests; } Diag;

/* aabb.zig:109-127.  Each axis is tested against the caller's [t_min, t_max]
 * on its own (the interval is not narrowed across axes). */
static int aabb_hit(const AABB* box, const Ray* ray, float t_min, float t_max) {
  for (int i = 0; i < 3; ++i) {
    const float inv_d = 1.0f / v_elem(ray->direction, i);
    float t0 = (v_elem(box->min, i) - v_elem(ray->origin, i)) * inv_d;
    float t1 = (v_elem(box->max, i) - v_elem(ray->origin, i)) * inv_d;
    if (inv_d < 0.0f) { const float tmp = t0; t0 = t1; t1 = tmp; }
    const float tmin = zs_max(t0, t_min);
    const float tmax = zs_min(t1, t_max);
    if (tmax <= tmin) return 0;
  }
  return 1;
}

/* ---- texture.zig / material.zig ----------------------------------------- */
typedef struct {
  uint32_t kind;            /* ZRT_TEX_* */
  V3 color;
  const zrt_image* image;
  float u_offset, v_offset;
} Texture;

typedef struct {
  uint32_t kind;            /* ZRT_MAT_* */
  Texture texture;
  float index_of_refraction;
} Material;

/* @floatToInt(u64, f) as it executes for the values that can reach it: a
 * non-negative finite value truncates; NaN and out-of-range values convert to
 * 2^63 on x86-64 (cvttss2si), which the clamp then maps to the last texel. */
static uint64_t float_to_u64(float f) {
  if (f >= 0.0f && f < 18446744073709551616.0f) return (uint64_t)f;
  if (f < 0.0f && f > -1.0f) return 0;
  return 0x8000000000000000ULL;
}

/* texture.zig:52-74 (the V wrap tests uu_first, as the reference does: :66) */
static V3 image_albedo(const zrt_image* img, float u_offset, float v_offset, V2 tc) {
  const float uu_first = 1.0f - tc.u + u_offset;
  float uu = uu_first;
  if (uu_first > 1.0f) uu = uu_first - 1.0f;
  else if (uu_first < 0.0f) uu = uu_first + 1.0f;
  const float vv_first = tc.v + v_offset;
  float vv = vv_first;
  if (vv_first > 1.0f) vv = vv_first - 1.0f;
  else if (uu_first < 0.0f) vv = vv_first + 1.0f;
  uint64_t x = float_to_u64(uu * (float)img->width);
  uint64_t y = float_to_u64(vv * (float)img->height);
  if (x > (uint64_t)(img->width - 1)) x = img->width - 1;
  if (y > (uint64_t)(img->height - 1)) y = img->height - 1;
  const float* p = img->pixels + 3 * (y * img->width + x);
  return v3(p[0], p[1], p[2]);
}

/* texture.zig:20-27 */
static V3 texture_albedo(const Texture* t, V2 tc) {
  if (t->kind == ZRT_TEX_COLOR) return t->color;
  return image_albedo(t->image, t->u_offset, t->v_offset, tc);
}

/* ---- surfaces ------------------------------------------------------------ */
enum { S_SPHERE = 0, S_TRIANGLE = 1, S_BVH = 2 };

typedef struct Surface Surface;
typedef struct {
  V3 center; float radius; const Material* material; AABB aabb;
} Sphere;
typedef struct {
  V3 a, b, c, e1, e2, face_normal, face_unit_normal; const Material* material; AABB aabb;
} Triangle;
typedef struct {
  AABB aabb; const Surface* left; const Surface* right;
} BVHNode;
struct Surface {
  int kind;
  int32_t index;  /* prim: reference list index; node: export index */
  union { Sphere sphere; Triangle triangle; BVHNode node; } u;
};

typedef struct {
  V3 location, normal;
  float t;
  int front_face;
  const Surface* surface;
  V2 texture_coords;
} HitRecord;

/* hit_record.zig:28-41 */
static void hit_record_init(HitRecord* h, const Ray* ray, V3 location, V3 outward_normal,
                            float t, const Surface* s, V2 tc) {
  h->location = location;
  h->t = t;
  h->surface = s;
  h->texture_coords = tc;
  if (v_dot(ray->direction, outward_normal) > 0.0f) {
    h->normal = v_neg(outward_normal);
    h->front_face = 0;
  } else {
    h->normal = outward_normal;
    h->front_face = 1;
  }
}

/* sphere.zig:24-29 */
static void sphere_init(Surface* s, V3 center, float radius, const Material* m) {
  s->kind = S_SPHERE;
  s->u.sphere.center = center;
  s->u.sphere.radius = radius;
  s->u.sphere.material = m;
  s->u.sphere.aabb = aabb_min_max(v_sub(center, v3(radius, radius, radius)),
                                  v_add(center, v3(radius, radius, radius)));
}

/* triangle.zig:32-44 */
static void triangle_init(Surface* s, V3 a, V3 b, V3 c, const Material* m) {
  Triangle* t = &s->u.triangle;
  s->kind = S_TRIANGLE;
  t->aabb = aabb_union(aabb_min_max(a, b), aabb_min_max(a, c));
  t->a = a; t->b = b; t->c = c;
  t->e1 = v_sub(b, a);
  t->e2 = v_sub(c, a);
  t->face_normal = v_cross(t->e1, t->e2);
  t->face_unit_normal = v_unit(t->face_normal);
  t->material = m;
}

/* sphere.zig:31-71 */
static int sphere_hit(const Surface* s, const Ray* ray, float t_min, float t_max, HitRecord* out) {
  const Sphere* sp = &s->u.sphere;
  const V3 oc = v_sub(ray->origin, sp->center);
  const float half_b = v_dot(oc, ray->direction);
  const float c = v_len2(oc) - (sp->radius * sp->radius);
  const float discriminant = half_b * half_b - c;
  if (discriminant < 0.0f) return 0;
  const float root = zs_sqrt(discriminant);
  const float roots[2] = {-half_b - root, -half_b + root};
  for (int k = 0; k < 2; ++k) {
    const float t = roots[k];
    if (t < t_max && t > t_min) {
      const V3 location = ray_at(ray, t);
      const V3 outward_normal = v_scale(v_sub(location, sp->center), 1.0f / sp->radius);
      const float theta = zs_acos(-outward_normal.y);
      const float phi = zs_atan2(-outward_normal.z, -outward_normal.x) + (float)M_PI;
      V2 tc;
      tc.u = phi / (float)(2.0 * M_PI);
      tc.v = theta / (float)M_PI;
      hit_record_init(out, ray, location, outward_normal, t, s, tc);
      return 1;
    }
  }
  return 0;
}

/* triangle.zig:48-70 (single sided: det >= 1e-6) */
static int triangle_hit(const Surface* s, const Ray* ray, float t_min, float t_max, HitRecord* out) {
  const Triangle* tr = &s->u.triangle;
  const float det = -v_dot(ray->direction, tr->face_normal);
  const float inv_det = 1.0f / det;
  const V3 ao = v_sub(ray->origin, tr->a);
  const V3 dao = v_cross(ao, ray->direction);
  const float u = v_dot(tr->e2, dao) * inv_det;
  const float v = -v_dot(tr->e1, dao) * inv_det;
  const float t = v_dot(ao, tr->face_normal) * inv_det;
  const int is_hit = det >= 1e-6f && t > t_min && t < t_max && u >= 0.0f && v >= 0.0f &&
                     (u + v) <= 1.0f;
  if (!is_hit) return 0;
  const V3 location = v_add(ray->origin, v_scale(ray->direction, t));
  V2 tc = {u, v};
  hit_record_init(out, ray, location, tr->face_unit_normal, t, s, tc);
  return 1;
}

/* surface.zig:28-36 + bvh.zig:187-205 */
static int surface_hit(const Surface* s, const Ray* ray, float t_min, float t_max, HitRecord* out,
                       Diag* dg) {
  switch (s->kind) {
    case S_SPHERE:
      dg->prim_tests++;
      return sphere_hit(s, ray, t_min, t_max, out);
    case S_TRIANGLE:
      dg->prim_tests++;
      return triangle_hit(s, ray, t_min, t_max, out);
    default: {
      const BVHNode* n = &s->u.node;
      dg->node_visits++;
      if (!aabb_hit(&n->aabb, ray, t_min, t_max)) return 0;
      HitRecord hl;
      if (!surface_hit(n->left, ray, t_min, t_max, &hl, dg))
        return surface_hit(n->right, ray, t_min, t_max, out, dg);
      HitRecord hr;
      if (surface_hit(n->right, ray, t_min, hl.t, &hr, dg)) { *out = hr; return 1; }
      *out = hl;
      return 1;
    }
  }
}

/* surface.zig:39-48 */
static const Material* surface_material(const Surface* s) {
  return s->kind == S_SPHERE ? s->u.sphere.material : s->u.triangle.material;
}
/* surface.zig:51-60 */
static AABB surface_aabb(const Surface* s) {
  switch (s->kind) {
    case S_SPHERE: return s->u.sphere.aabb;
    case S_TRIANGLE: return s->u.triangle.aabb;
    default: return s->u.node.aabb;
  }
}

/* ---- bvh.zig build -------------------------------------------------------- */
typedef struct {
  Surface* pool;
  uint32_t n, cap;
  uint64_t max_depth;
} Builder;

static Surface* builder_alloc(Builder* b) { return &b->pool[b->n++]; }

/* bvh.zig:162-169 create */
static Surface* bvh_create(Builder* b, const Surface* left, const Surface* right) {
  Surface* s = builder_alloc(b);
  s->kind = S_BVH;
  s->index = -1;
  s->u.node.aabb = aabb_union(surface_aabb(left), surface_aabb(right));
  s->u.node.left = left;
  s->u.node.right = right;
  return s;
}

/* std.sort.sort is a stable (block) sort; a stable merge sort gives the
 * identical order for the same comparator. */
static int g_axis;
static int less_axis(const Surface* a, const Surface* b) {
  return v_elem(surface_aabb(a).midpoint, g_axis) < v_elem(surface_aabb(b).midpoint, g_axis);
}
static void merge_sort(Surface** a, Surface** tmp, size_t n) {
  if (n < 2) return;
  const size_t h = n / 2;
  merge_sort(a, tmp, h);
  merge_sort(a + h, tmp, n - h);
  size_t i = 0, j = h, k = 0;
  while (i < h && j < n) {
    if (less_axis(a[j], a[i])) tmp[k++] = a[j++];
    else tmp[k++] = a[i++];
  }
  while (i < h) tmp[k++] = a[i++];
  while (j < n) tmp[k++] = a[j++];
  memcpy(a, tmp, n * sizeof(*a));
}
static void sort_axis(int axis, Surface** s, size_t n, Surface** tmp) {
  g_axis = axis;
  merge_sort(s, tmp, n);
}

/* bvh.zig:62-69 surfaces_to_aabb -> aabb.zig:73-81 initAabbList -> :44-65 initVertexes */
static AABB surfaces_to_aabb(Surface** s, size_t n) {
  float mnx = INFINITY, mny = INFINITY, mnz = INFINITY;
  float mxx = -INFINITY, mxy = -INFINITY, mxz = -INFINITY;
  for (size_t i = 0; i < n; ++i) {
    const AABB b = surface_aabb(s[i]);
    const V3 vs[2] = {b.min, b.max};
    for (int k = 0; k < 2; ++k) {
      mnx = zs_min(mnx, vs[k].x); mny = zs_min(mny, vs[k].y); mnz = zs_min(mnz, vs[k].z);
      mxx = zs_max(mxx, vs[k].x); mxy = zs_max(mxy, vs[k].y); mxz = zs_max(mxz, vs[k].z);
    }
  }
  return aabb_min_max(v3(mnx, mny, mnz), v3(mxx, mxy, mxz));
}

/* bvh.zig:85-120 optimal_axis_divide; returns the split, leaves `s` sorted
 * by the best axis (re-sorted from the order the last trial left). */
static size_t optimal_axis_divide(Surface** s, size_t n, Surface** tmp) {
  int best_axis = 0;
  float best_ratio = INFINITY;
  size_t best_split = n / 2;
  const float total_area = aabb_area(surfaces_to_aabb(s, n));
  size_t splits[3];
  int n_splits = 1;
  splits[0] = n / 2;
  if (n >= 4) {
    splits[0] = n / 4; splits[1] = n / 2; splits[2] = n / 4 + n / 2;
    n_splits = 3;
  }
  for (int axis = 0; axis < 3; ++axis) {
    for (int k = 0; k < n_splits; ++k) {
      const size_t split = splits[k];
      sort_axis(axis, s, n, tmp);
      const AABB right = surfaces_to_aabb(s + split, n - split);
      const AABB left = surfaces_to_aabb(s, split);
      const float area = aabb_area(right) + aabb_area(left);
      const float ratio = area / total_area;
      if (ratio < best_ratio) {
        best_ratio = ratio;
        best_axis = axis;
        best_split = split;
      }
    }
  }
  sort_axis(best_axis, s, n, tmp);
  return best_split;
}

/* bvh.zig:129-160 divide */
static Surface* bvh_divide(Builder* b, Surface** s, size_t n, uint64_t depth, Surface** tmp) {
  if (b->max_depth < depth) b->max_depth = depth;
  if (n == 1) return bvh_create(b, s[0], s[0]);
  if (n == 2) return bvh_create(b, s[1], s[0]);
  const size_t split = optimal_axis_divide(s, n, tmp);
  Surface* left = bvh_divide(b, s, split, depth + 1, tmp);
  Surface* right = bvh_divide(b, s + split, n - split, depth + 1, tmp);
  return bvh_create(b, left, right);
}

/* ---- scene ----------------------------------------------------------------- */
typedef struct {
  Material* materials;
  Surface* prims;        /* reference list order */
  uint32_t n_prims;
  Builder bvh;           /* nodes */
  const Surface* root;   /* BVH root or NULL (surface list) */
  uint32_t n_top;
  const Surface** top;   /* the list rayColor loops over (raytrace.zig:75) */
} Scene;

static void scene_free(Scene* sc) {
  free(sc->materials);
  free(sc->prims);
  free(sc->bvh.pool);
  free((void*)sc->top);
  memset(sc, 0, sizeof(*sc));
}

static int scene_build(Scene* sc, const zrt_scene* in, int use_bvh_param) {
  memset(sc, 0, sizeof(*sc));
  sc->materials = (Material*)calloc(in->n_materials ? in->n_materials : 1, sizeof(Material));
  sc->prims = (Surface*)calloc(in->n_prims ? in->n_prims : 1, sizeof(Surface));
  if (!sc->materials || !sc->prims) return ZRT_E_NOMEM;
  for (uint32_t i = 0; i < in->n_materials; ++i) {
    const zrt_material* m = &in->materials[i];
    Material* o = &sc->materials[i];
    o->kind = m->kind;
    o->index_of_refraction = m->index_of_refraction;
    if (m->kind != ZRT_MAT_DIELECTRIC) {
      if (m->texture >= in->n_textures) return ZRT_E_INVALID;
      const zrt_texture* t = &in->textures[m->texture];
      o->texture.kind = t->kind;
      o->texture.color = v3(t->color.x, t->color.y, t->color.z);
      o->texture.u_offset = t->u_offset;
      o->texture.v_offset = t->v_offset;
      if (t->kind == ZRT_TEX_IMAGE) {
        if (t->image >= in->n_images) return ZRT_E_INVALID;
        o->texture.image = &in->images[t->image];
      }
    }
  }
  sc->n_prims = in->n_prims;
  for (uint32_t i = 0; i < in->n_prims; ++i) {
    const zrt_prim* p = &in->prims[i];
    if (p->material >= in->n_materials) return ZRT_E_INVALID;
    const Material* m = &sc->materials[p->material];
    if (p->kind == ZRT_PRIM_SPHERE)
      sphere_init(&sc->prims[i], v3(p->center.x, p->center.y, p->center.z), p->radius, m);
    else if (p->kind == ZRT_PRIM_TRIANGLE)
      triangle_init(&sc->prims[i], v3(p->a.x, p->a.y, p->a.z), v3(p->b.x, p->b.y, p->b.z),
                    v3(p->c.x, p->c.y, p->c.z), m);
    else
      return ZRT_E_INVALID;
    sc->prims[i].index = (int32_t)i;
  }
  /* raytrace.zig:124-133 preprocessSufraces */
  if (use_bvh_param && in->n_prims > 10) {
    Surface** ptrs = (Surface**)malloc(in->n_prims * sizeof(Surface*));
    Surface** tmp = (Surface**)malloc(in->n_prims * sizeof(Surface*));
    sc->bvh.cap = 2 * in->n_prims;
    sc->bvh.pool = (Surface*)calloc(sc->bvh.cap, sizeof(Surface));
    if (!ptrs || !tmp || !sc->bvh.pool) { free(ptrs); free(tmp); return ZRT_E_NOMEM; }
    for (uint32_t i = 0; i < in->n_prims; ++i) ptrs[i] = &sc->prims[i];
    sc->root = bvh_divide(&sc->bvh, ptrs, in->n_prims, 1, tmp);
    free(ptrs);
    free(tmp);
    sc->n_top = 1;
    sc->top = (const Surface**)malloc(sizeof(Surface*));
    sc->top[0] = sc->root;
  } else {
    sc->n_top = in->n_prims;
    sc->top = (const Surface**)malloc((in->n_prims ? in->n_prims : 1) * sizeof(Surface*));
    for (uint32_t i = 0; i < in->n_prims; ++i) sc->top[i] = &sc->prims[i];
  }
  return ZRT_OK;
}

/* ---- sample.zig ---------------------------------------------------------- */
/* sample.zig:47-53 randomHemisphere: phi = 2.0*pi*r2, the comptime product
 * 2*pi coerced to f32 first. */
static V3 random_hemisphere(zs_rng* r) {
  const float r1 = zs_random_float(r);
  const float r2 = zs_random_float(r);
  const float rr = zs_sqrt(1.0f - r1 * r1);
  const float phi = (float)(2.0 * M_PI) * r2;
  return v3(zs_cos(phi) * rr, zs_sin(phi) * rr, r1);
}
/* sample.zig:55-61 */
static V3 random_unit_vector(zs_rng* r) {
  const V3 v = random_hemisphere(r);
  if (zs_random_boolean(r)) return v;
  return v3(v.x, v.y, v.z * -1.0f);
}

/* ---- material.zig --------------------------------------------------------- */
typedef struct { Ray scattered; V3 attenuation; } Scattering;

/* material.zig:122-128 (r0 is not squared in the reference) */
static float reflectance(float cosine, float ref_idx) {
  const float r0 = (1.0f - ref_idx) / (1.0f + ref_idx);
  return r0 + (1.0f - r0) * zs_pow(1.0f - cosine, 5.0f);
}

/* material.zig:43-52 + 71-120 */
static int scatter(const Material* m, const Ray* ray, const HitRecord* h, zs_rng* rng,
                   Scattering* out) {
  switch (m->kind) {
    case ZRT_MAT_LAMBERTIAN: {
      const V3 dir = v_add(h->normal, random_unit_vector(rng));
      out->scattered = ray_init(h->location, dir);
      out->attenuation = texture_albedo(&m->texture, h->texture_coords);
      return 1;
    }
    case ZRT_MAT_METAL: {
      const V3 reflected = v_reflect(v_unit(ray->direction), h->normal);
      out->scattered = ray_init(h->location, reflected);
      if (v_dot(out->scattered.direction, h->normal) > 0.0f) {
        out->attenuation = texture_albedo(&m->texture, h->texture_coords);
        return 1;
      }
      return 0;
    }
    default: {
      out->attenuation = v3(1.0f, 1.0f, 1.0f);
      const float ratio = h->front_face ? (1.0f / m->index_of_refraction) : m->index_of_refraction;
      const V3 unit_direction = v_unit(ray->direction);
      const float cos_theta = zs_min(v_dot(v_neg(unit_direction), h->normal), 1.0f);
      const float sin_theta = zs_sqrt(1.0f - cos_theta * cos_theta);
      const int cannot_refract = ratio * sin_theta > 1.0f;
      if (cannot_refract || (double)reflectance(cos_theta, ratio) > (double)zs_random_float(rng)) {
        out->scattered = ray_init(h->location, v_reflect(unit_direction, h->normal));
        return 1;
      }
      out->scattered = ray_init(h->location, v_refract(unit_direction, h->normal, ratio));
      return 1;
    }
  }
}

/* ---- raytrace.zig --------------------------------------------------------- */
typedef struct {
  uint64_t recursion_depth_hits, reflections, background_hits, pixels, samples, rays;
} Progress;

typedef struct {
  const Scene* scene;
  zs_rng* rng;
  Progress p;
  Diag dg;
} Ctx;

/* raytrace.zig:53-58 */
static V3 background_color(const Ray* ray) {
  const V3 u = v_unit(ray->direction);
  const float t = 0.5f * (u.y + 1.0f);
  const V3 white = v_scale(v3(1.0f, 1.0f, 1.0f), 1.0f - t);
  return v_add(white, v_scale(v3(0.5f, 0.7f, 1.0f), t));
}

/* raytrace.zig:62-100 (recursive; attenuation * rayColor(scattered)) */
static V3 ray_color(Ctx* c, const Ray* ray, uint32_t depth) {
  if (depth == 0) {
    c->p.recursion_depth_hits++;
    return v3(0.0f, 0.0f, 0.0f);
  }
  c->p.rays++;
  const float t_min = 0.001f;
  float t_max = INFINITY;
  HitRecord closest;
  int have = 0;
  for (uint32_t i = 0; i < c->scene->n_top; ++i) {
    HitRecord h;
    if (surface_hit(c->scene->top[i], ray, t_min, t_max, &h, &c->dg)) {
      closest = h;
      have = 1;
      t_max = closest.t;
    }
  }
  if (!have) {
    c->p.background_hits++;
    return background_color(ray);
  }
  Scattering s;
  if (!scatter(surface_material(closest.surface), ray, &closest, c->rng, &s))
    return v3(0.0f, 0.0f, 0.0f);
  c->p.reflections++;
  return c_mul(s.attenuation, ray_color(c, &s.scattered, depth - 1));
}

/* camera.zig:46-52 */
static Ray camera_get_ray(const zrt_camera* cam, float u, float v) {
  const V3 llc = v3(cam->lower_left_corner.x, cam->lower_left_corner.y, cam->lower_left_corner.z);
  const V3 hor = v3(cam->horizontal.x, cam->horizontal.y, cam->horizontal.z);
  const V3 ver = v3(cam->vertical.x, cam->vertical.y, cam->vertical.z);
  const V3 org = v3(cam->origin.x, cam->origin.y, cam->origin.z);
  const V3 dir = v_sub(v_add(v_add(llc, v_scale(hor, u)), v_scale(ver, v)), org);
  return ray_init(org, dir);
}

static int validate(const zrt_scene* scene, const zrt_camera* camera, const zrt_params* p) {
  if (!scene || !camera || !p) return ZRT_E_INVALID;
  if (p->width == 0 || p->height == 0 || p->samples_per_pixel == 0) return ZRT_E_INVALID;
  if (p->width > 65535 || p->height > 65535 || p->samples_per_pixel > 65535 || p->max_depth > 65535)
    return ZRT_E_INVALID;  /* RenderParams fields are u16 (raytrace.zig:102-108) */
  /* raytrace.zig:168 loops x over image.height; with height > width the last
   * row's writes fall past the end of the pixel slice. */
  if (p->height > p->width) return ZRT_E_INVALID;
  if (scene->n_prims && !scene->prims) return ZRT_E_INVALID;
  return ZRT_OK;
}

static double now_ms(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6;
}

static uint64_t counter_key(uint64_t pixel, uint32_t sample, uint64_t seed) {
  return ((pixel << 16) | (uint64_t)sample) + seed * 0x9E3779B97F4A7C15ULL;
}

static int render_rows_impl(const zrt_scene* scene, const zrt_camera* camera, const zrt_params* p,
                            uint32_t y0, uint32_t y1, float* out, zrt_stats* stats, zrt_scanline* rows) {
  int rc = validate(scene, camera, p);
  if (rc) return rc;
  if (y1 > p->height || y0 > y1) return ZRT_E_INVALID;
  if (p->rng_mode == ZRT_RNG_REFERENCE_STREAM && y0 != 0) return ZRT_E_INVALID;
  const double t_start = now_ms();
  Scene sc;
  rc = scene_build(&sc, scene, p->bounded_volume_hierarchy != 0);
  if (rc) { scene_free(&sc); return rc; }
  const double t_built = now_ms();  /* raytrace.zig:150: preprocess timed apart from rendering */

  zs_rng global;
  zs_rng_init(&global, (int)p->prng, p->seed);
  Ctx c;
  memset(&c, 0, sizeof(c));
  c.scene = &sc;
  const float f_width = (float)p->width;
  const float f_height = (float)p->height;
  const float color_scale = 1.0f / (float)p->samples_per_pixel;
  const uint32_t chunk = p->sample_chunk ? p->sample_chunk : ZRT_DEFAULT_SAMPLE_CHUNK;
  for (uint32_t y = y0; y < y1; ++y) {
    const float f_y = (float)y;
    const Progress prev = c.p;  /* raytrace.zig:185 progress_prev */
    for (uint32_t x = 0; x < p->height; ++x) {  /* raytrace.zig:168 bound */
      const uint64_t offset = (uint64_t)y * p->width + x;
      V3 acc = v3(0.0f, 0.0f, 0.0f);
      V3 chunk_acc = v3(0.0f, 0.0f, 0.0f);
      for (uint32_t s = 0; s < p->samples_per_pixel; ++s) {
        zs_rng local;
        if (p->rng_mode == ZRT_RNG_COUNTER) {
          zs_rng_init(&local, (int)p->prng, counter_key(offset, s, p->seed));
          c.rng = &local;
        } else {
          c.rng = &global;
        }
        const float u = ((float)x + zs_random_float(c.rng) - 0.5f) / f_width;
        const float v = (f_y + zs_random_float(c.rng) - 0.5f) / f_height;
        const Ray ray = camera_get_ray(camera, u, v);
        const V3 col = ray_color(&c, &ray, p->max_depth);
        if (p->rng_mode == ZRT_RNG_COUNTER) {
          /* zrt.h sample_chunk: chunk sums, added in chunk order */
          chunk_acc.x += col.x; chunk_acc.y += col.y; chunk_acc.z += col.z;
          if ((s + 1) % chunk == 0 || s + 1 == p->samples_per_pixel) {
            acc.x += chunk_acc.x; acc.y += chunk_acc.y; acc.z += chunk_acc.z;
            chunk_acc = v3(0.0f, 0.0f, 0.0f);
          }
        } else {
          /* raytrace.zig:177 color_acc.addMutate: one sequential sum */
          acc.x += col.x; acc.y += col.y; acc.z += col.z;
        }
        c.p.samples++;
      }
      c.p.pixels++;
      const V3 px = v_scale(acc, color_scale);
      out[3 * offset + 0] = px.x;
      out[3 * offset + 1] = px.y;
      out[3 * offset + 2] = px.z;
    }
    if (rows) {  /* printProgress(y + 1, ...) (raytrace.zig:37-50, 184): this scanline's deltas */
      zrt_scanline* r = &rows[y];
      r->recursion_depth_hits = c.p.recursion_depth_hits - prev.recursion_depth_hits;
      r->reflections = c.p.reflections - prev.reflections;
      r->background_hits = c.p.background_hits - prev.background_hits;
      r->pixels = c.p.pixels - prev.pixels;
      r->samples = c.p.samples - prev.samples;
      r->rays = c.p.rays - prev.rays;
    }
  }
  if (stats) {
    memset(stats, 0, sizeof(*stats));
    stats->recursion_depth_hits = c.p.recursion_depth_hits;
    stats->reflections = c.p.reflections;
    stats->background_hits = c.p.background_hits;
    stats->pixels_processed = c.p.pixels;
    stats->samples_processed = c.p.samples;
    stats->rays_processed = c.p.rays;
    stats->node_visits = c.dg.node_visits;
    stats->prim_tests = c.dg.prim_tests;
    stats->used_bvh = sc.root != NULL;
    stats->bvh_nodes = sc.bvh.n;
    stats->bvh_max_depth = (uint32_t)sc.bvh.max_depth;
    stats->n_gpus = 0;
    stats->preprocess_ms = t_built - t_start;
    stats->render_ms = now_ms() - t_built;
  }
  scene_free(&sc);
  return ZRT_OK;
}

int oracle_render_rows(const zrt_scene* scene, const zrt_camera* camera, const zrt_params* p,
                       uint32_t y0, uint32_t y1, float* out, zrt_stats* stats) {
  return render_rows_impl(scene, camera, p, y0, y1, out, stats, NULL);
}

int oracle_render_scanlines(const zrt_scene* scene, const zrt_camera* camera, const zrt_params* p,
                            float* out, zrt_stats* stats, zrt_scanline* rows) {
  if (!p || !rows) return ZRT_E_INVALID;
  if (out && p->width && p->height)
    memset(out, 0, sizeof(float) * 3 * (size_t)p->width * p->height);
  memset(rows, 0, sizeof(zrt_scanline) * p->height);
  return render_rows_impl(scene, camera, p, 0, p->height, out, stats, rows);
}

int oracle_render(const zrt_scene* scene, const zrt_camera* camera, const zrt_params* p,
                  float* out, zrt_stats* stats) {
  if (!p) return ZRT_E_INVALID;
  if (out && p->width && p->height)
    memset(out, 0, sizeof(float) * 3 * (size_t)p->width * p->height);  /* Image.init: black */
  return oracle_render_rows(scene, camera, p, 0, p->height, out, stats);
}

/* ---- BVH export ------------------------------------------------------------ */
static int32_t export_node(const Surface* s, zrt_bvh_node* nodes, uint32_t* n) {
  const uint32_t me = (*n)++;
  const BVHNode* b = &s->u.node;
  nodes[me].min.x = b->aabb.min.x; nodes[me].min.y = b->aabb.min.y; nodes[me].min.z = b->aabb.min.z;
  nodes[me].max.x = b->aabb.max.x; nodes[me].max.y = b->aabb.max.y; nodes[me].max.z = b->aabb.max.z;
  int32_t l, r;
  l = b->left->kind == S_BVH ? export_node(b->left, nodes, n) : -(b->left->index + 1);
  r = b->right->kind == S_BVH ? export_node(b->right, nodes, n) : -(b->right->index + 1);
  nodes[me].left = l;
  nodes[me].right = r;
  return (int32_t)me;
}

int oracle_bvh_build(const zrt_scene* scene, zrt_bvh_node** nodes, uint32_t* n_nodes,
                     uint32_t* max_depth) {
  if (!scene || !nodes || !n_nodes) return ZRT_E_INVALID;
  *nodes = NULL;
  *n_nodes = 0;
  if (scene->n_prims == 0) return ZRT_E_INVALID;
  Scene sc;
  memset(&sc, 0, sizeof(sc));
  zrt_scene copy = *scene;
  int rc = scene_build(&sc, &copy, 0);
  if (rc) { scene_free(&sc); return rc; }
  /* build regardless of the n>10 rule so small cases can be compared too */
  Surface** ptrs = (Surface**)malloc(sc.n_prims * sizeof(Surface*));
  Surface** tmp = (Surface**)malloc(sc.n_prims * sizeof(Surface*));
  sc.bvh.cap = 2 * sc.n_prims;
  sc.bvh.pool = (Surface*)calloc(sc.bvh.cap, sizeof(Surface));
  for (uint32_t i = 0; i < sc.n_prims; ++i) ptrs[i] = &sc.prims[i];
  const Surface* root = bvh_divide(&sc.bvh, ptrs, sc.n_prims, 1, tmp);
  free(ptrs);
  free(tmp);
  zrt_bvh_node* out = (zrt_bvh_node*)calloc(sc.bvh.n, sizeof(zrt_bvh_node));
  uint32_t n = 0;
  export_node(root, out, &n);
  *nodes = out;
  *n_nodes = n;
  if (max_depth) *max_depth = (uint32_t)sc.bvh.max_depth;
  scene_free(&sc);
  return ZRT_OK;
}

/* ---- camera.zig:17-35 ------------------------------------------------------- */
void oracle_camera_init(const float from[3], const float at[3], const float vup_[3], float vfov,
                        float aspect, zrt_camera* out) {
  const float theta = (float)M_PI * vfov / 180.0f;
  const float h = tanf(theta / 2.0f);
  const float viewport_height = 2.0f * h;
  const float viewport_width = aspect * viewport_height;
  const V3 look_from = v3(from[0], from[1], from[2]);
  const V3 look_at = v3(at[0], at[1], at[2]);
  const V3 vup = v3(vup_[0], vup_[1], vup_[2]);
  const V3 w = v_unit(v_sub(look_from, look_at));
  const V3 u = v_unit(v_cross(vup, w));
  const V3 v = v_cross(w, u);
  const V3 horizontal = v_scale(u, viewport_width);
  const V3 vertical = v_scale(v, viewport_height);
  const V3 llc = v_sub(v_sub(v_sub(look_from, v_scale(horizontal, 1.0f / 2.0f)),
                             v_scale(vertical, 1.0f / 2.0f)), w);
  out->origin.x = look_from.x; out->origin.y = look_from.y; out->origin.z = look_from.z;
  out->lower_left_corner.x = llc.x; out->lower_left_corner.y = llc.y; out->lower_left_corner.z = llc.z;
  out->horizontal.x = horizontal.x; out->horizontal.y = horizontal.y; out->horizontal.z = horizontal.z;
  out->vertical.x = vertical.x; out->vertical.y = vertical.y; out->vertical.z = vertical.z;
}

/* ---- KAT hooks ---------------------------------------------------------------- */
void oracle_prng_u64(uint32_t prng, uint64_t seed, uint64_t* out, int n) {
  zs_rng r;
  zs_rng_init(&r, (int)prng, seed);
  for (int i = 0; i < n; ++i) out[i] = zs_rng_next(&r);
}
void oracle_prng_f32(uint32_t prng, uint64_t seed, float* out, int n) {
  zs_rng r;
  zs_rng_init(&r, (int)prng, seed);
  for (int i = 0; i < n; ++i) out[i] = zs_random_float(&r);
}

/* sample.zig:9-44 (the unused variants are restated for their golden tests) */
static V3 random_vector(zs_rng* r) {
  const float x = zs_random_float(r) * 2.0f - 1.0f;
  const float y = zs_random_float(r) * 2.0f - 1.0f;
  const float z = zs_random_float(r) * 2.0f - 1.0f;
  return v3(x, y, z);
}
static V3 random_in_unit_sphere(zs_rng* r) {
  for (;;) {
    const V3 p = random_vector(r);
    if (v_len2(p) > 1.0f) continue;
    return p;
  }
}
/* raytrace.zig:71-81 (the closest-hit part of rayColor) for a batch of rays */
int oracle_trace(const zrt_scene* scene, int use_bvh, const float* rays, uint32_t n, float* out_t,
                 int32_t* out_prim) {
  Scene sc;
  int rc = scene_build(&sc, scene, use_bvh);
  if (rc) { scene_free(&sc); return rc; }
  Diag dg = {0, 0};
  for (uint32_t i = 0; i < n; ++i) {
    const float* q = rays + 6 * (size_t)i;
    const Ray ray = ray_init(v3(q[0], q[1], q[2]), v3(q[3], q[4], q[5]));
    float t_max = INFINITY;
    HitRecord closest;
    int have = 0;
    for (uint32_t k = 0; k < sc.n_top; ++k) {
      HitRecord h;
      if (surface_hit(sc.top[k], &ray, 0.001f, t_max, &h, &dg)) {
        closest = h;
        have = 1;
        t_max = closest.t;
      }
    }
    out_t[i] = have ? closest.t : INFINITY;
    out_prim[i] = have ? closest.surface->index : -1;
  }
  scene_free(&sc);
  return ZRT_OK;
}

/* bvh.zig:234-247 (createSurfaces) and bvh.zig:280-281 on one stream */
void oracle_bvh_test_data(uint32_t prng, uint64_t seed, uint32_t n_spheres, uint32_t n_rays, float* spheres,
                          float* rays) {
  zs_rng r;
  zs_rng_init(&r, (int)prng, seed);
  for (uint32_t i = 0; i < n_spheres; ++i) {
    const float x = (zs_random_float(&r) - 0.5f) * 100.0f;
    const float y = (zs_random_float(&r) - 0.5f) * 100.0f;
    const float z = (zs_random_float(&r) - 0.5f) * 100.0f;
    const float radius = zs_random_float(&r) * 10.0f + 0.01f;
    spheres[4 * (size_t)i + 0] = x;
    spheres[4 * (size_t)i + 1] = y;
    spheres[4 * (size_t)i + 2] = z;
    spheres[4 * (size_t)i + 3] = radius;
  }
  for (uint32_t i = 0; i < n_rays; ++i) {
    const V3 o = v_scale(random_unit_vector(&r), 100.0f);
    const V3 d = random_unit_vector(&r);
    float* q = rays + 6 * (size_t)i;
    q[0] = o.x; q[1] = o.y; q[2] = o.z;
    q[3] = d.x; q[4] = d.y; q[5] = d.z;
  }
}

void oracle_sample_vector(uint32_t prng, uint64_t seed, int which, float out[3]) {
  zs_rng r;
  zs_rng_init(&r, (int)prng, seed);
  V3 v;
  switch (which) {
    case 0: v = random_vector(&r); break;
    case 1: v = random_in_unit_sphere(&r); break;
    case 2:
      for (;;) {
        v = v_unit(random_in_unit_sphere(&r));
        if (!isnan(v.x)) break;
      }
      break;
    default: v = random_unit_vector(&r); break;
  }
  out[0] = v.x; out[1] = v.y; out[2] = v.z;
}

float oracle_math1(int fn, float x) {
  switch (fn) {
    case 0: return zs_sin(x);
    case 1: return zs_cos(x);
    case 2: return zs_acos(x);
    case 3: return zs_atan(x);
    default: return zs_sqrt(x);
  }
}
float oracle_math2(int fn, float y, float x) { return fn == 0 ? zs_atan2(y, x) : zs_pow(y, x); }

void oracle_ray_at(const float o[3], const float d[3], float t, float out[3]) {
  const Ray r = ray_init(v3(o[0], o[1], o[2]), v3(d[0], d[1], d[2]));
  const V3 p = ray_at(&r, t);
  out[0] = p.x; out[1] = p.y; out[2] = p.z;
}
void oracle_unit_vector(const float v[3], float out[3]) {
  const V3 u = v_unit(v3(v[0], v[1], v[2]));
  out[0] = u.x; out[1] = u.y; out[2] = u.z;
}

static void pack_hit(const HitRecord* h, float out[9]) {
  out[0] = h->location.x; out[1] = h->location.y; out[2] = h->location.z;
  out[3] = h->normal.x; out[4] = h->normal.y; out[5] = h->normal.z;
  out[6] = h->t; out[7] = (float)h->front_face;
  out[8] = 0.0f;
}
int oracle_triangle_hit(const float a[3], const float b[3], const float c[3], const float o[3],
                        const float d[3], float t_min, float t_max, float out[9]) {
  static const Material black = {ZRT_MAT_METAL, {ZRT_TEX_COLOR, {0, 0, 0}, NULL, 0, 0}, 0};
  Surface s;
  triangle_init(&s, v3(a[0], a[1], a[2]), v3(b[0], b[1], b[2]), v3(c[0], c[1], c[2]), &black);
  const Ray r = ray_init(v3(o[0], o[1], o[2]), v3(d[0], d[1], d[2]));
  HitRecord h;
  if (!triangle_hit(&s, &r, t_min, t_max, &h)) return 0;
  pack_hit(&h, out);
  return 1;
}
int oracle_sphere_hit(const float center[3], float radius, const float o[3], const float d[3],
                      float t_min, float t_max, float out[9]) {
  static const Material black = {ZRT_MAT_METAL, {ZRT_TEX_COLOR, {0, 0, 0}, NULL, 0, 0}, 0};
  Surface s;
  sphere_init(&s, v3(center[0], center[1], center[2]), radius, &black);
  const Ray r = ray_init(v3(o[0], o[1], o[2]), v3(d[0], d[1], d[2]));
  HitRecord h;
  if (!sphere_hit(&s, &r, t_min, t_max, &h)) return 0;
  pack_hit(&h, out);
  out[7] = h.texture_coords.u;  /* front_face is implied by the normal; report uv */
  out[8] = h.texture_coords.v;
  return 1;
}
int oracle_aabb_hit(const float c1[3], const float c2[3], const float o[3], const float d[3],
                    float t_min, float t_max) {
  const AABB b = aabb_min_max(v3(c1[0], c1[1], c1[2]), v3(c2[0], c2[1], c2[2]));
  const Ray r = ray_init(v3(o[0], o[1], o[2]), v3(d[0], d[1], d[2]));
  return aabb_hit(&b, &r, t_min, t_max);
}
float oracle_aabb_surface_area(const float c1[3], const float c2[3]) {
  return aabb_area(aabb_min_max(v3(c1[0], c1[1], c1[2]), v3(c2[0], c2[1], c2[2])));
}
void oracle_texture_albedo(const zrt_image* img, float u_off, float v_off, float u, float v,
                           float out[3]) {
  V2 tc = {u, v};
  const V3 c = image_albedo(img, u_off, v_off, tc);
  out[0] = c.x; out[1] = c.y; out[2] = c.z;
}

void oracle_free(void* p) { free(p); }
