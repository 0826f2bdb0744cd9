/*
 * ORACLE — test infrastructure only.  Nothing under oracle/ is linked into or
 * called by the product (zraytrace_amd/libzrt.so); only tests/, the smoke()
 * check in __graft_entry__.py and bench.py's cpu_baseline leg load it.
 *
 * zig_std.h — restatement of the parts of the Zig standard library (0.9.0-dev,
 * 2021, the toolchain the reference's HEAD needs: SURVEY.md §0.4) that the
 * reference's hot path calls.  The library is not vendored in the reference
 * (no lockfile); each function below restates its published algorithm:
 *
 *   std.rand.SplitMix64 / Xoroshiro128 (= DefaultPrng in the toolchain the
 *     reference's tests were written for; pinned by src/sample.zig:70-118) and
 *     Xoshiro256 (DefaultPrng from Zig 0.8 on; unpinned);
 *   std.rand.Random.float(f32) / .boolean();
 *   std.math.sin / cos (Go port of Cephes sin.go/cos.go, used by Zig <= 0.9),
 *   acos / atan / atan2 (musl acosf/atanf/atan2f ports), pow (Go port),
 *   sqrt (@sqrt: IEEE correctly rounded).
 *
 * Parity status: the RNG + float conversion + hemisphere sampling are pinned
 * by the four golden vectors of src/sample.zig:70-118 (tests/golden).  The
 * transcendental restatements are "parity unpinned" beyond those vectors'
 * 0.01 tolerance: no Zig toolchain exists here to compare against.
 */
#ifndef ZRT_ORACLE_ZIG_STD_H
#define ZRT_ORACLE_ZIG_STD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- std.rand ----------------------------------------------------------- */
typedef struct zs_rng {
  int kind;          /* 0 = Xoroshiro128 (+), 1 = Xoshiro256 (++) */
  uint64_t s[4];
} zs_rng;

uint64_t zs_splitmix64_next(uint64_t* state);
void zs_rng_init(zs_rng* r, int kind, uint64_t init_s); /* DefaultPrng.init(init_s) */
uint64_t zs_rng_next(zs_rng* r);
float zs_random_float(zs_rng* r);   /* Random.float(f32) */
int zs_random_boolean(zs_rng* r);   /* Random.boolean() */

/* ---- std.math (f32) ----------------------------------------------------- */
float zs_sqrt(float x);
float zs_sin(float x);
float zs_cos(float x);
float zs_acos(float x);
float zs_atan(float x);
float zs_atan2(float y, float x);
float zs_pow(float x, float y);   /* integral y only (the path uses y = 5) */
float zs_min(float x, float y);   /* math.min: x < y ? x : y */
float zs_max(float x, float y);   /* math.max: x > y ? x : y */

#ifdef __cplusplus
}
#endif
#endif
