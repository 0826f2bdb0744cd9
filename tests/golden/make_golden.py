"""Generate tests/golden/golden.json (run in the build container; committed).

Two kinds of fixtures:

1. Known answers copied from the reference's own unit tests (data only):
     sample.zig:70-118   RNG + Random.float + the four sample vectors (tol 0.01)
     ray.zig:32-39       rayAt(2) of Ray((1,1,1),(1,2,3))
     triangle.zig:84-118 hit / miss
     aabb.zig:151-254    initMinMax / initAabb / surfaceArea / hitAabb
     vector.zig:169-255  dot / unitVector
     texture.zig:90-103  earthmap texel lookups at (u, v) with zero offsets
2. PRNG output streams from an independent pure-Python emulation of Zig's
   std.rand (SplitMix64 seeding, Xoroshiro128+, Xoshiro256++, Random.float):
   they pin the C oracle and the device RNG to the published algorithms.
   The emulation is this file; no reference code is executed.
"""
import json
import os
import struct

HERE = os.path.dirname(os.path.abspath(__file__))
M = (1 << 64) - 1


def rotl(x, k):
    return ((x << k) | (x >> (64 - k))) & M


def splitmix(state):
    state = (state + 0x9E3779B97F4A7C15) & M
    z = state
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
    return state, z ^ (z >> 31)


class Xoroshiro128:
    def __init__(self, seed):
        g = seed & M
        g, a = splitmix(g)
        g, b = splitmix(g)
        self.s = [a, b]

    def next(self):
        s0, s1 = self.s
        r = (s0 + s1) & M
        s1 ^= s0
        self.s = [rotl(s0, 55) ^ s1 ^ ((s1 << 14) & M), rotl(s1, 36)]
        return r


class Xoshiro256:
    def __init__(self, seed):
        g = seed & M
        self.s = []
        for _ in range(4):
            g, v = splitmix(g)
            self.s.append(v)

    def next(self):
        s = self.s
        r = (rotl((s[0] + s[3]) & M, 23) + s[0]) & M
        t = (s[1] << 17) & M
        s[2] ^= s[0]
        s[3] ^= s[1]
        s[1] ^= s[2]
        s[0] ^= s[3]
        s[2] ^= t
        s[3] = rotl(s[3], 45)
        return r


def rand_float(g):
    u = g.next() & 0xFFFFFFFF
    bits = 0x3F800000 | (u >> 9)
    f = struct.unpack("<f", struct.pack("<I", bits))[0]
    return struct.unpack("<f", struct.pack("<f", f - 1.0))[0]


def main():
    gold = {"source": "tests/golden/make_golden.py", "reference_tests": {}, "streams": {}}
    R = gold["reference_tests"]
    # sample.zig:70-118 (DefaultPrng.init(0), tolerance 0.01)
    R["sample"] = {
        "seed": 0, "tol": 0.01,
        "randomVector": [-0.7746, 0.3873, -0.7065],
        "randomVectorInUnitSphere": [0.1846, 0.8305, -0.0479],
        "randomUnitVector_old": [0.2167, 0.9746, -0.0562],
        "randomUnitVector": [-0.344, -0.932, 0.113],
    }
    # ray.zig:32-39 (exact)
    R["ray_at"] = {"origin": [1, 1, 1], "direction": [1, 2, 3], "t": 2.0,
                   "expected": [1.53452253e+00, 2.06904506e+00, 2.60356736e+00]}
    # vector.zig:213-218
    R["unit_vector"] = [{"v": [1, 0, 0], "expected": [1, 0, 0]},
                        {"v": [3, -4, 0], "expected": [0.6, -0.8, 0.0]}]
    # triangle.zig:84-118
    R["triangle_miss"] = {"a": [1, 0, 0], "b": [0, 1, 0], "c": [0, 0, 1],
                          "origin": [1, 1, 1], "direction": [1, 1, 1], "t_min": 0.1, "t_max": 10000.0}
    R["triangle_hit"] = {"a": [10, 5, 1], "b": [-10, -10, 1], "c": [-10, 10, 1],
                         "origin": [0, 0, -10], "direction": [0, 0, 1], "t_min": 0.1, "t_max": 10000.0,
                         "location": [0, 0, 1], "normal": [0, 0, -1], "t": 11.0, "front_face": True}
    # aabb.zig:151-254
    R["aabb_min_max"] = {"c1": [-1, 2, 3], "c2": [4, -3, 7], "min": [-1, -3, 3], "max": [4, 2, 7]}
    R["aabb_union"] = {"box1": [[-1, 2, 3], [4, -3, 7]], "box2": [[7, 1, 11], [0, -3, -2]],
                       "min": [-1, -3, -2], "max": [7, 2, 11]}
    R["aabb_surface_area"] = {"c1": [0, 0, 0], "c2": [1, -2, 3], "expected": 28.0}
    R["aabb_hit"] = {"c1": [-1, -1, -1], "c2": [1, 1, 1], "origin": [-10, 0, 0], "t_min": 0.0,
                     "t_max": 100000.0, "cases": [{"direction": [-1, 0, 0], "hit": False},
                                                  {"direction": [1, 0, 0], "hit": True}]}
    # texture.zig:90-103 (earthmap, Texture.initImageOpts(image, 0, 0); exact)
    R["texture_earthmap"] = {"file": "assets/earthmap.png", "u_offset": 0.0, "v_offset": 0.0, "cases": [
        {"uv": [0.0, 0.0], "expected": [9.21568632e-01, 9.37254905e-01, 9.49019610e-01]},
        {"uv": [0.1, 0.1], "expected": [9.25490200e-01, 9.45098042e-01, 9.56862747e-01]},
        {"uv": [0.5, 0.5], "expected": [0.0, 7.84313771e-03, 2.07843139e-01]},
        {"uv": [1.0, 1.0], "expected": [1.0, 1.0, 1.0]}]}
    # README.md:50-61: statistics of the 7-spheres showcase run
    R["readme_7spheres"] = {"width": 1000, "height": 1000, "spp": 1000, "max_depth": 30,
                            "reflections": 1144753226, "background_hits": 999892115,
                            "samples": 1000000000, "rays": 2144645362, "runtime_s": 617.41}

    S = gold["streams"]
    for name, cls in (("xoroshiro128", Xoroshiro128), ("xoshiro256", Xoshiro256)):
        for seed in (0, 42, 0x123456789ABCDEF):
            g = cls(seed)
            S[f"{name}_u64_seed{seed}"] = [str(g.next()) for _ in range(64)]
            g = cls(seed)
            S[f"{name}_f32_seed{seed}"] = [rand_float(g) for _ in range(64)]
    # counter-mode keys: ((pixel << 16) | sample) + seed * 0x9E3779B97F4A7C15
    keys = []
    for pixel, sample in ((0, 0), (1, 0), (0, 1), (4095, 15), (2048 * 2048 - 1, 1023)):
        key = (((pixel << 16) | sample) + 42 * 0x9E3779B97F4A7C15) & M
        g = Xoroshiro128(key)
        keys.append({"pixel": pixel, "sample": sample, "key": str(key),
                     "u64": [str(g.next()) for _ in range(8)]})
    S["counter_keys_seed42"] = keys
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(gold, f, indent=1)
    print("wrote", os.path.join(HERE, "golden.json"))


if __name__ == "__main__":
    main()
