"""The caller-side image writers (png_image.zig:96-148, ppm_image.zig) and the
command line (main.zig) over the C ABI, and the PNG reader (png_image.zig:19-94).
CPU-only except the marked test."""
import os
import re
import struct
import subprocess
import zlib

import numpy as np
import pytest

import zraytrace_amd as z
from zraytrace_amd import _ffi

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(REPO, "zraytrace_amd", "zrt-raytrace")


def png_quantize(img):
    """u8(std.math.clamp(255.999 * c, 0, 255)) in f32, math.min/max as `x < y ? x : y`."""
    v = (np.float32(255.999) * img.astype(np.float32)).astype(np.float32)
    m = np.where(v < 255, v, np.float32(255))        # min(v, 255): NaN -> 255
    c = np.where(np.float32(0) > m, np.float32(0), m)  # max(0, m)
    return np.trunc(c).astype(np.uint8)[::-1]         # top row first


def ppm_quantize(img):
    x = (img.astype(np.float32) * np.float32(255.999)).astype(np.float32)
    out = np.where(x >= 0, np.minimum(np.trunc(np.nan_to_num(x, nan=0.0, posinf=255.0)), 255), 0)
    return out.astype(np.uint32)[::-1]


def decode_png(path):
    data = open(path, "rb").read()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat, ihdr = 8, b"", None
    while pos < len(data):
        n, typ = struct.unpack(">I4s", data[pos:pos + 8])
        body = data[pos + 8:pos + 8 + n]
        crc, = struct.unpack(">I", data[pos + 8 + n:pos + 12 + n])
        assert crc == zlib.crc32(typ + body) & 0xffffffff
        if typ == b"IHDR":
            ihdr = struct.unpack(">IIBBBBB", body)
        elif typ == b"IDAT":
            idat += body
        pos += 12 + n
    w, h, bits, color, _, _, interlace = ihdr
    assert (bits, color, interlace) == (8, 2, 0)
    raw = np.frombuffer(zlib.decompress(idat), np.uint8).reshape(h, 1 + 3 * w)
    assert (raw[:, 0] == 0).all()  # filter type None on every row
    return raw[:, 1:].reshape(h, w, 3)


def test_png_matches_reference_quantization(tmp_path):
    rng = np.random.default_rng(3)
    img = rng.uniform(-0.2, 1.2, (13, 17, 3)).astype(np.float32)
    img[0, 0] = [np.nan, -0.0, 1.0]
    img[0, 1] = [np.inf, -np.inf, 0.999]
    img[1, 0] = [1.0 / 255.999, 0.5, 254.5 / 255.999]
    p = str(tmp_path / "out.png")
    z.write_png(p, img)
    np.testing.assert_array_equal(decode_png(p), png_quantize(img))


def test_ppm_matches_reference_format(tmp_path):
    rng = np.random.default_rng(4)
    img = rng.uniform(0.0, 1.0, (5, 7, 3)).astype(np.float32)
    p = str(tmp_path / "out.ppm")
    z.write_ppm(p, img)
    text = open(p).read()
    head = f"P3\n# filename: {p}\n# The P3 = colors are in ASCII\n# Image width and height\n7 5\n" \
           "# Max color value\n255\n# RGB triplets\n"
    assert text.startswith(head)
    rows = text[len(head):].split("\n")[:-1]
    want = ppm_quantize(img)
    for y, row in enumerate(rows):
        assert row == "".join(f"{r:>3} {g:>3} {b:>3}  " for r, g, b in want[y])


# ---- png_image.readFile (png_image.zig:19-94): zrt_image_read_png ------------------

ADAM7 = ((0, 0, 8, 8), (4, 0, 8, 8), (0, 4, 4, 8), (2, 0, 4, 4), (0, 2, 2, 4), (1, 0, 2, 2), (0, 1, 1, 2))


def _filter_row(row, prev, bpp, ftype):
    """PNG spec §9 filters applied to one scanline (uint8 arrays)."""
    r = row.astype(np.int32)
    p = prev.astype(np.int32) if prev is not None else np.zeros_like(r)
    a = np.concatenate([np.zeros(bpp, np.int32), r[:-bpp]])
    c = np.concatenate([np.zeros(bpp, np.int32), p[:-bpp]])
    if ftype == 0:
        out = r
    elif ftype == 1:
        out = r - a
    elif ftype == 2:
        out = r - p
    elif ftype == 3:
        out = r - (a + p) // 2
    else:
        est = a + p - c
        pa, pb, pc = np.abs(est - a), np.abs(est - p), np.abs(est - c)
        out = r - np.where((pa <= pb) & (pa <= pc), a, np.where(pb <= pc, p, c))
    return (out & 0xFF).astype(np.uint8)


def encode_test_png(pixels, interlace=False, color_type=None, depth=8, rng=None):
    """A PNG of `pixels` (uint8 [h, w, 3 or 4], top row first) with a random
    filter type per scanline, optionally Adam7-interlaced."""
    h, w, ch = pixels.shape
    bpp = ch
    color_type = color_type if color_type is not None else (6 if ch == 4 else 2)
    passes = ADAM7 if interlace else ((0, 0, 1, 1),)
    raw = bytearray()
    for x0, y0, dx, dy in passes:
        sub = pixels[y0::dy, x0::dx]
        if sub.shape[0] == 0 or sub.shape[1] == 0:
            continue
        prev = None
        for row in sub.reshape(sub.shape[0], -1):
            ft = int(rng.integers(0, 5))
            raw.append(ft)
            raw += _filter_row(row, prev, bpp, ft).tobytes()
            prev = row

    def chunk(t, d):
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)
    ihdr = struct.pack(">IIBBBBB", w, h, depth, color_type, 0, 0, 1 if interlace else 0)
    return (b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", ihdr) + chunk(b"tEXt", b"Comment\x00test")
            + chunk(b"IDAT", zlib.compress(bytes(raw))) + chunk(b"IEND", b""))


@pytest.mark.parametrize("interlace", [False, True], ids=["progressive", "adam7"])
@pytest.mark.parametrize("channels", [3, 4], ids=["rgb", "rgba"])
def test_png_reader_filters(tmp_path, interlace, channels):
    """Every filter type, both color types png_image.zig:44 accepts, Adam7 and
    sizes smaller than an interlace block: rows flipped, c / 255 (png_image.zig:86-87)."""
    rng = np.random.default_rng(11 + channels)
    for h, w in ((1, 1), (5, 7), (17, 33), (64, 9)):
        px = rng.integers(0, 256, (h, w, channels), dtype=np.uint8)
        p = tmp_path / f"t{h}x{w}.png"
        p.write_bytes(encode_test_png(px, interlace=interlace, rng=rng))
        got = z.read_png(str(p))
        want = (px[::-1, :, :3].astype(np.float32) / np.float32(255.0)).astype(np.float32)
        assert got.shape == (h, w, 3)
        assert (got.view(np.uint32) == want.view(np.uint32)).all(), (h, w)


def test_png_reader_rejects(tmp_path):
    """png_image.zig:44-51: UnsupportedPngFeature for grey / palette / 16-bit;
    a missing file or a damaged stream is an I/O error."""
    rng = np.random.default_rng(5)
    grey = tmp_path / "grey.png"
    grey.write_bytes(encode_test_png(rng.integers(0, 256, (4, 4, 1), dtype=np.uint8), color_type=0, rng=rng))
    deep = tmp_path / "deep.png"
    deep.write_bytes(encode_test_png(rng.integers(0, 256, (4, 4, 6), dtype=np.uint8), color_type=2, depth=16,
                                     rng=rng))
    for p in (grey, deep):
        with pytest.raises(z.ZrtError) as e:
            z.read_png(str(p))
        assert e.value.code == _ffi.ZRT_E_UNSUPPORTED
    good = encode_test_png(rng.integers(0, 256, (4, 4, 3), dtype=np.uint8), rng=rng)
    bad = bytearray(good)
    bad[-20] ^= 0xFF  # inside IDAT: its CRC no longer matches
    (tmp_path / "bad.png").write_bytes(bytes(bad))
    for p in (tmp_path / "bad.png", tmp_path / "missing.png"):
        with pytest.raises(z.ZrtError) as e:
            z.read_png(str(p))
        assert e.value.code == _ffi.ZRT_E_IO


def test_reference_pngs_decode():
    """The reference's own textures (models/images) and showcase render, as
    copied into assets/: sizes and the README showcase's channel means."""
    assert z.read_png(os.path.join(REPO, "assets", "earthmap.png")).shape == (512, 1024, 3)
    assert z.read_png(os.path.join(REPO, "assets", "nitor-logo-25.png")).shape == (439, 1000, 3)  # RGBA
    show = z.read_png(os.path.join(REPO, "assets", "showcase-7-spheres.png"))
    assert show.shape == (1000, 1000, 3)
    means = np.rint(show.astype(np.float64) * 255.0).reshape(-1, 3).mean(axis=0)
    np.testing.assert_allclose(means, [102.455496, 177.713237, 149.453943], atol=1e-5)


def test_writer_errors(tmp_path):
    img = np.zeros((2, 2, 3), np.float32)
    with pytest.raises(z.ZrtError) as e:
        z.write_png(str(tmp_path / "no" / "such" / "dir.png"), img)
    assert e.value.code == _ffi.ZRT_E_IO


def test_cli_arguments_and_no_device():
    r = subprocess.run([CLI, "32", "70000", "4", "5", "1", "x.png"], capture_output=True, text=True)
    assert r.returncode == 1
    assert r.stderr.startswith("raytrace\nUSAGE;\nraytrace width heigth samples depth scene_index filename\n")
    assert "error: Overflow" in r.stderr
    r = subprocess.run([CLI, "32", "32"], capture_output=True, text=True)
    assert r.returncode == 1 and "error: missing argument" in r.stderr
    import torch
    if not torch.cuda.is_available():  # the HIP path fails loudly, no CPU fallback
        r = subprocess.run([CLI, "8", "8", "1", "2", "1", "x.png"], capture_output=True, text=True)
        assert r.returncode == 1 and "no HIP device" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("devices", [None, "0", "0,0,0"])
def test_cli_renders_oracle_image(tmp_path, scenes, devices):
    """main.zig end to end: the CLI's PNG is the oracle image through
    png_image.zig's quantization, and its summary lines carry the counters.
    ZRT_DEVICES renders through zrt_render_multi (RCCL gather for "0")."""
    from oracle import oracle_py as O
    out = str(tmp_path / "scene1.png")
    env = dict(os.environ)
    env.pop("ZRT_DEVICES", None)
    if devices:
        env["ZRT_DEVICES"] = devices
    r = subprocess.run([CLI, "40", "40", "4", "12", "1", out], capture_output=True, text=True, timeout=300,
                       env=env)
    assert r.returncode == 0, r.stderr
    s = scenes(1)
    ref, rs = O.render(s.view, s.camera, z.RenderParams(40, 40, 4, 12))
    np.testing.assert_array_equal(decode_png(out), png_quantize(ref))
    summary = {}
    for line in r.stderr.splitlines():
        if line.startswith("  Total ") and line.count(":") == 1:
            label, value = line.split(":")
            summary[label.strip()] = value.strip()
    for label, key in (("Total rays", "rays_processed"), ("Total samples", "samples_processed"),
                       ("Total background hits", "background_hits"), ("Total pixels", "pixels_processed"),
                       ("Total reflections", "reflections")):
        assert int(summary[label]) == rs[key], label
    # printProgress after every scanline (raytrace.zig:37-50, 184): the reference's
    # line format, running pixels / samples / rays, per-row deltas of the rest
    _, _, rows = O.render_scanlines(s.view, s.camera, z.RenderParams(40, 40, 4, 12))
    pat = re.compile(r"^Scanline: (\d+)/(\d+) Pixels: (\d+) Samples: (\d+) Rays: (\d+) Recursion limit: (\d+) "
                     r"Reflections: (\d+) Background hits: (\d+) Pixels/s: \d+\.\d$")
    lines = [pat.match(line) for line in r.stderr.splitlines() if line.startswith("Scanline:")]
    assert len(lines) == 40 and all(lines)
    cum = np.cumsum(rows, axis=0)
    for y, m in enumerate(lines):
        v = [int(g) for g in m.groups()]
        assert v[:2] == [y + 1, 40]
        assert v[2:5] == [cum[y, 3], cum[y, 4], cum[y, 5]], y  # pixels, samples, rays so far
        assert v[5:8] == [rows[y, 0], rows[y, 1], rows[y, 2]], y  # this row's limit / reflections / sky
    order = [line.split(":")[0] for line in r.stderr.splitlines()]
    assert order.index("Preprocess time") < order.index("Scanline") < order.index("Rendering ready")
