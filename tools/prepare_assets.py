"""Copy the reference's scene data into ``assets/`` (run once, in the build container).

The reference loads OBJ meshes and PNG textures from ``/root/reference/models``
(scenes.zig:38, 66-69, 110; obj_reader.zig:114).  That directory never reaches
the GPU box, so the data files are copied here:

* OBJ files are copied byte-for-byte (they are data, parsed by our own reader).
* PNG textures are decoded with Pillow and written as binary PPM (P6, RGB8).
  The reference decodes with libpng, drops alpha (``png_set_filler``) and keeps
  the raw 8-bit RGB samples (png_image.zig:44-89); no gamma is applied by either
  decoder, so the P6 bytes are exactly the samples the reference reads.  The
  row flip and the ``c/255`` f32 conversion happen at load time in the host
  layer, as png_image.zig:86 does.
* ``showcase/7-spheres.png`` (README.md:39, the only image-level golden) is
  stored as P6 as well, for the statistical parity test.
"""
import os
import shutil
import sys

from PIL import Image

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
ASSETS = os.path.join(os.path.dirname(HERE), "assets")


def write_p6(src, dst):
    im = Image.open(src)
    if im.mode not in ("RGB", "RGBA"):
        raise SystemExit(f"{src}: unsupported mode {im.mode} (reference accepts RGB/RGBA 8-bit only)")
    rgb = im.convert("RGB") if im.mode == "RGBA" else im
    w, h = rgb.size
    with open(dst, "wb") as f:
        f.write(b"P6\n%d %d\n255\n" % (w, h))
        f.write(rgb.tobytes())


def main():
    os.makedirs(ASSETS, exist_ok=True)
    for rel, name in [("models/bunny/bunny.obj", "bunny.obj"),
                      ("models/teapot/teapot.obj", "teapot.obj"),
                      ("models/man/Man.obj", "Man.obj")]:
        shutil.copyfile(os.path.join(REF, rel), os.path.join(ASSETS, name))
    for rel, name in [("models/images/earthmap.png", "earthmap.ppm"),
                      ("models/images/nitor-logo-25.png", "nitor-logo-25.ppm"),
                      ("showcase/7-spheres.png", "showcase-7-spheres.ppm")]:
        write_p6(os.path.join(REF, rel), os.path.join(ASSETS, name))
    print("assets written to", ASSETS)


if __name__ == "__main__":
    sys.exit(main())
