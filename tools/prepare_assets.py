"""Copy the reference's scene data into ``assets/`` (run once, in the build container).

The reference loads OBJ meshes and PNG textures from ``/root/reference/models``
(scenes.zig:38, 66-69, 110; obj_reader.zig:114).  That directory never reaches
the GPU box, so the data files are copied here:

* OBJ files and PNG textures are copied byte-for-byte (they are data; libzrt
  parses the OBJs and decodes the PNGs itself: scene_io.cpp, image_io.cpp's
  restatement of png_image.zig:19-94).
* ``showcase/7-spheres.png`` (README.md:39, the only image-level golden) is
  copied as well, for the statistical parity test.
"""
import os
import shutil
import sys

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
ASSETS = os.path.join(os.path.dirname(HERE), "assets")


def main():
    os.makedirs(ASSETS, exist_ok=True)
    for rel, name in [("models/bunny/bunny.obj", "bunny.obj"),
                      ("models/teapot/teapot.obj", "teapot.obj"),
                      ("models/man/Man.obj", "Man.obj"),
                      ("models/images/earthmap.png", "earthmap.png"),
                      ("models/images/nitor-logo-25.png", "nitor-logo-25.png"),
                      ("showcase/7-spheres.png", "showcase-7-spheres.png")]:
        shutil.copyfile(os.path.join(REF, rel), os.path.join(ASSETS, name))
    print("assets written to", ASSETS)


if __name__ == "__main__":
    sys.exit(main())
