"""Decode the reference sample's image data/images/albert.jpg (public domain, see its LICENSE.txt)
with PIL in the build container and store a 768x1024 grayscale copy as a binary PGM (P5) fixture,
tests/golden/albert_768x1024.pgm, that the sample program and bench.py read on the GPU box (where
/root/reference does not exist). The reference loads the full 3250x4333 image with stbi_loadf (RGBA
float, 8-bit values linearised with gamma 2.2, stbi_wrapper.cpp:37-44); the consumers apply the same
linearisation to these 8-bit values. Downscaled with PIL's BOX filter to keep the fixture < 1 MB.

usage: python tools/make_albert_fixture.py [/root/reference/data/images/albert.jpg]
"""
import os
import sys

from PIL import Image

SRC = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/data/images/albert.jpg"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "albert_768x1024.pgm")

im = Image.open(SRC).convert("L")
assert im.size == (3250, 4333), im.size
small = im.resize((768, 1024), Image.BOX)
with open(OUT, "wb") as f:
    f.write(b"P5\n768 1024\n255\n")
    f.write(small.tobytes())
print(OUT, os.path.getsize(OUT))
