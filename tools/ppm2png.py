"""Convert an f64 canvas / P3 PPM to PNG for a quick look (dev tool, stdlib only)."""
import struct
import sys
import zlib

import numpy as np


def write_png(path, rgb8):
    h, w, _ = rgb8.shape
    raw = b"".join(b"\x00" + rgb8[y].tobytes() for y in range(h))
    def chunk(tag, data):
        c = struct.pack(">I", len(data)) + tag + data
        return c + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)
    png = b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 0))
    png += chunk(b"IDAT", zlib.compress(raw, 9)) + chunk(b"IEND", b"")
    open(path, "wb").write(png)


def read_ppm(path):
    tok = open(path, "rb").read().split()
    assert tok[0] == b"P3"
    w, h = int(tok[1]), int(tok[2])
    v = np.array([int(t) for t in tok[4:4 + w * h * 3]], dtype=np.uint8)
    return v.reshape(h, w, 3)


if __name__ == "__main__":
    write_png(sys.argv[2], read_ppm(sys.argv[1]))
