"""Minimal PNG writer (stdlib zlib) for eyeballing frames: write_png(path, uint8 HxWx{3,4})."""
import struct
import zlib

import numpy as np


def write_png(path, img):
    img = np.ascontiguousarray(img[..., :3].astype(np.uint8))
    h, w, _ = img.shape
    raw = b"".join(b"\x00" + img[y].tobytes() for y in range(h))

    def chunk(tag, data):
        return struct.pack(">I", len(data)) + tag + data + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)

    with open(path, "wb") as f:
        f.write(b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 0))
                + chunk(b"IDAT", zlib.compress(raw, 6)) + chunk(b"IEND", b""))
