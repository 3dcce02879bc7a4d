"""Minimal PNG writer for `--save_last_image` (the reference writes the frame with cv2.imwrite,
common/base/RolloutBase.py:541-561; cv2 is not part of this stack): 8-bit RGB, no interlace,
filter type 0, zlib-compressed IDAT, CRC-checked chunks (PNG spec, ISO/IEC 15948)."""

import struct
import zlib

import numpy as np


def _chunk(tag, data):
    return struct.pack(">I", len(data)) + tag + data + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)


def encode_png(rgb):
    """uint8 [H, W, 3] -> PNG bytes."""
    rgb = np.ascontiguousarray(rgb, dtype=np.uint8)
    if rgb.ndim != 3 or rgb.shape[2] != 3:
        raise ValueError("encode_png expects an [H, W, 3] uint8 image")
    h, w, _ = rgb.shape
    raw = np.concatenate([np.zeros((h, 1), dtype=np.uint8), rgb.reshape(h, w * 3)], axis=1)
    ihdr = struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 0)
    return b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", ihdr) + _chunk(b"IDAT", zlib.compress(raw.tobytes(), 6)) + _chunk(b"IEND", b"")


def write_png(path, rgb):
    with open(path, "wb") as f:
        f.write(encode_png(rgb))


def decode_png(data):
    """PNG bytes -> uint8 [H, W, C] (C = 1 grey, 2 grey + alpha, 3 RGB, 4 RGBA; palette images
    expanded to RGB / RGBA): 8-bit samples, no interlace, every scanline filter of the PNG spec
    (None, Sub, Up, Average, Paeth; ISO/IEC 15948 §9).  The model compiler reads the reference's
    texture files with it (mjcf/compiler.py); the tests read back encode_png's output."""
    if data[:8] != b"\x89PNG\r\n\x1a\n":
        raise ValueError("not a PNG file")
    pos, idat, plte, trns = 8, b"", None, None
    w = h = depth = ctype = interlace = None
    while pos < len(data):
        (n,) = struct.unpack(">I", data[pos:pos + 4])
        tag, body = data[pos + 4:pos + 8], data[pos + 8:pos + 8 + n]
        (crc,) = struct.unpack(">I", data[pos + 8 + n:pos + 12 + n])
        if crc != zlib.crc32(tag + body) & 0xFFFFFFFF:
            raise ValueError(f"PNG chunk {tag!r}: CRC mismatch")
        if tag == b"IHDR":
            w, h, depth, ctype, _, _, interlace = struct.unpack(">IIBBBBB", body[:13])
        elif tag == b"PLTE":
            plte = np.frombuffer(body, dtype=np.uint8).reshape(-1, 3)
        elif tag == b"tRNS":
            trns = np.frombuffer(body, dtype=np.uint8)
        elif tag == b"IDAT":
            idat += body
        elif tag == b"IEND":
            break
        pos += 12 + n
    if depth != 8 or interlace != 0:
        raise ValueError(f"unsupported PNG: bit depth {depth}, interlace {interlace} (8-bit, non-interlaced only)")
    chans = {0: 1, 2: 3, 3: 1, 4: 2, 6: 4}[ctype]
    stride = w * chans
    raw = np.frombuffer(zlib.decompress(idat), dtype=np.uint8).reshape(h, 1 + stride)
    out = np.zeros((h, stride), dtype=np.uint8)
    prev = np.zeros(stride, dtype=np.int32)
    for y in range(h):
        f, line = raw[y, 0], raw[y, 1:].astype(np.int32)
        if f == 0:
            cur = line
        elif f == 1:  # Sub: cumulative per channel along the row, mod 256
            cur = np.cumsum(line.reshape(w, chans), axis=0).reshape(-1) & 255
        elif f == 2:  # Up
            cur = (line + prev) & 255
        elif f in (3, 4):  # Average / Paeth: sequential along the row (left neighbour)
            cur = np.zeros(stride, dtype=np.int32)
            for x in range(0, stride, chans):
                a = cur[x - chans:x] if x else np.zeros(chans, dtype=np.int32)
                b = prev[x:x + chans]
                if f == 3:
                    cur[x:x + chans] = (line[x:x + chans] + ((a + b) >> 1)) & 255
                else:
                    c = prev[x - chans:x] if x else np.zeros(chans, dtype=np.int32)
                    p = a + b - c
                    pa, pb, pc = np.abs(p - a), np.abs(p - b), np.abs(p - c)
                    pred = np.where((pa <= pb) & (pa <= pc), a, np.where(pb <= pc, b, c))
                    cur[x:x + chans] = (line[x:x + chans] + pred) & 255
        else:
            raise ValueError(f"bad PNG filter type {f}")
        out[y] = cur
        prev = cur
    img = out.reshape(h, w, chans)
    if ctype == 3:  # palette
        rgb = plte[img[..., 0]]
        if trns is not None:
            alpha = np.full(len(plte), 255, dtype=np.uint8)
            alpha[: len(trns)] = trns
            return np.concatenate([rgb, alpha[img[..., 0]][..., None]], axis=2)
        return rgb
    return img
