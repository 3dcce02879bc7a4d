"""PNG writer used by --save_last_image (CPU)."""

import zlib

import numpy as np

from robomanipbaselines_amd.common.image_io import decode_png, encode_png


def test_png_roundtrip_and_header():
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, (37, 53, 3), dtype=np.uint8)
    data = encode_png(img)
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    assert data[12:16] == b"IHDR" and int.from_bytes(data[16:20], "big") == 53 and int.from_bytes(data[20:24], "big") == 37
    np.testing.assert_array_equal(decode_png(data), img)
    assert zlib.crc32(data[-8:-4]) & 0xFFFFFFFF == int.from_bytes(data[-4:], "big")  # IEND CRC
