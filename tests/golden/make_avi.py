"""Writes the tiny uncompressed AVI fixtures under tests/golden/avi/ (committed):
cam0_image.avi / cam1_image.avi -- 5 frames of 20 x 12, 8-bit palettised gray
(BI_RGB, bottom-up rows padded to 4 bytes, '00db' chunks, an idx1 index, a
JUNK chunk and an odd-sized strn chunk to exercise padding), and bgr24.avi --
3 frames of 7 x 5, 24-bit BGR top-down (negative biHeight, '00dc' chunks,
each row padded 21 -> 24 bytes), plus the pixel arrays expected from them
(frames.npz) and image_data.csv.  This writer is independent of the reader
in uasl_motion_estimation_amd/file_io.py: it packs the RIFF structure by hand.

    python tests/golden/make_avi.py
"""
import os
import struct

import numpy as np

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "avi")


def chunk(cid: bytes, data: bytes) -> bytes:
    pad = b"\0" if len(data) & 1 else b""
    return cid + struct.pack("<I", len(data)) + data + pad


def lst(kind: bytes, body: bytes) -> bytes:
    return b"LIST" + struct.pack("<I", len(body) + 4) + kind + body


def write_avi(path: str, frames, bits: int, top_down: bool = False, fourcc: bytes = b"00db"):
    n = len(frames)
    h, w = frames[0].shape[:2]
    stride = ((w * bits // 8) + 3) & ~3
    payload = []
    for f in frames:
        rows = f if top_down else f[::-1]
        buf = bytearray()
        for r in rows:
            b = r.tobytes() if bits == 8 else r[:, :3].tobytes()
            buf += b + b"\0" * (stride - len(b))
        payload.append(bytes(buf))
    avih = struct.pack("<IIIIIIIIIIIIII", 40000, 0, 0, 0x10, n, 0, 1, stride * h, w, h, 0, 0, 0, 0)
    strh = b"vids" + b"DIB " + struct.pack("<IHHIIIIIIIIhhhh", 0, 0, 0, 0, 1, 25, 0, n, stride * h, 0xFFFFFFFF, 0,
                                           0, 0, w, h)
    ncol = 256 if bits == 8 else 0
    bih = struct.pack("<IiiHHIIiiII", 40, w, -h if top_down else h, 1, bits, 0, stride * h, 0, 0, ncol, 0)
    pal = b"".join(struct.pack("<BBBB", i, i, i, 0) for i in range(ncol))
    strl = lst(b"strl", chunk(b"strh", strh) + chunk(b"strf", bih + pal) + chunk(b"strn", b"cam\0\0"))
    hdrl = lst(b"hdrl", chunk(b"avih", avih) + strl)
    movi_body = b"".join(chunk(fourcc, p) for p in payload)
    movi = lst(b"movi", movi_body)
    idx = b""
    off = 4
    for p in payload:
        idx += fourcc + struct.pack("<III", 0x10, off, len(p))
        off += 8 + len(p) + (len(p) & 1)
    body = b"AVI " + hdrl + chunk(b"JUNK", b"\0" * 13) + movi + chunk(b"idx1", idx)
    with open(path, "wb") as fh:
        fh.write(b"RIFF" + struct.pack("<I", len(body)) + body)


def main():
    os.makedirs(OUT, exist_ok=True)
    rng = np.random.default_rng(20261018)
    g0 = rng.integers(0, 256, (5, 12, 20), dtype=np.uint8)
    g1 = rng.integers(0, 256, (5, 12, 20), dtype=np.uint8)
    c3 = rng.integers(0, 256, (3, 5, 7, 3), dtype=np.uint8)  # B, G, R planes
    write_avi(os.path.join(OUT, "cam0_image.avi"), list(g0), 8)
    write_avi(os.path.join(OUT, "cam1_image.avi"), list(g1), 8)
    write_avi(os.path.join(OUT, "bgr24.avi"), list(c3), 24, top_down=True, fourcc=b"00dc")
    np.savez(os.path.join(OUT, "frames.npz"), cam0=g0, cam1=g1, bgr24=c3)
    with open(os.path.join(OUT, "image_data.csv"), "w") as fh:
        fh.write("#img_nb,timestamp\n" + "".join(f"{i},{1000 + 40 * i}\n" for i in range(5)))


if __name__ == "__main__":
    main()
