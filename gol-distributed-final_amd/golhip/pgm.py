"""PGM P5 codec with the reference's byte layout and error messages (gol/io.go:42-126).

Boards are written by the engine on the device side (gol_engine_write_pgm);
this module is the host-side reader used to feed images/<W>x<H>.pgm to it.
"""
from __future__ import annotations

import numpy as np

from ._lib import GOL_EFORMAT, GolError

_SPACE = b" \t\n\v\f\r"


def read_pgm(path: str, width: int | None = None, height: int | None = None) -> np.ndarray:
    """io.go:90-126: fields = strings.Fields(data); "P5", width, height, 255, pixels."""
    with open(path, "rb") as f:
        data = f.read()
    fields, i, n = [], 0, len(data)
    while i < n and len(fields) < 4:
        while i < n and data[i] in _SPACE:
            i += 1
        j = i
        while j < n and data[j] not in _SPACE:
            j += 1
        if j > i:
            fields.append(data[i:j])
        i = j
    if not fields or fields[0] != b"P5":
        raise GolError(GOL_EFORMAT, "Not a pgm file")
    try:
        W, H, maxval = int(fields[1]), int(fields[2]), int(fields[3])
    except (IndexError, ValueError):
        raise GolError(GOL_EFORMAT, "Not a pgm file")
    if width is not None and W != width:
        raise GolError(GOL_EFORMAT, "Incorrect width")
    if height is not None and H != height:
        raise GolError(GOL_EFORMAT, "Incorrect height")
    if maxval != 255:
        raise GolError(GOL_EFORMAT, "Incorrect maxval/bit depth")
    # one whitespace byte separates maxval from the raster
    pix = np.frombuffer(data, dtype=np.uint8, count=W * H, offset=i + 1) if n >= i + 1 + W * H else None
    if pix is None:
        raise GolError(GOL_EFORMAT, "pixel data shorter than W*H")
    return pix.reshape(H, W).copy()


def write_pgm_bytes(board: np.ndarray) -> bytes:
    """io.go:52-81 byte stream: "P5\\n<W> <H>\\n255\\n" + H*W raster bytes."""
    H, W = board.shape
    return b"P5\n%d %d\n255\n" % (W, H) + np.ascontiguousarray(board, dtype=np.uint8).tobytes()
