"""PGM P5 codec with the reference's byte layout and error messages (gol/io.go:42-126).

Boards are written by the engine on the device side (gol_engine_write_pgm);
this module is the host-side reader used to feed images/<W>x<H>.pgm to it.
"""
from __future__ import annotations

import numpy as np

from ._lib import GOL_EFORMAT, GolError

_SPACE = b" \t\n\v\f\r"


def go_atoi(field: bytes) -> int:
    """strconv.Atoi with its error dropped (io.go:104-116): an optional sign and ASCII digits;
    anything else is 0, out of range is the clamped int64."""
    digits = field[1:] if field[:1] in (b"+", b"-") else field
    if not digits or any(c < 0x30 or c > 0x39 for c in digits):
        return 0
    v = int(digits.decode("ascii")) * (-1 if field[:1] == b"-" else 1)
    return max(-(1 << 63), min((1 << 63) - 1, v))


def pgm_header(head: bytes, width: int | None = None, height: int | None = None) -> tuple[int, int, int]:
    """io.go:90-126 header rules on the first bytes of a P5 file: fields = strings.Fields(data);
    "P5", width, height, 255.  Returns (W, H, offset of the first raster byte)."""
    fields, i, n = [], 0, len(head)
    while i < n and len(fields) < 4:
        while i < n and head[i] in _SPACE:
            i += 1
        j = i
        while j < n and head[j] not in _SPACE:
            j += 1
        if j > i:
            fields.append(head[i:j])
        i = j
    if not fields or fields[0] != b"P5":
        raise GolError(GOL_EFORMAT, "Not a pgm file")
    if len(fields) < 4:
        raise GolError(GOL_EFORMAT, "Not a pgm file")
    W, H, maxval = go_atoi(fields[1]), go_atoi(fields[2]), go_atoi(fields[3])
    if width is not None and W != width:
        raise GolError(GOL_EFORMAT, "Incorrect width")
    if height is not None and H != height:
        raise GolError(GOL_EFORMAT, "Incorrect height")
    if maxval != 255:
        raise GolError(GOL_EFORMAT, "Incorrect maxval/bit depth")
    while i < n and head[i] in _SPACE:  # the raster is fields[4]: it starts at the next non-space byte
        i += 1
    return W, H, i


def _check_raster(raster: np.ndarray) -> None:
    """The reference takes the raster as strings.Fields(data)[4] (io.go:98-119): a whitespace byte
    inside it would end the field early (and the reference would then wait for the missing
    pixels), so such files are rejected here instead of read differently."""
    if np.isin(raster, np.frombuffer(_SPACE, dtype=np.uint8)).any():
        raise GolError(GOL_EFORMAT, "pixel data shorter than W*H (a whitespace byte ends the field)")


def read_pgm(path: str, width: int | None = None, height: int | None = None) -> np.ndarray:
    """io.go:90-126 readPgmImage: the whole raster as an (H, W) uint8 array."""
    with open(path, "rb") as f:
        data = f.read()
    W, H, off = pgm_header(data[:4096], width, height)
    if len(data) < off + W * H:
        raise GolError(GOL_EFORMAT, "pixel data shorter than W*H")
    raster = np.frombuffer(data, dtype=np.uint8, count=W * H, offset=off).reshape(H, W).copy()
    _check_raster(raster)
    return raster


def pgm_rows(path: str, y0: int, y1: int, width: int | None = None, height: int | None = None):
    """Rows [y0, y1) of a P5 file as a read-only (y1-y0, W) memory map: a rank of a sharded
    board reads only its own rows (a 2^20 x 2^20 image is 1 TiB)."""
    with open(path, "rb") as f:
        head = f.read(4096)
        f.seek(0, 2)
        size = f.tell()
    W, H, off = pgm_header(head, width, height)
    if size < off + W * H:
        raise GolError(GOL_EFORMAT, "pixel data shorter than W*H")
    if not 0 <= y0 <= y1 <= H:
        raise ValueError(f"rows [{y0}, {y1}) outside the {H}-row image")
    return np.memmap(path, dtype=np.uint8, mode="r", offset=off + y0 * W, shape=(y1 - y0, W))


def write_pgm_bytes(board: np.ndarray) -> bytes:
    """io.go:52-81 byte stream: "P5\\n<W> <H>\\n255\\n" + H*W raster bytes."""
    H, W = board.shape
    return b"P5\n%d %d\n255\n" % (W, H) + np.ascontiguousarray(board, dtype=np.uint8).tobytes()
