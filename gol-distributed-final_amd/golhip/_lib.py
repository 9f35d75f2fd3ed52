"""ctypes binding of libgolhip.so (include/golhip.h).

The library is the product: it is built in-tree by ``__graft_entry__.build()``
(hipcc, gfx950) next to this file.  There is no fallback -- if the shared
object is missing or fails to load, every entry point raises.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libgolhip.so")

GOL_OK = 0
GOL_EINVAL = -1
GOL_EHIP = -2
GOL_ENOMEM = -3
GOL_EIO = -4
GOL_EFORMAT = -5
GOL_ESTATE = -6
GOL_EQUIT = -7
GOL_ECOMM = -8
GOL_COUNT_SLOTS = 256
GOL_RCCL_ID_BYTES = 128
GOL_TIMING_EXCHANGE = 2
GOL_IPC_ID_BYTES = 128
GOL_IPC_MAX_RANKS = 16
GOL_LAYOUT_AUTO, GOL_LAYOUT_STANDARD, GOL_LAYOUT_BAND, GOL_LAYOUT_BYTES = 0, 1, 2, 3
LAYOUTS = {"auto": GOL_LAYOUT_AUTO, "standard": GOL_LAYOUT_STANDARD, "band": GOL_LAYOUT_BAND,
           "bytes": GOL_LAYOUT_BYTES}
GOL_TRANSPORT_AUTO, GOL_TRANSPORT_LOOPBACK, GOL_TRANSPORT_RCCL, GOL_TRANSPORT_LOCAL, GOL_TRANSPORT_IPC = 0, 1, 2, 3, 4
TRANSPORTS = {"auto": GOL_TRANSPORT_AUTO, "loopback": GOL_TRANSPORT_LOOPBACK, "rccl": GOL_TRANSPORT_RCCL,
              "ipc": GOL_TRANSPORT_IPC}
TRANSPORT_NAMES = {GOL_TRANSPORT_LOOPBACK: "loopback", GOL_TRANSPORT_RCCL: "rccl", GOL_TRANSPORT_LOCAL: "local",
                   GOL_TRANSPORT_IPC: "ipc"}
GOL_SHARDS_SAME_DEVICE = 1
GOL_STEP_SERIAL, GOL_STEP_EDGE_FIRST, GOL_STEP_OVERLAP = 2, 4, 8
STEP_MODES = {"auto": 0, "serial": GOL_STEP_SERIAL, "edge_first": GOL_STEP_EDGE_FIRST, "overlap": GOL_STEP_OVERLAP}
GOL_HALO_SEND, GOL_HALO_RECV = 0, 1
GOL_LAUNCH_MAIN, GOL_LAUNCH_EDGE = 0, 1

_NAMES = {
    GOL_EINVAL: "EINVAL", GOL_EHIP: "EHIP", GOL_ENOMEM: "ENOMEM", GOL_EIO: "EIO",
    GOL_EFORMAT: "EFORMAT", GOL_ESTATE: "ESTATE", GOL_EQUIT: "EQUIT", GOL_ECOMM: "ECOMM",
}


class GolError(RuntimeError):
    def __init__(self, code: int, message: str):
        super().__init__(f"{_NAMES.get(code, code)}: {message}")
        self.code = code


class gol_config(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("turns_per_launch", ctypes.c_int32),
                ("strip_rows", ctypes.c_int32), ("cells_per_lane", ctypes.c_int32),
                ("layout", ctypes.c_int32), ("shards", ctypes.c_int32), ("transport", ctypes.c_int32),
                ("flags", ctypes.c_int32)]


class gol_request(ctypes.Structure):
    _fields_ = [("World", ctypes.c_void_p), ("world_stride", ctypes.c_int64),
                ("Turns", ctypes.c_int64), ("ImageHeight", ctypes.c_int64),
                ("ImageWidth", ctypes.c_int64), ("Threads", ctypes.c_int64),
                ("EndY", ctypes.c_int64), ("StartY", ctypes.c_int64), ("Worker", ctypes.c_int64)]


class gol_response(ctypes.Structure):
    _fields_ = [("Alive", ctypes.c_void_p), ("alive_cap", ctypes.c_int64),
                ("alive_len", ctypes.c_int64), ("AliveCount", ctypes.c_int64),
                ("TurnsCompleted", ctypes.c_int64), ("World", ctypes.c_void_p),
                ("world_stride", ctypes.c_int64), ("WorkSlice", ctypes.c_void_p),
                ("work_stride", ctypes.c_int64), ("Worker", ctypes.c_int64)]


# int (*gol_write_fn)(void *user, int64_t offset, const uint8_t *data, int64_t len)
GOL_WRITE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64)


class gol_halo_op(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("peer", ctypes.c_int32), ("row", ctypes.c_int64), ("rows", ctypes.c_int64)]


class gol_launch(ctypes.Structure):
    _fields_ = [("stream", ctypes.c_int32), ("needs_halo", ctypes.c_int32), ("row0", ctypes.c_int64),
                ("rows", ctypes.c_int64)]


_i64 = ctypes.c_int64
_i32 = ctypes.c_int32
_u64 = ctypes.c_uint64
_vp = ctypes.c_void_p
_P = ctypes.POINTER

# (name, restype, argtypes) -- one row per declaration in include/golhip.h
SIGNATURES = [
    ("gol_abi_version", ctypes.c_int, []),
    ("gol_last_error", ctypes.c_char_p, []),
    ("gol_device_count", ctypes.c_int, [_P(ctypes.c_int)]),
    ("gol_next_state_slab", ctypes.c_int, [_vp, _i64, _i64, _i64, _i64, _i64, _vp, _i64]),
    ("gol_partition_rows", ctypes.c_int, [_i64, _i64, _i64, _P(_i64), _P(_i64)]),
    ("gol_engine_create", ctypes.c_int, [_i64, _i64, _P(gol_config), _P(_vp)]),
    ("gol_rccl_unique_id", ctypes.c_int, [_vp, _i64]),
    ("gol_ipc_unique_id", ctypes.c_int, [_vp, _i64]),
    ("gol_engine_create_rank", ctypes.c_int, [_i64, _i64, _i32, _i32, _vp, _P(gol_config), _P(_vp)]),
    ("gol_engine_destroy", None, [_vp]),
    ("gol_engine_topology", ctypes.c_int, [_vp, _P(_i32), _P(_i32), _P(_i32), _P(_i32)]),
    ("gol_engine_shard", ctypes.c_int, [_vp, _i32, _P(_i32), _P(_i64), _P(_i64)]),
    ("gol_engine_load_bytes", ctypes.c_int, [_vp, _vp, _i64]),
    ("gol_engine_load_pgm", ctypes.c_int, [_vp, ctypes.c_char_p]),
    ("gol_engine_load_random", ctypes.c_int, [_vp, _u64]),
    ("gol_engine_step", ctypes.c_int, [_vp, _i64]),
    ("gol_engine_step_counted", ctypes.c_int, [_vp, _i64, _i64, _vp, _i64]),
    ("gol_engine_turn", ctypes.c_int, [_vp, _P(_i64)]),
    ("gol_engine_alive_count", ctypes.c_int, [_vp, _P(_u64)]),
    ("gol_engine_store_bytes", ctypes.c_int, [_vp, _vp, _i64]),
    ("gol_engine_store_rows", ctypes.c_int, [_vp, _i64, _i64, _vp, _i64]),
    ("gol_engine_alive_cells", ctypes.c_int, [_vp, _vp, _i64, _P(_i64)]),
    ("gol_engine_step_flips", ctypes.c_int, [_vp, _vp, _i64, _P(_i64)]),
    ("gol_engine_write_pgm", ctypes.c_int, [_vp, ctypes.c_char_p]),
    ("gol_engine_write_pgm_to", ctypes.c_int, [_vp, _vp, _vp]),
    ("gol_engine_load_words", ctypes.c_int, [_vp, _i64, _i64, _vp, _i64]),
    ("gol_engine_store_words", ctypes.c_int, [_vp, _i64, _i64, _vp, _i64]),
    ("gol_engine_hash", ctypes.c_int, [_vp, _P(_u64)]),
    ("gol_engine_info", ctypes.c_int, [_vp, _P(_i32), _P(_i32), _P(_i32), _P(_i32)]),
    ("gol_engine_device_bits", ctypes.c_int, [_vp, _P(_vp), _P(_i64)]),
    ("gol_engine_set_timing", ctypes.c_int, [_vp, _i32]),
    ("gol_engine_timing", ctypes.c_int, [_vp, _P(_i64), _P(ctypes.c_double), _P(ctypes.c_double)]),
    ("gol_engine_exchange_timing", ctypes.c_int, [_vp, _P(_i64), _P(ctypes.c_double)]),
    ("gol_engine_exchange_split", ctypes.c_int, [_vp, _P(_i64), _P(ctypes.c_double), _P(ctypes.c_double)]),
    ("gol_halo_plan", ctypes.c_int, [_i64, _i32, _i32, _i32, _P(gol_halo_op), _i32, _P(_i32)]),
    ("gol_step_plan", ctypes.c_int, [_i64, _i32, _i32, _i32, _P(gol_launch), _i32, _P(_i32)]),
    ("gol_dev_bits_step", ctypes.c_int,
     [_vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _i32, _i32, _i32, _vp, _vp]),
    ("gol_dev_random_fill", ctypes.c_int, [_vp, _i64, _i64, _i64, _i64, _u64, _vp]),
    ("gol_dev_popcount", ctypes.c_int, [_vp, _i64, _i64, _i64, _vp, _vp]),
    ("gol_dev_hash", ctypes.c_int, [_vp, _i64, _i64, _i64, _i64, _vp, _vp]),
    ("gol_dev_pack", ctypes.c_int, [_vp, _i64, _i64, _i64, _vp, _i64, _vp, _vp]),
    ("gol_dev_unpack", ctypes.c_int, [_vp, _i64, _i64, _i64, _vp, _i64, _vp]),
    ("gol_dev_bytes_step", ctypes.c_int, [_vp, _i64, _i64, _i64, _i64, _i64, _vp, _i64, _vp]),
    ("gol_dev_bytes_step_k", ctypes.c_int,
     [_vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _i32, _i32, _vp, _vp]),
    ("gol_dev_band_step", ctypes.c_int,
     [_vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _i32, _i32, _i32, _vp, _vp]),
    ("gol_band_max_k", ctypes.c_int, [_i32]),
    ("gol_dev_band_convert", ctypes.c_int, [_i32, _vp, _vp, _i64, _i64, _i64, _i64, _vp]),
    ("gol_dev_error", ctypes.c_int, [_i32, _P(ctypes.c_uint32)]),
    ("gol_broker_create", ctypes.c_int, [_P(gol_config), _P(_vp)]),
    ("gol_broker_destroy", None, [_vp]),
    ("gol_broker_run", ctypes.c_int, [_vp, _P(gol_request), _P(gol_response)]),
    ("gol_broker_retrieve", ctypes.c_int, [_vp, _P(gol_request), _P(gol_response)]),
    ("gol_broker_pause", ctypes.c_int, [_vp]),
    ("gol_broker_quit", ctypes.c_int, [_vp]),
    ("gol_broker_superquit", ctypes.c_int, [_vp]),
    ("gol_broker_paused", ctypes.c_int, [_vp, _P(_i32)]),
    ("gol_worker_update", ctypes.c_int, [_P(gol_request), _P(gol_response)]),
]

_lib = None


def _one_hip_runtime():
    """libgolhip.so links ROCm's libamdhip64.so.7; PyTorch ships its own copy with the same soname.
    The first one loaded serves the whole process, and torch's GPU initialisation fails on the
    other one, so torch (when installed) is loaded first: then both use torch's runtime (the two
    are ABI-compatible: every GPU test passes torch tensors to the library)."""
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def load(path: str, strict: bool = True):
    """Bind the C ABI of the shared object at `path` (raises if it is missing).  strict=False
    (same-box A/B builds of older revisions, tools/ab.py) skips entry points it lacks."""
    _one_hip_runtime()
    if not os.path.exists(path):
        raise GolError(GOL_ESTATE, f"{path} is missing: run __graft_entry__.build() "
                                   "(hipcc --offload-arch=gfx950); there is no CPU fallback")
    L = ctypes.CDLL(path)
    for name, res, args in SIGNATURES:
        if not strict and not hasattr(L, name):
            continue
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    return L


def lib():
    """libgolhip.so, the product library (built in-tree next to this file)."""
    global _lib
    if _lib is None:
        _lib = load(LIB_PATH)
    return _lib


def check(rc: int) -> None:
    if rc != GOL_OK:
        raise GolError(rc, lib().gol_last_error().decode(errors="replace"))


def halo_plan(H: int, nranks: int, rank: int, k: int) -> list[tuple[str, int, int, int]]:
    """gol_halo_plan: the halo exchange of `rank` in issue order, as (kind "send"/"recv", peer,
    first shard-local row, rows).  Host code: no GPU needed."""
    ops = (gol_halo_op * 4)()
    n = ctypes.c_int32()
    check(lib().gol_halo_plan(H, nranks, rank, k, ops, 4, ctypes.byref(n)))
    return [("send" if o.kind == GOL_HALO_SEND else "recv", o.peer, o.row, o.rows) for o in ops[:n.value]]


def step_plan(R: int, k: int, kx: int, mode: str = "overlap") -> list[tuple[str, bool, int, int]]:
    """gol_step_plan: the launches of one k-turn step of an R-row shard in launch order, as
    (stream "main"/"edge", needs_halo, first output row, rows); mode "overlap", "edge_first" or
    "serial"."""
    out = (gol_launch * 3)()
    n = ctypes.c_int32()
    check(lib().gol_step_plan(R, k, kx, STEP_MODES[mode], out, 3, ctypes.byref(n)))
    return [("edge" if L.stream == GOL_LAUNCH_EDGE else "main", bool(L.needs_halo), L.row0, L.rows)
            for L in out[:n.value]]


def device_count() -> int:
    n = ctypes.c_int()
    check(lib().gol_device_count(ctypes.byref(n)))
    return n.value
