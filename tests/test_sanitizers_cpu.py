"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer (the reference has no
race/sanitizer checks; the build runs its host code under ASan/UBSan here, CPU only -- GPU
sanitizers are not available).

`make -C gol-distributed-final_amd/csrc asan` (run by __graft_entry__.build()) instruments
gol_abi.cpp, gol_engine.cpp and gol_host.cpp:
  * golhip/libgolhip_asan.so -- the C ABI with instrumented host code, driven here through ctypes in
    a child Python with the clang ASan runtime preloaded: every entry point that runs without a GPU
    (partition, argument and state errors, the worker's and broker's request checks, engine
    creation failing cleanly);
  * build/asan/pgm_header_check -- the native P5 header parser (io.go:97-117 rules) on random and
    mutated headers, each verdict compared with golhip.pgm.pgm_header (differential).
Any sanitizer report fails the test (UBSan without recovery, ASan aborts).
"""
import glob
import os
import random
import struct
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "gol-distributed-final_amd")
ASAN_LIB = os.path.join(PKG, "golhip", "libgolhip_asan.so")
HEADER_CHECK = os.path.join(PKG, "build", "asan", "pgm_header_check")
RUNTIME = sorted(glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so"))

pytestmark = pytest.mark.skipif(not RUNTIME or not os.path.exists(ASAN_LIB) or not os.path.exists(HEADER_CHECK),
                                reason="sanitizer build missing (make -C gol-distributed-final_amd/csrc asan)")


def _env(preload=True):
    env = dict(os.environ)
    if preload:  # the child Python is not instrumented; the driver binary links its runtime statically
        env["LD_PRELOAD"] = RUNTIME[-1]
    env["ASAN_OPTIONS"] = "detect_leaks=0:abort_on_error=0:exitcode=23"
    env["UBSAN_OPTIONS"] = "print_stacktrace=1:halt_on_error=1:exitcode=24"
    return env


CHILD = r"""
import ctypes, sys
sys.path[:0] = [%(root)r, %(pkg)r]
import numpy as np
import golhip._lib as L
L._lib = L.load(%(lib)r)
import golhip as G
from golhip._lib import gol_config, gol_request, gol_response, lib
from oracle import oracle as O

assert lib().gol_abi_version() == 6
for H in (0, 1, 2, 10, 17, 512, 1 << 20):
    for T in (1, 2, 3, 7, 16):
        for i in range(T):
            assert G.partition_rows(H, T, i) == O.partition(H, T, i)
for args in [(16, 0, 0), (16, 4, 4), (16, 4, -1), (-1, 2, 0), (1 << 62, 3, 1)]:
    try:
        G.partition_rows(*args)
    except G.GolError:
        pass
assert lib().gol_partition_rows(16, 4, 0, None, None) != 0
assert isinstance(lib().gol_last_error(), bytes)
n = ctypes.c_int(-1)
lib().gol_device_count(ctypes.byref(n))
# engine entry points on a NULL handle: EINVAL, no crash
h = ctypes.c_void_p()
for name, args in [("gol_engine_step", (h, 1)), ("gol_engine_load_random", (h, 1)), ("gol_engine_turn", (h, None)),
                   ("gol_engine_alive_count", (h, None)), ("gol_engine_hash", (h, None)),
                   ("gol_engine_load_pgm", (h, None)), ("gol_engine_write_pgm", (h, None)),
                   ("gol_engine_set_timing", (h, 1)), ("gol_engine_step_counted", (h, 1, 1, None, 0))]:
    assert getattr(lib(), name)(*args) != 0, name
lib().gol_engine_destroy(h)
# engine / broker creation without a GPU fails cleanly; bad shapes are EINVAL first
for H, W in [(16, 16), (0, 16), (16, -1), (1 << 40, 1 << 40)]:
    try:
        G.Engine(H, W)
    except G.GolError:
        pass
cfg = gol_config(device=-1)
b = ctypes.c_void_p()
if lib().gol_broker_create(ctypes.byref(cfg), ctypes.byref(b)) == 0:
    lib().gol_broker_destroy(b)
# the worker's Update checks its request before any HIP call
world = np.zeros((16, 16), np.uint8)
res = gol_response()
for (y0, y1, H, W, stride) in [(5, 2, 16, 16, 16), (0, 17, 16, 16, 16), (-1, 4, 16, 16, 16), (0, 4, 16, 16, 8),
                               (0, 4, 0, 16, 16), (0, 4, 16, 0, 16)]:
    req = gol_request(World=world.ctypes.data, world_stride=stride, Turns=1, ImageHeight=H, ImageWidth=W,
                      Threads=1, StartY=y0, EndY=y1)
    assert lib().gol_worker_update(ctypes.byref(req), ctypes.byref(res)) != 0
req = gol_request(World=None, world_stride=16, Turns=1, ImageHeight=16, ImageWidth=16, Threads=1, StartY=0, EndY=4)
assert lib().gol_worker_update(ctypes.byref(req), ctypes.byref(res)) != 0
assert lib().gol_worker_update(None, None) != 0
print("sanitized ok")
"""


def test_abi_host_paths_under_asan_ubsan():
    code = CHILD % {"root": ROOT, "pkg": PKG, "lib": ASAN_LIB}
    p = subprocess.run([sys.executable, "-c", code], env=_env(), capture_output=True, text=True, timeout=600)
    report = p.stderr[-4000:]
    assert p.returncode == 0 and "sanitized ok" in p.stdout, report
    assert "AddressSanitizer" not in p.stderr and "runtime error" not in p.stderr, report


def _mutations(rng):
    base = [b"P5\n16 16\n255\n", b"P5 16 16 255 ", b"P5\r\n16\t16\v255\f\x00", b"P2\n16 16\n255\n", b"P5\n16 16\n15\n",
            b"P5\n+16 16\n255\n", b"P5\n-16 16\n255\n", b"P5\n16abc 16\n255\n", b"P5\n1_6 16\n255\n",
            b"P5\n99999999999999999999 16\n255\n", b"P5\n16 16\n255", b"P5\n16 16\n255\n\n\n", b"", b"P5", b" \n\t",
            b"P5\n16 16 255\xff\x00", b"P5\n0016 016\n0255\n"]
    out = list(base)
    for _ in range(1500):
        s = bytearray(rng.choice(base))
        for _ in range(rng.randint(0, 4)):
            op = rng.randint(0, 2)
            if op == 0 and s:
                del s[rng.randrange(len(s))]
            elif op == 1:
                s.insert(rng.randint(0, len(s)), rng.choice(b" \t\n\r\v\f0123456789+-P5\x00\xff"))
            elif s:
                s[rng.randrange(len(s))] = rng.randrange(256)
        out.append(bytes(s))
    return out


def test_native_pgm_header_parser_matches_python_under_asan():
    from golhip._lib import GOL_OK, GolError
    from golhip.pgm import pgm_header
    rng = random.Random(5)
    cases = _mutations(rng)
    blob = b"".join(struct.pack("<qqI", 16, 16, len(h)) + h for h in cases)
    p = subprocess.run([HEADER_CHECK], input=blob, env=_env(preload=False), capture_output=True, timeout=300)
    assert p.returncode == 0, p.stderr.decode(errors="replace")[-4000:]
    got = [tuple(int(x) for x in ln.split()) for ln in p.stdout.decode().splitlines()]
    assert len(got) == len(cases)
    for h, (rc, off) in zip(cases, got):
        try:
            W, H, want_off = pgm_header(h, 16, 16)
            want = (GOL_OK, want_off if want_off < len(h) else None)
        except GolError as e:
            want = (e.code, -1)
        if want[0] == GOL_OK and want[1] is None:
            want = (rc, off) if rc != GOL_OK else want  # no raster byte after the header: native says so
        assert (rc, off) == want, (h, rc, off, want)
