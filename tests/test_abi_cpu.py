"""CPU-side checks of the drop-in boundary (no GPU needed):

* libgolhip.so loads and exports every symbol include/golhip.h declares, and the
  ctypes table binds each of them;
* the header is valid C and C++;
* host logic that runs without a device: the partition (broker.go:135-206),
  error codes instead of crashes, PGM codec, wire names of stubs.go.
"""
import os
import sys
import re
import subprocess

import numpy as np
import pytest

from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "golhip.h")


@pytest.fixture(scope="module")
def G():
    import golhip
    golhip.lib()
    return golhip


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(gol_[a-z_0-9]+)\s*\(", text)))


def test_library_exports_every_declared_symbol(G):
    import ctypes
    lib = ctypes.CDLL(G._lib.LIB_PATH)
    decl = declared_functions()
    assert len(decl) >= 30
    for name in decl:
        assert hasattr(lib, name), name
    assert sorted(n for n, _, _ in G._lib.SIGNATURES) == decl


def test_nm_exports_match_header(G):
    out = subprocess.run(["nm", "-D", "--defined-only", G._lib.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = sorted({l.split()[-1] for l in out.splitlines() if l.split()[-1].startswith("gol_")})
    assert exported == declared_functions()


@pytest.mark.parametrize("compiler,lang", [("gcc", "c"), ("g++", "c++")])
def test_header_compiles(tmp_path, compiler, lang):
    src = tmp_path / ("t.c" if lang == "c" else "t.cpp")
    src.write_text('#include "golhip.h"\nint main(void){ return gol_abi_version() == GOL_ABI_VERSION ? 0 : 1; }\n')
    subprocess.run([compiler, "-fsyntax-only", "-Wall", "-Werror", "-I", os.path.dirname(HEADER), str(src)],
                   check=True)


def test_abi_version(G):
    assert G.lib().gol_abi_version() == 6


def test_ipc_unique_id_host_only(G):
    """gol_ipc_unique_id needs no GPU: 128 bytes, the IPC magic, 16 random bytes naming the ranks'
    shared-memory segment; two ids differ; a short buffer is EINVAL."""
    import ctypes
    a, b = G.engine.ipc_unique_id(), G.engine.ipc_unique_id()
    assert len(a) == len(b) == G._lib.GOL_IPC_ID_BYTES == 128
    assert a[:8] == b"GOLIPC1\0" and b[:8] == a[:8]
    assert a[8:24] != b[8:24] and a[24:] == bytes(104)
    assert G.engine.unique_id("ipc")[:8] == a[:8]
    buf = (ctypes.c_uint8 * 16)()
    assert G.lib().gol_ipc_unique_id(buf, 16) == G._lib.GOL_EINVAL


@pytest.mark.parametrize("n", [0, 24, 127, 129])
def test_rank_id_of_wrong_length_is_einval(G, n):
    """Engine.rank checks the id's length before the C call (which reads 128 bytes of it): a short
    or long id is EINVAL, not an out-of-bounds read."""
    with pytest.raises(G.GolError) as ei:
        G.Engine.rank(64, 64, 2, 0, bytes(n), transport="ipc")
    assert ei.value.code == G._lib.GOL_EINVAL
    assert "128 bytes" in str(ei.value)


@pytest.mark.parametrize("H,T", [(512, 4), (512, 16), (16, 3), (64, 7), (17, 5), (10, 16), (1, 1), (0, 3)])
def test_partition_matches_broker_formula(G, H, T):
    for i in range(T):
        assert G.partition_rows(H, T, i) == O.partition(H, T, i)


def test_partition_errors(G):
    for args in [(16, 0, 0), (16, 4, 4), (16, 4, -1), (-1, 2, 0)]:
        with pytest.raises(G.GolError) as ei:
            G.partition_rows(*args)
        assert ei.value.code == G._lib.GOL_EINVAL


def test_no_gpu_calls_fail_cleanly(G):
    import torch
    if torch.cuda.is_available():
        pytest.skip("has a GPU")
    with pytest.raises(G.GolError):
        G.Engine(16, 16)
    with pytest.raises(G.GolError):
        G.next_state_slab(np.zeros((16, 16), np.uint8), 0, 16)
    with pytest.raises(G.GolError):
        G.next_state_slab(np.zeros((16, 16), np.uint8), 5, 2)  # bad bounds: EINVAL before any HIP call


def test_pgm_reader_matches_oracle_and_errors(G, golden_dir, tmp_path):
    for name in os.listdir(os.path.join(golden_dir, "check", "images")):
        p = os.path.join(golden_dir, "check", "images", name)
        assert np.array_equal(G.read_pgm(p), O.read_pgm(p)[2])
        assert G.write_pgm_bytes(G.read_pgm(p)) == open(p, "rb").read()
    bad = tmp_path / "bad.pgm"
    bad.write_bytes(b"P2\n2 2\n255\n\x00\x00\x00\x00")
    with pytest.raises(G.GolError, match="Not a pgm file"):
        G.read_pgm(str(bad))
    bad.write_bytes(b"P5\n2 2\n15\n\x00\x00\x00\x00")
    with pytest.raises(G.GolError, match="Incorrect maxval"):
        G.read_pgm(str(bad))
    p = os.path.join(golden_dir, "images", "16x16.pgm")
    with pytest.raises(G.GolError, match="Incorrect width"):
        G.read_pgm(p, width=17)
    # io.go takes the raster as strings.Fields(data)[4]: any whitespace after maxval is skipped,
    # and a whitespace byte inside the raster would end the field (rejected)
    good = tmp_path / "crlf.pgm"
    good.write_bytes(b"P5\n2 2\n255\r\n\xff\x00\x00\xff")
    assert G.read_pgm(str(good)).tolist() == [[255, 0], [0, 255]]
    bad.write_bytes(b"P5\n2 2\n255\n\xff\x20\x00\xff")
    with pytest.raises(G.GolError, match="whitespace"):
        G.read_pgm(str(bad))


def test_stub_names_match_reference(G):
    """stubs.go:5-11 method names (the net/rpc ABI a Go drop-in keeps)."""
    s = G.stubs if hasattr(G, "stubs") else __import__("golhip.stubs", fromlist=["x"])
    assert s.GameOfLifeUpdate == "GameOfLifeOperations.Update"
    assert s.BrokeOps == "Operations.Run"
    assert s.Retrieve == "Operations.RetrieveCurrentData"
    assert s.Pause == "Operations.Pause" and s.Quit == "Operations.Quit"
    assert s.SuperQuit == "Operations.SuperQuit" and s.WorkerQuit == "GameOfLifeOperations.WorkerQuit"
    req = s.Request()
    for f in ["World", "Turns", "ImageHeight", "ImageWidth", "Threads", "EndY", "StartY", "Worker"]:
        assert hasattr(req, f)
    res = s.Response()
    for f in ["Alive", "AliveCount", "TurnsCompleted", "World", "WorkSlice", "Worker"]:
        assert hasattr(res, f)


def test_cell_list_reads_as_cells(G):
    """A Response's alive list (CellList over the device's (x, y) pairs) reads like the
    reference's []util.Cell: length, indexing, slicing, iteration and equality."""
    from golhip.stubs import Cell, CellList
    xy = np.array([[3, 0], [0, 1], [7, 1], [2, 5]], dtype=np.int32)
    cl = CellList(xy)
    want = [Cell(3, 0), Cell(0, 1), Cell(7, 1), Cell(2, 5)]
    assert len(cl) == 4 and list(cl) == want and cl == want and want == list(cl)
    assert cl[0] == Cell(3, 0) and cl[-1] == Cell(2, 5) and cl[1].X == 0 and cl[1].Y == 1
    assert cl[1:3] == want[1:3] and isinstance(cl[1:3], CellList)
    assert cl != want[:3] and cl != [Cell(3, 0), Cell(0, 1), Cell(7, 1), Cell(2, 6)]
    assert cl == CellList(xy.copy()) and Cell(7, 1) in cl and Cell(1, 7) not in cl
    assert sorted(cl, key=lambda c: (c.Y, c.X)) == want
    assert len(CellList()) == 0 and list(CellList()) == [] and CellList() == []
    assert all(type(c.X) is int for c in cl)
    np.testing.assert_array_equal(cl.array(), xy)


def test_pipe_kernels_wait_before_reading_lds(tmp_path):
    """The pipe kernels' inline-asm LDS reads: no instruction may read a destination
    VGPR before its s_waitcnt (a compiler copy there read stale rows once:
    tools/check_lds_wait.py).  Compiles gol_kernels.hip to gfx950 assembly (~20 s)."""
    import shutil
    if shutil.which("/opt/rocm/bin/hipcc") is None:
        pytest.skip("hipcc not present")
    r = subprocess.run(["python", os.path.join(ROOT, "tools", "check_lds_wait.py")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "0 hazards" in r.stdout


@pytest.mark.parametrize("unit,flags", [("gol_band_pipe.hip", "BANDFLAGS"), ("gol_bytes_pipe.hip", "BYTEFLAGS")])
def test_pipe_units_compile_with_test_defines(tmp_path, unit, flags):
    """The pipeline units under the test builds' defines (`make spintest`: GOL_SPIN_LIMIT=0;
    `make mispair` changes host code only): their inline asm takes wave-uniform ("s") operands,
    which another control flow can leave in VGPRs -- the spin-limit build of the byte loader's
    SGPR-base loads once failed to assemble while the product built."""
    import re
    import shutil
    if shutil.which("/opt/rocm/bin/hipcc") is None:
        pytest.skip("hipcc not present")
    csrc = os.path.join(ROOT, "gol-distributed-final_amd", "csrc")
    mk = open(os.path.join(csrc, "Makefile")).read()
    sched = re.search(r"^%s = (.*)$" % flags, mk, re.M).group(1).split()
    r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                        "-mllvm", "-amdgpu-atomic-optimizer-strategy=None"] + sched +
                       ["-DGOL_SPIN_LIMIT=0", "-I" + os.path.join(ROOT, "include"), "-I" + csrc,
                        "--cuda-device-only", "-c", os.path.join(csrc, unit), "-o", str(tmp_path / "u.o")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]


def test_valu_hazard_checker_catches_asm_hazards():
    """tools/check_lds_wait.py's VALU-hazard scan (round 6) on hand-made assembly: a v_dot4 result
    read at once, a DPP move of a register an asm VALU just wrote, an asm LDS DMA right after an
    M0 write -- and the same sequences padded with s_nop, or produced by compiler code (which
    hipcc pads itself), pass."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import check_lds_wait as C

    def scan(text):
        return C.valu_hazards(text)
    bad_dot = ";;#ASMSTART\n\tv_dot4_i32_i8 v1, v2, v3, v4\n;;#ASMEND\n\tv_add_u32_e32 v5, v1, v6\n"
    assert len(scan(bad_dot)) == 1
    assert not scan(bad_dot.replace(";;#ASMEND", "\ts_nop 2\n;;#ASMEND"))
    bad_dpp = (";;#ASMSTART\n\tv_bcnt_u32_b32 v7, v8, v7\n;;#ASMEND\n"
               "\tv_mov_b32_dpp v9, v7 wave_shr:1 row_mask:0xf bank_mask:0xf\n")
    assert len(scan(bad_dpp)) == 1
    assert not scan(bad_dpp.replace(";;#ASMEND\n", ";;#ASMEND\n\ts_nop 1\n"))
    assert not scan(bad_dpp.replace(";;#ASMSTART\n", "").replace(";;#ASMEND\n", ""))  # hipcc's own: padded by it
    bad_m0 = ";;#ASMSTART\n\ts_mov_b32 m0, s4\n\tglobal_load_lds_dwordx4 v[2:3], off\n;;#ASMEND\n"
    assert len(scan(bad_m0)) == 1
    assert not scan(bad_m0.replace("\tglobal_load", "\ts_nop 0\n\tglobal_load"))
    fall = "\tv_bcnt_u32_b32 v7, v8, v7\n.LBB0_1:\n;;#ASMSTART\n\tv_mov_b32_dpp v9, v7 row_shr:1\n;;#ASMEND\n"
    assert len(scan(fall)) == 1  # a label is also a fall-through
    assert not scan(fall.replace(".LBB0_1:", "\ts_branch .LBB0_2\n.LBB0_1:"))


def test_go_shims_use_only_declared_c_symbols():
    """The cgo drop-ins under go/ (not compiled here: no Go toolchain) call only functions, types
    and constants golhip.h declares, and fill only fields of its structs."""
    header = open(HEADER).read()
    decl = set(declared_functions())
    names = set(re.findall(r"\b(gol_[a-z_0-9]+|GOL_[A-Z_0-9]+)\b", header))
    used, fields = set(), set()
    for dirpath, _, files in os.walk(os.path.join(ROOT, "go")):
        for f in files:
            if f.endswith(".go"):
                text = open(os.path.join(dirpath, f)).read()
                used |= set(re.findall(r"\bC\.(gol_[a-z_0-9]+|GOL_[A-Z_0-9]+)", text))
                for lit in re.findall(r"C\.gol_(?:config|request|response)\{([^}]*)\}", text):
                    fields |= set(re.findall(r"(\w+):", lit))
                fields |= set(re.findall(r"\bc(?:req|res)\.(\w+)\b", text))
    assert used and used <= (names | decl), sorted(used - names - decl)
    struct_text = " ".join(re.findall(r"typedef struct gol_(?:config|request|response) \{(.*?)\}", header, re.S))
    for f in fields:
        assert re.search(r"\b%s\b" % f, struct_text), f


def test_layout_constants_match_header(G):
    """gol_config.layout values (golhip.h) and the binding's names agree, GOL_LAYOUT_BYTES
    included (round 5: the byte board as a layout)."""
    text = open(HEADER).read()
    vals = {m.group(1): int(m.group(2)) for m in re.finditer(r"#define GOL_LAYOUT_([A-Z]+) (\d+)", text)}
    assert vals == {"AUTO": 0, "STANDARD": 1, "BAND": 2, "BYTES": 3}
    assert G._lib.LAYOUTS == {k.lower(): v for k, v in vals.items()}
