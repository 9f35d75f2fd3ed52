"""Per-workgroup timeline of the pipeline kernels (measurement only).

Builds a copy of libgolhip.so whose band_pipe_kernel / bytes_pipe_kernel write, per wave, the
s_memrealtime stamps (100 MHz, chip-wide) of kernel entry and exit plus the HW_ID / XCC_ID
registers into the count-slot buffer (which the launch is given instead of count slots), runs
one launch of a workload and summarises when workgroups start and end: how much of the kernel
span the waves are resident, the dispatch ramp, and the tail.

    python tools/timeline.py build [-DFLAG=..] [--out NAME]  # here (hipcc), -> tools/variants/libNAME.so
        # (default libtimeline; the patched sources are built in a temporary directory and removed)
    python tools/timeline.py run bit64k|byte16k|weak|strong2|strong8|strong262k [--strip N] [--wrap] [--pre N]
        # on the GPU box; --wrap: wrap rows read from the board (LOCAL launch), else ghost rows;
        # --pre N: a fill kernel over N x 4096 floats right before the launch
    python tools/timeline.py build -DGOL_EXP_CLOCK --out libclock   # then, on the box:
    GOL_TL_LIB=tools/variants/libclock.so python tools/timeline.py clock WORKLOAD
        # the shader clock under load: every wave's s_memtime / s_memrealtime (100 MHz) deltas over
        # its life in the last of >= 2 s of back-to-back launches on a random board (median over
        # waves; MI355X_MICROARCH.md 'DVFS give-back' item 6), for dispatches too short for
        # GRBM_GUI_ACTIVE / 8 / time
"""
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "gol-distributed-final_amd", "csrc")
VARIANTS = os.path.join(ROOT, "tools", "variants")
LIB = os.environ.get("GOL_TL_LIB") or os.path.join(VARIANTS, "libtimeline.so")

ENTRY = "    const int lane = threadIdx.x & 63;\n"
STAMP_T0 = ENTRY + "    const uint64_t tl_t0 = __builtin_amdgcn_s_memrealtime();\n    const uint64_t tl_c0 = __builtin_amdgcn_s_memtime(); (void)tl_c0;\n"
COUNT_LINE = "    if (COUNT && wv == P - 1) slot_add(a.slots, alive);\n"
STORE = """    {  // timeline: (t0, t1, hw_id, xcc_id) per wave, slot = linear workgroup id * P + wave
        const uint64_t tl_t1 = __builtin_amdgcn_s_memrealtime();
        const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
        const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);
        const uint64_t i = ((uint64_t)blockIdx.y * gridDim.x + blockIdx.x) * (blockDim.x >> 6) + (threadIdx.x >> 6);
        if ((threadIdx.x & 63) == 0) {
            a.slots[4 * i] = tl_t0; a.slots[4 * i + 1] = tl_t1;
#ifdef GOL_EXP_PROF
            a.slots[4 * i] = tl_c0; a.slots[4 * i + 1] = __builtin_amdgcn_s_memtime();
            a.slots[4 * i + 2] = prof_a; a.slots[4 * i + 3] = prof_b | ((uint64_t)wv << 56); (void)hw; (void)xcc;
#elif defined(GOL_EXP_CLOCK)
            a.slots[4 * i + 2] = tl_c0; a.slots[4 * i + 3] = __builtin_amdgcn_s_memtime(); (void)hw; (void)xcc;
#else
            a.slots[4 * i + 2] = hw; a.slots[4 * i + 3] = xcc | ((uint64_t)wv << 56) | ((uint64_t)(threadIdx.x >> 6) << 48);
#endif
        }
        (void)alive;
    }
"""


PROF_SPINS = (  # -DGOL_EXP_PROF: cycles each wave spends in its flag waits (ready -> a, free -> b)
    ("seen_free = spin_until_ge(consumed_l + wv + 1, b + 1 - NS);", "prof_b"),
    ("seen_ready = spin_until_ge(ready_l + wv, b + 2);", "prof_a"),
    ("seen_ready = spin_until_ge(ready_l + wv, b + 1);", "prof_a"),
    ("seen_ready = spin_until_ge(ready_l + wv, 1);", "prof_a"),
)


def build(flags="", name="libtimeline"):
    import shutil
    import tempfile
    os.makedirs(VARIANTS, exist_ok=True)
    OUT = tempfile.mkdtemp(prefix="gol_tl_")
    src = open(os.path.join(CSRC, "gol_kernels.hip")).read()
    if "GOL_EXP_PROF" in flags:
        for stmt, acc in PROF_SPINS:
            if stmt not in src:
                continue
            src = src.replace(stmt, "{ const uint64_t pt_ = __builtin_amdgcn_s_memtime(); " + stmt +
                              f" {acc} += __builtin_amdgcn_s_memtime() - pt_; }}")
        for kern in ("band_pipe_kernel(BitsArgs a)", "bytes_pipe_kernel(BytesKArgs a)"):
            i = src.index(kern)
            j = src.index("    uint32_t alive = 0;\n", i)
            src = src[:j] + "    uint64_t prof_a = 0, prof_b = 0;\n" + src[j:]
    for kern in ("band_pipe_kernel(BitsArgs a)", "bytes_pipe_kernel(BytesKArgs a)"):
        i = src.index(kern)
        j = src.index(ENTRY, i)
        src = src[:j] + STAMP_T0 + src[j + len(ENTRY):]
        k = src.index(COUNT_LINE, j)  # the kernel's final fused-count slot_add: the stamps replace it
        src = src[:k] + STORE + src[k + len(COUNT_LINE):]
    open(os.path.join(OUT, "gol_kernels.hip"), "w").write(src)
    for f in os.listdir(CSRC):
        if f.endswith((".cpp", ".h")) or f == "Makefile" or (f.endswith(".hip") and f != "gol_kernels.hip"):
            with open(os.path.join(CSRC, f)) as a, open(os.path.join(OUT, f), "w") as b:
                b.write(a.read())
    lib = os.path.join(VARIANTS, name + ".so")
    try:
        subprocess.run(["make", "-s", "-j8", "-C", OUT, "ARCH=gfx950", "BUILD=./obj", f"OUT={lib}",
                        f"CXXFLAGS=-O3 -std=c++17 -fPIC -Wall -I{ROOT}/include -I. {flags}", f"INC={ROOT}/include"], check=True)
    finally:
        shutil.rmtree(OUT, ignore_errors=True)  # (the patched copy of the sources is not kept)
    print(lib)


def run(workload, strip, wrap=False, pre=0):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "gol-distributed-final_amd")]
    import ctypes

    import numpy as np
    import torch

    import golhip._lib as L
    lib = L.load(LIB)
    st = torch.cuda.current_stream().cuda_stream
    if workload == "byte16k":
        H = W = 16384
        k, P = 32, 8
        a = torch.zeros((H, W), dtype=torch.uint8, device="cuda")
        b = torch.empty_like(a)
        ngroups = (W // 32 + 61) // 62
        buf = torch.zeros(4 * P * ngroups * H, dtype=torch.int64, device="cuda")  # generous
        launch = lambda: lib.gol_dev_bytes_step_k(a[H - k:].data_ptr(), a.data_ptr(), a.data_ptr(), b.data_ptr(), H, W,  # noqa: E731
                                                  W, 0, H, k, strip, buf.data_ptr(), st)
    else:
        H, W = {"bit64k": (65536, 65536), "weak": (1 << 17, 1 << 20), "strong2": (131072, 262144),
                "strong8": (32768, 262144), "strong262k": (262144, 262144)}[workload]
        k, P = 12, 16  # buffer sized for up to 16 waves per work item
        Wd = W // 32
        g = 16
        a = torch.zeros((H + 2 * g, Wd), dtype=torch.int32, device="cuda")
        b = torch.zeros_like(a)
        mid = a[g:g + H]
        ngroups = (Wd + 231) // 232
        buf = torch.zeros(4 * P * ngroups * min(H, 8192), dtype=torch.int64, device="cuda")
        # --wrap: the torus wrap rows read from the board itself (the LOCAL engine's launch);
        # else from ghost rows right above and below (contiguous: the N-GPU launch)
        top = mid[H - k:] if wrap else a[g - k:]
        bot = mid if wrap else a[g + H:]
        launch = lambda: lib.gol_dev_band_step(top.data_ptr(), mid.data_ptr(), bot.data_ptr(),  # noqa: E731
                                               b[g:].data_ptr(), H, Wd, Wd, 0, H, k, 128, strip, buf.data_ptr(), st)
    pre_t = torch.empty(max(1, pre) * 4096, dtype=torch.float32, device="cuda")
    for _ in range(3):
        assert launch() == 0
    torch.cuda.synchronize()
    buf.zero_()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if pre:  # a kernel of some other grid right before the launch, on the same stream
        pre_t.fill_(1.0)
    e0.record()
    assert launch() == 0
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    v = buf.view(-1, 4).cpu().numpy().astype(np.int64)
    v = v[v[:, 1] > 0]
    t0, t1 = v[:, 0], v[:, 1]
    base = t0.min()
    s, e = (t0 - base) / 100.0, (t1 - base) / 100.0  # microseconds (100 MHz)
    span = e.max()
    hw, xcc = v[:, 2], v[:, 3] & 0xFFFF
    cu = (hw >> 8) & 0xF
    se = (hw >> 13) & 0x7
    simd = (hw >> 4) & 0x3
    key = xcc * 1000 + se * 100 + cu
    per_cu = {}
    for kk in np.unique(key):
        m = key == kk
        per_cu[int(kk)] = (int(m.sum()), float(e[m].max()))
    life = e - s
    out = {"workload": workload, "strip": strip, "wrap": wrap, "pre": pre, "event_ms": round(ms, 4), "waves": int(len(v)), "span_us": round(float(span), 1),
           "resident_frac": round(float(life.sum() / (span * 16 * 256)), 3),
           "start_us_pct": [round(float(np.percentile(s, q)), 1) for q in (0, 10, 50, 90, 99, 100)],
           "end_us_pct": [round(float(np.percentile(e, q)), 1) for q in (0, 1, 10, 50, 90, 100)],
           "life_us_pct": [round(float(np.percentile(life, q)), 1) for q in (0, 10, 50, 90, 100)],
           "cus_used": len(per_cu), "waves_per_cu": sorted({c for c, _ in per_cu.values()}),
           "cu_end_us_pct": [round(float(np.percentile([x for _, x in per_cu.values()], q)), 1) for q in (0, 10, 50, 90, 100)],
           "simd_hist": np.bincount(simd, minlength=4).tolist()}
    if not os.environ.get("GOL_TL_PROF"):
        # pipeline roles per SIMD (role = wv, the wave's position in its pipeline) and how the
        # wave index maps to the SIMD
        role = (v[:, 3] >> 56) & 0xFF
        widx = (v[:, 3] >> 48) & 0xFF
        out["simd_of_wave_index"] = {int(w): np.bincount(simd[widx == w], minlength=4).tolist() for w in np.unique(widx)}
        # for every CU: at each wave's start, the roles resident on its SIMD (same CU) -- the
        # fraction of waves that share their SIMD with another wave of the same role
        same = 0
        order = np.argsort(s)
        for kk in np.unique(key):
            idx = np.where(key == kk)[0]
            for i in idx:
                live = idx[(s[idx] <= s[i]) & (e[idx] > s[i]) & (simd[idx] == simd[i]) & (idx != i)]
                same += int((role[live] == role[i]).any())
        out["share_simd_with_same_role"] = round(same / len(v), 3)
        out["role_simd_hist"] = {int(r): np.bincount(simd[role == r], minlength=4).tolist() for r in np.unique(role)}
    if os.environ.get("GOL_TL_PROF"):  # prof build: slots = (c0, c1, ready-wait, free-wait | role << 56) in shader cycles
        life_c = (v[:, 1] - v[:, 0]).astype(np.float64)
        role = (v[:, 3] >> 56) & 0xFF
        out["prof"] = {int(r): {"waves": int((role == r).sum()), "life_Mcyc_med": round(float(np.median(life_c[role == r])) / 1e6, 3),
                                "ready_wait_frac": round(float(v[role == r, 2].sum() / life_c[role == r].sum()), 4),
                                "free_wait_frac": round(float((v[role == r, 3] & ((1 << 56) - 1)).sum() / life_c[role == r].sum()), 4)}
                       for r in np.unique(role)}
        out["start_us_pct"] = out["end_us_pct"] = out["life_us_pct"] = None
    print(json.dumps(out))
    np.save(os.path.join(ROOT, "gpurun_out", f"timeline_{workload}_{strip}_{int(wrap)}_{pre}.npy"), v)


def clock(workload, seconds=2.0):
    """Median in-kernel shader clock of the step kernel of `workload` on a random board."""
    sys.path[:0] = [ROOT, os.path.join(ROOT, "gol-distributed-final_amd")]
    import time

    import numpy as np
    import torch

    import golhip._lib as L
    lib = L.load(LIB)
    st = torch.cuda.current_stream().cuda_stream
    if workload == "byte16k":
        H = W = 16384
        k, P = 32, 8
        bits = torch.empty((H, W // 32), dtype=torch.int32, device="cuda")
        assert lib.gol_dev_random_fill(bits.data_ptr(), H, 0, W, W // 32, 1, st) == 0
        a = torch.empty((H, W), dtype=torch.uint8, device="cuda")
        assert lib.gol_dev_unpack(bits.data_ptr(), H, W, W // 32, a.data_ptr(), W, st) == 0
        b = torch.empty_like(a)
        buf = torch.zeros(4 * P * ((W // 32 + 61) // 62) * H, dtype=torch.int64, device="cuda")
        bufs = [(a, b), (b, a)]
        launch = lambda s, d: lib.gol_dev_bytes_step_k(s[H - k:].data_ptr(), s.data_ptr(), s.data_ptr(), d.data_ptr(),  # noqa: E731
                                                       H, W, W, 0, H, k, 0, buf.data_ptr(), st)
    else:
        H, W = {"bit64k": (65536, 65536), "weak": (1 << 17, 1 << 20), "strong262k": (262144, 262144)}[workload]
        k, P = 12, 16
        Wd = W // 32
        a = torch.empty((H, Wd), dtype=torch.int32, device="cuda")
        b = torch.empty_like(a)
        assert lib.gol_dev_random_fill(a.data_ptr(), H, 0, W, Wd, 1, st) == 0
        buf = torch.zeros(4 * P * ((Wd + 231) // 232) * H, dtype=torch.int64, device="cuda")
        bufs = [(a, b), (b, a)]
        launch = lambda s, d: lib.gol_dev_band_step(s[H - k:].data_ptr(), s.data_ptr(), s.data_ptr(), d.data_ptr(),  # noqa: E731
                                                    H, Wd, Wd, 0, H, k, 128, 0, buf.data_ptr(), st)
    torch.cuda.synchronize()
    t0, n = time.perf_counter(), 0
    while time.perf_counter() - t0 < seconds:  # back-to-back launches (the board evolves: random data)
        for _ in range(8):
            s, d = bufs[n & 1]
            assert launch(s, d) == 0
            n += 1
        torch.cuda.synchronize()
    buf.zero_()
    s, d = bufs[n & 1]
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    assert launch(s, d) == 0
    e1.record()
    torch.cuda.synchronize()
    v = buf.view(-1, 4).cpu().numpy().astype(np.int64)
    v = v[(v[:, 1] > v[:, 0]) & (v[:, 3] > v[:, 2])]
    ghz = (v[:, 3] - v[:, 2]) / ((v[:, 1] - v[:, 0]) / 100.0) / 1e3  # cycles per us / 1000
    out = {"workload": workload, "launches_before": n, "event_ms": round(e0.elapsed_time(e1), 4), "waves": int(len(v)),
           "clock_GHz_median": round(float(np.median(ghz)), 3),
           "clock_GHz_pct": [round(float(np.percentile(ghz, q)), 3) for q in (5, 25, 50, 75, 95)],
           "method": "per wave: delta s_memtime / delta s_memrealtime x 100 MHz over its life, in the last of "
                     f"{n + 1} back-to-back launches ({seconds} s) on a random board"}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "clock":
        clock(sys.argv[2])
        sys.exit(0)
    if sys.argv[1] == "build":
        args = sys.argv[2:]
        name = "libtimeline"
        if "--out" in args:
            i = args.index("--out")
            name = args[i + 1]
            del args[i:i + 2]
        build(" ".join(args), name)  # extra compiler flags, e.g. -DGOL_EXP_CLOCK
    else:
        strip = int(sys.argv[sys.argv.index("--strip") + 1]) if "--strip" in sys.argv else 0
        pre = int(sys.argv[sys.argv.index("--pre") + 1]) if "--pre" in sys.argv else 0
        run(sys.argv[2], strip, "--wrap" in sys.argv, pre)
