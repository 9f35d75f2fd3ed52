"""Check the split-issue LDS reads and the inline-asm VALU hazards of the pipeline kernels in the
gfx950 assembly.

The pipe kernels issue ds_read from inline asm and wait for it in a later asm
statement (lds_*_issue / lds_wait*), so the compiler does not see the read as
asynchronous.  If it copies or reads the destination VGPRs between the issue
and the s_waitcnt lgkmcnt(0), the kernel reads stale data (this happened in
bytes_pipe_kernel: `v_mov v79, v78` between `ds_read_b32 v78` and the wait).
This script scans every kernel whose name matches a pattern and reports any
instruction that reads an in-flight register before the wait.

    python tools/check_lds_wait.py [asm.s] [--pattern REGEX]

Without an argument it compiles gol_kernels.hip to device assembly first.
Exit status 1 if a hazard is found.
"""
import argparse
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "gol-distributed-final_amd", "csrc")


def compile_asm(out):
    """The kernel translation units with the Makefile's flags (KFLAGS; the pipeline units also
    BANDFLAGS / BYTEFLAGS, their schedulers), concatenated into one assembly file."""
    parts = []
    mk = open(os.path.join(CSRC, "Makefile")).read()
    flags = {v: re.search(r"^%s = (.*)$" % v, mk, re.M).group(1).split() for v in ("BANDFLAGS", "BYTEFLAGS")}
    for src, extra in (("gol_kernels.hip", []), ("gol_band_pipe.hip", flags["BANDFLAGS"]),
                       ("gol_bytes_pipe.hip", flags["BYTEFLAGS"])):
        part = out + "." + src + ".s"
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                        "-mllvm", "-amdgpu-atomic-optimizer-strategy=None"] + extra +  # as the Makefile
                       ["-I" + os.path.join(ROOT, "include"), "-I" + CSRC, "--cuda-device-only", "-S",
                        os.path.join(CSRC, src), "-o", part], check=True, stderr=subprocess.DEVNULL)
        parts.append(open(part).read())
    with open(out, "w") as f:
        f.write("\n".join(parts))


def regs(text):
    """VGPR numbers named in an operand string (v7, v[8:11])."""
    out = set()
    for m in re.finditer(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b", text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def kernels(asm, pattern):
    for m in re.finditer(r"^(_Z\S+):.*$", asm, re.M):
        name = m.group(1)
        if not re.search(pattern, name):
            continue
        end = asm.find(".Lfunc_end", m.end())  # the whole function: a kernel may have several s_endpgm
        yield name, asm[m.end():end]


def check(body):
    """Straight-line scan of the LDS counter: outstanding LDS operations are kept in issue
    order (they complete in order); `s_waitcnt lgkmcnt(N)` retires all but the youngest N.
    A vector instruction that reads the destination of an outstanding ds_read is a hazard,
    and so is a partial wait (N > 0) while a scalar load is outstanding (scalar loads share
    the counter but complete out of order).  Labels do not reset the state, so the scan is
    an approximation of the control flow: straight-line and fall-through paths are tracked,
    code after an unconditional branch starts from an empty counter."""
    hazards = []
    out = []  # (kind, regs) in issue order
    for i, line in enumerate(body.splitlines()):
        s = line.split(";")[0].strip()
        if not s or s.endswith(":") or s.startswith("."):
            continue
        op, _, rest = s.partition(" ")
        if op == "s_waitcnt":
            m = re.search(r"lgkmcnt\((\d+)\)", rest)
            if m:
                n = int(m.group(1))
                if n < len(out):
                    if n > 0 and any(k == "smem" for k, _ in out):
                        hazards.append((i, s, ["partial lgkmcnt wait with a scalar load outstanding"]))
                    out = out[len(out) - n:] if n else []
            continue
        if op.startswith(("s_load", "s_buffer_load")):
            out.append(("smem", set()))
            continue
        if op in ("s_branch", "s_setpc_b64"):
            out = []  # the next instruction is reached from elsewhere: state unknown, assume drained
            continue
        if op.startswith("s_"):
            continue
        pending = set().union(*(r for _, r in out)) if out else set()
        if op.startswith("ds_read"):
            dst, _, src = rest.partition(",")
            used = regs(src)
        elif op.startswith(("ds_write", "buffer_store", "global_store", "flat_store")):
            used = regs(rest)
        else:
            _, _, srcs = rest.partition(",")
            used = regs(srcs)
        bad = used & pending
        if bad:
            hazards.append((i, s, sorted(bad)))
        if op.startswith("ds_read"):
            out.append(("ds", regs(dst)))
        elif op.startswith("ds_"):
            out.append(("ds", set()))
    return hazards


# VALU hazards the compiler cannot see (round 6): hipcc pads the wait states of the
# instructions it emits itself, but not those whose producer or consumer sits inside an inline-asm
# statement (cdna_hip_programming.md §5.7 item 2).  Rules checked, as (consumer, states after a
# VALU write of the register it reads):
#   DPP source (v_mov_b32_dpp ... row_/wave_ controls)     2   (VALU write VGPR -> DPP read)
#   v_readfirstlane / v_readlane source VGPR               1
#   v_permlane16/32_swap either operand                    2
#   any VALU source after a v_dot* result                  3   (the round-5 stale-sum bug)
#   global_load_lds / buffer_load ... lds after an M0 write 1  (SALU write M0 -> LDS DMA)
# Wait states: every instruction between producer and consumer counts 1, s_nop N counts N + 1.
# The scan is straight-line (fall-through across labels; an unconditional branch resets it); it reports
# only pairs with an end inside an ASMSTART/ASMEND region -- the compiler pads the rest.
HAZARD_RULES = (
    ("dpp", 2), ("readlane", 1), ("permlane", 2), ("dot", 3),
)


def _dsts_srcs(op, rest):
    dst, _, src = rest.partition(",")
    return regs(dst), regs(src)


def valu_hazards(body):
    out = []
    last_write = {}   # vgpr -> (instruction position in wait states, producer kind, in_asm)
    m0_write = None   # position of the last M0 write
    pos = 0
    in_asm = False
    for i, line in enumerate(body.splitlines()):
        t = line.strip()
        if t.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if t.startswith(";;#ASMEND"):
            in_asm = False
            continue
        s = line.split(";")[0].strip()
        if not s or s.startswith(".") or s.endswith(":"):
            continue  # (labels: a fall-through keeps the state -- conservative)
        op, _, rest = s.partition(" ")
        if op in ("s_branch", "s_setpc_b64"):
            last_write.clear()  # the next instruction is reached only by a branch
            m0_write = None
            continue
        if op == "s_nop":
            pos += int(rest.strip() or "0", 0) + 1
            continue
        pos += 1
        if op.startswith("v_"):
            dsts, srcs = _dsts_srcs(op, rest)
            dpp = "_dpp" in op or re.search(r"\b(row_|wave_|quad_perm|row_bcast)", rest)
            kinds = []
            if dpp:
                kinds.append(("dpp", 2))
            if op.startswith(("v_readfirstlane", "v_readlane")):
                kinds.append(("readlane", 1))
            if op.startswith("v_permlane"):
                kinds.append(("permlane", 2))
                srcs = srcs | dsts
            for r in srcs:
                w = last_write.get(r)
                if not w:
                    continue
                wpos, wkind, wasm = w
                need = max([n for _, n in kinds] + ([3] if wkind == "dot" else []) + [0])
                if need and pos - wpos - 1 < need and (wasm or in_asm):
                    out.append((i, s, f"v{r} written {pos - wpos - 1} wait states before, needs {need}"))
            kind = "dot" if op.startswith("v_dot") else "valu"
            for r in dsts:
                last_write[r] = (pos, kind, in_asm)
        elif op.startswith("s_") and re.match(r"\s*m0\b", rest):
            m0_write = (pos, in_asm)
        elif (op.startswith("global_load_lds") or (op.startswith("buffer_load") and " lds" in rest)) and m0_write:
            mpos, masm = m0_write
            if pos - mpos - 1 < 1 and (masm or in_asm):
                out.append((i, s, "M0 written 0 wait states before an LDS DMA, needs 1"))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm", nargs="?")
    ap.add_argument("--pattern", default=r"pipe_kernel")
    args = ap.parse_args()
    path = args.asm
    if path is None:
        path = os.path.join(tempfile.mkdtemp(), "k.s")
        compile_asm(path)
    asm = open(path).read()
    bad = 0
    n = 0
    for name, body in kernels(asm, args.pattern):
        n += 1
        for i, s, r in check(body):
            bad += 1
            print(f"{name}: line {i}: reads in-flight v{r}: {s}")
        for i, s, why in valu_hazards(body):
            bad += 1
            print(f"{name}: line {i}: VALU hazard ({why}): {s}")
    # the pipeline kernels must not spill: scratch traffic inside the pipeline loop costs more
    # than the kernel's whole LDS hand-off (and reads in-flight registers, as above)
    for blk in re.findall(r"- \.agpr_count.*?(?=\n  - \.agpr_count|\namdhsa\.target)", asm, re.S):
        name = re.search(r"\.name:\s+(\S+)", blk).group(1)
        scratch = re.search(r"\.private_segment_fixed_size:\s+(\d+)", blk)
        if re.search(args.pattern, name) and scratch and int(scratch.group(1)):
            bad += 1
            print(f"{name}: {scratch.group(1)} bytes of scratch (register spills)")
    print(f"{n} kernels checked, {bad} hazards")
    return 1 if bad or n == 0 else 0


if __name__ == "__main__":
    sys.exit(main())
