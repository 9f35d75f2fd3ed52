"""Check the split-issue LDS reads of the pipeline kernels in the gfx950 assembly.

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
