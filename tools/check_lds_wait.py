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
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                    "-I" + os.path.join(ROOT, "include"), "-I" + CSRC, "--cuda-device-only", "-S",
                    os.path.join(CSRC, "gol_kernels.hip"), "-o", out], check=True,
                   stderr=subprocess.DEVNULL)


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
        end = asm.find("s_endpgm", m.end())
        yield name, asm[m.end():end]


def check(body):
    """Straight-line scan: after an asm ds_read, any use of its destination before an
    lgkmcnt(0) wait is a hazard.  Branch targets reset the in-flight set only when a wait
    is seen, so a hazard across a label is still reported (conservative)."""
    hazards = []
    pending = {}  # vgpr -> line of the ds_read
    in_asm = False
    for i, line in enumerate(body.splitlines()):
        s = line.split(";")[0].strip()
        if ";;#ASMSTART" in line:
            in_asm = True
            continue
        if ";;#ASMEND" in line:
            in_asm = False
            continue
        if not s or s.endswith(":") or s.startswith("."):
            continue
        op, _, rest = s.partition(" ")
        if op == "s_waitcnt" and "lgkmcnt(0)" in rest:
            pending.clear()
            continue
        if op.startswith("ds_read") and in_asm:
            dst, _, src = rest.partition(",")
            for r in regs(dst):
                pending[r] = i
            continue
        if op.startswith("s_"):
            continue
        # sources: everything after the first operand for VALU / stores; all operands for
        # stores and ds_write (they have no destination VGPR)
        if op.startswith(("ds_write", "buffer_store", "global_store", "flat_store")):
            used = regs(rest)
        else:
            _, _, srcs = rest.partition(",")
            used = regs(srcs)
        bad = used & pending.keys()
        if bad:
            hazards.append((i, s, sorted(bad)))
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
    print(f"{n} kernels checked, {bad} hazards")
    return 1 if bad or n == 0 else 0


if __name__ == "__main__":
    sys.exit(main())
