"""Scan the built gfx950 code objects for packed-FP32 instructions whose high half reads the
destination's low register.

A v_pk_{fma,mul,add}_f32 / v_pk_mov_b32 writes a 64-bit register pair v[a:a+1]; its high half
reads register b + op_sel_hi of each source pair v[b:b+1].  When that register is a (the
destination's low half), the instruction's result depended on timing on MI355X: the fast g = 0
replay built this way (a broadcast constant whose register the compiler reused as the
destination, v_pk_fma_f32 v[48:49], v[54:55], v[48:49], v[48:49] op_sel_hi:[1,0,1]) gave
run-to-run different table rows when it ran beside the feature MLP's GEMMs, and bit-identical
ones with the operands laid out as pairs (profiles/r04_replay_pk_overlap.txt).  The library's
build refuses such instructions: csrc/Makefile compiles the files whose auto-vectorised code
produced them with -fno-slp-vectorize, and hand-written packed code reads pair operands.

Usage: python tools/check_pk_operands.py BUILD_DIR   (exit status 1 and a list when found)
"""

from __future__ import annotations

import re
import subprocess
import sys
import tempfile
from pathlib import Path

LLVM = Path("/opt/rocm/lib/llvm/bin")
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
PK = re.compile(r"^\s*(v_pk_(?:fma|mul|add)_f32|v_pk_mov_b32)\s+v\[(\d+):\d+\],\s*(.*?)(?://.*)?$")
FUNC = re.compile(r"^[0-9a-f]+ <(\S+)>:")


def hazards_in_listing(lines) -> list[tuple[str, str]]:
    """(function, instruction) pairs whose high half reads the destination's low register."""
    out = []
    func = "?"
    for line in lines:
        m = FUNC.match(line)
        if m:
            func = m.group(1)
            continue
        m = PK.match(line)
        if not m:
            continue
        op, dst, rest = m.group(1), int(m.group(2)), m.group(3)
        nsrc = 3 if "fma" in op else (1 if "mov" in op else 2)
        srcs = [s.strip() for s in re.split(r",\s*", re.split(r"\s(?:op_sel|neg_)", rest)[0])][:nsrc]
        hi = [1, 1, 1]
        mm = re.search(r"op_sel_hi:\[([\d,]+)\]", rest)
        if mm:
            hi = [int(x) for x in mm.group(1).split(",")] + [1, 1, 1]
        for j, s in enumerate(srcs):
            ms = re.match(r"v\[(\d+):\d+\]", s)
            if ms and int(ms.group(1)) + hi[j] == dst:
                out.append((func, line.strip().split("//")[0].strip()))
    return out


# library objects that hold kernels: finding no gfx950 code in one of them means the section or
# bundle naming changed under a toolchain update and the scan would check nothing -> fail
KERNEL_OBJECTS = {"rows.o", "optim.o", "cal.o", "gemm.o", "gate.o", "gate16.o", "inbatch.o", "retrieval.o",
                  "sampler.o", "data.o", "route.o"}


def scan_object(obj: Path) -> tuple[list[tuple[str, str]], int]:
    """(hazards, number of device functions disassembled); (.., 0) when the object has no gfx950 code."""
    with tempfile.TemporaryDirectory() as td:
        fat = Path(td) / "fatbin"
        co = Path(td) / "co"
        r = subprocess.run(["objcopy", f"--dump-section", f".hip_fatbin={fat}", str(obj)], capture_output=True)
        if r.returncode != 0 or not fat.exists():
            return [], 0  # no device code
        subprocess.run([str(LLVM / "clang-offload-bundler"), "--type=o", f"--targets={TARGET}", f"--input={fat}",
                        f"--output={co}", "--unbundle"], check=True, capture_output=True)
        dis = subprocess.run([str(LLVM / "llvm-objdump"), "-d", str(co)], check=True, capture_output=True, text=True)
        lines = dis.stdout.splitlines()
        return hazards_in_listing(lines), sum(1 for ln in lines if FUNC.match(ln))


def main(argv: list[str]) -> int:
    build = Path(argv[1]) if len(argv) > 1 else Path(__file__).resolve().parents[1] / \
        "two-tower-augmented-with-adaptive-mimic-mechanism_amd" / "build"
    bad = 0
    for obj in sorted(build.glob("*.o")):
        hazards, nfunc = scan_object(obj)
        if nfunc == 0 and obj.name in KERNEL_OBJECTS:
            print(f"{obj.name}: no gfx950 device code found (.hip_fatbin / {TARGET}): the scan would check nothing")
            bad += 1
        for func, ins in hazards:
            print(f"{obj.name}: {func}: {ins}")
            bad += 1
    if bad:
        print(f"{bad} problem(s): packed-FP32 instructions reading their own destination's low register across "
              "halves, or kernel objects without scannable device code")
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
