#!/usr/bin/env python
"""Audit the built library's gfx950 ISA for the mixed-shape MFMA chain hazard
(dstd-gcn_amd/csrc/dstd_hilo.h, "a gfx950 MFMA hazard hipcc does not pad";
reproducer scripts/micro/mfma_read_hazard.hip): an MFMA whose C operand is
exactly the previous MFMA's destination, with a DIFFERENT MFMA opcode, fewer
than 5 wait states after it.  hipcc (ROCm 7.2) pads nothing there, and
gfx950 then accumulates onto a stale C.

  python scripts/mfma_hazard_audit.py [lib.so]   -> exit 1 and a listing if any

How: the gfx950 code object is taken out of the library's clang offload
bundle (.hip_fatbin), disassembled with llvm-objdump, and every function is
walked in layout order (a linear approximation of control flow: a dependency
across a taken branch back into a loop is not followed).  Wait states between
two instructions: 1 per instruction, N + 1 per s_nop N.
"""
import os
import re
import subprocess
import sys
import tempfile

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
NEED = 5  # wait states that made every mixed pair exact (mfma_read_hazard.hip)
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def code_objects(lib_path, arch="gfx950"):
    """Every gfx950 code object of the library (one offload bundle per
    translation unit in .hip_fatbin)."""
    data = open(lib_path, "rb").read()
    out, i = [], data.find(MAGIC)
    while i >= 0:
        n = int.from_bytes(data[i + 24:i + 32], "little")
        p = i + 32
        for _ in range(n):
            off, size, tlen = (int.from_bytes(data[p + 8 * k:p + 8 * k + 8], "little") for k in range(3))
            triple = data[p + 24:p + 24 + tlen].decode(errors="replace")
            p += 24 + tlen
            if "amdgcn" in triple and arch in triple:
                out.append(data[i + off:i + off + size])
        i = data.find(MAGIC, i + 24)
    if not out:
        raise RuntimeError(f"{lib_path}: no {arch} code object in an offload bundle")
    return out


REG = re.compile(r"^(?:v|a)\[(\d+):(\d+)\]$|^(?:v|a)(\d+)$")


def reg_range(tok):
    m = REG.match(tok.strip())
    if not m:
        return None
    if m.group(1) is not None:
        return int(m.group(1)), int(m.group(2))
    r = int(m.group(3))
    return r, r


def audit(lib_path):
    txt = ""
    for co in code_objects(lib_path):
        with tempfile.NamedTemporaryFile(suffix=".co", delete=False) as f:
            f.write(co)
            path = f.name
        try:
            txt += subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", "--no-show-raw-insn", path], check=True,
                                  capture_output=True, text=True).stdout
        finally:
            os.unlink(path)
    findings, n_mfma, n_funcs = [], 0, 0
    func = None
    insns = []  # (mnemonic, operands) of the current function

    def flush():
        nonlocal n_mfma
        last = {}  # (lo, hi) destination range -> (index, opcode)
        pos = 0  # running wait-state position
        at = []
        for k, (mn, ops) in enumerate(insns):
            at.append(pos)
            pos += int(ops[0]) + 1 if mn == "s_nop" and ops else 1
        for k, (mn, ops) in enumerate(insns):
            if not mn.startswith("v_mfma"):
                continue
            n_mfma += 1
            if len(ops) >= 4:
                dst, srcc = reg_range(ops[0]), reg_range(ops[3])
                if srcc is not None and srcc in last:
                    j, opc = last[srcc]
                    gap = at[k] - at[j] - 1
                    if opc != mn and gap < NEED:
                        findings.append((func, j, k, opc, mn, ops[3], gap))
                if dst is not None:
                    for key in [r for r in last if not (r[1] < dst[0] or r[0] > dst[1])]:
                        del last[key]
                    last[dst] = (k, mn)

    for line in txt.splitlines():
        m = re.match(r"^[0-9a-f]+ <([^>]+)>:$", line)
        if m:
            if func is not None:
                flush()
            func, insns = m.group(1), []
            n_funcs += 1
            continue
        s = line.split("//")[0].strip()
        if not s or func is None or s.endswith(":"):
            continue
        parts = s.split(None, 1)
        ops = [o.strip() for o in parts[1].split(",")] if len(parts) > 1 else []
        insns.append((parts[0], ops))
    if func is not None:
        flush()
    return findings, n_mfma, n_funcs


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))), "dstd-gcn_amd", "libdstd_gcn.so")
    findings, n_mfma, n_funcs = audit(lib)
    print(f"{os.path.basename(lib)}: {n_funcs} functions, {n_mfma} MFMAs, "
          f"{len(findings)} mixed-shape C-chain pairs closer than {NEED} wait states")
    for f in findings[:40]:
        print("  %s: insn %d %s -> insn %d %s (C = %s), %d wait states" % (f[0][:80], f[1], f[3], f[2], f[4], f[5], f[6]))
    return 1 if findings else 0


if __name__ == "__main__":
    sys.exit(main())
