"""Instruction mix of each loop (backward branch) of one kernel in a built
library: python scripts/isa_loops.py lib.so <mangled-name substring>"""
import collections
import re
import subprocess
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from mfma_hazard_audit import OBJDUMP, code_objects  # noqa: E402


def kernel_lines(lib, key):
    for co in code_objects(lib):
        open("/tmp/_isa.co", "wb").write(co)
        txt = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", "--no-show-raw-insn", "/tmp/_isa.co"],
                             capture_output=True, text=True).stdout
        for f in re.split(r"\n(?=[0-9a-f]+ <)", txt):
            head = f.split("\n")[0]
            if key in head and "ZZN" not in head:
                out = []
                for l in f.split("\n")[1:]:
                    m = re.match(r"\s*(\S.*?)\s*//\s*([0-9A-Fa-f]+):", l)
                    if m:
                        out.append((int(m.group(2), 16), m.group(1)))
                return head, out
    raise SystemExit("kernel not found")


def cls(ins):
    op = ins.split()[0]
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("buffer_", "global_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    head, lines = kernel_lines(sys.argv[1], sys.argv[2])
    print(head[:160], len(lines), "instructions")
    addr = [a for a, _ in lines]
    for i, (a, ins) in enumerate(lines):
        m = re.match(r"s_c?branch\S*\s+(\d+)", ins)
        if not m:
            continue
        off = int(m.group(1))
        if off >= 32768:
            off -= 65536
        tgt = a + 4 + 4 * off
        if tgt < a:  # backward: loop body [tgt, a]
            body = [ins2 for a2, ins2 in lines if tgt <= a2 <= a]
            c = collections.Counter(cls(x) for x in body)
            valu = collections.Counter(x.split()[0] for x in body if cls(x) == "valu")
            print(f"loop {tgt:#x}-{a:#x}: {len(body)} insts", dict(c))
            print("   top VALU:", valu.most_common(14))
    c = collections.Counter(cls(x) for _, x in lines)
    print("whole kernel:", dict(c))


if __name__ == "__main__":
    main()
