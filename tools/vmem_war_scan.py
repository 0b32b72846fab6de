"""Scan gfx950 assembly for a VALU instruction that overwrites a VGPR read by a
vector-memory instruction issued just before it (write-after-read on the VMEM's address
or store-data operands), per kernel.  (diagnostic / test helper)

Packed-FP32 VALU (v_pk_add/mul/fma_f32) doing this was caught corrupting the last 16
lanes of such loads under concurrent GPU load: kernels must not contain
a packed-FP32 write to a VGPR that a VMEM instruction among the preceding `--window`
instructions reads.

    python tools/vmem_war_scan.py file.s [--window 6] [--all]
"""
import argparse
import re
import sys

VREG = re.compile(r"v\[(\d+):(\d+)\]|v(\d+)\b")


def regs(spec):
    out = set()
    for m in VREG.finditer(spec):
        if m.group(1):
            out |= set(range(int(m.group(1)), int(m.group(2)) + 1))
        else:
            out.add(int(m.group(3)))
    return out


def vmem_reads(ins):
    """VGPRs a global/buffer/flat memory instruction reads (address, store data)."""
    op, _, rest = ins.partition(" ")
    ops = [o.strip() for o in rest.split(",")]
    if op.startswith(("global_load", "flat_load", "buffer_load")):
        return regs(ops[1]) if len(ops) > 1 else set()
    if op.startswith(("global_store", "flat_store", "buffer_store", "global_atomic")):
        return regs(ops[0]) | (regs(ops[1]) if len(ops) > 1 else set())
    return None


def scan(path, window=6, packed_only=True):
    hits = []
    kern = None
    recent = []
    for raw in open(path):
        line = raw.split(";")[0].strip()
        if not line or line.startswith("."):
            continue
        if line.endswith(":") and not line.startswith("."):
            if not line.startswith(".L") and not line.startswith("$"):
                kern = line[:-1]
                recent = []
            continue
        r = vmem_reads(line)
        if r is not None:
            recent.append((line, r))
            recent = recent[-window:]
            continue
        if line.startswith("v_"):
            op, _, rest = line.partition(" ")
            dst = regs(rest.split(",")[0])
            if (not packed_only or re.match(r"v_pk_\w+_f32", op)) and dst:
                for vm, rr in recent:
                    if dst & rr:
                        hits.append((kern, vm, line))
        if line.startswith(("s_waitcnt", "s_endpgm")) and "vmcnt(0)" in line:
            recent = []
        recent = recent[-window:]
    return hits


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("--window", type=int, default=6)
    ap.add_argument("--all", action="store_true", help="any VALU, not only packed FP32")
    a = ap.parse_args()
    hits = scan(a.asm, a.window, not a.all)
    for k, vm, v in hits:
        print(f"{k}: {vm}  <-  {v}")
    print(f"{len(hits)} hits")
    sys.exit(1 if hits else 0)


if __name__ == "__main__":
    main()
