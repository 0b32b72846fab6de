"""Instruction mix of every loop in one kernel of a hipcc --save-temps gfx950 .s file.

A loop is a label and the last backward branch to it; the counts are of the static
instructions between them (each executes once per iteration unless branched around).

    python tools/asm_mix.py conv_x6-hip-amdgcn-amd-amdhsa-gfx950.s <mangled symbol> [--min 40]
"""
import argparse
import collections
import re


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith("ds_"):
        return "lds"
    if op == "s_barrier":
        return "barrier"
    if op == "s_waitcnt" or op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("symbol")
    ap.add_argument("--min", type=int, default=40)
    a = ap.parse_args()
    lines = open(a.asm).read().splitlines()
    i0 = next(i for i, l in enumerate(lines) if l.startswith(a.symbol + ":"))
    i1 = next(i for i in range(i0 + 1, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
    labels = {}
    for i in range(i0, i1):
        m = re.match(r"^(\.LBB\w+):", lines[i])
        if m:
            labels[m.group(1)] = i
    loops = {}
    for i in range(i0, i1):
        m = re.match(r"^\s+(s_branch|s_cbranch_\w+)\s+(\.LBB\w+)", lines[i])
        if m and m.group(2) in labels and labels[m.group(2)] < i:
            loops[m.group(2)] = i
    total = collections.Counter()
    for i in range(i0, i1):
        s = lines[i].strip()
        if s and not s.startswith((".", ";")) and not s.endswith(":"):
            total[classify(s.split()[0])] += 1
    print(f"{a.symbol}: whole kernel {dict(total)}")
    for lab, end in sorted(loops.items(), key=lambda kv: labels[kv[0]]):
        beg = labels[lab]
        c = collections.Counter()
        for i in range(beg, end + 1):
            s = lines[i].strip()
            if s and not s.startswith((".", ";")) and not s.endswith(":"):
                c[classify(s.split()[0])] += 1
        if sum(c.values()) >= a.min:
            print(f"  loop {lab} lines {beg + 1}-{end + 1}: {sum(c.values())} instr {dict(c)}")


if __name__ == "__main__":
    main()
