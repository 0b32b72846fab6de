"""Audit of the untracked-load discipline in a kernel's assembly (-save-temps .s).

The loader waves issue global_load_dwordx4 from inline asm (gld16): hipcc counts the
destination as written at the asm statement, so it could copy, reuse or spill that
register before the data lands (cdna_hip_programming.md, 'What hipcc does not do' 1).
This builds the kernel's control-flow graph, tracks the outstanding vector-memory
operations in issue order (loads, LDS-DMA, stores) along every path, retires them at
each `s_waitcnt vmcnt(N)`, and reports any instruction that reads or writes a register
of a load that may still be in flight (at a join, the longer in-flight list wins).

    python tools/asm_audit.py file.s KERNEL_SYMBOL
"""
import argparse
import re
import sys

# (scratch_* count in vmcnt too: a spill reload inside a loader pipeline would shift every
# counted wait after it)
VMEM = re.compile(r"^(global_load\w*|global_store\w*|buffer_\w+|global_atomic\w*|flat_\w+|scratch_\w+)\b")
WAIT = re.compile(r"s_waitcnt\s+vmcnt\((\d+)\)")
REG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")
LABEL = re.compile(r"^(\.?[\w.$]+):")


def regs(text):
    out = set()
    for m in REG.finditer(text):
        if m.group(1) is not None:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
        else:
            out.add(int(m.group(3)))
    return frozenset(out)


def parse(lines, i0, i1):
    blocks, cur, order = {}, None, []
    for i in range(i0, i1 + 1):
        raw = lines[i].split(";")[0].rstrip()
        s = raw.strip()
        m = LABEL.match(s)
        if m and not s.startswith(".p2align"):
            cur = m.group(1)
            blocks[cur] = []
            order.append(cur)
            continue
        if cur is None:
            cur = "__entry"
            blocks[cur] = []
            order.append(cur)
        if s and not s.startswith("."):
            blocks[cur].append((i, s))
    succ = {}
    for n, b in enumerate(order):
        ins = blocks[b]
        nxt = order[n + 1] if n + 1 < len(order) else None
        last = ins[-1][1] if ins else ""
        if last.startswith("s_branch"):
            succ[b] = [last.split()[1]]
        elif last.startswith("s_cbranch"):
            succ[b] = [last.split()[1]] + ([nxt] if nxt else [])
        elif last.startswith("s_endpgm"):
            succ[b] = []
        else:
            succ[b] = [nxt] if nxt else []
    return order, blocks, succ


def step(state, s, line, report):
    w = WAIT.search(s)
    if w:
        keep = int(w.group(1))
        return state[len(state) - keep:] if keep else ()
    ops = s.split(None, 1)
    operands = ops[1] if len(ops) > 1 else ""
    m = VMEM.match(s)
    if m:
        parts = [p.strip() for p in operands.split(",")]
        if (m.group(1).startswith("global_load") or m.group(1).startswith("scratch_load")) \
                and "lds" not in m.group(1):
            dst, srcs = regs(parts[0]), regs(",".join(parts[1:]))
        else:
            dst, srcs = frozenset(), regs(operands)
        for d, ln in state:
            if d & srcs:
                report(line, ln, d & srcs, s)
        return (state + ((dst, line),))[-64:]  # vmcnt counts at most 63 in flight
    used = regs(operands)
    for d, ln in state:
        if d & used:
            report(line, ln, d & used, s)
    return state


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("symbol")
    a = ap.parse_args()
    lines = open(a.asm).read().splitlines()
    i0 = next(i for i, l in enumerate(lines) if l.startswith(a.symbol + ":"))
    i1 = next(i for i in range(i0 + 1, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
    order, blocks, succ = parse(lines, i0 + 1, i1 - 1)
    found = {}

    def report(line, ln, r, s):
        found.setdefault(line, (ln, sorted(r), s))

    entry = {order[0]: ()}
    work = [order[0]]
    seen = 0
    while work and seen < 20000:
        seen += 1
        b = work.pop()
        st = entry[b]
        for line, s in blocks[b]:
            st = step(st, s, line, report)
        for t in succ.get(b, []):
            if t not in blocks:
                continue
            old = entry.get(t)
            new = st if old is None or len(st) > len(old) else old
            if old is None or new != old:
                entry[t] = new
                work.append(t)
    for line, (ln, r, s) in sorted(found.items()):
        print(f"line {line + 1}: in-flight v{r} (load at line {ln + 1}): {s}")
    print(f"{a.symbol}: {len(found)} problem(s)")
    sys.exit(1 if found else 0)


if __name__ == "__main__":
    main()
