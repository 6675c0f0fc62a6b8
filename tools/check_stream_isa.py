#!/usr/bin/env python3
"""Build-time check of the dense phase-B stream's hand-scheduled loads.

The stream's loads are issued as inline asm (gpk_kernels.hip slot_load), so
the compiler's wait-count pass does not see them, and the kernel waits for
them itself (slot_wait). That is correct only if the compiled code leaves a
slot's registers alone while its load is in flight: a register copy, spill
or reuse of an in-flight register reads or clobbers stale data. The register
allocator is free to insert such copies (it believes the asm produced the
value at once), so every build is checked here instead of trusted.

Input: the device assembly of gpk_kernels.hip (hipcc -S --cuda-device-only,
same flags as the library). For every kernel, the instructions are walked
along the control-flow graph (basic blocks, branches, loops; iterated to a
fixed point) with the set of in-flight stream registers: an asm
buffer_load_dwordx4 ... nt puts its destination in flight; every later
vector-memory instruction ages it by one; s_waitcnt vmcnt(k) retires the
loads with at least k younger vector-memory operations behind them. Any
instruction that names an in-flight register on some path is a violation.

    python tools/check_stream_isa.py kernels.s      exit 1 on a violation
"""
import re
import sys

REG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")
VMEM = ("buffer_", "global_", "scratch_", "flat_")


def regs(operands):
    out = set()
    for m in REG.finditer(operands):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def parse_blocks(lines):
    """Basic blocks of one function: [(instrs, successors)], instrs as
    (line number, mnemonic, operands, inside inline asm)."""
    blocks, labels, cur, in_asm = [], {}, [], False
    ends = []  # per block: the label of the block it starts at (None = unlabeled)

    def close():
        nonlocal cur
        if cur or (ends and ends[-1] is not None and len(blocks) < len(ends)):
            blocks.append(cur)
        cur = []

    for ln, raw in lines:
        line = raw.strip()
        if line.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if line.startswith(";;#ASMEND"):
            in_asm = False
            continue
        m = re.match(r"^(\.?[\w$.]+):", line)
        if m and not line.startswith(";"):
            if cur:
                blocks.append(cur)
                cur = []
            labels[m.group(1)] = len(blocks)
            continue
        code = line.split(";")[0].strip()
        if not code or code.startswith("."):
            continue
        mnem, _, ops = code.partition(" ")
        cur.append((ln, mnem, ops, in_asm))
        if mnem == "s_branch" or mnem.startswith("s_cbranch") or mnem in ("s_endpgm", "s_setpc_b64"):
            blocks.append(cur)
            cur = []
    if cur:
        blocks.append(cur)
    out = []
    for i, ins in enumerate(blocks):
        last = ins[-1][1] if ins else ""
        tgt = ins[-1][2].strip() if ins else ""
        if last == "s_branch":
            succ = [labels[tgt]] if tgt in labels else []
        elif last.startswith("s_cbranch"):
            succ = ([labels[tgt]] if tgt in labels else []) + ([i + 1] if i + 1 < len(blocks) else [])
        elif last in ("s_endpgm", "s_setpc_b64"):
            succ = []
        else:
            succ = [i + 1] if i + 1 < len(blocks) else []
        out.append((ins, succ))
    return out


def transfer(name, ins, state, bad):
    """Walk one block from the in-flight state {load line: (registers, younger
    vector-memory operations)}; record violations; return the out state."""
    st = dict(state)
    nloads = 0
    for ln, mnem, ops, in_asm in ins:
        code = (mnem + " " + ops).strip()
        if mnem == "s_waitcnt":
            m = re.search(r"vmcnt\((\d+)\)", ops)
            k = int(m.group(1)) if m else (0 if ops.strip() == "0" else None)
            if k is not None:
                st = {o: v for o, v in st.items() if v[1] < k}
            continue
        used = regs(ops)
        for o, (r, _) in st.items():
            if used & r:
                bad.add("%s: line %d: '%s' touches v%s, in flight since line %d" % (name, ln, code, sorted(used & r), o))
        if mnem.startswith(VMEM):
            st = {o: (r, min(c + 1, 64)) for o, (r, c) in st.items()}
            if in_asm and mnem == "buffer_load_dwordx4" and re.search(r"\bnt\b", ops):
                st[ln] = (frozenset(regs(ops.split(",")[0])), 0)
                nloads += 1
    return st, nloads


def check_function(name, lines):
    """Follows the control flow (branches, loops) to a fixed point: the state
    entering a block is the union of its predecessors' (a load counts as
    still in flight with the fewest younger operations any path gives it)."""
    blocks = parse_blocks(lines)
    if not blocks:
        return [], 0
    ins_state = [None] * len(blocks)
    ins_state[0] = {}
    work = [0]
    bad = set()
    nloads = sum(1 for ins, _ in blocks for x in ins if x[3] and x[1] == "buffer_load_dwordx4" and re.search(r"\bnt\b", x[2]))
    while work:
        b = work.pop()
        out, _ = transfer(name, blocks[b][0], ins_state[b], bad)
        for s in blocks[b][1]:
            cur = ins_state[s]
            if cur is None:
                ins_state[s] = dict(out)
                work.append(s)
                continue
            changed = False
            for o, (r, c) in out.items():
                if o not in cur or c < cur[o][1]:
                    cur[o] = (r, c)
                    changed = True
            if changed:
                work.append(s)
    return sorted(bad), nloads


def main(path):
    text = open(path).read().split("\n")
    funcs, cur, start = {}, None, 0
    for i, l in enumerate(text):
        m = re.match(r"^(_Z\w*decode_(?:sb_)?kernel\w*):", l)
        if m:
            cur, start = m.group(1), i
        elif cur and l.startswith(".Lfunc_end"):
            funcs[cur] = [(k + 1, text[k]) for k in range(start, i)]
            cur = None
    if not funcs:
        print("check_stream_isa: no decode_kernel in %s" % path)
        return 1
    errors = 0
    for name, lines in funcs.items():
        bad, n = check_function(name, lines)
        for b in bad[:10]:
            print(b)
        errors += len(bad)
    print("check_stream_isa: %d kernels, %d violations" % (len(funcs), errors))
    return 1 if errors else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
