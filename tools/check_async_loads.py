"""Static check of explicit async loads in the k_ingest ISA.

For every inline-asm global_load (between ;;#ASMSTART/;;#ASMEND), follow all
control-flow paths until an `s_waitcnt` with vmcnt(0); report any instruction
that reads or writes the load's destination VGPRs before that point.
Usage: python tools/check_async_loads.py <file.s> <kernel-symbol-prefix>
"""
import re
import sys


def regs_of(tok):
    m = re.fullmatch(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.fullmatch(r"v(\d+)", tok)
    if m:
        return {int(m.group(1))}
    return set()


def main(path, prefix):
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(prefix) and l.rstrip().endswith(":") or
                 (l.startswith(prefix) and ":" in l and "@" in l))
    body = []
    for l in lines[start + 1:]:
        body.append(l)
        if "s_endpgm" in l:
            break
    # blocks
    labels = {}
    insts = []  # (text, is_asm)
    in_asm = False
    for l in body:
        s = l.strip()
        if s.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if s.startswith(";;#ASMEND"):
            in_asm = False
            continue
        m = re.match(r"^(\.LBB\w+):", s)
        if m:
            labels[m.group(1)] = len(insts)
            continue
        if not s or s.startswith(";"):
            continue
        insts.append((s.split(";")[0].strip(), in_asm))
    succ = {}
    for i, (t, _) in enumerate(insts):
        op = t.split()[0]
        tgt = re.search(r"(\.LBB\w+)", t)
        if op == "s_branch":
            succ[i] = [labels[tgt.group(1)]]
        elif op.startswith("s_cbranch"):
            succ[i] = [labels[tgt.group(1)], i + 1]
        elif op == "s_endpgm" or op == "s_setpc_b64":
            succ[i] = []
        else:
            succ[i] = [i + 1]
    bad = 0
    nloads = 0
    for i, (t, is_asm) in enumerate(insts):
        if not (is_asm and t.startswith("global_load")):
            continue
        nloads += 1
        dst = regs_of(t.split()[1].rstrip(","))
        seen = set()
        stack = list(succ[i])
        while stack:
            j = stack.pop()
            if j in seen or j >= len(insts):
                continue
            seen.add(j)
            tj, _ = insts[j]
            if tj.startswith("s_waitcnt") and "vmcnt(0)" in tj:
                continue
            toks = re.findall(r"v\[\d+:\d+\]|v\d+", tj)
            used = set()
            for tk in toks:
                used |= regs_of(tk)
            if used & dst:
                print("VIOLATION load@%d %r -> %d %r" % (i, t, j, tj))
                bad += 1
                continue
            stack.extend(succ.get(j, []))
    print("%s: %d asm loads, %d violations" % (prefix, nloads, bad))
    return bad


if __name__ == "__main__":
    sys.exit(1 if main(sys.argv[1], sys.argv[2]) else 0)
