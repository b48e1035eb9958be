"""Audit a kernel's ISA for in-flight asm loads: every instruction that reads or writes a VGPR whose
global / buffer load is still outstanding (not yet retired by an ``s_waitcnt vmcnt(N)``) is
reported.  Loads hipcc emits itself are included (the compiler never touches them early); the
point is the inline-asm loads of the strip engine, whose destinations hipcc believes written at
issue (cdna_hip_programming.md §5.7 item 1).

    hipcc ... -save-temps ; python tools/asm_vmcnt_audit.py <file.s> <kernel symbol> [--copies]

``--copies`` reports only instructions other than MFMA reads -- the compiler's own moves, spills
and reuses of in-flight registers.  MFMA reads of ring registers are ordered after the waits by
the source's "+v" statements; what the CFG walk cannot tell apart is a wait whose count depends
on a counter carried between loop iterations (it walks every arm), so those paths show up as
MFMA reads.

vmcnt model: one in-order queue of vector-memory ops (loads, LDS-DMA loads, stores, atomics);
``s_waitcnt vmcnt(N)`` retires all but the N youngest.  The function is cut into basic blocks
(labels, branches, fall-through) and the possible queue states are propagated over the control-flow
graph to a fixed point, so a wait that sits in one arm of a branch only covers the paths through
that arm (a straight-line scan mixes arms that hipcc lays out far apart).  Exit status 1 when a
hazard is found.
"""
import re
import sys

VMEM = re.compile(r"^(global_load|global_store|global_atomic|buffer_load|buffer_store|buffer_atomic|"
                  r"flat_load|flat_store|global_load_lds)")
QMAX = 64                 # vmcnt counts to 63: anything older than that has retired by any wait
STATES_MAX = 256          # per block entry; beyond it the audit says so (never silently)


def regs(tok):
    m = re.fullmatch(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return frozenset(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.fullmatch(r"v(\d+)", tok)
    return frozenset({int(m.group(1))}) if m else frozenset()


def operands(line):
    code = line.split(";")[0].strip()
    parts = code.split(None, 1)
    if len(parts) < 2:
        return parts[0] if parts else "", []
    return parts[0], [t.strip() for t in parts[1].split(",")]


def blocks_of(body):
    """[(start, end, successors, last opcode)] with successors as block indices (taken target
    first for a conditional branch)."""
    starts = {0}
    label_at = {}
    for i, l in enumerate(body):
        m = re.match(r"^(\.LBB\S+):", l)
        if m:
            starts.add(i)
            label_at[m.group(1)] = i
        op, _ = operands(l)
        if op.startswith("s_cbranch") or op == "s_branch" or op == "s_endpgm":
            starts.add(i + 1)
    starts = sorted(s for s in starts if s < len(body))
    idx = {s: k for k, s in enumerate(starts)}
    out = []
    for k, s in enumerate(starts):
        e = starts[k + 1] if k + 1 < len(starts) else len(body)
        succ = []
        last_op, last_ops = "", []
        for i in range(s, e):
            op, ops = operands(body[i])
            if op and not op.startswith(".") and not op.endswith(":"):
                last_op, last_ops = op, ops
        if last_op == "s_endpgm":
            pass
        elif last_op == "s_branch":
            if last_ops and last_ops[0] in label_at:
                succ.append(idx[label_at[last_ops[0]]])
        else:
            if last_op.startswith("s_cbranch") and last_ops and last_ops[0] in label_at:
                succ.append(idx[label_at[last_ops[0]]])
            if k + 1 < len(starts):
                succ.append(k + 1)
        out.append((s, e, succ, last_op))
    return out


def sdst(tok):
    """Scalar destination key of an operand ("vcc", "s[0:1]", "s5") or None."""
    return tok if re.fullmatch(r"vcc|exec|s\[\d+:\d+\]|s\d+", tok or "") else None


def step(body, s, e, st, report):
    """Run block [s, e) from state (queue, known scalar values); returns (state, taken, fallthrough)
    where taken / fallthrough say whether the block's final conditional branch can go that way."""
    q, known = list(st[0]), dict(st[1])
    taken = fall = True
    for i in range(s, e):
        op, ops = operands(body[i])
        if not op or op.startswith(".") or op.endswith(":"):
            continue
        # the structurizer's flow blocks select arms through s_mov_b64 s[x:y], -1 / 0 and
        # s_andn2_b64 vcc, exec, s[x:y]; s_cbranch_vccnz: follow those constants (exec != 0)
        if op == "s_mov_b64" and len(ops) == 2 and ops[1] in ("-1", "0"):
            known[ops[0]] = int(ops[1])
            continue
        if op == "s_andn2_b64" and len(ops) == 3 and ops[0] == "vcc" and ops[1] == "exec" and ops[2] in known:
            known["vcc"] = 0 if known[ops[2]] == -1 else 1
            continue
        if op in ("s_cbranch_vccnz", "s_cbranch_vccz") and "vcc" in known:
            nz = known["vcc"] != 0
            taken = nz if op == "s_cbranch_vccnz" else not nz
            fall = not taken
            continue
        if ops and sdst(ops[0]) and not op.startswith(("s_cbranch", "s_branch", "s_waitcnt", "s_cmp")):
            known.pop(ops[0], None)
            if op.startswith("v_cmp") or op.startswith("s_and") or "vcc" in ops:
                known.pop("vcc", None)
        elif op.startswith("v_cmp"):
            known.pop("vcc", None)
        if op == "s_waitcnt":
            m = re.search(r"vmcnt\((\d+)\)", body[i])
            if m:
                keep = int(m.group(1))
                del q[: max(0, len(q) - keep)]
            continue
        touched = frozenset()
        for t in ops:
            touched |= regs(t)
        hit = touched & frozenset(r for d in q for r in d)
        if hit and report is not None:
            report[i] = (body[i].strip()[:110], sorted(hit)[:4])
        if VMEM.match(op):
            dst = regs(ops[0]) if op.startswith(("global_load", "buffer_load", "flat_load")) else frozenset()
            if op.startswith("global_load_lds") or " lds" in body[i]:
                dst = frozenset()
            q.append(dst)
            del q[: max(0, len(q) - QMAX)]
    return (tuple(q), frozenset(known.items())), taken, fall


def main(path, sym, copies=False):
    lines = open(path).read().split("\n")
    s = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
    e = next(i for i in range(s, len(lines)) if lines[i].startswith(".Lfunc_end"))
    body = lines[s:e]
    blocks = blocks_of(body)
    seen = [set() for _ in blocks]
    work = [(0, ((), frozenset()))]
    report = {}
    overflow = False
    while work:
        b, q = work.pop()
        if q in seen[b]:
            continue
        if len(seen[b]) >= STATES_MAX:
            overflow = True
            continue
        seen[b].add(q)
        bs, be, succ, last = blocks[b]
        out, taken, fall = step(body, bs, be, q, report)
        for n in succ:
            if last.startswith("s_cbranch") and len(succ) == 2:
                if n == succ[0] and not taken:
                    continue
                if n == succ[1] and not fall:
                    continue
            if out not in seen[n]:
                work.append((n, out))
    if copies:
        report = {i: v for i, v in report.items() if not v[0].startswith("v_mfma")}
    for i in sorted(report)[:40]:
        txt, rr = report[i]
        print(f"{i}: {txt}   in-flight v{rr}")
    if overflow:
        print(f"{sym}: WARNING more than {STATES_MAX} queue states at a block entry; audit incomplete")
    print(f"{sym}: {len(report)} instructions touch in-flight load destinations")
    return 1 if report or overflow else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1], sys.argv[2], "--copies" in sys.argv[3:]))
