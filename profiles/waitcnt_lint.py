#!/usr/bin/env python3
"""Conservative s_waitcnt checker for one kernel's gfx950 assembly (profiles/isa.sh
writes /tmp/kernel.s).  Basic blocks from labels and branches; per block entry the
set of memory results that may still be in flight, each with the minimum number of
same-counter operations issued after it (its "age"), merged over predecessors
(minimum age) to a fixpoint.  An s_waitcnt vmcnt(N) retires VMEM results of age >= N,
lgkmcnt(N) LDS results of age >= N (SMEM only at lgkmcnt(0), it returns out of order).
Reports every instruction that reads or writes a register whose load may be in flight.
Usage: waitcnt_lint.py [/tmp/kernel.s]"""
import re
import sys


def regs(tok):
    out = set()
    for m in re.finditer(r"\b([vsa])(\d+)\b|\b([vsa])\[(\d+):(\d+)\]", tok):
        if m.group(1):
            out.add((m.group(1), int(m.group(2))))
        else:
            for i in range(int(m.group(4)), int(m.group(5)) + 1):
                out.add((m.group(3), i))
    return out


def parse(path):
    blocks, cur, label = [], [], None
    order = []
    for n, raw in enumerate(open(path).read().split("\n"), 1):
        s = raw.split(";")[0].strip()
        if not s:
            continue
        if s.endswith(":"):
            if cur or label is not None:
                blocks.append((label, cur))
            label, cur = s[:-1], []
            continue
        if s.startswith("."):
            continue
        cur.append((n, s))
        op = s.split()[0]
        if op.startswith("s_cbranch") or op in ("s_branch", "s_endpgm", "s_setpc_b64"):
            blocks.append((label, cur))
            label, cur = None, []
    if cur:
        blocks.append((label, cur))
    return blocks


def classify(op, args):
    store = op.startswith(("global_store", "buffer_store", "scratch_store", "ds_write")) or (
        (op.startswith(("global_atomic", "buffer_atomic")) and " sc0" not in " " + args))
    if op.startswith("ds_") and not op.startswith("ds_read") and "rtn" not in op and not op.startswith("ds_bpermute") \
            and not op.startswith("ds_permute") and not op.startswith("ds_swizzle"):
        store = True
    kind = None
    if op.startswith("ds_"):
        kind = "lds"
    elif op.startswith(("s_load", "s_buffer_load")):
        kind = "smem"
    elif op.startswith(("global_", "buffer_", "scratch_")):
        kind = "vmem"
    return kind, store


def step(state, n, s, report):
    op = s.split()[0]
    args = s[len(op):].strip()
    if op == "s_waitcnt":
        vm = re.search(r"vmcnt\((\d+)\)", args)
        lg = re.search(r"lgkmcnt\((\d+)\)", args)
        if args == "0":
            return {}
        new = {}
        for key, (kind, age, rg) in state.items():
            if kind == "vmem" and vm and age >= int(vm.group(1)):
                continue
            if kind == "lds" and lg and age >= int(lg.group(1)):
                continue
            if kind == "smem" and lg and int(lg.group(1)) == 0:
                continue
            new[key] = (kind, age, rg)
        return new
    kind, store = classify(op, args)
    parts = [p.strip() for p in args.split(",")] if args else []
    dst, srcs = set(), set()
    if parts:
        if store or op.startswith(("s_cbranch", "s_branch", "s_endpgm", "s_barrier", "s_nop", "s_sleep", "s_setprio")):
            for p in parts:
                srcs |= regs(p)
        else:
            dst = regs(parts[0])
            for p in parts[1:]:
                srcs |= regs(p)
    touched = srcs | dst
    if report is not None:
        for key, (k2, age, rg) in state.items():
            if rg & touched:
                report.append((n, s, key, k2, sorted(rg & touched)[:4]))
    if kind:
        state = {key: (k2, age + (1 if k2 == kind or (kind == "smem" and k2 == "lds") or (kind == "lds" and k2 == "smem") else 0), rg)
                 for key, (k2, age, rg) in state.items()}
        if not store and dst:
            state[n] = (kind, 0, dst)
        elif store:
            state[n] = (kind, 0, set())
    return state


def merge(a, b):
    out = dict(a)
    for key, (k, age, rg) in b.items():
        if key in out:
            out[key] = (k, min(out[key][1], age), rg)
        else:
            out[key] = (k, age, rg)
    return out


def main(path="/tmp/kernel.s"):
    blocks = parse(path)
    idx = {lab: i for i, (lab, _) in enumerate(blocks) if lab}
    succ = []
    for i, (lab, ins) in enumerate(blocks):
        ss = []
        if ins:
            op = ins[-1][1].split()[0]
            tgt = ins[-1][1].split()[-1] if op.startswith(("s_cbranch", "s_branch")) else None
            if tgt in idx:
                ss.append(idx[tgt])
            if op not in ("s_branch", "s_endpgm", "s_setpc_b64") and i + 1 < len(blocks):
                ss.append(i + 1)
        elif i + 1 < len(blocks):
            ss.append(i + 1)
        succ.append(ss)
    entry = [None] * len(blocks)
    entry[0] = {}
    work = [0]
    it = 0
    while work and it < 200000:
        it += 1
        i = work.pop()
        st = dict(entry[i])
        for n, s in blocks[i][1]:
            st = step(st, n, s, None)
        for j in succ[i]:
            m = st if entry[j] is None else merge(entry[j], st)
            if entry[j] is None or m != entry[j]:
                entry[j] = m
                work.append(j)
    rep = []
    for i, (lab, ins) in enumerate(blocks):
        if entry[i] is None:
            continue
        st = dict(entry[i])
        for n, s in ins:
            st = step(st, n, s, rep)
    seen = set()
    for n, s, key, kind, r in rep:
        if (n, key) in seen:
            continue
        seen.add((n, key))
        print(f"{n}: {s}\n    {kind} result of line {key} may be in flight: {r}")
    print(f"{len(seen)} reports", file=sys.stderr)


if __name__ == "__main__":
    main(*sys.argv[1:2])
