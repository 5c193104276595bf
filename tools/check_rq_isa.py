#!/usr/bin/env python3
"""Check the prefetching register-resident kernels (qdc_rq.hpp, k_rq<*, *, true> and
k_rw<*, *, true>, VGPR and AGPR destinations): no
instruction may read or overwrite the destination registers of a hidden prefetch load
(inline-asm global_load_dwordx4 ... nt) on any control-flow path between the load and the
explicit asm s_waitcnt vmcnt that retires it (a copy or spill of an in-flight register would
read stale data; the compiler cannot know, the loads are invisible to it).

Walks the CFG of each kernel's device assembly (labels, branches, fall-through) from every
hidden load until an explicit asm vmcnt wait.  usage: tools/check_rq_isa.py [asm file]
(asm file: make -C differentiable-quantum-circuit-cuda_amd/csrc asm -> /tmp/qdc_f32.s)
"""
import re
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "/tmp/qdc_f32.s"
text = open(path).read().splitlines()


def regs(tok):
    """VGPRs and AGPRs named by an operand, as (class, index)."""
    m = re.match(r"-?([va])\[(\d+):(\d+)\]", tok)
    if m:
        return {(m.group(1), k) for k in range(int(m.group(2)), int(m.group(3)) + 1)}
    m = re.match(r"-?([va])(\d+)$", tok)
    return {(m.group(1), int(m.group(2)))} if m else set()


def parse(line):
    body = line.split(";")[0].strip()
    if not body:
        return "", []
    parts = body.split(None, 1)
    ops = [t.strip() for t in re.split(r",\s*(?![^\[]*\])", parts[1])] if len(parts) > 1 else []
    return parts[0], ops


STORES = ("global_store", "flat_store", "scratch_store", "buffer_store", "ds_write", "ds_store")


def reads_writes(op, ops):
    """(registers read, registers written) by one instruction (VGPRs only)."""
    if not ops:
        return set(), set()
    if op.startswith(STORES) or op.startswith("s_") or op.startswith("ds_bpermute") is False and op.startswith("ds_add"):
        return set().union(*[regs(t) for t in ops]), set()
    dst = regs(ops[0])
    src = set().union(*[regs(t) for t in ops[1:]]) if len(ops) > 1 else set()
    return src, dst


bad = 0
for start, line in enumerate(text):
    m = re.match(r"^(_ZN3qdc4k_r[qw]ILb[01]ELi\d+ELb1E\S*):", line)
    if not m:
        continue
    name = m.group(1)
    end = next(j for j in range(start + 1, len(text)) if text[j].startswith(".Lfunc_end"))
    lines = list(range(start + 1, end))
    label_at = {}
    for i in lines:
        lm = re.match(r"^(\.LBB\w+):", text[i])
        if lm:
            label_at[lm.group(1)] = i

    def succ(i):
        op, ops = parse(text[i])
        if op == "s_branch":
            return [label_at[ops[0]]]
        if op.startswith("s_cbranch"):
            return [label_at[ops[0]], i + 1]
        if op in ("s_endpgm", "s_setpc_b64"):
            return []
        return [i + 1] if i + 1 < end else []

    asm_end = {}  # ;;#ASMSTART line -> its ;;#ASMEND line (an asm statement is one step)
    for i in lines:
        if text[i].strip() == ";;#ASMSTART":
            asm_end[i] = next(j for j in range(i, end) if text[j].strip() == ";;#ASMEND")

    def is_wait(i):
        return i in asm_end and any(re.search(r"s_waitcnt vmcnt\(\d+\)", text[k])
                                    for k in range(i, asm_end[i]))

    n = 0
    for i in lines:
        op, ops = parse(text[i])
        if op != "global_load_dwordx4" or not text[i].rstrip().endswith("nt"):
            continue
        n += 1
        dst = regs(ops[0])
        seen, stack, hit = set(), [i + 1], None
        while stack and hit is None:
            j = stack.pop()
            if j in seen or j >= end:
                continue
            seen.add(j)
            if is_wait(j):
                continue
            if j in asm_end:
                # other asm statements (stage math, loads): check their operands, then skip
                for k in range(j + 1, asm_end[j]):
                    o2, a2 = parse(text[k])
                    if o2 == "global_load_dwordx4" and text[k].rstrip().endswith("nt"):
                        r, w = (regs(a2[1]) if len(a2) > 1 else set()), set()
                    else:
                        r, w = reads_writes(o2, a2)
                    if (r | w) & dst:
                        hit = k
                        break
                stack.append(asm_end[j] + 1)
                continue
            o2, a2 = parse(text[j])
            if o2 and not o2.startswith((".", ";")):
                if o2 == "global_load_dwordx4" and text[j].rstrip().endswith("nt"):
                    r, w = regs(a2[1]) if len(a2) > 1 else set(), set()
                else:
                    r, w = reads_writes(o2, a2)
                if (r | w) & dst:
                    hit = j
                    break
            stack.extend(succ(j))
        if hit is not None:
            print(f"{name[:50]}: load at line {i + 1} -> line {hit + 1}: {text[hit].strip()}")
            bad += 1
    print(f"{name[:60]}: {n} hidden loads checked")
print("FAIL" if bad else "OK")
sys.exit(1 if bad else 0)
