#!/usr/bin/env python3
"""SLP root-cause bisection: rewrite chosen
packed-FP32 instructions of one kernel in a device assembly file as the two
scalar instructions they stand for, lane by lane.

  slp_scalarize.py <in.s> <out.s> <function label|*> <indices|all|list> [temp VGPR]

<indices>: comma-separated positions among the function's packed instructions
(v_pk_add/mul/fma_f32, v_pk_mov_b32, v_mov_b64), in order of appearance; `list` prints
them.  A packed instruction computes lane lo from the operand halves op_sel
selects and lane hi from those op_sel_hi selects, negating per neg_lo /
neg_hi; the scalar pair does the same with VOP3 neg modifiers.  An
instruction whose destination's low register feeds its high lane and whose
high register feeds its low lane cannot be split in place: with a temp VGPR
(one below the kernel's allocated VGPR count, above its last used one) its
high lane goes through the temp, else it is left packed (reported).  If rewriting an instruction removes a divergence, the packed form
of that instruction (in that context) is what differs from the scalar IEEE
operations the IR asked for.
"""
import re
import sys

PK = re.compile(r"^(\s*)(v_pk_(add|mul|fma)_f32|v_pk_mov_b32|v_mov_b64_e32)\s+(.*?)\s*$")


def split_operands(text):
    ops, mods = [], {}
    parts = [p.strip() for p in re.split(r",(?![^\[]*\])", text)]
    # modifiers are appended after the last operand, separated by spaces
    last = parts[-1].split()
    parts[-1] = last[0]
    for m in last[1:]:
        k, v = m.split(":")
        mods[k] = [int(x) for x in v.strip("[]").split(",")]
    return parts, mods


def half(op, h):
    """register / value of half h (0 lo, 1 hi) of a 64-bit packed operand"""
    m = re.match(r"([vs])\[(\d+):(\d+)\]$", op)
    if m:
        return "%s%d" % (m.group(1), int(m.group(2)) + h), "%s%d" % (m.group(1), int(m.group(2)) + h)
    return op, None   # inline constant: the same value in either half as the compiler uses it (checked below)


def rewrite(indent, name, kind, text, temp=None):
    if name == "v_mov_b64_e32":   # 64-bit move of a register pair: two 32-bit moves (aligned pairs never overlap partly)
        m = re.match(r"v\[(\d+):\d+\],\s*([vs])\[(\d+):\d+\]$", text)
        if not m:
            return None, "unparsed"
        d, f, a = int(m.group(1)), m.group(2), int(m.group(3))
        return ["%sv_mov_b32_e32 v%d, %s%d" % (indent, d, f, a), "%sv_mov_b32_e32 v%d, %s%d" % (indent, d + 1, f, a + 1)], None
    ops, mods = split_operands(text)
    n = 3 if kind == "fma" else 2
    dst, srcs = ops[0], ops[1:1 + n]
    dm = re.match(r"v\[(\d+):(\d+)\]$", dst)
    if not dm or len(srcs) != n:
        return None, "unparsed"
    d = int(dm.group(1))
    op_sel = mods.get("op_sel", [0] * n)
    op_sel_hi = mods.get("op_sel_hi", [1] * n)
    neg_lo = mods.get("neg_lo", [0] * n)
    neg_hi = mods.get("neg_hi", [0] * n)
    for i, s in enumerate(srcs):   # a non-zero constant read through its high half: ambiguous, leave it
        if not re.match(r"[vs]\[", s) and op_sel_hi[i] and s not in ("0", "0.0"):
            return None, "constant read high"
    lanes = []
    for lane, sel, neg in ((0, op_sel, neg_lo), (1, op_sel_hi, neg_hi)):
        args, regs = [], set()
        for i, s in enumerate(srcs):
            v, r = half(s, sel[i])
            if r:
                regs.add(r)
            if name == "v_pk_mov_b32":
                args.append(v)
            else:
                args.append("neg(%s)" % v if neg[i] else v)
        lanes.append((lane, args, regs))
    if name == "v_pk_mov_b32":   # lo <- src0 half op_sel[0], hi <- src1 half op_sel[1]
        v0, r0 = half(srcs[0], op_sel[0])
        v1, r1 = half(srcs[1], op_sel[1])
        lanes = [(0, [v0], {r0} if r0 else set()), (1, [v1], {r1} if r1 else set())]
    lo_reg, hi_reg = "v%d" % d, "v%d" % (d + 1)
    order = [0, 1]
    out = []
    if lo_reg in lanes[1][2]:
        if hi_reg in lanes[0][2]:
            if temp is None:
                return None, "crossed halves"
            # high lane into the temp, low lane in place, temp to the high register
            _, hargs, _ = lanes[1]
            _, largs, _ = lanes[0]
            if name == "v_pk_mov_b32":
                return ["%sv_mov_b32_e32 %s, %s" % (indent, temp, hargs[0]), "%sv_mov_b32_e32 %s, %s" % (indent, lo_reg, largs[0]),
                        "%sv_mov_b32_e32 %s, %s" % (indent, hi_reg, temp)], None
            return ["%sv_%s_f32_e64 %s, %s" % (indent, kind, temp, ", ".join(hargs)),
                    "%sv_%s_f32_e64 %s, %s" % (indent, kind, lo_reg, ", ".join(largs)),
                    "%sv_mov_b32_e32 %s, %s" % (indent, hi_reg, temp)], None
        order = [1, 0]
    for k in order:
        lane, args, _ = lanes[k]
        reg = "v%d" % (d + lane)
        if name == "v_pk_mov_b32":
            out.append("%sv_mov_b32_e32 %s, %s" % (indent, reg, args[0]))
        else:
            out.append("%sv_%s_f32_e64 %s, %s" % (indent, kind, reg, ", ".join(args)))
    return out, None


def functions(lines, func):
    """[(start, end)] line ranges of the named function, or of every function for '*'"""
    out = []
    for i, l in enumerate(lines):
        m = re.match(r"^([A-Za-z_.$][\w.$]*):", l)
        if m and (m.group(1) == func or (func == "*" and "; @" in l)):
            end = next(j for j in range(i + 1, len(lines)) if lines[j].startswith(".Lfunc_end"))
            out.append((i, end))
    return out


def main():
    src, dst, func, which = sys.argv[1:5]
    temp = sys.argv[5] if len(sys.argv) > 5 else None
    lines = open(src).read().split("\n")
    idx = [i for a, b in functions(lines, func) for i in range(a, b) if PK.match(lines[i])]
    if which == "list":
        for k, i in enumerate(idx):
            print(k, i + 1, lines[i].strip())
        return
    chosen = range(len(idx)) if which == "all" else [int(x) for x in which.split(",") if x]
    kept = []
    for k in sorted(chosen, reverse=True):
        i = idx[k]
        m = PK.match(lines[i])
        new, why = rewrite(m.group(1), m.group(2), m.group(3) or "mov", m.group(4), temp if func != "*" else None)
        if new is None:
            kept.append((k, why, lines[i].strip()))
            continue
        lines[i:i + 1] = ["\t; scalarized: " + lines[i].strip()] + new
    open(dst, "w").write("\n".join(lines))
    for k, why, l in kept:
        print("left packed:", k, why, l)


if __name__ == "__main__":
    main()
