"""Per-opcode histogram of one loop (or line range) of a kernel in a hipcc -S
device assembly file, with each VALU opcode put in a class:

  flop  -- fp32 arithmetic the algorithm counts (add/sub/mul/fma, min/max,
           floor/rndne/fract, sqrt/rcp/exp, packed f32 ops count once here)
  conv  -- int <-> float conversions
  int   -- integer ALU: hashing, masks, shifts, integer adds (addressing)
  sel   -- compares and selects (v_cmp*, v_cndmask)
  move  -- v_mov, lane moves (readlane/readfirstlane/permlane)
and the gfx950 issue cost of tools/isa_cost.py.  Non-VALU instructions are
counted by class (LDS, VMEM, SALU).

    python tools/isa_hist.py FILE.s KERNEL_SUBSTRING FIRST_LINE LAST_LINE
        (lines relative to the kernel's label, as tools/isa_loops.py prints)
"""
import collections
import re
import sys

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.abspath(__file__)))
from isa_cost import cost  # noqa: E402

FLOP = re.compile(r"^v_(pk_)?(add|sub|subrev|mul|fma|fmac|fmamk|fmaak|mac|min|max|min3|max3|med3|floor|rndne|fract|"
                  r"sqrt|rcp|rsq|exp|log|ldexp|fma_mix)(_f32|_f16|_legacy_f32)?$")
CONV = re.compile(r"^v_cvt_")
SEL = re.compile(r"^v_(cmp|cmpx|cndmask)")
MOVE = re.compile(r"^v_(mov|pk_mov|readlane|readfirstlane|writelane|permlane|swap|accvgpr)")


def classify(op):
    if FLOP.match(op):
        return "flop"
    if CONV.match(op):
        return "conv"
    if SEL.match(op):
        return "sel"
    if MOVE.match(op):
        return "move"
    return "int"


def kernel_body(path, want):
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*:\s*(;.*)?$", l) and want in l)
    end = next(i for i in range(start + 1, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
    return lines[start:end]


def histogram(ins):
    ops = collections.Counter()
    cls = collections.Counter()
    cyc = collections.Counter()
    other = collections.Counter()
    for x in ins:
        op = re.sub(r"_e(32|64|64_dpp|32_dpp|_sdwa)$", "", x.split()[0])
        if op.startswith("v_"):
            c = classify(op)
            ops[op] += 1
            cls[c] += 1
            cyc[c] += cost(x)[0]
        elif op.startswith("ds_"):
            other["LDS"] += 1
        elif op.startswith(("buffer_", "global_", "flat_", "scratch_")):
            other["VMEM"] += 1
        elif op.startswith("s_"):
            other["SALU"] += 1
    return ops, cls, cyc, other


def main():
    path, want, a, b = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    body = kernel_body(path, want)
    seg = [x.strip() for x in body[a:b + 1]]
    ins = [x for x in seg if x and not x.startswith((".", ";")) and not x.endswith(":")]
    ops, cls, cyc, other = histogram(ins)
    n = sum(cls.values())
    print(f"{body[0].split(':')[0]} lines {a}-{b}: {n} VALU, {dict(other)}")
    for c in ("flop", "int", "conv", "sel", "move"):
        print(f"  {c:5s} {cls[c]:4d} instr ({cls[c] / max(1, n):5.1%}), {cyc[c]:6.1f} issue cycles")
    for op, k in ops.most_common():
        print(f"    {op:28s} {k:4d}  {classify(op)}")


if __name__ == "__main__":
    main()
