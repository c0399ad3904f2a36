"""Issue-cycle model of a kernel's loops from its hipcc -S assembly, with the
gfx950 VALU costs measured by tools/valu_calib.hip (profiles/valu_calib.txt,
SIMD cycles per wave64 instruction at 8 waves/SIMD):

  ~2.2: f32 add/sub/mul/fma/fmac/fmamk/fmaak with VGPR, inline or literal
        operands; mov; and/or/xor; lshrrev/ashrrev; add/sub_u32; bitop3
  ~4.1: everything else -- lshlrev, packed f32, conversions, floor/fract/
        rndne, min/max/med3, cmp, cndmask, integer multiplies, 3-operand
        integer ops, fma_mix -- and ANY VALU op that reads an SGPR
  ~8.2: transcendentals (exp, log, rcp, rsq, sqrt)

    python tools/isa_cost.py FILE.s KERNEL_SUBSTRING [--hist LOOP_LABEL]
"""
import re
import sys

FAST = {"v_add_f32", "v_sub_f32", "v_subrev_f32", "v_mul_f32", "v_fma_f32", "v_fmac_f32", "v_fmamk_f32",
        "v_fmaak_f32", "v_mov_b32", "v_and_b32", "v_or_b32", "v_xor_b32", "v_lshrrev_b32", "v_ashrrev_i32",
        "v_add_u32", "v_sub_u32", "v_subrev_u32", "v_bitop3_b32", "v_not_b32", "v_mac_f32"}
TRANS = ("v_exp_", "v_log_", "v_rcp_", "v_rsq_", "v_sqrt_", "v_sin_", "v_cos_")


def cost(line):
    parts = line.split(None, 1)
    op = re.sub(r"_e(32|64)$", "", parts[0])
    if not op.startswith("v_"):
        return 0.0, op
    if op.startswith(TRANS):
        return 8.2, op
    args = parts[1] if len(parts) > 1 else ""
    sgpr = re.search(r"(^|[\s,\-|])s(\d+|\[\d+:\d+\])", args) is not None
    if op in FAST and not sgpr:
        return 2.2, op
    return 4.1, op


def loops(path, want):
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*:\s*(;.*)?$", l) and want in l)
    end = next(i for i in range(start + 1, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
    body = lines[start:end]
    labels = {m.group(1): i for i, l in enumerate(body) if (m := re.match(r"^(\.LBB\S+):", l))}
    out = []
    for i, l in enumerate(body):
        m = re.search(r"s_cbranch_\w+\s+(\.LBB\S+)|s_branch\s+(\.LBB\S+)", l)
        if m:
            tgt = m.group(1) or m.group(2)
            if tgt in labels and labels[tgt] < i:
                seg = [x.strip() for x in body[labels[tgt]:i + 1]]
                out.append((tgt, [x for x in seg if x and not x.startswith((".", ";")) and not x.endswith(":")]))
    return body[0].split(":")[0], out


def main():
    path, want = sys.argv[1], sys.argv[2]
    hist = sys.argv[4] if len(sys.argv) > 4 and sys.argv[3] == "--hist" else None
    name, ls = loops(path, want)
    print(name)
    for tgt, ins in ls:
        c = [cost(x) for x in ins]
        valu = [x for x in c if x[0] > 0]
        slow = sum(1 for x in valu if x[0] > 3)
        print(f"loop {tgt}: {len(valu)} VALU, {slow} at >=4 cycles, model {sum(x[0] for x in valu):.0f} SIMD cycles")
        if hist == tgt:
            agg = {}
            for (cy, op), x in zip(c, ins):
                if cy > 3:
                    key = op + (" (sgpr)" if cy == 4.1 and op in FAST else "")
                    agg[key] = agg.get(key, 0) + 1
            for k, v in sorted(agg.items(), key=lambda kv: -kv[1]):
                print(f"   {v:4d} x {k}")


if __name__ == "__main__":
    main()
