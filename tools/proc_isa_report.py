"""Per-evaluation VALU mix of the procedural density (verdict r04 #3), from a
hipcc -S device assembly file: the octave loop (8 LDS reads + the lattice
load), the rest of one sample (fractions, Worley cube, combine), and the
27-cell Worley block that (cells - 8) / 27 of the samples also run.  Each
region's opcodes are classed by tools/isa_hist.py (flop / int / conv / sel /
move) and costed with the calibrated gfx950 issue cycles (tools/isa_cost.py).

    python tools/proc_isa_report.py FILE.s [KERNEL_SUBSTRING ...] [--octaves 4] [--cells 8.68]

With PMC numbers (SQ_INSTS_VALU per launch, density evaluations per launch,
GRBM_GUI_ACTIVE) it also gives the measured wave-instructions per 64
evaluations and the model's VALU issue utilisation (instructions per SIMD
cycle x calibrated cycles per instruction): --pmc INSTS,EVALS,GUI_ACTIVE.
"""
import argparse
import collections
import re
import sys

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.abspath(__file__)))
from isa_cost import cost  # noqa: E402
from isa_hist import classify, kernel_body  # noqa: E402


def loops(body):
    labels = {m.group(1): i for i, l in enumerate(body) if (m := re.match(r"^(\.LBB\S+):", l))}
    out = []
    for i, l in enumerate(body):
        m = re.search(r"s_cbranch_\w+\s+(\.LBB\S+)|s_branch\s+(\.LBB\S+)", l)
        if m:
            tgt = m.group(1) or m.group(2)
            if tgt in labels and labels[tgt] < i:
                out.append((labels[tgt], i))
    # several back edges to one header are one loop (to its last back edge)
    last = {}
    for a, b in out:
        last[a] = max(b, last.get(a, b))
    return sorted(last.items())


def instrs(body, lines):
    for i in sorted(lines):
        x = body[i].strip()
        if x and not x.startswith((".", ";")) and not x.endswith(":"):
            yield x


def count(body, lines):
    n = collections.Counter()
    for x in instrs(body, lines):
        op = x.split()[0]
        if op.startswith("ds_"):
            n["LDS"] += 1
        elif op.startswith(("buffer_", "global_")):
            n["VMEM"] += 1
        elif op.startswith("v_"):
            n["VALU"] += 1
    return n


def mix(body, lines):
    cls, cyc, ops = collections.Counter(), collections.Counter(), collections.Counter()
    for x in instrs(body, lines):
        op = re.sub(r"_e(32|64|64_dpp|32_dpp|_sdwa)$", "", x.split()[0])
        if op.startswith("v_"):
            c = classify(op)
            cls[c] += 1
            cyc[c] += cost(x)[0]
            ops[op] += 1
    return cls, cyc, ops


def basic_blocks(body, lo, hi):
    """Label-delimited line ranges [a, b) inside [lo, hi]."""
    cuts = [i for i in range(lo, hi + 1) if re.match(r"^\.LBB\S+:", body[i])]
    # a block also ends after a branch (exec-masked ifs fall through)
    cuts += [i + 1 for i in range(lo, hi) if re.search(r"\bs_(cbranch_\w+|branch)\b", body[i])]
    edges = sorted(set([lo] + cuts + [hi + 1]))
    return [(a, b) for a, b in zip(edges, edges[1:]) if b > a]


def report(path, want, octaves, cells, pmc):
    body = kernel_body(path, want)
    ls = loops(body)
    regions = [(a, b, count(body, range(a, b + 1))) for a, b in ls]
    p_full = max(0.0, (cells - 8.0) / 27.0)
    allb = basic_blocks(body, 0, len(body) - 1)
    nld = lambda a, b: sum(1 for x in instrs(body, range(a, b)) if x.startswith("buffer_load_dwordx2"))
    fb = max(allb, key=lambda ab: nld(*ab))
    if nld(*fb) < 2:   # the octave loop (fbm_lat<0>) is the hot one
        oct_ = max((r for r in regions if r[2]["LDS"] == 8 and r[2]["VMEM"] == 1), key=lambda r: r[2]["VALU"])
        samp = min((r for r in regions if r[2]["LDS"] >= 16 and r[0] <= oct_[0] and r[1] >= oct_[1]),
                   key=lambda r: r[1] - r[0])
        L_oct = set(range(oct_[0], oct_[1] + 1))
        L_samp = set(range(samp[0], samp[1] + 1))
        if samp[2]["LDS"] >= 43:   # the 27-cell block inside the sample loop: its rintf blocks
            L_full = set()
            for a, b in basic_blocks(body, samp[0], samp[1]):
                if not (L_oct & set(range(a, b))) and any(x.startswith("v_rndne_f32") for x in instrs(body, range(a, b))):
                    L_full |= set(range(a, b))
        else:   # a loop of its own around the sample loop
            full = min((r for r in regions if r[2]["LDS"] >= 43 and r[0] <= samp[0] and r[1] >= samp[1]),
                       key=lambda r: r[1] - r[0])
            L_full = set(range(full[0], full[1] + 1)) - L_samp
        L_rest = L_samp - L_oct - L_full
        parts = [("octave x %d" % octaves, L_oct, octaves), ("rest of the sample", L_rest, 1.0),
                 ("27-cell block x %.3f" % p_full, L_full, p_full)]
    else:
        # fbm_lat<OCT> fully unrolled: the basic block with the lattice loads of
        # every octave; the sample loop is the smallest loop around it (its
        # nested loops -- the p.octaves != OCT fallback -- and the fallback's
        # other lattice-load blocks excluded), and the 27-cell block its basic
        # blocks of >= 20 LDS reads
        samp = min((r for r in regions if r[0] <= fb[0] and r[1] >= fb[1] - 1), key=lambda r: r[1] - r[0])
        inner = [r for r in regions if samp[0] <= r[0] and r[1] <= samp[1] and (r[0], r[1]) != (samp[0], samp[1])]
        blocks = basic_blocks(body, samp[0], samp[1])
        L_oct = set(range(*fb))
        L_full = set()
        excl = set()
        for a, b in blocks:
            if (a, b) != fb and any(x.startswith("v_rndne_f32") for x in instrs(body, range(a, b))):
                L_full |= set(range(a, b))   # cellular_table9_full: rintf per axis
            elif (a, b) != fb and nld(a, b):
                excl |= set(range(a, b))
        if not L_full:   # the 27-cell block without rintf of its own: its >= 20 LDS reads
            for a, b in blocks:
                if (a, b) != fb and sum(1 for x in instrs(body, range(a, b)) if x.startswith("ds_read")) >= 20:
                    L_full |= set(range(a, b))
            excl -= L_full
        for a, b, _ in inner:
            excl |= set(range(a, b + 1))
        L_rest = set(range(samp[0], samp[1] + 1)) - L_oct - L_full - excl
        parts = [("fbm, %d octaves unrolled" % octaves, L_oct, 1.0), ("rest of the sample", L_rest, 1.0),
                 ("27-cell block x %.3f" % p_full, L_full, p_full)]
    tot_cls, tot_cyc = collections.Counter(), collections.Counter()
    print(f"{body[0].split(':')[0]}")
    for name, L, w in parts:
        cls, cyc, ops = mix(body, L)
        print(f"  {name:24s} per pass: {sum(cls.values()):4d} VALU, {sum(cyc.values()):7.1f} issue cycles; "
              + ", ".join(f"{k} {cls[k]}" for k in ("flop", "int", "conv", "sel", "move")))
        if name.startswith(("octave", "fbm", "rest")):
            print("      " + ", ".join(f"{op} {k}" for op, k in ops.most_common(12)))
        for k in cls:
            tot_cls[k] += w * cls[k]
            tot_cyc[k] += w * cyc[k]
    n, c = sum(tot_cls.values()), sum(tot_cyc.values())
    print(f"  per density evaluation (static, all lanes active): {n:.1f} VALU, {c:.1f} issue cycles "
          f"({c / n:.2f} per instruction)")
    for k in ("flop", "int", "conv", "sel", "move"):
        print(f"    {k:5s} {tot_cls[k]:6.1f} instr ({tot_cls[k] / n:5.1%}), {tot_cyc[k]:7.1f} cycles ({tot_cyc[k] / c:5.1%})")
    if pmc:
        insts, evals, gui = pmc
        per64 = insts / evals * 64
        cyc_xcd = gui / 8
        ipc = insts / (1024 * cyc_xcd)
        print(f"  PMC: {per64:.1f} wave-instructions per 64 evaluations (static {n:.1f}: lane use {n / per64:.2f}); "
              f"{ipc:.3f} VALU instructions per SIMD-cycle; x {c / n:.2f} calibrated cycles = VALU issue "
              f"utilisation {ipc * c / n:.2f}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("kernels", nargs="*", default=["march_proc_sortedILb0ELb0ELi3", "proc_shadow_evalILi3ELb0"])
    ap.add_argument("--octaves", type=int, default=4)
    ap.add_argument("--cells", type=float, default=8.68)
    ap.add_argument("--pmc", default=None, help="INSTS,EVALS,GUI_ACTIVE (one kernel)")
    a = ap.parse_args()
    pmc = tuple(float(v) for v in a.pmc.split(",")) if a.pmc else None
    for k in a.kernels:
        report(a.asm, k, a.octaves, a.cells, pmc)


if __name__ == "__main__":
    main()
