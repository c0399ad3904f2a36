"""List the loops of one kernel in a hipcc -S device assembly file, with
instruction counts by class (VALU / VMEM / LDS / SALU / other) per loop body.

    python tools/isa_loops.py FILE.s KERNEL_SUBSTRING
"""
import re
import sys


def main():
    path, want = sys.argv[1], sys.argv[2]
    lines = open(path).read().split("\n")
    start = None
    for i, l in enumerate(lines):
        if re.match(r"^_Z\S*:\s*(;.*)?$", l) and want in l:
            start = i
            break
    if start is None:
        sys.exit("kernel not found")
    end = next(i for i in range(start + 1, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
    body = lines[start:end]
    labels = {}
    for i, l in enumerate(body):
        m = re.match(r"^(\.LBB\S+):", l)
        if m:
            labels[m.group(1)] = i
    print(body[0].strip())
    for i, l in enumerate(body):
        m = re.search(r"s_cbranch_\w+\s+(\.LBB\S+)|s_branch\s+(\.LBB\S+)", l)
        if not m:
            continue
        tgt = m.group(1) or m.group(2)
        if tgt in labels and labels[tgt] < i:
            seg = [x.strip() for x in body[labels[tgt]:i + 1]]
            ins = [x for x in seg if x and not x.startswith((".", ";")) and not x.endswith(":")]
            cls = {"VALU": 0, "VMEM": 0, "LDS": 0, "SALU": 0, "other": 0}
            for x in ins:
                op = x.split()[0]
                if op.startswith("v_"):
                    cls["VALU"] += 1
                elif op.startswith(("buffer_", "global_", "flat_")):
                    cls["VMEM"] += 1
                elif op.startswith("ds_"):
                    cls["LDS"] += 1
                elif op.startswith("s_"):
                    cls["SALU"] += 1
                else:
                    cls["other"] += 1
            print(f"loop {tgt} lines {labels[tgt]}-{i}: {len(ins)} instr {cls}")


if __name__ == "__main__":
    main()
