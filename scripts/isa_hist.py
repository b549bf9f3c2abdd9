"""Instruction histogram of one kernel in a hipcc -S listing (tuning aid).

usage: python3 scripts/isa_hist.py file.s NAME_SUBSTRING [top]
Counts the instructions of the first function whose symbol contains
NAME_SUBSTRING, and of its innermost loop bodies (the blocks between a loop
header label and its backward branch), so a change's effect on the per-window
instruction mix can be read without a GPU."""
import collections
import re
import sys


def main():
    path, key = sys.argv[1], sys.argv[2]
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    lines = [l.split(";")[0].rstrip() for l in open(path).read().splitlines()]
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l) and key in l)
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
    body = lines[start:end]
    ins = [(i, l.strip()) for i, l in enumerate(body)
           if l.strip() and not l.strip().startswith((".", ";", "_")) and not l.strip().endswith(":")]
    c = collections.Counter(l.split()[0] for _, l in ins)
    print(body[0].split(":")[0][:90], "instructions", len(ins))
    for op, n in c.most_common(top):
        print(f"  {op:30s}{n}")
    labels = {l.strip()[:-1]: i for i, l in enumerate(body) if l.strip().endswith(":") and l.strip().startswith(".LBB")}
    for i, l in ins:
        m = re.match(r"s_cbranch_\w+\s+(\.LBB\S+)|s_branch\s+(\.LBB\S+)", l)
        if not m:
            continue
        tgt = m.group(1) or m.group(2)
        j = labels.get(tgt)
        if j is None or j >= i:
            continue
        loop = [x for k, x in ins if j <= k <= i]
        lc = collections.Counter(x.split()[0] for x in loop)
        cls = collections.Counter()
        for op, n in lc.items():
            cls["valu" if op.startswith("v_") else "lds" if op.startswith("ds_") else
                "vmem" if op.startswith(("global_", "buffer_")) else "salu" if op.startswith("s_") else "other"] += n
        print(f"loop {tgt} ({len(loop)} instructions): {dict(cls)}")
        for op, n in lc.most_common(12):
            print(f"    {op:28s}{n}")


if __name__ == "__main__":
    main()
