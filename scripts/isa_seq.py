"""Memory-instruction / wait sequence of one kernel in a hipcc -S listing
(tuning aid): global/LDS operations and s_waitcnt in program order, runs of
the same instruction compressed, so the batching of loads against their waits
can be read without a GPU.  usage: python3 scripts/isa_seq.py file.s NAME [max_lines]"""
import re
import sys


def main():
    path, key = sys.argv[1], sys.argv[2]
    lim = int(sys.argv[3]) if len(sys.argv) > 3 else 400
    lines = open(path).read().splitlines()
    st = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l) and key in l)
    en = next(i for i in range(st, len(lines)) if lines[i].startswith(".Lfunc_end"))
    seq, valu = [], 0
    for l in lines[st + 1:en]:
        t = l.split(";")[0].strip()
        if not t:
            continue
        if t.endswith(":"):
            seq.append(("L " + t, 0))
            continue
        if t.startswith("."):
            continue
        op = t.split()[0]
        if op.startswith("v_"):
            valu += 1
            continue
        if op.startswith(("global_", "buffer_", "ds_", "s_waitcnt", "s_cbranch", "s_branch", "s_barrier")):
            seq.append((t if op == "s_waitcnt" else op, valu))
            valu = 0
    out, prev, cnt, v = [], None, 0, 0
    for k, nv in seq:
        if k == prev and nv == 0:
            cnt += 1
            continue
        if prev:
            out.append(f"{prev}{' x%d' % cnt if cnt > 1 else ''}{'   (+%d valu before)' % v if v else ''}")
        prev, cnt, v = k, 1, nv
    out.append(prev)
    print("\n".join(out[:lim]))


if __name__ == "__main__":
    main()
