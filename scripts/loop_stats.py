"""Loop bodies of a disassembled gfx950 code object (llvm-objdump -d --no-show-raw-insn output): per
kernel, every backward branch's body length in instructions and its scratch (spill) accesses --
to check that a hand-scheduled inner loop stays spill-free after a change.
usage: python3 scripts/loop_stats.py <disasm.s> [min_len] [max_len]   (LOOP_MIX=n: the n commonest
opcodes of each loop too)"""
import collections
import os
import re
import sys


def main():
    txt = open(sys.argv[1]).read()
    lo = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    hi = int(sys.argv[3]) if len(sys.argv) > 3 else 4000
    for part in re.split(r"\n(?=[0-9a-f]+ <_Z)", txt):
        m = re.match(r"([0-9a-f]+) <(_Z[^>]+)>:", part)
        if not m:
            continue
        base = int(m.group(1), 16)
        ins = []
        for line in part.split("\n")[1:]:
            mm = re.match(r"\s+(\S.*?)\s*//\s*([0-9A-F]+):", line)
            if mm:
                ins.append((int(mm.group(2), 16), mm.group(1)))
        idx = {a: i for i, (a, _) in enumerate(ins)}
        loops = set()
        for line in part.split("\n"):
            mm = re.match(r"\s+(s_c?branch\S*).*//\s*([0-9A-F]+):.*\+0x([0-9a-f]+)>", line)
            if mm:
                a, tgt = int(mm.group(2), 16), base + int(mm.group(3), 16)
                if tgt < a and tgt in idx:
                    body = ins[idx[tgt]:idx[a] + 1]
                    if lo <= len(body) <= hi:
                        mix = collections.Counter(x.split()[0] for _, x in body)
                        loops.add((len(body), sum(1 for _, x in body if x.startswith("scratch_")), hex(tgt),
                                   tuple(mix.most_common(int(os.environ.get("LOOP_MIX", "0"))))))
        print(m.group(2), "instructions", len(ins), "scratch", sum(1 for _, x in ins if x.startswith("scratch_")))
        for n, sc, t, mix in sorted(loops):
            print(f"  loop at {t}: {n} instructions, {sc} scratch")
            if mix:
                print("    " + " ".join(f"{k} {v}" for k, v in mix))


if __name__ == "__main__":
    main()
