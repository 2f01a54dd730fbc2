"""Instruction mix of one kernel in a hipcc -S listing: per basic block (label) counts of MFMA,
VALU, LDS, VMEM, SALU, waitcnt, barrier; the blocks inside loops are what the tile loop runs.
usage: isa_mix.py listing.s kernel-name-substring [min_instr]"""
import re
import sys
from collections import Counter

path, want = sys.argv[1], sys.argv[2]
min_n = int(sys.argv[3]) if len(sys.argv) > 3 else 50
lines = open(path).read().split("\n")
start = None
for i, l in enumerate(lines):
    if ":" in l and l.split(":")[0] .endswith(want.split("*")[-1]) is False and False:
        pass
    if re.match(r"^[_A-Za-z0-9]+:", l) and want in l:
        start = i
        break
if start is None:
    sys.exit(f"{want} not found")
blocks, cur, name = [], Counter(), lines[start][:-1]
for l in lines[start + 1:]:
    s = l.strip()
    if s.startswith(".Lfunc_end"):
        break
    if re.match(r"^\.LBB\d+_\d+:", s):
        blocks.append((name, cur))
        name, cur = s[:-1], Counter()
        continue
    if not s or s.startswith((";", ".", "//")):
        continue
    op = s.split()[0]
    if op.startswith("v_mfma"):
        cur["mfma"] += 1
    elif op.startswith("v_"):
        cur["valu"] += 1
        if any(t in op for t in ("exp", "log", "rcp", "rsq", "sqrt")):
            cur["trans"] += 1
        if op.startswith("v_cvt"):
            cur["cvt"] += 1
    elif op.startswith("ds_"):
        cur["lds"] += 1
    elif op.startswith(("buffer_", "global_", "flat_", "scratch_")):
        cur["vmem"] += 1
    elif op.startswith("s_waitcnt"):
        cur["wait"] += 1
    elif op.startswith("s_barrier"):
        cur["barrier"] += 1
    elif op.startswith("s_nop"):
        cur["nop"] += 1
    elif op.startswith("s_"):
        cur["salu"] += 1
blocks.append((name, cur))
tot = Counter()
for n, c in blocks:
    tot += c
    if sum(c.values()) >= min_n:
        print(f"{n:14s} " + " ".join(f"{k}={c[k]}" for k in ("mfma", "valu", "trans", "cvt", "lds", "vmem", "salu", "wait", "nop", "barrier")))
print("total          " + " ".join(f"{k}={tot[k]}" for k in ("mfma", "valu", "trans", "cvt", "lds", "vmem", "salu", "wait", "nop", "barrier")))
