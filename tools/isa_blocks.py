"""List the large basic blocks of a kernel in a hipcc --save-temps .s: VALU / SALU / memory op counts.
usage: python tools/isa_blocks.py file.s kernel_symbol_substring [min_instrs]"""
import collections
import re
import sys

path, key = sys.argv[1], sys.argv[2]
mn = int(sys.argv[3]) if len(sys.argv) > 3 else 300
s = open(path).read()
syms = [m.group(1) for m in re.finditer(r"^(\S+):[ \t]*(;.*)?$", s, re.M) if key in m.group(1) and not m.group(1).startswith(".")]
for sym in syms:
    start = s.index(sym + ":")
    end = s.index(".Lfunc_end", start)
    body = s[start:end].splitlines()
    print("==", sym)
    cur, cnt, n = None, collections.Counter(), 0
    out = []
    for line in body[1:]:
        t = line.strip()
        if re.match(r"^\.LBB\d+_\d+:", t):
            if cur:
                out.append((cur, n, cnt))
            cur, cnt, n = t.split(":")[0], collections.Counter(), 0
            continue
        if not t or t.startswith((";", ".")):
            continue
        op = t.split()[0]
        cls = "v" if op.startswith("v_") else "s" if op.startswith("s_") else "m"
        cnt[cls] += 1
        cnt[op] += 1
        n += 1
    out.append((cur, n, cnt))
    for b, n, c in out:
        if n >= mn:
            print(f"  {b:12s} n={n:5d} valu={c['v']:5d} salu={c['s']:4d} mem/lds={c['m']:3d} alignbit={c['v_alignbit_b32']:4d} "
                  f"mad64={c['v_mad_u64_u32']:3d} mov={c['v_mov_b32_e32']:3d}")
