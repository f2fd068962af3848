"""Scan a gfx950 ISA listing (hipcc --save-temps .s, or --cuda-device-only -S) for two VMEM hazards
that the compiler counts for its own instructions but not into inline asm (EmitLines::flush stores
through an asm global_store_dwordx4):

  (1) store data: a store with more than 64 bits of data reads its data VGPRs after issue; a VALU
      that rewrites them must wait one state (distance 1 = hazard, one instruction or s_nop between
      = safe);
  (2) a VMEM instruction reading an SGPR (its saddr) that a VALU wrote (v_readfirstlane) needs 5
      wait states;
  (3) (round 3) a MUBUF store of more than 64 bits with a REGISTER soffset.  LLVM assumes such a
      store has no store-data hazard and schedules a VALU that rewrites the data VGPRs right
      behind it; on gfx950 the store then writes the new value.  The kernels pass soffset 0
      (buf_store16 in cz_kernels.hip), so the compiler inserts the wait state itself; any
      register soffset is reported, whatever the schedule around it.

The scan is linear over the text (it ignores branches), so it may over-report, never under-report
a straight-line case.  usage: python tools/isa_store_hazard.py file.s"""
import re
import sys


def _vregs(tok):
    m = re.match(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", tok)
    return {int(m.group(1))} if m else set()


def _instrs(text):
    out = []
    for line in text.splitlines():
        t = line.strip()
        if not t or t.startswith((";", ".")) or re.match(r"^\S+:", t):
            continue
        out.append(t)
    return out


def scan(text):
    """-> (store-data hazards, VALU-SGPR -> VMEM hazards, wide MUBUF stores with a register
    soffset): lists of (store, offending instruction) and of stores."""
    ins = _instrs(text)
    data_hz, sgpr_hz, soff_reg = [], [], []
    for i, t in enumerate(ins):
        op = t.split()[0]
        if not op.startswith(("global_", "buffer_", "flat_")):
            continue
        ops = [o.strip() for o in t.split(None, 1)[1].split(",")] if " " in t else []
        if op.startswith(("global_store_dwordx", "buffer_store_dwordx", "flat_store_dwordx")) and len(ops) > 1:
            # data operand: global/flat "vaddr, vdata, ..."; buffer (MUBUF) "vdata, vaddr, srsrc, soffset"
            data = _vregs(ops[0] if op.startswith("buffer_") else ops[1])
            if op.startswith("buffer_") and len(data) > 2 and len(ops) > 3 and re.match(r"s\d+$", ops[3].split()[0]):
                soff_reg.append(t)
            if len(data) > 2 and i + 1 < len(ins):  # > 64 bits of store data
                u = ins[i + 1]
                if u.startswith("v_") and " " in u and _vregs(u.split(None, 1)[1].split(",")[0].strip()) & data:
                    data_hz.append((t, u))
        m = re.search(r"s\[(\d+):(\d+)\]", t)
        if not m:
            continue
        sg = {int(m.group(1)), int(m.group(2))}
        ws = 0
        for k in range(i - 1, max(-1, i - 8), -1):
            u = ins[k]
            o = u.split()[0]
            if o == "s_nop":
                ws += int(u.split()[1], 0) + 1
                continue
            if o.startswith("v_") and " " in u:
                d = u.split(None, 1)[1].split(",")[0].strip()
                mm = re.match(r"s(\d+)$", d) or re.match(r"s\[(\d+):(\d+)\]", d)
                if mm and {int(x) for x in mm.groups() if x} & sg and ws < 5:
                    sgpr_hz.append((t, u))
                    break
            ws += 1
            if ws >= 5:
                break
    return data_hz, sgpr_hz, soff_reg


if __name__ == "__main__":
    d, s, r = scan(open(sys.argv[1]).read())
    print("store-data hazards (VALU rewrites store data at distance 1):", len(d))
    print("VALU-written SGPR read as a VMEM address within 5 wait states:", len(s))
    print("wide MUBUF stores with a register soffset:", len(r))
    for h in (d + s + r)[:10]:
        print("  ", h)
    sys.exit(1 if d or s or r else 0)
