"""Scan a hipcc --save-temps .s for the VMEM store-data hazard: a global_store_dwordx4 whose data
VGPRs a VALU rewrites within the next two instructions (one intervening instruction or an
s_nop is the required wait state; distance 1 is the hazard).  usage: python tools/isa_store_hazard.py file.s"""
import re,sys
lines=open(sys.argv[1]).read().splitlines()
cur=None; hits=0; total=0; ex=[]; allx=[]
def regs(tok):
    m=re.match(r"v\[(\d+):(\d+)\]",tok)
    if m: return set(range(int(m.group(1)),int(m.group(2))+1))
    m=re.match(r"v(\d+)$",tok)
    return {int(m.group(1))} if m else set()
for i,l in enumerate(lines):
    t=l.strip()
    if t.startswith("global_store_dwordx4"):
        ops=[o.strip() for o in t.split(None,1)[1].split(",")]
        data=regs(ops[1]); total+=1
        # next real instructions
        k=i+1; seen=0
        while k<len(lines) and seen<2:
            u=lines[k].strip(); k+=1
            if not u or u.startswith((";",".")): continue
            seen+=1
            op=u.split()[0]
            if op.startswith("s_nop"): break
            if op.startswith("v_"):
                dst=u.split(None,1)[1].split(",")[0].strip()
                if regs(dst)&data:
                    hits+=1
                    allx.append((i,t,u,seen))
                    if len(ex)<5: ex.append((i,t,u,seen))
print("stores", total, "VALU overwrites of store data at distance 2 (safe):", sum(1 for e in allx if e[3] == 2),
      "at distance 1 (HAZARD):", sum(1 for e in allx if e[3] == 1))
for e in allx:
    if e[3] == 1:
        print("hazard:", e)
