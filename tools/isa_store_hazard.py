"""Scan a hipcc --save-temps .s for two VMEM hazards the compiler does not count into inline asm.
(1) store data: a global_store_dwordx4 whose data
VGPRs a VALU rewrites within the next two instructions (one intervening instruction or an
s_nop is the required wait state; distance 1 is the hazard); (2) a VALU-written SGPR read as a VMEM
address needs 5 wait states.  usage: python tools/isa_store_hazard.py file.s"""
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

# second check: a VALU-written SGPR (v_readfirstlane) read as a VMEM address within 5 wait states
L=[l.strip() for l in open(sys.argv[1]).read().splitlines()]
ins=[l for l in L if l and not l.startswith((";",".")) and not re.match(r"^\S+:",l)]
bad=0
for i,t in enumerate(ins):
    op=t.split()[0]
    if not (op.startswith("global_") or op.startswith("buffer_") or op.startswith("flat_")): continue
    m=re.search(r"s\[(\d+):(\d+)\]",t)
    if not m: continue
    sg={int(m.group(1)),int(m.group(2))}
    ws=0
    for k in range(i-1,max(-1,i-8),-1):
        u=ins[k]; o=u.split()[0]
        if o.startswith("s_nop"):
            ws+=int(u.split()[1])+1; continue
        if o.startswith("v_") :
            d=u.split(None,1)[1].split(",")[0].strip()
            mm=re.match(r"s(\d+)$",d) or re.match(r"s\[(\d+):(\d+)\]",d)
            if mm and (set(int(x) for x in mm.groups() if x)&sg) and ws<5:
                bad+=1
                if bad<=5: print("VALU-SGPR -> VMEM within",ws,"states:",u,"|",t)
                break
        ws+=1
print("VALU-written SGPR used as VMEM address within 5 states:",bad)
