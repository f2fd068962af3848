#!/usr/bin/env python3
"""How far each vector-memory load runs ahead of the s_waitcnt that first waits for it, per
kernel of a built library (linear scan of the llvm-objdump listing; branches ignored).

A load whose wait comes a few VALU instructions after it exposes its whole latency to the wave
(round 4: the box-layout seal's line loads had been sunk next to their uses, the dense open
funnelled its loads right after issuing them).  Lists, per kernel, the loads waited for within
`--near` VALU instructions.

  python tools/isa_loadwait.py jeromq_amd/libcurvezmq_mi355x.so [--near 100] [--kernel k_open]
"""
import argparse
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def kernels(text):
    cur, lines = None, []
    for ln in text.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", ln)
        if m:
            if cur:
                yield cur, lines
            cur, lines = m.group(1), []
        elif cur:
            t = ln.split("//")[0].strip()
            m = re.search(r"//\s*([0-9A-Fa-f]+):", ln)
            if t:
                lines.append((int(m.group(1), 16) if m else -1, t))
    if cur:
        yield cur, lines


def loop_mask(lines):
    """instruction i is inside a loop: between the target of a backward branch and the branch"""
    idx = {a: i for i, (a, _) in enumerate(lines)}
    mask = [False] * len(lines)
    for i, (a, t) in enumerate(lines):
        op = t.split()[0]
        if op.startswith(("s_branch", "s_cbranch")) and len(t.split()) > 1:
            off = int(t.split()[1])
            off = off - 65536 if off >= 32768 else off
            tgt = a + 4 + 4 * off
            if off < 0 and tgt in idx:
                for k in range(idx[tgt], i + 1):
                    mask[k] = True
    return mask


def scan(lines, loops_only=False):
    """-> list of (load text, VALU instructions between the load and its first wait)"""
    out, pend = [], []  # pend: [is_load, text, valu count since issue]
    mask = loop_mask(lines)
    for k, (_, t) in enumerate(lines):
        if loops_only and not mask[k]:
            pend = []
            continue
        op = t.split()[0]
        if op.startswith(("global_load", "buffer_load", "global_store", "buffer_store", "flat_")):
            pend.append([op.startswith(("global_load", "buffer_load")), t, 0])
        elif op.startswith("v_"):
            for p in pend:
                p[2] += 1
        elif op == "s_waitcnt":
            m = re.search(r"vmcnt\((\d+)\)", t)
            if m:
                keep = int(m.group(1))
                done, pend = pend[:max(0, len(pend) - keep)], pend[max(0, len(pend) - keep):]
                out += [(p[1], p[2]) for p in done if p[0]]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--near", type=int, default=100)
    ap.add_argument("--kernel", default="")
    ap.add_argument("--all", action="store_true", help="count loads outside loops too")
    a = ap.parse_args()
    from jeromq_amd import build
    for co in build.device_code_objects(a.lib):
        import subprocess
        import tempfile
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(co)
            f.flush()
            text = subprocess.run([os.path.join(build.LLVM_BIN, "llvm-objdump"), "-d", "--mcpu=gfx950", f.name],
                                  check=True, capture_output=True, text=True).stdout
        for name, lines in kernels(text):
            if a.kernel not in name:
                continue
            res = scan(lines, loops_only=not a.all)
            near = [r for r in res if r[1] < a.near]
            wide = [r for r in near if "dwordx4" in r[0]]
            print(f"{len(res):5d} loads, {len(near):4d} waited within {a.near} VALU ({len(wide)} dwordx4)  {name}")


if __name__ == "__main__":
    main()
