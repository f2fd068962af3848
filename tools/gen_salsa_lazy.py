#!/usr/bin/env python3
"""Generate jeromq_amd/csrc/cz_salsa_lazy.h: Salsa20 rounds 3..20 as one gfx950 inline-asm
block with LAZY XORS (fewer VALU instructions per 64-byte block).

Why.  On gfx950 every int32 VALU wave-instruction occupies its SIMD for 4 cycles,
whatever the opcode (tools/diag/salsa_ub.hip, profiles/r01/ubench_salsa_issue.log), so
the seal kernel's time is its VALU instruction count.  A Salsa20 quarter-round step is
    b ^= rotl(a + d, r)          (v_add_u32, v_alignbit_b32, v_xor_b32)
and 1/3 of the 960 ARX instructions of a block are those xors.  gfx950 has two 3-input
ops that absorb a pending xor for free:
    v_xad_u32    D = (S0 ^ S1) + S2   -- an add whose operand is still "m ^ delta"
    v_bitop3_b32 D = S0 ^ S1 ^ S2      -- an update that folds two deltas at once
So a word updated by `w ^= R` can keep R as a pending delta (0 instructions) as long as
  * every add that reads it has at most one such lazy operand (v_xad_u32), and
  * it has at most one pending delta when updated again (then v_bitop3_b32 folds the
    old delta and the new R in one instruction).
Which updates to defer is a small 0/1 program over the 16 words x 18 rounds (solved
here with scipy's MILP): about half of the xors.  Rounds 1 and 2 stay in C: with the
key, constants, block counter and high nonce word wave-uniform, the compiler moves 3 of
round 1's quarter-rounds and part of round 2 to the scalar unit and reads the uniform
words as SGPR operands (an asm block would need a v_mov per uniform word).  Words left
lazy after round 20 are absorbed by the feed-forward add (v_xad_u32).

Operands of the generated asm: %0..%15 state words m_w ("+v"), %16..%31 deltas d_w
("=&v"), %32..%35 temps ("=&v").  CZ_LAZY_PENDING has bit w set when d_w is pending at the
end: the true word is m_w ^ d_w.

The generator checks its own output: a small interpreter runs the emitted instructions
on random states and compares with a plain Salsa20 round function.
usage: python tools/gen_salsa_lazy.py
"""
import os
import random

import numpy as np

COL = [(0, 4, 8, 12), (5, 9, 13, 1), (10, 14, 2, 6), (15, 3, 7, 11)]
ROW = [(0, 1, 2, 3), (5, 6, 7, 4), (10, 11, 8, 9), (15, 12, 13, 14)]
ROT = [7, 9, 13, 18]
W = 16
FIRST = 3   # first Salsa round (1-based) done in asm; rounds 1..FIRST-1 stay in C
ROUNDS = 21 - FIRST


def groups_of(r):  # r = 0..ROUNDS-1 <-> Salsa round r + FIRST (odd rounds are column rounds)
    return COL if (r + FIRST) % 2 == 1 else ROW


def solve():
    """S = pending at round start, A = pending during pre-update uses, F = fold at update,
    M = materialise at round start (cost 1 when S = 1 and A = 0)."""
    from scipy.optimize import Bounds, LinearConstraint, milp
    R = ROUNDS

    def idx(kind, w, r):
        return ("SAFM".index(kind) * W + w) * R + r
    n = 4 * W * R
    c = np.zeros(n)
    rows, lo, hi = [], [], []

    def add(coefs, l, h):
        v = np.zeros(n)
        for k, val in coefs:
            v[k] += val
        rows.append(v)
        lo.append(l)
        hi.append(h)
    for w in range(W):
        add([(idx("S", w, 0), 1)], 0, 0)
        for r in range(R):
            S, A, F, M = (idx(k, w, r) for k in "SAFM")
            c[F] = c[M] = 1
            add([(A, 1), (S, -1)], -np.inf, 0)         # A <= S
            add([(M, 1), (S, -1), (A, 1)], 0, np.inf)  # M >= S - A
            add([(A, 1), (F, -1)], -np.inf, 0)         # defer only from A = 0
            if r + 1 < R:
                add([(idx("S", w, r + 1), 1), (F, 1)], 1, 1)  # S' = 1 - F
    for r in range(R):
        for (a, b, cc, d) in groups_of(r):
            Af = lambda w: idx("A", w, r)  # noqa: E731
            Ff = lambda w: idx("F", w, r)  # noqa: E731  pending after update = 1 - F
            add([(Af(a), 1), (Af(d), 1)], -np.inf, 1)   # a_old + d_old
            add([(Af(a), 1), (Ff(b), -1)], -np.inf, 0)  # b_new + a_old
            add([(Ff(cc), 1), (Ff(b), 1)], 1, np.inf)   # c_new + b_new
            add([(Ff(d), 1), (Ff(cc), 1)], 1, np.inf)   # d_new + c_new
    res = milp(c, constraints=LinearConstraint(np.array(rows), lo, hi), integrality=np.ones(n),
               bounds=Bounds(0, 1), options={"time_limit": 300})
    assert res.status == 0, res.message
    x = np.round(res.x).astype(int)
    get = lambda k: [[int(x[idx(k, w, r)]) for w in range(W)] for r in range(R)]  # noqa: E731
    return get("A"), get("F"), int(round(res.fun))


def emit(A, F):
    m = lambda w: f"%{w}"        # noqa: E731
    d = lambda w: f"%{16 + w}"   # noqa: E731
    tmp = lambda i: f"%{32 + i}"  # noqa: E731
    pend = [0] * W
    out = []
    starts = []  # index of each round's first instruction

    def val(w):  # operand list of word w's current value: (m,) or (m, d)
        return (m(w), d(w)) if pend[w] else (m(w),)

    def add_into(dst, u, v):
        vu, vv = val(u), val(v)
        assert len(vu) + len(vv) <= 3, "two lazy add operands"
        if len(vu) == 2:
            out.append(f"v_xad_u32 {dst}, {vu[0]}, {vu[1]}, {vv[0]}")
        elif len(vv) == 2:
            out.append(f"v_xad_u32 {dst}, {vv[0]}, {vv[1]}, {vu[0]}")
        else:
            out.append(f"v_add_u32 {dst}, {vu[0]}, {vv[0]}")

    for r in range(ROUNDS):
        groups = groups_of(r)
        starts.append(len(out))
        # materialise at round start where the schedule clears a pending delta without a fold
        for w in range(W):
            if pend[w] and not A[r][w]:
                out.append(f"v_xor_b32 {m(w)}, {m(w)}, {d(w)}")
                pend[w] = 0
        for k in range(4):
            steps = []
            for i, q in enumerate(groups):
                dst, s1, s2 = q[(k + 1) % 4], q[k], q[(k + 3) % 4]
                fold = F[r][dst]
                reg = tmp(i) if (fold or pend[dst]) else d(dst)
                steps.append((dst, s1, s2, reg, fold))
            for dst, s1, s2, reg, fold in steps:
                add_into(reg, s1, s2)
            for dst, s1, s2, reg, fold in steps:
                out.append(f"v_alignbit_b32 {reg}, {reg}, {reg}, {32 - ROT[k]}")
            for dst, s1, s2, reg, fold in steps:
                if fold:
                    if pend[dst]:
                        out.append(f"v_bitop3_b32 {m(dst)}, {m(dst)}, {d(dst)}, {reg} bitop3:0x96")
                    else:
                        out.append(f"v_xor_b32 {m(dst)}, {m(dst)}, {reg}")
                    pend[dst] = 0
                else:
                    assert not pend[dst] and reg == d(dst), "deferred update on a pending word"
                    pend[dst] = 1
    return out, pend, starts


# ---------------------------------------------------------------------------- check
M32 = 0xffffffff


def rotl(v, c):
    return ((v << c) | (v >> (32 - c))) & M32


def ref_rounds(x, first_round, nrounds):
    x = list(x)
    for r in range(first_round, first_round + nrounds):
        for (a, b, c, d) in (COL if r % 2 == 0 else ROW):
            x[b] ^= rotl((x[a] + x[d]) & M32, 7)
            x[c] ^= rotl((x[b] + x[a]) & M32, 9)
            x[d] ^= rotl((x[c] + x[b]) & M32, 13)
            x[a] ^= rotl((x[d] + x[c]) & M32, 18)
    return x


def interpret(lines, regs):
    def v(tok):
        return regs[int(tok.strip(",").lstrip("%"))]
    for ln in lines:
        op, *a = ln.replace(",", " ").split()
        dst = int(a[0].lstrip("%"))
        if op == "v_add_u32":
            regs[dst] = (v(a[1]) + v(a[2])) & M32
        elif op == "v_xad_u32":
            regs[dst] = ((v(a[1]) ^ v(a[2])) + v(a[3])) & M32
        elif op == "v_alignbit_b32":
            s = int(a[3])
            regs[dst] = ((((v(a[1]) << 32) | v(a[2])) >> s) & M32)
        elif op == "v_xor_b32":
            regs[dst] = v(a[1]) ^ v(a[2])
        elif op == "v_bitop3_b32":
            assert a[4] == "bitop3:0x96"
            regs[dst] = v(a[1]) ^ v(a[2]) ^ v(a[3])
        else:
            raise ValueError(op)
    return regs


def main():
    A, F, cost = solve()
    lines, pend, starts = emit(A, F)
    rng = random.Random(1)
    for _ in range(200):
        x = [rng.getrandbits(32) for _ in range(W)]
        before = ref_rounds(x, 0, FIRST - 1)
        regs = before + [rng.getrandbits(32) for _ in range(20)]
        regs = interpret(lines, regs)
        got = [regs[w] ^ (regs[16 + w] if pend[w] else 0) for w in range(W)]
        assert got == ref_rounds(x, 0, 20), "lazy schedule mismatch"
    ops = {}
    for ln in lines:
        ops[ln.split()[0]] = ops.get(ln.split()[0], 0) + 1
    mask = sum(1 << w for w in range(W) if pend[w])
    here = os.path.dirname(os.path.abspath(__file__))
    path = os.path.join(here, "..", "jeromq_amd", "csrc", "cz_salsa_lazy.h")
    body = " \\\n".join(f'    "{s}\\n"' for s in lines)
    bounds = starts + [len(lines)]
    rounds = "\n".join(
        f"#define CZ_SALSA_LAZY_ROUND_{i} \\\n" + " \\\n".join(f'    "{s}\\n"' for s in lines[bounds[i]:bounds[i + 1]])
        for i in range(ROUNDS))
    hdr = f"""// cz_salsa_lazy.h -- GENERATED by tools/gen_salsa_lazy.py (do not edit).
// Salsa20 rounds {FIRST}..20 with lazy xors: {len(lines)} VALU instructions
// ({", ".join(f"{k} {v}" for k, v in sorted(ops.items()))})
// instead of {48 * ROUNDS} ({ROUNDS} rounds x 48).  Fold/materialise instructions: {cost} (vs {16 * ROUNDS} xors).
// Operands: %0..%15 state m_w ("+v"), %16..%31 deltas d_w ("=&v"), %32..%35 temps ("=&v").
// After the block, word w = m_w ^ d_w for every bit w of CZ_LAZY_PENDING, else m_w.
#pragma once
#define CZ_LAZY_PENDING 0x{mask:04x}u
#define CZ_LAZY_FIRST_ROUND {FIRST}
#define CZ_SALSA_LAZY_ASM \\
{body}

// The same instructions one Salsa20 round per macro (rounds {FIRST}..20), so the compiler can
// place independent work (the previous block's Poly1305, loads, stores) between rounds.
{rounds}
"""
    with open(path, "w") as f:
        f.write(hdr)
    print(f"wrote {os.path.normpath(path)}: {len(lines)} instructions, pending mask 0x{mask:04x}, {ops}")


if __name__ == "__main__":
    main()
