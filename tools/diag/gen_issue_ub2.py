"""Generate tools/diag/issue_ub2.inc: asm bodies for tools/diag/issue_ub2.hip (diagnostics only).

Single-opcode bodies (16 independent accumulators v8..v23, operands v4..v7), fast/slow mixing
patterns, and one Salsa20 double round in two forms:
  ALIGN  t = a + d; t = alignbit(t, t, 32 - r); b ^= t           (v_add, v_alignbit, v_xor)
  SHIFT  t = a + d; u = t << r; t = t >> (32 - r); b = b ^ u ^ t  (v_add, v_lshlrev, v_lshrrev, v_bitop3)
State words x0..x15 in v8..v23, temporaries v24..v31; the 4 quarter-rounds of a round are
interleaved step by step."""
import os

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "issue_ub2.inc")

SINGLE = {
    "v_lshlrev_b32_e32": "v_lshlrev_b32_e32 v{n}, 7, v{n}",
    "v_lshrrev_b32_e32": "v_lshrrev_b32_e32 v{n}, 7, v{n}",
    "v_or_b32_e32": "v_or_b32_e32 v{n}, v4, v{n}",
    "v_and_b32_e32": "v_and_b32_e32 v{n}, v4, v{n}",
    "v_sub_u32_e32": "v_sub_u32_e32 v{n}, v4, v{n}",
    "v_add_u32_e64": "v_add_u32_e64 v{n}, v4, v{n}",
    "v_add_u32 sgpr": "v_add_u32_e32 v{n}, s2, v{n}",
    "v_add_u32 literal": "v_add_u32_e32 v{n}, 0x12345678, v{n}",
    "v_lshlrev_b32_e64": "v_lshlrev_b32_e64 v{n}, 7, v{n}",
    "v_cndmask_b32_e32": "v_cndmask_b32_e32 v{n}, v4, v{n}, vcc",
    "v_alignbyte_b32": "v_alignbyte_b32 v{n}, v{n}, v4, 3",
    "v_bfi_b32": "v_bfi_b32 v{n}, v4, v{n}, v5",
    "v_not_b32": "v_not_b32_e32 v{n}, v{n}",
    "v_max_u32": "v_max_u32_e32 v{n}, v4, v{n}",
    "v_mul_u32_u24": "v_mul_u32_u24_e32 v{n}, v4, v{n}",
    "v_mul_hi_u32": "v_mul_hi_u32 v{n}, v4, v{n}",
    "v_addc_co_u32_e32": "v_addc_co_u32_e32 v{n}, vcc, v4, v{n}, vcc",
    "v_lshl_or_b32": "v_lshl_or_b32 v{n}, v{n}, 7, v4",
    "v_and_or_b32": "v_and_or_b32 v{n}, v{n}, v4, v5",
    "v_or3_b32": "v_or3_b32 v{n}, v{n}, v4, v5",
    "v_bitop3 3 vgprs": "v_bitop3_b32 v{n}, v{n}, v{m}, v{p} bitop3:0x96",
    "v_add_u32 2 vgprs": "v_add_u32_e32 v{n}, v{m}, v{n}",
    "v_cvt_f32_u32": "v_cvt_f32_u32_e32 v{n}, v{n}",
    "v_mul_f32_e32": "v_mul_f32_e32 v{n}, v4, v{n}",
    "v_fma_f64": "v_fma_f64 v[{a}:{b}], v[{a}:{b}], v[4:5], v[6:7]",
    "v_lshrrev_b64": "v_lshrrev_b64 v[{a}:{b}], 7, v[{a}:{b}]",
    "v_pk_mov_b32": "v_pk_mov_b32 v[{a}:{b}], v[4:5], v[{a}:{b}] op_sel:[0,1]",
    "v_bfe_u32": "v_bfe_u32 v{n}, v{n}, 3, 20",
    "v_min3_u32": "v_min3_u32 v{n}, v{n}, v4, v5",
    # left-shift candidates (v_lshlrev_b32 issues in 4 cycles, v_lshrrev_b32 in 2)
    "v_lshlrev_b32 vgpr amt": "v_lshlrev_b32_e32 v{n}, v6, v{n}",
    "v_lshrrev_b32 vgpr amt": "v_lshrrev_b32_e32 v{n}, v6, v{n}",
    "v_ashrrev_i32_e32": "v_ashrrev_i32_e32 v{n}, 7, v{n}",
    "v_lshlrev_b16_e32": "v_lshlrev_b16_e32 v{n}, 7, v{n}",
    "v_lshrrev_b16_e32": "v_lshrrev_b16_e32 v{n}, 7, v{n}",
    "v_add_u16_e32": "v_add_u16_e32 v{n}, v4, v{n}",
    "v_mul_lo_u16_e32": "v_mul_lo_u16_e32 v{n}, v4, v{n}",
    "v_bfrev_b32": "v_bfrev_b32_e32 v{n}, v{n}",
    "v_subrev_u32_e32": "v_subrev_u32_e32 v{n}, v4, v{n}",
    "v_add_u32 sdwa w1": "v_add_u32_sdwa v{n}, v{n}, v{n} dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:DWORD",
    "v_xor_b32 sdwa": "v_xor_b32_sdwa v{n}, v{n}, v4 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD",
    "v_lshlrev_b32 sdwa": "v_lshlrev_b32_sdwa v{n}, v6, v{n} dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:DWORD",
    "v_xor_b32 dpp": "v_xor_b32_dpp v{n}, v{n}, v4 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf",
    "v_mul_f32 imm": "v_mul_f32_e32 v{n}, 0x43000000, v{n}",
    "v_ldexp_f32": "v_ldexp_f32 v{n}, v{n}, 7",
    "v_cndmask_b32 sgpr": "v_cndmask_b32_e64 v{n}, v4, v{n}, s[0:1]",
    "v_max_f32": "v_max_f32_e32 v{n}, v4, v{n}",
    "v_med3_f32": "v_med3_f32 v{n}, v{n}, v4, v5",
    "v_exp_f32": "v_exp_f32_e32 v{n}, v{n}",
}
PAIRED = {"v_fma_f64", "v_lshrrev_b64", "v_pk_mov_b32"}

FAST = "v_xor_b32_e32 v{n}, v4, v{n}"
SLOW = "v_alignbit_b32 v{n}, v{n}, v{n}, 7"
MIX = {  # pattern of F / S over 16 instructions
    "mix F1S1": "FS" * 8,
    "mix F2S2": "FFSS" * 4,
    "mix F4S4": "FFFFSSSS" * 2,
    "mix F8S8": "F" * 8 + "S" * 8,
    "mix F2S1": "FFSFFSFFSFFSFFSF",
    "mix F3S1": "FFFS" * 4,
    "mix F15S1": "F" * 15 + "S",
    "mix F7S1": "FFFFFFFS" * 2,
}


def body_single(tpl, paired):
    lines = []
    if paired:
        for k in range(8):
            a = 8 + 2 * k
            lines.append(tpl.format(a=a, b=a + 1))
    else:
        for k in range(16):
            n = 8 + k
            lines.append(tpl.format(n=n, m=8 + (k + 5) % 16, p=8 + (k + 11) % 16))
    return lines


def body_mix(pat):
    return [(FAST if c == "F" else SLOW).format(n=8 + k) for k, c in enumerate(pat)]


COLS = [(0, 4, 8, 12), (5, 9, 13, 1), (10, 14, 2, 6), (15, 3, 7, 11)]
ROWS = [(0, 1, 2, 3), (5, 6, 7, 4), (10, 11, 8, 9), (15, 12, 13, 14)]
STEPS = [(1, 0, 3, 7), (2, 1, 0, 9), (3, 2, 1, 13), (0, 3, 2, 18)]  # target, x, y, rot: w[t] ^= rotl(w[x] + w[y])


def salsa_round(quads, form):
    v = lambda i: f"v{8 + i}"
    out = []
    for (t, x, y, r) in STEPS:
        for q, quad in enumerate(quads):
            T, U = f"v{24 + q}", f"v{28 + q}"
            a, d, b = quad[x], quad[y], quad[t]
            out.append(f"v_add_u32_e32 {T}, {v(a)}, {v(d)}")
            if form == "ALIGN":
                out.append(f"v_alignbit_b32 {T}, {T}, {T}, {32 - r}")
                out.append(f"v_xor_b32_e32 {v(b)}, {v(b)}, {T}")
            else:
                out.append(f"v_lshlrev_b32_e32 {U}, {r}, {T}")
                out.append(f"v_lshrrev_b32_e32 {T}, {32 - r}, {T}")
                out.append(f"v_bitop3_b32 {v(b)}, {v(b)}, {U}, {T} bitop3:0x96")
    return out


def cstr(lines):
    return " \\\n    ".join('"' + l + '\\n"' for l in lines)


def main():
    with open(OUT, "w") as f:
        f.write("// generated by tools/diag/gen_issue_ub2.py -- do not edit\n")
        names = []
        for i, (name, tpl) in enumerate(SINGLE.items()):
            f.write(f"#define UB_BODY_{i} {cstr(body_single(tpl, name in PAIRED))}\n")
            names.append((name, 8 if name in PAIRED else 16))
        base = len(SINGLE)
        for j, (name, pat) in enumerate(MIX.items()):
            f.write(f"#define UB_BODY_{base + j} {cstr(body_mix(pat))}\n")
            names.append((name, 16))
        f.write(f"#define UB_NSINGLE {len(names)}\n")
        f.write("template <int I> __device__ __forceinline__ void ub_body();\n")
        for i in range(len(names)):
            f.write(f"template <> __device__ __forceinline__ void ub_body<{i}>() {{ asm volatile(UB_BODY_{i} ::: UB_CLOB); }}\n")
        f.write("static const char *UB_NAMES[] = {" + ", ".join(f'"{n}"' for n, _ in names) + "};\n")
        f.write("static const int UB_PER[] = {" + ", ".join(str(p) for _, p in names) + "};\n")
        for form in ("ALIGN", "SHIFT"):
            dr = salsa_round(COLS, form) + salsa_round(ROWS, form)
            f.write(f"#define SALSA_DR_{form} {cstr(dr)}\n")
            f.write(f"#define SALSA_DR_{form}_N {len(dr)}\n")


if __name__ == "__main__":
    main()
