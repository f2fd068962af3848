// cz_kernels.hip -- batched CurveZMQ MESSAGE seal/open kernels for MI355X (gfx950).
//
// Reference path:
//   CurveClientMechanism.encode / CurveServerMechanism.encode
//     (CurveClientMechanism.java:126-163, CurveServerMechanism.java:127-163)
//     -> Curve.afternm (Curve.java:129-137) -> jnacl crypto_box_afternm
//   CurveClientMechanism.decode / CurveServerMechanism.decode
//     (CurveClientMechanism.java:165-224, CurveServerMechanism.java:165-224)
//     -> Curve.openAfternm (Curve.java:139-147) -> jnacl crypto_box_open_afternm
//
// Work mapping: ONE FRAME PER LANE.  A lane walks its frame's Salsa20 blocks in
// order with the 64-byte block state in VGPRs and runs Poly1305 as a serial
// Horner chain, so there are no cross-lane reductions and no r^k tables (the
// Poly1305 key differs per frame, a power table would never amortise).
//
// Memory (measured on MI355X, tools/diag): lane-wise 16-byte loads stream at
// ~4.9 TB/s, but lane-wise 16-byte STORES reach only ~2.8 TB/s because every
// 128-byte line is written piecewise; a store instruction that writes whole,
// aligned 128-byte lines reaches ~4.5 TB/s.  So loads stay lane-wise and the
// output is staged through LDS by an "emitter":
//   EmitLines  (large frames, slot stride % 128 == 0): each lane writes its
//              64-byte chunks into an 8 KiB per-wave LDS line buffer; every 2
//              chunks the wave flushes one full line per frame, 8 frames per
//              store instruction (XOR-swizzled, bank-conflict free both ways);
//   EmitRegion (small frames, 64 slots <= 16 KiB): the wave's whole output
//              region is assembled in LDS and stored with 1 KiB contiguous
//              store instructions;
//   EmitDirect byte-exact per-lane stores (descriptor batches, partial waves,
//              unaligned frames).
// The 33-byte MESSAGE header shift (flags byte + 32-byte NaCl zero prefix) is
// absorbed with v_alignbyte_b32 funnel shifts and a 1-dword (seal) / 8-dword
// (open) carry.
//
// Layout (box coordinates, mlen = 33 + n for a MESSAGE):
//   box[0:32]   = NaCl ZEROBYTES (keystream bytes 0..31 are the Poly1305 key)
//   box[32]     = flags (MORE=1, COMMAND=2),  box[33:33+n] = payload
//   body[i]     = box[i] for i >= 16; body[0:8] = "\x07MESSAGE", body[8:16] = BE64(counter)
//   tag         = Poly1305(box[32:mlen]) stored at body[16:32]
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "cz_device.h"
#include "cz_diag.h"
#include "../../include/curvezmq_mi355x.h"

// The file compiles as one translation unit (CZ_KPART undefined) or as three that build in parallel
// (jeromq_amd/build.py: -DCZ_KPART=1 the uniform seal kernels and launchers, 2 the uniform opens,
// 3 everything else and the run-time knobs); each part instantiates only its own kernels.
#ifndef CZ_KPART
#define CZ_KPART 0
#endif
#define CZ_KPART_HAS(n) (CZ_KPART == 0 || CZ_KPART == (n))

using namespace cz;

namespace {

// MODE_BOX: MESSAGE output (as MODE_ZMQ) from input already in the reference's box layout,
// m = 0^32 || flags || payload (CurveClientMechanism.java:144-153 builds exactly this and hands it
// to Curve.afternm): box blocks are read where they lie, no funnel shift, no carried words.
enum Mode { MODE_ZMQ = 0, MODE_NACL = 1, MODE_BOX = 2 };

// "\x07MESSAGE" as two little-endian words
constexpr u32 HDR0 = 0x53454d07u, HDR1 = 0x45474153u;

constexpr int BLOCK = 256;              // threads per workgroup (4 waves)
// Build-time occupancy knobs (CZ_EXTRA_FLAGS): CZ_UNIFORM_WAVES_PER_EU=n caps the VGPRs of the
// uniform seal/open kernels so that n waves fit per SIMD, CZ_SEG_WAVES_PER_EU=n the segment
// kernel's; CZ_SEAL_WAVES_PER_EU=n sets both.
#ifdef CZ_SEAL_WAVES_PER_EU
#ifndef CZ_UNIFORM_WAVES_PER_EU
#define CZ_UNIFORM_WAVES_PER_EU CZ_SEAL_WAVES_PER_EU
#endif
#ifndef CZ_SEG_WAVES_PER_EU
#define CZ_SEG_WAVES_PER_EU CZ_SEAL_WAVES_PER_EU
#endif
#endif
#ifdef CZ_UNIFORM_WAVES_PER_EU
#define CZ_OCC __attribute__((amdgpu_waves_per_eu(CZ_UNIFORM_WAVES_PER_EU, CZ_UNIFORM_WAVES_PER_EU)))
#else
#define CZ_OCC
#endif
// k_seal_segments_lines: 3 waves per SIMD unless CZ_SEG_LINES_WAVES_PER_EU says otherwise
#ifndef CZ_SEG_LINES_WAVES_PER_EU
#define CZ_SEG_LINES_WAVES_PER_EU 3
#endif
#define CZ_SEG_LINES_OCC __attribute__((amdgpu_waves_per_eu(CZ_SEG_LINES_WAVES_PER_EU, CZ_SEG_LINES_WAVES_PER_EU)))
// k_open_segments: 3 waves per SIMD (left alone, the funnelled EmitShiftLines path took it to
// 178 VGPRs, 2 waves)
#ifndef CZ_OPEN_SEG_WAVES_PER_EU
#define CZ_OPEN_SEG_WAVES_PER_EU 3
#endif
#define CZ_OPEN_SEG_OCC __attribute__((amdgpu_waves_per_eu(CZ_OPEN_SEG_WAVES_PER_EU, CZ_OPEN_SEG_WAVES_PER_EU)))
#ifndef CZ_UNIFORM_WAVES_PER_EU
#define CZ_OPEN_UNI_OCC __attribute__((amdgpu_waves_per_eu(3)))
#else
#define CZ_OPEN_UNI_OCC
#endif
// k_open_uniform_carry: two aligned lines carried per lane (64 VGPRs) -- 2 waves per SIMD
#ifndef CZ_OPEN_CARRY_WAVES_PER_EU
#define CZ_OPEN_CARRY_WAVES_PER_EU 2
#endif
#define CZ_OPEN_CARRY_OCC __attribute__((amdgpu_waves_per_eu(CZ_OPEN_CARRY_WAVES_PER_EU, CZ_OPEN_CARRY_WAVES_PER_EU)))
#ifdef CZ_SEG_WAVES_PER_EU
#define CZ_SEG_OCC __attribute__((amdgpu_waves_per_eu(CZ_SEG_WAVES_PER_EU, CZ_SEG_WAVES_PER_EU)))
#else
#define CZ_SEG_OCC
#endif
constexpr int WAVES = BLOCK / 64;
constexpr u32 LINE_LDS_BYTES = 64 * 128; // EmitLines: one 128-byte line per frame
constexpr u32 HOLD_LDS_BYTES = 64 * 64;  // EmitLines (seal): block 1 of every frame, until tag()
constexpr u32 REGION_MAX = 16384;       // EmitRegion: 64 slots per wave

struct V4 {
    u32 x, y, z, w;
};

__device__ __forceinline__ V4 zero4() { return V4{0u, 0u, 0u, 0u}; }

// Byte-granular pieces of a 16-byte unit.  gfx950 executes unaligned global and LDS
// accesses (the compiler emits them for align-1 types), so a clipped edge unit leaves in at
// most 4 stores (8, 4, 2, 1 bytes) instead of a byte loop.
typedef uint64_t u64_ua __attribute__((aligned(1)));
typedef uint32_t u32_ua __attribute__((aligned(1)));
typedef uint16_t u16_ua __attribute__((aligned(1)));
struct __attribute__((packed)) U16ua {
    uint4 v;
};

// Stores through pointers rebuilt from integers (ds_bpermute'd bases, SGPR line bases) would
// compile to flat_* instructions, which also count against lgkmcnt: every LDS wait of an
// emitter would then wait for them too.  These go out as global_* stores.
typedef unsigned v4u_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) v4u_t g_uint4;
typedef __attribute__((address_space(1))) uint8_t g_u8;
typedef __attribute__((address_space(1))) u64_ua g_u64_ua;
typedef __attribute__((address_space(1))) u32_ua g_u32_ua;
typedef __attribute__((address_space(1))) u16_ua g_u16_ua;
typedef v4u_t v4u_ua __attribute__((aligned(1)));
typedef uint4 u4_a4 __attribute__((aligned(4)));  // a 16-byte load from a dword-aligned address
typedef __attribute__((address_space(1))) v4u_ua g_v4u_ua;

// Cache policy of the line stores (gfx940 encoding: 1 sc0, 2 nt, 16 sc1).  Seal emitters store
// non-temporal: interleaved A/B, Zipf seal +1.4%, dense seal +1.9%, headline +0.3%; the open's
// 4 KiB plaintext slots lose 1.4% with it and keep the default.
#ifndef CZ_SEAL_STORE_CPOL
#define CZ_SEAL_STORE_CPOL 2
#endif
#ifndef CZ_OPEN_STORE_CPOL
#define CZ_OPEN_STORE_CPOL 0
#endif
// opens of bodies off 16-byte alignment, of plaintext at any byte offset, and of segments: nt
// (dense open +2.2%, Zipf open +1.5% / +2.1% at the 8-byte table; the aligned open into 4 KiB
// plaintext slots and the carried-line open keep the default: -0.7..-1.4% / +-0 with nt)
#ifndef CZ_OPEN_ANY_STORE_CPOL
#define CZ_OPEN_ANY_STORE_CPOL 2
#endif
// 16-byte line store through a buffer resource: `base` wave-uniform (SGPRs), `voff` this lane's
// 32-bit offset, soffset the constant 0.  Never give these stores a REGISTER soffset: LLVM's
// hazard recognizer assumes a MUBUF store with a register soffset has no store-data hazard and
// lets the next VALU rewrite the data VGPRs right behind the store, and on gfx950 the store then
// writes the new value (round 3: one dword per 16 bytes replaced by an LDS address, a few lines
// per 2^20-frame Zipf batch).  With soffset 0 it inserts the wait state, and
// tests/test_isa_hazards.py checks the listing for any MUBUF store with a register soffset.
template <int CP = CZ_OPEN_STORE_CPOL>
__device__ __forceinline__ void buf_store16(u64 base, u32 voff, uint4 v)
{
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>((uintptr_t)base), 0, (int)0xffffffffu, 0x00020000);
    CZ_DIAG_STORE_GUARD(v)  // (cz_diag.h: compiled out of the product library)
    __builtin_amdgcn_raw_buffer_store_b128(v4u_t{v.x, v.y, v.z, v.w}, rs, (int)voff, 0, CP);
}

// wave-uniform copy of a 64-bit value (each half through u32: readfirstlane returns int, and a low
// half with bit 31 set would sign-extend over the high one)
__device__ __forceinline__ u64 uniform64(u64 v)
{
    return ((u64)(u32)__builtin_amdgcn_readfirstlane((u32)(v >> 32)) << 32) |
           (u64)(u32)__builtin_amdgcn_readfirstlane((u32)v);
}

// store bytes [a, b) (0 <= a <= b <= 16) of the unit v whose byte 0 belongs at p
__device__ void st_range16(uint8_t *p, uint4 v, u32 a, u32 b)
{
    if (b <= a)
        return;
    u64 lo = ((u64)v.y << 32) | v.x, hi = ((u64)v.w << 32) | v.z;
    if (a >= 8u) {
        lo = hi >> (8u * (a - 8u));
        hi = 0;
    } else if (a) {
        lo = (lo >> (8u * a)) | (hi << (64u - 8u * a));
        hi >>= 8u * a;
    }
    uint8_t *q = p + a;
    const u32 n = b - a;
    if (n == 16u) {
        reinterpret_cast<U16ua *>(q)->v = v;
        return;
    }
    if (n & 8u) {
        *reinterpret_cast<u64_ua *>(q) = lo;
        q += 8;
        lo = hi;
    }
    if (n & 4u) {
        *reinterpret_cast<u32_ua *>(q) = (u32)lo;
        q += 4;
        lo >>= 32;
    }
    if (n & 2u) {
        *reinterpret_cast<u16_ua *>(q) = (uint16_t)lo;
        q += 2;
        lo >>= 16;
    }
    if (n & 1u)
        *q = (uint8_t)lo;
}

// Load 16 bytes from p.  avail = bytes of the object remaining at p.
// AL: p is 16-byte aligned, so reading the whole aligned chunk once any byte of
// it is valid cannot cross a page; bytes past the object are ignored by callers.
template <bool AL>
__device__ __forceinline__ V4 ld16(const uint8_t *__restrict__ p, u64 avail)
{
    if (avail == 0)
        return zero4();
    if constexpr (AL) {
        uint4 v = *reinterpret_cast<const uint4 *>(p);
        return V4{v.x, v.y, v.z, v.w};
    } else {
        if (avail >= 16u) {  // every byte valid: one unaligned load (cannot touch an unmapped page)
            const uint4 v = reinterpret_cast<const U16ua *>(p)->v;
            return V4{v.x, v.y, v.z, v.w};
        }
        u32 w[4] = {0u, 0u, 0u, 0u};
        u32 lim = avail < 16 ? (u32)avail : 16u;
        for (u32 i = 0; i < lim; i++)
            w[i >> 2] |= (u32)p[i] << (8 * (i & 3));
        return V4{w[0], w[1], w[2], w[3]};
    }
}

template <bool AL>
__device__ __forceinline__ u32 ld32(const uint8_t *__restrict__ p)
{
    if constexpr (AL)
        return *reinterpret_cast<const u32 *>(p);
    else
        return (u32)p[0] | ((u32)p[1] << 8) | ((u32)p[2] << 16) | ((u32)p[3] << 24);
}

// Unguarded full-chunk load (caller proved all 16 bytes valid).
template <bool AL>
__device__ __forceinline__ V4 ld16f(const uint8_t *__restrict__ p)
{
    if constexpr (AL) {
        uint4 v = *reinterpret_cast<const uint4 *>(p);
        return V4{v.x, v.y, v.z, v.w};
    } else {
        return ld16<false>(p, 16);
    }
}

// 8-byte aligned input (the open of bodies packed at 8-byte offsets): a
// 16-byte chunk as two naturally aligned 8-byte loads.  ld16_8 reads the second half only when the
// object reaches into it (an aligned 8-byte piece holding a valid byte cannot cross a page).
// the seal's payload loads (non-temporal loads measured -27..-35% on every seal: DESIGN.md section 6)
template <bool AL>
__device__ __forceinline__ V4 ld16f_in(const uint8_t *__restrict__ p)
{
    return ld16f<AL>(p);
}
__device__ __forceinline__ V4 ld16f_8(const uint8_t *__restrict__ p)
{
    const uint2 a = reinterpret_cast<const uint2 *>(p)[0], b = reinterpret_cast<const uint2 *>(p)[1];
    return V4{a.x, a.y, b.x, b.y};
}
__device__ __forceinline__ V4 ld16_8(const uint8_t *__restrict__ p, u64 avail)
{
    if (avail == 0)
        return zero4();
    const uint2 a = reinterpret_cast<const uint2 *>(p)[0];
    const uint2 b = avail > 8u ? reinterpret_cast<const uint2 *>(p)[1] : make_uint2(0u, 0u);
    return V4{a.x, a.y, b.x, b.y};
}

template <bool AL>
__device__ __forceinline__ void st16(uint8_t *__restrict__ p, u32 a, u32 b, u32 c, u32 d)
{
    if constexpr (AL) {
        *reinterpret_cast<uint4 *>(p) = make_uint4(a, b, c, d);
    } else {
        reinterpret_cast<U16ua *>(p)->v = make_uint4(a, b, c, d);
    }
}

// Store the first nb (0..16) bytes of a 16-byte chunk.
__device__ __forceinline__ void st_bytes(uint8_t *__restrict__ p, u32 a, u32 b, u32 c, u32 d, u32 nb)
{
    st_range16(p, make_uint4(a, b, c, d), 0u, nb);
}

__device__ __forceinline__ u32 funnel(u32 hi, u32 lo, u32 sh) { return __builtin_amdgcn_alignbyte(hi, lo, sh); }

// keep the first `valid` bytes (0..64) of a 64-byte chunk, zero the rest
__device__ __forceinline__ void mask_chunk(u32 D[16], u32 valid)
{
#pragma unroll
    for (int k = 0; k < 16; k++) {
        int rel = (int)valid - 4 * k;
        u32 keep = rel >= 4 ? 0xffffffffu : (rel <= 0 ? 0u : ((1u << (8 * rel)) - 1u));
        D[k] &= keep;
    }
}

// ---------------------------------------------------------------------------
// Emitters.  A frame's output arrives as 64-byte chunks q = 0, 1, 2, ... (bytes
// [64q, 64q+64) of the output object, `total` bytes long).  Bytes >= total in
// the last chunk are don't-care in D.  tag() (seal only) writes output bytes
// 16..31 after the chunk stream; chunk 0 carries zeros there.
// ---------------------------------------------------------------------------
template <bool AL>
struct EmitDirect {
    static constexpr bool cooperative = false;
    uint8_t *dst;
    u32 total;

    __device__ __forceinline__ void emit(u32 q, const u32 D[16])
    {
        const u32 base = 64u * q;
        uint8_t *p = dst + base;
        if (base + 64u <= total) {
            st16<AL>(p, D[0], D[1], D[2], D[3]);
            st16<AL>(p + 16, D[4], D[5], D[6], D[7]);
            st16<AL>(p + 32, D[8], D[9], D[10], D[11]);
            st16<AL>(p + 48, D[12], D[13], D[14], D[15]);
        } else {
#pragma unroll
            for (int c = 0; c < 4; c++) {
                u32 s = base + 16u * c;
                if (s < total) {
                    u32 nb = total - s;
                    if (nb >= 16)
                        st16<AL>(dst + s, D[4 * c], D[4 * c + 1], D[4 * c + 2], D[4 * c + 3]);
                    else
                        st_bytes(dst + s, D[4 * c], D[4 * c + 1], D[4 * c + 2], D[4 * c + 3], nb);
                }
            }
        }
    }
    // chunk q lies entirely inside the object (64q + 64 <= total): no tail handling
    __device__ __forceinline__ void emit_full(u32 q, const u32 D[16])
    {
        uint8_t *p = dst + 64u * q;
        st16<AL>(p, D[0], D[1], D[2], D[3]);
        st16<AL>(p + 16, D[4], D[5], D[6], D[7]);
        st16<AL>(p + 32, D[8], D[9], D[10], D[11]);
        st16<AL>(p + 48, D[12], D[13], D[14], D[15]);
    }
    __device__ __forceinline__ void tag(const u32 t[4]) { st16<AL>(dst + 16, t[0], t[1], t[2], t[3]); }
    __device__ __forceinline__ void finish() {}
    __device__ __forceinline__ void close(bool bad)
    {
        if (bad)
            poison();
    }
    __device__ void poison()
    {
        for (u32 o = 0; o < total; o += 16) {
            u32 nb = total - o < 16 ? total - o : 16;
            if (nb == 16)
                st16<AL>(dst + o, 0u, 0u, 0u, 0u);
            else
                st_bytes(dst + o, 0u, 0u, 0u, 0u, nb);
        }
    }
};

// Whole-line staging for a full wave of equal-length frames whose slots are
// 128-byte multiples (stride % 128 == 0, base 16-byte aligned).  Each frame
// owns its slot: bytes of the last line beyond `total` are written as zero.
template <int CP>
struct EmitLinesT {
    static constexpr bool cooperative = true;  // every lane of the wave must run the same chunk sequence
    uint4 *lds;        // this wave's 64 x 8 chunks
    uint8_t *wbase;    // slot of frame 0 of this wave
    uint8_t *mine;     // this lane's slot
    u64 stride;
    u32 lane, total, last_q;
    bool tag_slot;     // seal: line 0 (header, nonce, tag, first 96 ciphertext bytes) leaves whole in tag()
    uint4 *hold;       // seal: this wave's 64 x 64 bytes, block 1 of every frame
    u32 head[12];      // seal: block 0's words 0..3 and 8..15
    u32 tagw[4];       // seal: the tag, staged with line 0 by close()

    __device__ __forceinline__ void flush(u32 line, bool whole = false)
    {
        const u32 c = lane & 7u;
        const u32 r = lane >> 3;
        // A buffer store (buf_store16): the j-th frame group's line base lb + j * 8 * stride in
        // the resource (SGPRs, advanced by the scalar unit), this lane's 32-bit offset in a VGPR
        // computed once -- no VALU address arithmetic at all per store (plain C stores cost a
        // v_lshl_add_u64 each, +8 VALU and 16 VGPRs per block pair).  It is a compiler builtin,
        // not inline asm, so the backend counts the store's wait states itself (round 2's asm
        // store was outside its hazard recognizer, and a rescheduled Poly1305 v_mad_u64_u32
        // rewrote one store's data VGPRs one state after issue: DESIGN.md section 6).  The
        // launcher keeps 64 * stride < 2^31.
        const u64 lb = uniform64((u64)(uintptr_t)wbase) + 128ull * line;
        const u32 voff = r * (u32)stride + 16u * c;
        const u32 step = 8u * (u32)stride;
        // seal: line 0 leaves whole from close(), one full 128-byte line written once, not a
        // 112-byte line and a late 16-byte tag (partial lines cost L2 fills)
        const bool skip = tag_slot && line == 0 && !whole;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the other lanes' ds_writes of this line
#pragma unroll
        for (u32 j = 0; j < 8; j++) {
            const u32 F = 8u * j + r;
            uint4 v = lds[F * 8u + (c ^ (F & 7u))];
            if (!skip)
                buf_store16<CP>(lb + (u64)(j * step), voff, v);
        }
    }
    __device__ __forceinline__ void emit(u32 q, const u32 Din[16])
    {
        u32 D[16];
#pragma unroll
        for (int k = 0; k < 16; k++)
            D[k] = Din[k];
        if (64u * q + 64u > total)
            mask_chunk(D, total > 64u * q ? total - 64u * q : 0u);
        emit_full(q, D);
    }
    // chunk q lies entirely inside the object: no masking, so no branch (and no register
    // copies merging masked and unmasked chunks) between the producer and the LDS writes
    __device__ __forceinline__ void emit_full(u32 q, const u32 D[16])
    {
        if (tag_slot && q == 0u) {
#pragma unroll
            for (int k = 0; k < 4; k++)
                head[k] = D[k];
#pragma unroll
            for (int k = 0; k < 8; k++)
                head[4 + k] = D[8 + k];
        }
        if (tag_slot && q == 1u) {
#pragma unroll
            for (u32 c = 0; c < 4; c++)
                hold[lane * 4u + c] = make_uint4(D[4 * c], D[4 * c + 1], D[4 * c + 2], D[4 * c + 3]);
        }
        const u32 h = q & 1u;
        const u32 sw = lane & 7u;
#pragma unroll
        for (u32 c = 0; c < 4; c++)
            lds[lane * 8u + ((4u * h + c) ^ sw)] = make_uint4(D[4 * c], D[4 * c + 1], D[4 * c + 2], D[4 * c + 3]);
        if (h)
            flush(q >> 1);
        last_q = q;
    }
    __device__ __forceinline__ void tag(const u32 t[4])
    {
#pragma unroll
        for (int k = 0; k < 4; k++)
            tagw[k] = t[k];
    }
    // seal, converged, after the last line's flush: line 0 = block 0 (header, nonce, tag,
    // 32 ciphertext bytes) + block 1 (held in LDS; zero if the frame has one block), staged
    // and written with the same full-line stores as every other line
    __device__ __forceinline__ void line0()
    {
        const u32 sw = lane & 7u;
        const bool one = last_q == 0u;
        uint4 b1[4];
#pragma unroll
        for (u32 c = 0; c < 4; c++)
            b1[c] = one ? make_uint4(0u, 0u, 0u, 0u) : hold[lane * 4u + c];
        lds[lane * 8u + (0u ^ sw)] = make_uint4(head[0], head[1], head[2], head[3]);
        lds[lane * 8u + (1u ^ sw)] = make_uint4(tagw[0], tagw[1], tagw[2], tagw[3]);
        lds[lane * 8u + (2u ^ sw)] = make_uint4(head[4], head[5], head[6], head[7]);
        lds[lane * 8u + (3u ^ sw)] = make_uint4(head[8], head[9], head[10], head[11]);
#pragma unroll
        for (u32 c = 0; c < 4; c++)
            lds[lane * 8u + ((4u + c) ^ sw)] = b1[c];
        flush(0, true);
    }
    __device__ __forceinline__ void finish()
    {
        if ((last_q & 1u) == 0) {
            const u32 sw = lane & 7u;
#pragma unroll
            for (u32 c = 4; c < 8; c++)
                lds[lane * 8u + (c ^ sw)] = make_uint4(0u, 0u, 0u, 0u);
            flush(last_q >> 1);
        }
    }
    // converged: flush the last line (and the seal's line 0), then zero rejected frames' slots
    __device__ __forceinline__ void close(bool bad)
    {
        finish();
        if (tag_slot)
            line0();
        if (bad)
            poison();
    }
    __device__ void poison()
    {
        // the plaintext already left through other lanes' stores: make this lane's zeros land after them
        __threadfence_block();
        for (u32 o = 0; o < total; o += 16)
            *reinterpret_cast<uint4 *>(mine + o) = make_uint4(0u, 0u, 0u, 0u);
    }
};
using EmitLines = EmitLinesT<CZ_OPEN_STORE_CPOL>;
using EmitLinesSeal = EmitLinesT<CZ_SEAL_STORE_CPOL>;


// Whole-region staging for a full wave of small equal-length frames: the wave's
// 64 slots (64 * stride <= REGION_MAX, stride % 16 == 0) are assembled in LDS
// and written with contiguous 1 KiB store instructions.  Slot bytes beyond
// `total` are written as zero.
template <int CP>
struct EmitRegionT {
    static constexpr bool cooperative = true;
    uint4 *lds;        // 64 * stride bytes
    uint8_t *wbase;
    u32 stride, lane, total;

    __device__ __forceinline__ void emit(u32 q, const u32 Din[16])
    {
        u32 D[16];
#pragma unroll
        for (int k = 0; k < 16; k++)
            D[k] = Din[k];
        if (64u * q + 64u > total)
            mask_chunk(D, total > 64u * q ? total - 64u * q : 0u);
        const u32 base = (lane * stride + 64u * q) >> 4;
#pragma unroll
        for (u32 c = 0; c < 4; c++)
            if (64u * q + 16u * c < stride)
                lds[base + c] = make_uint4(D[4 * c], D[4 * c + 1], D[4 * c + 2], D[4 * c + 3]);
    }
    __device__ __forceinline__ void emit_full(u32 q, const u32 D[16])
    {
        const u32 base = (lane * stride + 64u * q) >> 4;  // 64q + 64 <= total <= stride
#pragma unroll
        for (u32 c = 0; c < 4; c++)
            lds[base + c] = make_uint4(D[4 * c], D[4 * c + 1], D[4 * c + 2], D[4 * c + 3]);
    }
    __device__ __forceinline__ void tag(const u32 t[4]) { lds[(lane * stride + 16u) >> 4] = make_uint4(t[0], t[1], t[2], t[3]); }
    __device__ __forceinline__ void finish()
    {
        // zero this slot's chunks after the last emitted one
        const u32 done = ((total + 63u) & ~63u) < stride ? ((total + 63u) & ~63u) : stride;
        for (u32 o = done; o < stride; o += 16u)
            lds[(lane * stride + o) >> 4] = make_uint4(0u, 0u, 0u, 0u);
        const u32 n16 = (64u * stride) >> 4;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the other lanes' ds_writes of the region
        for (u32 k = lane; k < n16; k += 64u) {
            const uint4 v = lds[k];
            if constexpr (CP == 2)
                __builtin_nontemporal_store(v4u_t{v.x, v.y, v.z, v.w}, reinterpret_cast<v4u_t *>(wbase) + k);
            else
                reinterpret_cast<uint4 *>(wbase)[k] = v;
        }
    }
    // zero a rejected frame's slot in LDS (per lane), then the converged region store
    __device__ __forceinline__ void close(bool bad)
    {
        if (bad)
            poison();
        finish();
    }
    __device__ void poison()
    {
        for (u32 o = 0; o < stride; o += 16u)
            lds[(lane * stride + o) >> 4] = make_uint4(0u, 0u, 0u, 0u);
    }
};
using EmitRegion = EmitRegionT<CZ_OPEN_STORE_CPOL>;
using EmitRegionSeal = EmitRegionT<CZ_SEAL_STORE_CPOL == 2 ? 2 : 0>;

// --------------------------------------------------------------------------
// SEAL one frame.
//   MODE_ZMQ : in = payload (n bytes), output = MESSAGE body (33 + n bytes)
//   MODE_NACL: in = m (n = mlen bytes, m[0:32] ignored), output = c (mlen bytes)
// key = Salsa20 subkey (HSalsa20 already applied), nonce words from `counter`
// (ZMQ: BE64 counter; NaCl: the caller passes n[16:24] read big-endian).
// --------------------------------------------------------------------------
// UN0: the caller guarantees that the high nonce word (bswap of the counter's top
// 32 bits) and the key are the same in every lane of the wave.  With the block
// counter also wave-uniform, only state word 7 is per-lane when a block starts,
// and the compiler's uniformity analysis moves everything that does not depend
// on it -- 3 of the 4 first column quarter-rounds and 1 of the first row
// quarter-rounds -- to the scalar unit (about 60 of the block's 960 VALU ops).
// INA (MODE_ZMQ): the payload's alignment class.  16: 16-byte aligned (AL as given); 8 / 1 (AL
// true): payloads at 8-byte / any byte offsets (messages packed back to back), read from the
// first dword boundary at or above the payload, `in + d` (d = -in & 3), with 16-byte loads.
// The box funnel then shifts by sh = (in + 3) & 3 instead of 3, and the dword before the window,
// P[-1] (flags << 24 for aligned payloads), holds the flags byte at byte sh and the first d
// payload bytes above it.  Same VALU count as the aligned kernel.
template <int MODE, bool AL, class EM, bool PAIR = false, bool UN0 = false, bool LAZY = true, int INA = 16>
__device__ __forceinline__ void seal_frame(const uint8_t *__restrict__ in0, u32 n, u32 flags, u64 counter,
                                           const u32 key[8], EM &em)
{
    static_assert(INA == 16 || (MODE == MODE_ZMQ && AL), "INA 8/1: MESSAGE seal on the AL code paths");
    const u32 ina_a = INA == 1 ? (u32)(uintptr_t)in0 & 3u : 0u;
    const u32 ina_d = (4u - ina_a) & 3u;
    const uint8_t *__restrict__ in = in0 + ina_d;  // dword-aligned for INA 8/1
    const u32 sh = ina_a ? ina_a - 1u : 3u;
    u32 pm1 = flags << 24;  // P[-1]
    if constexpr (INA == 1) {
        if (ina_a) {
            const u32 r = *reinterpret_cast<const u32 *>(in0 - ina_a);
            pm1 = (r & ~(0xffu << (8u * sh))) | (flags << (8u * sh));
        }
    }
    auto ldF = [&](const uint8_t *p) -> V4 {  // all 16 bytes inside the payload
        if constexpr (INA == 16) {
            return ld16f_in<AL>(p);
        } else {
            const uint4 r = *reinterpret_cast<const u4_a4 *>(p);
            return V4{r.x, r.y, r.z, r.w};
        }
    };
    auto ldP = [&](const uint8_t *p, u64 avail) -> V4 {  // avail bytes inside the payload
        if constexpr (INA == 16)
            return ld16<AL>(p, avail);
        else
            return avail >= 16u ? ldF(p) : ld16<false>(p, avail);
    };
    // ZMQ funnel: box dword k of block b = alignbyte(P[16b+k-8], P[16b+k-9], 3)
    // where P[i] is payload dword i; block b's window is P[16b-8 .. 16b+7]
    // (payload bytes [64b-32, 64b+32)) and P[16b-9] is carried from block b-1.
    // MODE_BOX: n = payload bytes, `in` = the box (mlen bytes; box bytes 0..31 are not read, the
    // flags byte is box byte 32 and `flags` is ignored)
    const u32 mlen = (MODE == MODE_ZMQ || MODE == MODE_BOX) ? n + 33u : n;
    const u32 nfull = mlen >> 6;
    const u32 tailv = mlen & 63u;
    // bytes from `in`; a payload shorter than d lies wholly in P[-1] (pm1)
    const u64 inlen = MODE == MODE_BOX ? (u64)mlen : (n > ina_d ? (u64)(n - ina_d) : 0ull);
    u32 n0, n1;
    counter_nonce(counter, n0, n1);
    if constexpr (UN0)
        n0 = __builtin_amdgcn_readfirstlane(n0);

    // keystream block c0 (c1 = 0): UN0 kernels take rounds 1-2 from the per-frame words
    [[maybe_unused]] SalsaFrame sf{};
    if constexpr (UN0 && LAZY)
        sf = salsa_frame(key, n0, n1);
    auto ksblock = [&](u32 *xs, u32 c0, u32 c1) {
        if constexpr (UN0 && LAZY)
            salsa20_block_frame(xs, sf, key, n0, n1, c0);
        else
            salsa20_block<LAZY>(xs, key, n0, n1, c0, c1);
    };
    // keystream words 0..3 of block c0 only (a last block with <= 16 box bytes)
    auto ksblock_w03 = [&](u32 *xs, u32 c0) {
        if constexpr (UN0 && LAZY)
            salsa20_block_frame_w03(xs, sf, key, n0, n1, c0);
        else
            salsa20_block_w03<LAZY>(xs, key, n0, n1, c0, 0u);
    };
    u32 x[16], C[16];
    ksblock(x, 0u, 0u);
    Poly P;
    poly_init(P, x[0], x[1], x[2], x[3], x[4], x[5], x[6], x[7]);

    // ZMQ, one full block b >= 1 from its 17-dword window W = P[16b-9 .. 16b+7]; STEADY: a block of
    // the pair loop (b >= 2), emitted through the emitter's steady-state form if it has one
    auto zmq_block = [&](u32 blk, const u32 *W, auto steady) {
        ksblock(x, blk, 0u);
#pragma unroll
        for (int k = 0; k < 16; k++)
            C[k] = funnel(W[k + 1], W[k], sh) ^ x[k];
        poly_block(P, C[0], C[1], C[2], C[3], 1u);
        poly_block(P, C[4], C[5], C[6], C[7], 1u);
        poly_block(P, C[8], C[9], C[10], C[11], 1u);
        poly_block(P, C[12], C[13], C[14], C[15], 1u);
        if constexpr (decltype(steady)::value)
            emit_steady(em, blk, C);
        else
            em.emit_full(blk, C);
    };
    auto zmq_full_block = [&](u32 blk, const u32 *W) { zmq_block(blk, W, std::false_type{}); };

    // box-aligned input, one full block b >= 1 from its 16 dwords
    [[maybe_unused]] auto box_full_block = [&](u32 blk, const u32 *W) {
        ksblock(x, blk, 0u);
#pragma unroll
        for (int k = 0; k < 16; k++)
            C[k] = W[k] ^ x[k];
        poly_block(P, C[0], C[1], C[2], C[3], 1u);
        poly_block(P, C[4], C[5], C[6], C[7], 1u);
        poly_block(P, C[8], C[9], C[10], C[11], 1u);
        poly_block(P, C[12], C[13], C[14], C[15], 1u);
        em.emit_full(blk, C);
    };

    u32 carry = 0;
    u32 blk = 1;
    if constexpr (MODE == MODE_BOX && AL && PAIR) {
        // Whole-line input straight from the box: line k = box blocks 2k and 2k+1 (line 0: bytes
        // 32..63 of block 0 and block 1), 8 back-to-back loads per line, nothing carried.
        u32 L[32];
#pragma unroll
        for (int c = 2; c < 8; c++) {
            V4 v = ld16<AL>(in + 16 * c, inlen > 16u * c ? inlen - 16u * c : 0);
            L[4 * c] = v.x; L[4 * c + 1] = v.y; L[4 * c + 2] = v.z; L[4 * c + 3] = v.w;
        }
#pragma unroll
        for (int k = 8; k < 16; k++)
            C[k] = L[k] ^ x[k];
        C[0] = HDR0; C[1] = HDR1; C[2] = n0; C[3] = n1;
        C[4] = C[5] = C[6] = C[7] = 0u;
        if (nfull >= 1) {
            poly_block(P, C[8], C[9], C[10], C[11], 1u);
            poly_block(P, C[12], C[13], C[14], C[15], 1u);
        } else {
            const u32 nb = mlen - 32u;
            if (nb >= 16u) {
                poly_block(P, C[8], C[9], C[10], C[11], 1u);
                if (nb > 16u)
                    poly_block_partial(P, C[12], C[13], C[14], C[15], nb - 16u);
            } else {
                poly_block_partial(P, C[8], C[9], C[10], C[11], nb);
            }
        }
        em.emit(0, C);
        if (nfull >= 2) {
            box_full_block(1, L + 16);
            for (u32 k = 1; 2u * k + 1u < nfull; k++) {
                const uint8_t *src = in + 128u * k;
#pragma unroll
                for (int c = 0; c < 8; c++) {
                    V4 v = ld16f_in<AL>(src + 16 * c);
                    L[4 * c] = v.x; L[4 * c + 1] = v.y; L[4 * c + 2] = v.z; L[4 * c + 3] = v.w;
                }
                // (The scheduler sinks each of these loads to just before its first use, with a vmcnt(0)
                // behind it, so a line is read in pieces and L2 re-fetches it: FETCH 1.20x the box
                // bytes.  A sched_barrier here keeps the 8 loads together and the first wait ~1570
                // instructions later -- and measured 14% SLOWER (interleaved A/B).)
                box_full_block(2u * k, L);
                box_full_block(2u * k + 1u, L + 16);
                blk = 2u * k + 2u;
            }
            if (blk < 2u)
                blk = 2u;
        } else {
            blk = nfull > 1 ? nfull : 1u;
        }
    } else if constexpr (MODE == MODE_ZMQ && AL && PAIR) {
        // Whole-line input: each lane reads payload line k = [128k, 128k+128) with
        // 8 back-to-back loads and uses it for blocks 2k and 2k+1 (block 2k's
        // window starts 36 bytes into line k-1: a 9-dword carry), so both halves
        // of every 128-byte line are consumed while it is in flight instead of
        // one step (~10 us) apart, which made L2 re-fetch half the lines.
        u32 L[32];
#pragma unroll
        for (int c = 0; c < 8; c++) {
            V4 v = ldP(in + 16 * c, inlen > 16u * c ? inlen - 16u * c : 0);
            L[4 * c] = v.x; L[4 * c + 1] = v.y; L[4 * c + 2] = v.z; L[4 * c + 3] = v.w;
        }
        // block 0
        {
            C[8] = funnel(L[0], pm1, sh) ^ x[8];
#pragma unroll
            for (int k = 9; k < 16; k++)
                C[k] = funnel(L[k - 8], L[k - 9], sh) ^ x[k];
            C[0] = HDR0; C[1] = HDR1; C[2] = n0; C[3] = n1;
            C[4] = C[5] = C[6] = C[7] = 0u;
            if (nfull >= 1) {
                poly_block(P, C[8], C[9], C[10], C[11], 1u);
                poly_block(P, C[12], C[13], C[14], C[15], 1u);
            } else {
                u32 nb = mlen - 32u;
                if (nb >= 16u) {
                    poly_block(P, C[8], C[9], C[10], C[11], 1u);
                    if (nb > 16u)
                        poly_block_partial(P, C[12], C[13], C[14], C[15], nb - 16u);
                } else {
                    poly_block_partial(P, C[8], C[9], C[10], C[11], nb);
                }
            }
            em.emit(0, C);
        }
        carry = L[7];
        if (nfull >= 2) {
            // Chunks 6 and 7 of a line (bytes 96..127) matter only as the carry of the next
            // iteration; past the payload end they are not loaded and the registers keep stale,
            // unused words (no zero fill: -8 v_mov per pair).  (Loading line k + 1 at the end of
            // iteration k, ahead of the line stores, measured 2% slower.)
            auto load_line = [&](u32 k) {
                const uint8_t *src = in + 128u * k;
                const u32 o = 128u * k;
#pragma unroll
                for (int c = 0; c < 6; c++) {
                    V4 v = ldF(src + 16 * c);
                    L[4 * c] = v.x; L[4 * c + 1] = v.y; L[4 * c + 2] = v.z; L[4 * c + 3] = v.w;
                }
#pragma unroll
                for (int c = 6; c < 8; c++) {
                    if (inlen > o + 16u * c) {
                        V4 v = INA == 16 ? ld16f_in<AL>(src + 16 * c) : ldP(src + 16 * c, inlen - o - 16u * c);
                        L[4 * c] = v.x; L[4 * c + 1] = v.y; L[4 * c + 2] = v.z; L[4 * c + 3] = v.w;
                    }
                }
            };
            u32 cy[9];
            zmq_full_block(1, L + 7);
#pragma unroll
            for (int q = 0; q < 9; q++)
                cy[q] = L[23 + q];
            blk = 2;
            for (u32 k = 1; 2u * k + 1u < nfull; k++) {
                load_line(k);
                u32 W[17];
#pragma unroll
                for (int q = 0; q < 9; q++)
                    W[q] = cy[q];
#pragma unroll
                for (int q = 0; q < 8; q++)
                    W[9 + q] = L[q];
                zmq_block(2u * k, W, std::true_type{});
                zmq_block(2u * k + 1u, L + 7, std::true_type{});
#pragma unroll
                for (int q = 0; q < 9; q++)
                    cy[q] = L[23 + q];
                blk = 2u * k + 2u;
            }
            carry = cy[0];  // P[16*blk - 9] for the per-block path below
        } else {
            blk = nfull > 1 ? nfull : 1u;
        }
    } else {
        if constexpr (MODE == MODE_ZMQ) {
            V4 a = ldP(in, inlen);
            V4 b = ldP(in + 16, inlen > 16 ? inlen - 16 : 0);
            u32 W[9] = {pm1, a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};  // P[-1 .. 7]
#pragma unroll
            for (int k = 8; k < 16; k++)
                C[k] = funnel(W[k - 7], W[k - 8], sh) ^ x[k];
            carry = b.w;
            C[0] = HDR0; C[1] = HDR1; C[2] = n0; C[3] = n1;
        } else {
            V4 a = ld16<AL>(in + 32, inlen > 32 ? inlen - 32 : 0);
            V4 b = ld16<AL>(in + 48, inlen > 48 ? inlen - 48 : 0);
            C[8] = a.x ^ x[8]; C[9] = a.y ^ x[9]; C[10] = a.z ^ x[10]; C[11] = a.w ^ x[11];
            C[12] = b.x ^ x[12]; C[13] = b.y ^ x[13]; C[14] = b.z ^ x[14]; C[15] = b.w ^ x[15];
            carry = 0;
            if constexpr (MODE == MODE_BOX) {
                C[0] = HDR0; C[1] = HDR1; C[2] = n0; C[3] = n1;
            } else {
                C[0] = C[1] = C[2] = C[3] = 0u;
            }
        }
        C[4] = C[5] = C[6] = C[7] = 0u;  // tag slot, written by em.tag()
        if (nfull >= 1) {
            poly_block(P, C[8], C[9], C[10], C[11], 1u);
            poly_block(P, C[12], C[13], C[14], C[15], 1u);
        } else {
            if (mlen > 32u) {
                u32 nb = mlen - 32u;
                if (nb >= 16u) {
                    poly_block(P, C[8], C[9], C[10], C[11], 1u);
                    if (nb > 16u)
                        poly_block_partial(P, C[12], C[13], C[14], C[15], nb - 16u);
                } else {
                    poly_block_partial(P, C[8], C[9], C[10], C[11], nb);
                }
            }
        }
        em.emit(0, C);
    }

    // steady state: remaining full 64-byte blocks, all inputs in range
    for (; blk < nfull; blk++) {
        V4 q0, q1, q2, q3;
        if constexpr (MODE == MODE_ZMQ) {
            const uint8_t *src = in + 64u * blk - 32u;
            q0 = ldF(src);
            q1 = ldF(src + 16);
            q2 = ldF(src + 32);
            q3 = ldP(src + 48, inlen - (64u * blk + 16u));  // may end inside this chunk
            u32 W[17] = {carry, q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w,
                         q2.x, q2.y, q2.z, q2.w, q3.x, q3.y, q3.z, q3.w};
            zmq_full_block(blk, W);
            carry = q3.w;
        } else {
            const uint8_t *src = in + 64u * blk;
            q0 = ld16f_in<AL>(src);
            q1 = ld16f_in<AL>(src + 16);
            q2 = ld16f_in<AL>(src + 32);
            q3 = ld16f_in<AL>(src + 48);
            ksblock(x, blk, 0u);
            u32 W[16] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w,
                         q2.x, q2.y, q2.z, q2.w, q3.x, q3.y, q3.z, q3.w};
#pragma unroll
            for (int k = 0; k < 16; k++)
                C[k] = W[k] ^ x[k];
            poly_block(P, C[0], C[1], C[2], C[3], 1u);
            poly_block(P, C[4], C[5], C[6], C[7], 1u);
            poly_block(P, C[8], C[9], C[10], C[11], 1u);
            poly_block(P, C[12], C[13], C[14], C[15], 1u);
            em.emit_full(blk, C);
        }
    }

    // final partial block with at most 16 box bytes (a 100-byte MESSAGE's 133-byte box ends 5
    // bytes into block 2): keystream words 0..3 only, from the tail schedule of rounds 19-20
    if (tailv != 0 && tailv <= 16u && nfull >= 1) {
        const u32 blk = nfull;
        const long o = (MODE == MODE_ZMQ) ? (long)(64u * blk) - 32 : (long)(64u * blk);
        const V4 q = ldP(in + o, (o >= 0 && (u64)o < inlen) ? inlen - (u64)o : 0);
        ksblock_w03(x, blk);
        if constexpr (MODE == MODE_ZMQ) {
            C[0] = funnel(q.x, carry, sh) ^ x[0];
            C[1] = funnel(q.y, q.x, sh) ^ x[1];
            C[2] = funnel(q.z, q.y, sh) ^ x[2];
            C[3] = funnel(q.w, q.z, sh) ^ x[3];
        } else {
            C[0] = q.x ^ x[0]; C[1] = q.y ^ x[1]; C[2] = q.z ^ x[2]; C[3] = q.w ^ x[3];
        }
#pragma unroll
        for (int k = 4; k < 16; k++)
            C[k] = 0u;
        if (tailv == 16u)
            poly_block(P, C[0], C[1], C[2], C[3], 1u);
        else
            poly_block_partial(P, C[0], C[1], C[2], C[3], tailv);
        em.emit(blk, C);
    } else if (tailv != 0 && nfull >= 1) {
        const u32 blk = nfull;
        V4 q[4];
#pragma unroll
        for (int c = 0; c < 4; c++) {
            long o = (MODE == MODE_ZMQ) ? (long)(64u * blk) - 32 + 16 * c : (long)(64u * blk) + 16 * c;
            u64 avail = (o >= 0 && (u64)o < inlen) ? inlen - (u64)o : 0;
            q[c] = ldP(in + o, avail);
        }
        ksblock(x, blk, 0u);
        u32 W[16] = {q[0].x, q[0].y, q[0].z, q[0].w, q[1].x, q[1].y, q[1].z, q[1].w,
                     q[2].x, q[2].y, q[2].z, q[2].w, q[3].x, q[3].y, q[3].z, q[3].w};
        if constexpr (MODE == MODE_ZMQ) {
            C[0] = funnel(W[0], carry, sh) ^ x[0];
#pragma unroll
            for (int k = 1; k < 16; k++)
                C[k] = funnel(W[k], W[k - 1], sh) ^ x[k];
        } else {
#pragma unroll
            for (int k = 0; k < 16; k++)
                C[k] = W[k] ^ x[k];
        }
#pragma unroll
        for (int j = 0; j < 4; j++) {
            u32 s = 16u * j;
            if (s < tailv) {
                u32 nb = tailv - s;
                if (nb >= 16)
                    poly_block(P, C[4 * j], C[4 * j + 1], C[4 * j + 2], C[4 * j + 3], 1u);
                else
                    poly_block_partial(P, C[4 * j], C[4 * j + 1], C[4 * j + 2], C[4 * j + 3], nb);
            }
        }
        em.emit(blk, C);
    }

    u32 tag[4];
    poly_finish(P, tag);
    em.tag(tag);
    em.close(false);
}

// Carry-line input for bodies off 16-byte alignment whose waves share one line phase (the
// phase-sorted open, k_open_uniform_carry).  A body's pair window k -- its bytes [128k, 128k + 128)
// plus the dword after, from the dword-aligned address at or below -- is dwords [s, s + 33) of the
// two aligned 128-byte lines Cur (line k) and Nxt (line k + 1), s = (in4 & 127) / 4 wave-uniform.
// Each aligned line is loaded once, whole, and carried in registers into the next pair, so no line
// is read in two parts a pair apart (L2 re-fetched most of them: FETCH 1.84x the body bytes).
// C[q] = funnel(window[BASE + q + 1], window[BASE + q], ina), q < 16; s selects among 32
// straight-line cases (wave-uniform branch), each with compile-time register indices.
template <int S, int BASE>
__device__ __forceinline__ void carry_window_s(u32 C[16], const u32 Cur[32], const u32 Nxt[32], u32 ina)
{
#pragma unroll
    for (int q = 0; q < 16; q++) {
        const int lo = BASE + q + S, hi = lo + 1;
        const u32 vlo = lo < 32 ? Cur[lo & 31] : Nxt[(lo - 32) & 31];
        const u32 vhi = hi < 32 ? Cur[hi & 31] : Nxt[(hi - 32) & 31];
        C[q] = funnel(vhi, vlo, ina);
    }
}
template <int BASE>
__device__ __forceinline__ void carry_window(u32 C[16], const u32 Cur[32], const u32 Nxt[32], u32 s, u32 ina)
{
    switch (s) {
#define CZ_CW(S) case S: carry_window_s<S, BASE>(C, Cur, Nxt, ina); break;
        CZ_CW(0) CZ_CW(1) CZ_CW(2) CZ_CW(3) CZ_CW(4) CZ_CW(5) CZ_CW(6) CZ_CW(7)
        CZ_CW(8) CZ_CW(9) CZ_CW(10) CZ_CW(11) CZ_CW(12) CZ_CW(13) CZ_CW(14) CZ_CW(15)
        CZ_CW(16) CZ_CW(17) CZ_CW(18) CZ_CW(19) CZ_CW(20) CZ_CW(21) CZ_CW(22) CZ_CW(23)
        CZ_CW(24) CZ_CW(25) CZ_CW(26) CZ_CW(27) CZ_CW(28) CZ_CW(29) CZ_CW(30)
        default: carry_window_s<31, BASE>(C, Cur, Nxt, ina); break;
#undef CZ_CW
    }
}

// --------------------------------------------------------------------------
// OPEN one frame.  Returns a CZ_STATUS_* code; the emitter receives the output:
//   MODE_ZMQ : in = MESSAGE body (size bytes), output = payload (size - 33 bytes);
//              *flags_out = box[32]; *nonce_out = BE64(body[8:16]).
//   MODE_NACL: in = c (size bytes), output = m (size bytes, m[0:32] = 0).
// The replay check of decode (CurveClientMechanism.java:186-193) compares the
// frame nonce against `floor` as signed 64-bit values, like Java's long.
// On a bad tag the emitted plaintext is overwritten with zeros (em.poison()).
// Frames rejected before decryption emit nothing.
// --------------------------------------------------------------------------
// INA: the input's alignment class.  16: 16-byte aligned (AL as given); 8 and 1 (AL true): bodies at
// any byte offset (the dense wire layout, V2Decoder.java:67-105 leaves bodies back to back), read
// with 16-byte loads from the dword-aligned address at or below and, for 1, one
// v_alignbyte_b32 per dword by (in & 3) with the dword after the 16 bytes (loaded only when
// in & 3 != 0); a whole line is 8 such loads plus that dword.  A chunk whose 16 bytes are all in
// the body never reads past the dword holding its last byte (a dword cannot cross a page) nor
// below the body's first dword (the buffer base is dword-aligned).
template <int MODE, bool AL, class EM, bool PAIR = false, bool UN0 = false, bool LAZY = true, int INA = 16,
          bool CARRY = false>
__device__ __forceinline__ u32 open_frame(const uint8_t *__restrict__ in, u32 size, const u32 key[8],
                                          bool check_floor, long long floor, u32 *flags_out, u64 *nonce_out,
                                          u64 nacl_counter, EM &em)
{
    static_assert(INA == 16 || (AL && (INA == 8 || INA == 1)), "INA 8/1 take the AL code paths");
    const u32 ina = INA == 1 ? (u32)(uintptr_t)in & 3u : 0u;
    const uint8_t *in4 = in - ina;
    // the 16 box bytes at `off`, every one inside the body
    auto LF = [&](u32 off) -> V4 {
        if constexpr (INA == 16) {
            return ld16f<AL>(in + off);
        } else {
            const uint4 r = *reinterpret_cast<const u4_a4 *>(in4 + off);
            if constexpr (INA == 8)
                return V4{r.x, r.y, r.z, r.w};
            const u32 r4 = ina ? *reinterpret_cast<const u32 *>(in4 + off + 16) : 0u;
            return V4{funnel(r.y, r.x, ina), funnel(r.z, r.y, ina), funnel(r.w, r.z, ina), funnel(r4, r.w, ina)};
        }
    };
    // the box bytes at `off`, avail of them inside the body
    auto LP = [&](u32 off, u64 avail) -> V4 {
        if constexpr (INA == 16)
            return ld16<AL>(in + off, avail);
        else
            return avail >= 16u ? LF(off) : ld16<false>(in + off, avail);
    };
    // A cooperative emitter needs every lane of the wave in the same chunk
    // sequence: a frame rejected before decryption then runs through the
    // (uniform-size) loop as a dead lane that emits zeros.
    constexpr bool COOP = EM::cooperative;
    u32 early = CZ_STATUS_OK;
    u32 n0, n1;
    if constexpr (MODE == MODE_ZMQ) {
        // Msgs.startsWith(msg, "MESSAGE", true) (zmq/io/Msgs.java:20-39): size >= 8,
        // byte 0 == 7, bytes 1..6 == "MESSAG" (its loop never reaches byte 7).
        V4 h = LP(0, size);
        if (size < 8u || h.x != HDR0 || (h.y & 0x00ffffffu) != (HDR1 & 0x00ffffffu))
            early = CZ_STATUS_COMMAND;
        else if (size < 33u)
            early = CZ_STATUS_MALFORMED;
        n0 = h.z;
        n1 = h.w;
        if (early == CZ_STATUS_OK) {
            u64 nonce = ((u64)bswap32(n0) << 32) | (u64)bswap32(n1);
            *nonce_out = nonce;
            if (check_floor && (long long)nonce <= floor)
                early = CZ_STATUS_SEQUENCE;
        }
    } else {
        if (size < 32u)
            early = CZ_STATUS_MALFORMED;
        counter_nonce(nacl_counter, n0, n1);
    }
    if (early != CZ_STATUS_OK && (!COOP || size < 33u))
        return early;  // cooperative callers only launch uniform sizes >= 33
    const bool dead = early != CZ_STATUS_OK;
    if constexpr (UN0)
        n0 = __builtin_amdgcn_readfirstlane(n0);  // caller checked: same in every lane
    // keystream block c0 (c1 = 0): UN0 kernels take rounds 1-2 from the per-frame words
    [[maybe_unused]] SalsaFrame sf{};
    if constexpr (UN0 && LAZY)
        sf = salsa_frame(key, n0, n1);
    auto ksblock = [&](u32 *xs, u32 c0, u32 c1) {
        if constexpr (UN0 && LAZY)
            salsa20_block_frame(xs, sf, key, n0, n1, c0);
        else
            salsa20_block<LAZY>(xs, key, n0, n1, c0, c1);
    };
    // keystream words 0..3 only (a last block holding <= 16 body bytes: 133-byte bodies of 100-byte
    // MESSAGEs end 5 bytes into block 2); words 4..15 are left unspecified, their bytes masked
    auto ksblock_w03 = [&](u32 *xs, u32 c0) {
        if constexpr (UN0 && LAZY)
            salsa20_block_frame_w03(xs, sf, key, n0, n1, c0);
        else
            salsa20_block_w03<LAZY>(xs, key, n0, n1, c0, 0u);
    };

    const u32 mlen = size;
    const u32 nblk = (mlen + 63u) >> 6;
    const u32 nfull = mlen >> 6;
    const u32 nout = (MODE == MODE_ZMQ) ? size - 33u : size;

    auto emit_open = [&](u32 q, u32 D[16], bool full) {
        if (COOP && dead) {
#pragma unroll
            for (int k = 0; k < 16; k++)
                D[k] = 0u;
        }
        if (full)
            em.emit_full(q, D);  // chunk q inside the output: no masking
        else
            em.emit(q, D);
    };

    // Whole-line input: body line 0 -- tag, block 0 and block 1 -- leaves L2 in ONE burst, before
    // block 0's keystream.  Read as before (block 1's half after block 0, ~6 us later under load)
    // the line was often evicted in between and fetched twice: open FETCH was 1.075x its slot
    // bytes against 1.03x for the seal, whose pair loop already reads whole lines.
    constexpr bool EARLY0 = PAIR && AL && MODE == MODE_ZMQ;
    const bool early0 = EARLY0 && nfull >= 2;
    [[maybe_unused]] V4 e_tin{}, e_a{}, e_b{};
    [[maybe_unused]] u32 L1[16];
    if constexpr (EARLY0) {
        if (early0) {
            e_tin = LF(16);
            e_a = LF(32);
            e_b = LF(48);
#pragma unroll
            for (int c = 0; c < 4; c++) {
                V4 v = LF(64 + 16 * c);
                L1[4 * c] = v.x; L1[4 * c + 1] = v.y; L1[4 * c + 2] = v.z; L1[4 * c + 3] = v.w;
            }
        }
    }
    u32 x[16], C[16], X[16];
    ksblock(x, 0u, 0u);
    Poly P;
    poly_init(P, x[0], x[1], x[2], x[3], x[4], x[5], x[6], x[7]);
    V4 tin = early0 ? e_tin : LP(16, size - 16u);

    // ZMQ: payload chunk m (bytes [64m, 64m+64)) = box [64m+33, 64m+97): dword t is
    // alignbyte(D[16m+t+9], D[16m+t+8], 1), D = plaintext box dwords.  It is emitted
    // after block m+1, from block m's dwords 8..15 (the carry) and block m+1's 0..8.
    u32 K[8];

    // block 0
    {
        V4 a = early0 ? e_a : LP(32, size > 32 ? size - 32u : 0);
        V4 b = early0 ? e_b : LP(48, size > 48 ? size - 48u : 0);
        C[8] = a.x; C[9] = a.y; C[10] = a.z; C[11] = a.w;
        C[12] = b.x; C[13] = b.y; C[14] = b.z; C[15] = b.w;
        if (nfull >= 1) {
            poly_block(P, C[8], C[9], C[10], C[11], 1u);
            poly_block(P, C[12], C[13], C[14], C[15], 1u);
        } else if (mlen > 32u) {
            u32 nb = mlen - 32u;
            if (nb >= 16u) {
                poly_block(P, C[8], C[9], C[10], C[11], 1u);
                if (nb > 16u)
                    poly_block_partial(P, C[12], C[13], C[14], C[15], nb - 16u);
            } else {
                poly_block_partial(P, C[8], C[9], C[10], C[11], nb);
            }
        }
#pragma unroll
        for (int k = 8; k < 16; k++)
            X[k] = C[k] ^ x[k];
        if constexpr (MODE == MODE_ZMQ) {
            *flags_out = X[8] & 0xffu;
#pragma unroll
            for (int k = 0; k < 8; k++)
                K[k] = X[8 + k];
        } else {
#pragma unroll
            for (int k = 0; k < 8; k++)
                X[k] = 0u;
            emit_open(0, X, false);
        }
    }

    // one block b >= 1 whose 64 ciphertext bytes are in C (full: all 64 valid).  drain: every
    // load in flight has landed by now (the block's keystream and MAC took ~1000 VALU); say so
    // before the emit, whose line flush issues stores -- vmcnt counts stores too, so otherwise
    // the next block's first use of the pair's second half waits for those stores to complete.
    // Rf (INA 1): the block's 17 raw dwords from the dword-aligned address below it; the byte
    // funnel into C runs after the keystream, so the wait for the loads comes ~800 VALU after they
    // were issued (funnelled ahead of the keystream, the loads' latency was exposed per pair)
    // fillC (carry path): writes C after the keystream, as Rf does
    auto open_block_f = [&](u32 blk, bool full, bool drain, const u32 *Rf, auto &&fillC) {
        if (!full && mlen - 64u * blk <= 16u)
            ksblock_w03(x, blk);
        else
            ksblock(x, blk, 0u);
        if (Rf) {
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int q = 0; q < 16; q++)
                C[q] = funnel(Rf[q + 1], Rf[q], ina);
        }
        fillC();
        if (full) {
            poly_block(P, C[0], C[1], C[2], C[3], 1u);
            poly_block(P, C[4], C[5], C[6], C[7], 1u);
            poly_block(P, C[8], C[9], C[10], C[11], 1u);
            poly_block(P, C[12], C[13], C[14], C[15], 1u);
        } else {
            const u32 tailv = mlen - 64u * blk;
#pragma unroll
            for (int j = 0; j < 4; j++) {
                u32 s = 16u * j;
                if (s < tailv) {
                    u32 nb = tailv - s;
                    if (nb >= 16)
                        poly_block(P, C[4 * j], C[4 * j + 1], C[4 * j + 2], C[4 * j + 3], 1u);
                    else
                        poly_block_partial(P, C[4 * j], C[4 * j + 1], C[4 * j + 2], C[4 * j + 3], nb);
                }
            }
        }
#pragma unroll
        for (int k = 0; k < 16; k++)
            X[k] = C[k] ^ x[k];
        if constexpr (MODE == MODE_ZMQ) {
            u32 O[16];
            u32 E[17] = {K[0], K[1], K[2], K[3], K[4], K[5], K[6], K[7], X[0], X[1], X[2], X[3], X[4], X[5], X[6],
                         X[7], X[8]};
#pragma unroll
            for (int t = 0; t < 16; t++)
                O[t] = funnel(E[t + 1], E[t], 1);
            if (drain)
                __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0), expcnt / lgkmcnt unchanged (gfx9 encoding)
            emit_open(blk - 1, O, full);
#pragma unroll
            for (int k = 0; k < 8; k++)
                K[k] = X[8 + k];
        } else {
            emit_open(blk, X, full);
        }
    };
    auto open_block = [&](u32 blk, bool full, bool drain = false, const u32 *Rf = nullptr) {
        open_block_f(blk, full, drain, Rf, [] {});
    };

    u32 blk = 1;
    if constexpr (PAIR && AL) {
        // whole-line input: blocks 2k, 2k+1 come from one 8-load burst of body line k
        if (nfull >= 2) {
#pragma unroll
            for (int k = 0; k < 16; k++)
                C[k] = L1[k];  // (loaded with the rest of line 0, above)
            open_block(1, true);
            blk = 2;
            if constexpr (CARRY) {
                static_assert(INA != 16, "carry-line input is for bodies off 16-byte alignment");
                // the caller sorted frames so that every lane of the wave has the same line phase
                const uint8_t *lb = reinterpret_cast<const uint8_t *>((uintptr_t)in4 & ~(uintptr_t)127);
                const u32 s = __builtin_amdgcn_readfirstlane(((u32)(uintptr_t)in4 & 127u) >> 2);
                u32 Cur[32], Nxt[32];
                auto load_line = [&](u32 *D, const uint8_t *p) {
#pragma unroll
                    for (int c = 0; c < 8; c++) {
                        const uint4 v = *reinterpret_cast<const uint4 *>(p + 16 * c);
                        D[4 * c] = v.x; D[4 * c + 1] = v.y; D[4 * c + 2] = v.z; D[4 * c + 3] = v.w;
                    }
                };
                // aligned line 1 (window 0 above read its first s + 1 dwords a moment ago)
                load_line(Cur, lb + 128);
                for (u32 k = 1; 2u * k + 1u < nfull; k++) {
                    // aligned line k + 1: it holds a body byte (2k + 2 <= nfull), so it is mapped
                    load_line(Nxt, lb + 128u * (k + 1u));
                    __builtin_amdgcn_sched_barrier(0);
                    open_block_f(2u * k, true, true, nullptr, [&] {
                        __builtin_amdgcn_sched_barrier(0);
                        carry_window<0>(C, Cur, Nxt, s, ina);
                    });
                    open_block_f(2u * k + 1u, true, false, nullptr, [&] {
                        __builtin_amdgcn_sched_barrier(0);
                        carry_window<16>(C, Cur, Nxt, s, ina);
                    });
#pragma unroll
                    for (int q = 0; q < 32; q++)
                        Cur[q] = Nxt[q];
                    blk = 2u * k + 2u;
                }
            }
            for (u32 k = 1; !CARRY && 2u * k + 1u < nfull; k++) {
                u32 M[32];
                if constexpr (INA == 1) {
                    // 8 loads from the dword-aligned line below and the dword after it, funnelled
                    // inside open_block (after the keystream)
                    const uint8_t *src4 = in4 + 128u * k;
                    u32 R[33];
#pragma unroll
                    for (int c = 0; c < 8; c++) {
                        const uint4 v = *reinterpret_cast<const u4_a4 *>(src4 + 16 * c);
                        R[4 * c] = v.x; R[4 * c + 1] = v.y; R[4 * c + 2] = v.z; R[4 * c + 3] = v.w;
                    }
                    R[32] = ina ? *reinterpret_cast<const u32 *>(src4 + 128) : 0u;  // (2k+2 <= nfull)
                    __builtin_amdgcn_sched_barrier(0);
                    open_block(2u * k, true, true, R);
                    open_block(2u * k + 1u, true, false, R + 16);
                    blk = 2u * k + 2u;
                    continue;
                } else {
#pragma unroll
                    for (int c = 0; c < 8; c++) {
                        V4 v = LF(128u * k + 16u * c);
                        M[4 * c] = v.x; M[4 * c + 1] = v.y; M[4 * c + 2] = v.z; M[4 * c + 3] = v.w;
                    }
                }
#pragma unroll
                for (int q = 0; q < 16; q++)
                    C[q] = M[q];
                open_block(2u * k, true, true);
#pragma unroll
                for (int q = 0; q < 16; q++)
                    C[q] = M[16 + q];
                open_block(2u * k + 1u, true);
                blk = 2u * k + 2u;
            }
        }
    }
    for (; blk < nblk; blk++) {
        const uint8_t *src = in + 64u * blk;
        V4 q0, q1, q2, q3;
        const bool full = blk < nfull;
        const u32 o = 64u * blk;
        if (full) {
            q0 = LF(o);
            q1 = LF(o + 16u);
            q2 = LF(o + 32u);
            q3 = LF(o + 48u);
        } else {
            q0 = LP(o, size - o);
            q1 = LP(o + 16u, o + 16u < size ? size - o - 16u : 0);
            q2 = LP(o + 32u, o + 32u < size ? size - o - 32u : 0);
            q3 = LP(o + 48u, o + 48u < size ? size - o - 48u : 0);
        }
        (void)src;
        C[0] = q0.x; C[1] = q0.y; C[2] = q0.z; C[3] = q0.w;
        C[4] = q1.x; C[5] = q1.y; C[6] = q1.z; C[7] = q1.w;
        C[8] = q2.x; C[9] = q2.y; C[10] = q2.z; C[11] = q2.w;
        C[12] = q3.x; C[13] = q3.y; C[14] = q3.z; C[15] = q3.w;
        open_block(blk, full);
    }
    if constexpr (MODE == MODE_ZMQ) {
        // last payload chunk nblk-1 (if any payload remains): block nblk is beyond the box
        if (64u * (nblk - 1u) < nout) {
            u32 O[16];
#pragma unroll
            for (int t = 0; t < 16; t++)
                O[t] = t < 7 ? funnel(K[t + 1], K[t], 1) : (t == 7 ? funnel(0u, K[7], 1) : 0u);
            emit_open(nblk - 1u, O, false);
        }
    }

    u32 tag[4];
    poly_finish(P, tag);
    u32 diff = (tag[0] ^ tin.x) | (tag[1] ^ tin.y) | (tag[2] ^ tin.z) | (tag[3] ^ tin.w);
    const bool bad = dead || diff != 0;
    em.close(bad);  // never release unauthenticated plaintext; converged for cooperative emitters
    if (dead)
        return early;
    return diff != 0 ? (u32)CZ_STATUS_CRYPTO : (u32)CZ_STATUS_OK;
}

__device__ __forceinline__ void load_key(const uint8_t *__restrict__ p, u32 k[8])
{
    const uint4 *q = reinterpret_cast<const uint4 *>(p);
    uint4 a = q[0], b = q[1];
    k[0] = a.x; k[1] = a.y; k[2] = a.z; k[3] = a.w;
    k[4] = b.x; k[5] = b.y; k[6] = b.z; k[7] = b.w;
}

__device__ __forceinline__ bool aligned16(const void *a, const void *b)
{
    return (((uintptr_t)a | (uintptr_t)b) & 15u) == 0;
}

// true when v is the same in every active lane of the wave
__device__ __forceinline__ bool wave_uniform(u32 v)
{
    return __builtin_amdgcn_ballot_w64(v != __builtin_amdgcn_readfirstlane(v)) == 0;
}

__device__ __forceinline__ u64 read_be64(const uint8_t *p)
{
    u64 v = 0;
    for (int b = 0; b < 8; b++)
        v = (v << 8) | p[b];
    return v;
}

// ---------------------------------------------------------------------------
// Segmented frames (ragged batches).  A frame longer than 1.5 x SEG blocks is
// split into SEG-block segments, one per lane, so a 64 KiB frame no longer pins
// one lane for 1025 sequential blocks (the Zipf batch's critical path).  A
// segment lane runs Poly1305 from h = 0 over its own blocks and writes a
// 64-byte partial record; k_*_combine joins a frame's records with r^m powers.
// Record: [0..4] h (2^32 radix, partially reduced), [5] poly blocks absorbed,
// [6] decrypted flags byte (open, segment 0), [7] early status (open, segment 0),
// [8..11] clamped r, [12..15] pad (segment 0).
//
// Both directions run ONE loop over the segment's output chunks with the emit
// at the loop's convergence point, so a wave whose lanes hold segments with
// the same chunk count can share the cooperative line emitter below.
// ---------------------------------------------------------------------------

// bytes [a, b) of unit v at global address p (st_range16 for a global pointer)
__device__ __forceinline__ void st_range16_g(u64 p, uint4 v, u32 a, u32 b)
{
    if (b <= a)
        return;
    u64 lo = ((u64)v.y << 32) | v.x, hi = ((u64)v.w << 32) | v.z;
    if (a >= 8u) {
        lo = hi >> (8u * (a - 8u));
        hi = 0;
    } else if (a) {
        lo = (lo >> (8u * a)) | (hi << (64u - 8u * a));
        hi >>= 8u * a;
    }
    u64 q = p + a;
    const u32 n = b - a;
    if (n == 16u) {
        *reinterpret_cast<g_v4u_ua *>(q) = v4u_t{v.x, v.y, v.z, v.w};
        return;
    }
    if (n & 8u) {
        *reinterpret_cast<g_u64_ua *>(q) = lo;
        q += 8;
        lo = hi;
    }
    if (n & 4u) {
        *reinterpret_cast<g_u32_ua *>(q) = (u32)lo;
        q += 4;
        lo >>= 32;
    }
    if (n & 2u) {
        *reinterpret_cast<g_u16_ua *>(q) = (uint16_t)lo;
        q += 2;
        lo >>= 16;
    }
    if (n & 1u)
        *reinterpret_cast<g_u8 *>(q) = (uint8_t)lo;
}

// unit v at global address p clipped to its bytes [a, b), minus [t0, t1) when t1 > t0.  Out of
// line (only an output's edge units take it), and one call per unit: the range store is inlined
// once, run for the part below the hole and then for the part above it.
__device__ __noinline__ void st_unit_clip(u64 p, uint4 v, u32 a, u32 b, u32 t0, u32 t1)
{
    const bool hole = t1 > t0;
    u32 lo = a, hi = hole && b > t0 ? t0 : b;
#pragma nounroll
    for (int part = 0; part < 2; part++) {
        st_range16_g(p, v, lo, hi);
        if (!hole)
            break;
        lo = a > t1 ? a : t1;
        hi = b;
    }
}

// zero n bytes at any alignment: 16-byte stores over the aligned interior
__device__ void zero_bytes(uint8_t *p, u32 n)
{
    const uint4 z = make_uint4(0u, 0u, 0u, 0u);
    const u32 head = (u32)((16u - ((uintptr_t)p & 15u)) & 15u);
    const u32 h = head < n ? head : n;
    st_range16(p + h - 16, z, 16u - h, 16u);
    u32 o = h;
    for (; o + 16u <= n; o += 16u)
        *reinterpret_cast<uint4 *>(p + o) = z;
    st_range16(p + o, z, 0u, n - o);
}

// Line staging for a wave of outputs at ANY byte offset (ragged segments, dense body
// packing, bodies interleaved with wire headers).  MI355X writes a 128-byte line fast only
// when one store instruction covers it whole (tools/diag: 4.5 TB/s against 2.8 TB/s for
// lines written piecewise), so lines are ABSOLUTE: lane L's output [mine, mine + total)
// starts d = mine & 127 bytes into its first line.  Its LDS row holds the line being built
// (bytes [0, 128)) plus up to 64 bytes of the next; chunk q lands at (d + 64q) & 127 with
// b128 / b64 writes when every offset in the wave is a multiple of 16 / 8, else four
// ds_write_b128 at the byte address (round 4; the dword funnel they replaced cost more VALU than
// the LDS's unaligned splits cost time), and completes a line when it reaches byte 128: at even q for
// "class A" outputs (d >= 64), at odd q for the others.  The wave then stores that line of 8
// outputs per global_store_dwordx4 (8 lanes x 16 bytes; each output's base and byte count
// come from its owner lane by ds_bpermute) and each completing lane moves its row's bytes
// [128, 192) to the front.  A wave whose lanes are all of one class (the kernels sort lanes
// by class, class_permute) flushes once per chunk pair like EmitLines; a mixed wave flushes
// at every chunk with the other class masked off.  Units that an output only partly covers
// -- its first and last, the tag slot -- are clipped to its bytes (st_range16): neighbouring
// outputs own the other bytes.  emit/finish/close must be reached by all 64 lanes together:
// ds_bpermute from an inactive lane returns garbage, not its base.
constexpr u32 SROW = 208;  // 16 headroom + 192 bytes used; 52 dwords apart: conflict-free 16-lane b128
constexpr u32 SHIFT_LDS_BYTES = 64 * SROW;  // EmitShiftLines: 13 KiB per wave
constexpr u32 SHEAD = 16;  // row bytes before line-space byte 0 (a chunk's first dword may start 4 early)
// the uniform seal's rows (EmitShiftLinesT WHOLE) + 16 bytes: the next body's header, written behind
// an output's end at row byte <= 192, may run 16 bytes past the last row
constexpr u32 SEAL_SHIFT_LDS_BYTES = WAVES * SHIFT_LDS_BYTES + 16u;
// EmitShiftLinesT keeps its flag bits 28..31 (tag_whole, ext_end, ext_start, tag slot) above the
// output's end d + total in `te`, so the launchers send an output to ST_SHIFT only when
// d + total < 2^28 with d < 128: total <= SHIFT_TOTAL_MAX.
constexpr u32 SHIFT_TE_FLAG_BITS = 0xf0000000u;
constexpr u32 SHIFT_TOTAL_MAX = (1u << 28) - 128u;
static_assert(((SHIFT_TOTAL_MAX + 127u) & SHIFT_TE_FLAG_BITS) == 0u, "te's end field overlaps its flag bits");
// UNI (uniform batches: output i at out + i * stride): every lane fetches, once per frame, the
// workgroup-relative frame index of the 8 outputs it stores for (ds_bpermute) and keeps their
// 128-byte line offsets from the workgroup's line-aligned base in 8 VGPRs, so the interior-line
// flush -- the hot one -- is 8 ds_read_b128 + 8 buffer stores with no per-store ds_bpermute and
// no VALU address arithmetic (the base lives in the SGPR resource, the line added to it by the scalar unit).
// The outputs of a wave of ragged segments as 32-bit offsets from one wave-uniform base, so that
// a line store is a buffer store (base + line in the SGPR resource) fed by one
// ds_bpermute of the owner's offset.  base = lane 0's output rounded down to 128, minus 2^30;
// ok when every output lies within [base, base + 2^31) -- the planner's stable sort keeps a
// wave's segments within a few MiB of each other, so the fallback (64-bit bases) is for
// far-apart caller buffers only.
struct WaveRel {
    u64 base;
    u32 rel;  // this lane's output - base
    bool ok;  // wave-uniform
    __device__ __forceinline__ void init(const uint8_t *mine)
    {
        const u64 a = (u64)(uintptr_t)mine;
        const u64 a0 = uniform64(a);
        base = (a0 & ~(u64)127) - (1ull << 30);
        const u64 d = a - base;
        const bool mine_ok = a0 >= (1ull << 30) + 128u && d < (1ull << 31);
        ok = __builtin_amdgcn_ballot_w64(!mine_ok) == 0;
        rel = (u32)d;
    }
};

// WHOLE (the uniform seal, round 5): no unit of an output is written byte by byte.  The tag slot's
// units (body bytes 16..31 and the header / ciphertext bytes that share their 16-byte units) are
// skipped by the line flushes and written whole by tag() from the header, the tag and the first
// ciphertext words kept since chunk 0.  Bodies back to back (out_stride == body length, the V2 wire
// layout): an output's last unit is completed with the next body's first header bytes (its
// "\x07MESSAGE" and nonce, known from the counter) and written whole, and the next output skips that
// unit (init_ext).  Only the batch's first and last outputs keep a clipped edge unit.
template <bool UNI, int CP = CZ_OPEN_STORE_CPOL, bool WHOLE = false>
struct EmitShiftLinesT {
    static constexpr bool cooperative = true;
    uint8_t *rows;   // this wave's 64 rows of SROW bytes
    uint8_t *mine;
    u32 lane, total, last_q;
    u32 te;          // end of the output in its line space, d + total | bit 31: leave output bytes 16..31 to tag()
    u32 mixed;       // the wave holds outputs of both classes
    u32 walign;      // largest of 16 / 8 / 1 that divides every output's line offset in the wave
    u64 ubase;       // UNI: the workgroup's first output address rounded down to 128 (wave-uniform)
    u32 loff[8];     // UNI: line offset from ubase of output F = 8j + lane / 8, plus 16 * (lane & 7)
    WaveRel wr;      // !UNI: 32-bit output offsets for the interior-line flush
    u32 hw[6];       // WHOLE: this body's nonce words (body dwords 2, 3) and ciphertext dwords 8..11

    // UNI: rel = this lane's workgroup-relative frame index, wg_out = the workgroup's frame-0 output
    // (the launcher keeps 256 * stride + the output length below 2^31)
    __device__ __forceinline__ void init_uniform(u32 rel, u32 stride, const uint8_t *wg_out)
    {
        const u64 wo = (u64)(uintptr_t)wg_out;
        const u64 wu = ((u64)(u32)__builtin_amdgcn_readfirstlane((u32)(wo >> 32)) << 32) |
                       (u64)(u32)__builtin_amdgcn_readfirstlane((u32)wo);
        ubase = wu & ~(u64)127;
        const u32 a = (u32)wu & 127u;
        const u32 c = lane & 7u, r = lane >> 3;
#pragma unroll
        for (u32 j = 0; j < 8; j++) {
            const u32 relF = (u32)__builtin_amdgcn_ds_bpermute((int)((8u * j + r) << 2), (int)rel);
            loff[j] = ((a + relF * stride) & ~127u) + 16u * c;
        }
    }

    // the launchers keep d + total below 2^28 (SHIFT_TOTAL_MAX): bits 28..31 of te are flags
    // tag_whole (WHOLE): tag() will write the tag slot's units whole (the flushes skip them; they
    // end by body byte 48, so the output must reach that far); otherwise a tag slot's bytes are
    // clipped out of the line stores and the tag is stored over them.  (The same for the segment
    // seal, tag-slot units whole where a frame is one segment, measured -1.4% / -0.7% / +0.5% on the
    // Zipf 8-byte table / 1-byte offsets / 128-byte slots: not shipped)
    __device__ __forceinline__ void init(bool tag_slot, bool tag_whole = false)
    {
        const u32 d = (u32)(uintptr_t)mine & 127u;
        walign = __builtin_amdgcn_ballot_w64((d & 15u) != 0u) == 0  ? 16u
                 : __builtin_amdgcn_ballot_w64((d & 7u) != 0u) == 0 ? 8u
                                                                     : 1u;
        te = (d + total) | (tag_slot ? 0x80000000u : 0u) | (WHOLE && tag_slot && tag_whole && total >= 48u ? 0x10000000u : 0u);
        const uint64_t a = __builtin_amdgcn_ballot_w64((((u32)(uintptr_t)mine) & 64u) != 0u);
        mixed = (a != 0 && ~a != 0) ? 1u : 0u;
        if constexpr (!UNI)
            wr.init(mine);
        else
            wr.ok = false;
    }
    // WHOLE, bodies back to back: ext_start -- the body before this one completes this output's
    // first unit (skip it); ext_end -- complete the last unit with the next body's header
    __device__ __forceinline__ void init_ext(bool ext_start, bool ext_end)
    {
        te |= (ext_start ? 0x40000000u : 0u) | (ext_end ? 0x20000000u : 0u);
    }
    // store, for every output F of the wave whose line completes now, its line k_F:
    // KIND FL_PHASE: a one-class wave after chunk q of its phase, every F's line k = q / 2;
    // KIND FL_MIXED: after chunk q, k_F = (d_F + 64q) / 128 for the F with bit 6 of d_F + 64q set;
    // KIND FL_FINAL: after the last chunk q, the line holding output bytes past chunk q's line.
    enum { FL_PHASE = 0, FL_MIXED = 1, FL_FINAL = 2 };
    template <int KIND>
    __device__ __forceinline__ void flush(u32 q)
    {
        const u32 c = lane & 7u;
        const u32 r = lane >> 3;
        const u64 mb = (u64)(uintptr_t)mine;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the other lanes' ds_writes of this line
        if constexpr (KIND == FL_PHASE) {
            // Line k = q / 2 strictly inside every output of the wave (past the lines holding the
            // tag slot, whole before the output's end): unclipped stores, only the base fetched.
            const u32 k = q >> 1;
            const bool inner = k >= 2u && 128u * (k + 1u) <= (te & ~SHIFT_TE_FLAG_BITS);
            if constexpr (UNI) {
                if (__builtin_amdgcn_ballot_w64(!inner) == 0) {
                    const u64 lb = ubase + (u32)__builtin_amdgcn_readfirstlane(128u * k);
#pragma unroll
                    for (u32 j = 0; j < 8; j++) {
                        const u32 F = 8u * j + r;
                        const uint4 v = *reinterpret_cast<const uint4 *>(rows + F * SROW + SHEAD + 16u * c);
                        buf_store16<CP>(lb, loff[j], v);
                    }
                    return;
                }
            }
            if (!UNI && wr.ok && __builtin_amdgcn_ballot_w64(!inner) == 0) {
                // as UNI, with each output's line offset fetched per store (one ds_bpermute + one
                // VALU instead of two ds_bpermutes and a 64-bit add)
                const u64 lb = wr.base + (u32)__builtin_amdgcn_readfirstlane(128u * k);
#pragma unroll
                for (u32 j = 0; j < 8; j++) {
                    const u32 F = 8u * j + r;
                    const uint4 v = *reinterpret_cast<const uint4 *>(rows + F * SROW + SHEAD + 16u * c);
                    const u32 lo = (u32)__builtin_amdgcn_ds_bpermute((int)(F << 2), (int)wr.rel);
                    buf_store16<CP>(lb, (lo & ~127u) | (16u * c), v);
                }
                return;
            }
            if (!UNI && __builtin_amdgcn_ballot_w64(!inner) == 0) {
#pragma unroll
                for (u32 j = 0; j < 8; j++) {
                    const u32 F = 8u * j + r;
                    const uint4 v = *reinterpret_cast<const uint4 *>(rows + F * SROW + SHEAD + 16u * c);
                    const int sel = (int)(F << 2);
                    const u32 blo = (u32)__builtin_amdgcn_ds_bpermute(sel, (int)(u32)mb);
                    const u32 bhi = (u32)__builtin_amdgcn_ds_bpermute(sel, (int)(u32)(mb >> 32));
                    const u64 p = ((((u64)bhi) << 32) | (blo & ~127u)) + 128u * k + 16u * c;
                    *reinterpret_cast<g_uint4 *>(p) = v4u_t{v.x, v.y, v.z, v.w};
                }
                return;
            }
        }
#pragma unroll
        for (u32 j = 0; j < 8; j++) {
            const u32 F = 8u * j + r;
            const uint4 v = *reinterpret_cast<const uint4 *>(rows + F * SROW + SHEAD + 16u * c);
            const int sel = (int)(F << 2);
            const u32 blo = (u32)__builtin_amdgcn_ds_bpermute(sel, (int)(u32)mb);
            const u32 bhi = (u32)__builtin_amdgcn_ds_bpermute(sel, (int)(u32)(mb >> 32));
            const u32 fe = (u32)__builtin_amdgcn_ds_bpermute(sel, (int)te);
            const u32 d = blo & 127u;           // output F's bytes are [d, e) of its line space
            const u32 e = fe & ~SHIFT_TE_FLAG_BITS;
            u32 k;
            bool act = true;
            if constexpr (KIND == FL_PHASE) {
                k = q >> 1;
            } else if constexpr (KIND == FL_MIXED) {
                const u32 t = d + 64u * q;
                k = t >> 7;
                act = (t & 64u) != 0u;
            } else {
                k = (d + 64u * (q + 1u)) >> 7;
                act = e > 128u * k;
            }
            const u32 u = 128u * k + 16u * c;  // this lane's unit of line k
            const u64 p = ((((u64)bhi) << 32) | (blo & ~127u)) + u;
            // overlaps the tag slot, output bytes 16..31: u + 16 > d + 16 && u < d + 32 (lines 0 and 1 only)
            const bool tg = (KIND != FL_PHASE || q < 4u) && (fe >> 31) && u > d && u < d + 32u;
            // WHOLE: units owned whole by a neighbour (ext) or by tag() are not this flush's
            const u32 dd = (WHOLE && (fe & 0x40000000u)) ? (d + 15u) & ~15u : d;
            const u32 ee = (WHOLE && (fe & 0x20000000u)) ? (e + 15u) & ~15u : e;
            if (act && u >= dd && u + 16u <= ee && !tg) {
                CZ_DIAG_STORE_GUARD(v)
                *reinterpret_cast<g_uint4 *>(p) = v4u_t{v.x, v.y, v.z, v.w};
            } else if (WHOLE && tg && (fe & 0x10000000u)) {
                // a unit of the tag slot: tag() writes it whole
            } else if (act && u < ee && u + 16u > dd) {
                // bytes [a, b) of this unit, minus the tag bytes [t0, t1) that stay for tag()
                const u32 a = dd > u ? dd - u : 0u, b = ee < u + 16u ? ee - u : 16u;
                const u32 t0 = tg ? (u < d + 16u ? d + 16u - u : 0u) : 0u;
                const u32 t1 = tg ? (d + 32u - u < 16u ? d + 32u - u : 16u) : 0u;
                if (((a | b | t0 | t1) & 7u) == 0u) {
                    // 8-byte boundaries (outputs on an 8-byte offset table): each half of the unit
                    // is kept whole or not at all, one aligned 8-byte store per kept half
                    const bool k0 = a == 0u && b >= 8u && !(t0 == 0u && t1 >= 8u);
                    const bool k1 = a <= 8u && b == 16u && !(t0 <= 8u && t1 == 16u);
                    CZ_DIAG_STORE_GUARD(v)
                    if (k0)
                        *reinterpret_cast<g_u64_ua *>(p) = ((u64)v.y << 32) | v.x;
                    CZ_DIAG_STORE_GUARD(v)
                    if (k1)
                        *reinterpret_cast<g_u64_ua *>(p + 8u) = ((u64)v.w << 32) | v.z;
                } else {
                    CZ_DIAG_STORE_GUARD(v)
                    st_unit_clip(p, v, a, b, t0, t1);
                }
            }
        }
    }
    // a lane whose line just left keeps the bytes it already holds past it, end - 128 of them,
    // for the next line (LDS ops of one wave execute in order: the flush's reads come first)
    __device__ __forceinline__ void shift_row(u32 end)
    {
        asm volatile("" ::: "memory");
        uint4 *row = reinterpret_cast<uint4 *>(rows + lane * SROW + SHEAD);
#pragma unroll
        for (u32 u = 0; u < 4; u++)
            if (128u + 16u * u < end)
                row[u] = row[8u + u];
        asm volatile("" ::: "memory");
    }
    __device__ __forceinline__ void emit(u32 q, const u32 D[16])
    {
        const u32 t = ((u32)(uintptr_t)mine & 127u) + 64u * q;
        const u32 pos = t & 127u;
        // chunk byte i belongs at line-space byte pos + i.  A wave whose offsets are all 16- or
        // 8-byte multiples writes the chunk with ds_write_b128 / b64 at aligned addresses; the
        // others with ds_write_b128 at the byte address (the dword funnel it replaced: DESIGN.md
        // section 4, "Byte-address LDS writes").
        // ds_write_b128 at any byte address (ROCm runs LDS in unaligned mode; the hardware splits
        // the access): the chunk's bytes land exactly at [pos, pos + 64), no funnel, no tail dword
        const u32 b = 0u;
        uint8_t *row0 = rows + lane * SROW + SHEAD;
        if (walign == 16u) {
#pragma unroll
            for (u32 c = 0; c < 4; c++)
                reinterpret_cast<uint4 *>(row0 + pos)[c] = make_uint4(D[4 * c], D[4 * c + 1], D[4 * c + 2], D[4 * c + 3]);
        } else if (walign == 8u) {
#pragma unroll
            for (u32 c = 0; c < 8; c++)
                reinterpret_cast<uint2 *>(row0 + pos)[c] = make_uint2(D[2 * c], D[2 * c + 1]);
        } else {
#pragma unroll
            for (u32 c = 0; c < 4; c++)
                *reinterpret_cast<v4u_ua *>(row0 + pos + 16u * c) = v4u_t{D[4 * c], D[4 * c + 1], D[4 * c + 2], D[4 * c + 3]};
        }
        if constexpr (WHOLE) {
            if (q == 0u) {
                hw[0] = D[2]; hw[1] = D[3];
                hw[2] = D[8]; hw[3] = D[9]; hw[4] = D[10]; hw[5] = D[11];
            }
            // the chunk holding the output's end: the next body's header right behind it (its first
            // bytes complete the last unit; the row has 16 bytes of slack past byte 192)
            if ((te & 0x20000000u) && total > 64u * q && total <= 64u * q + 64u) {
                const u64 nx = (((u64)bswap32(hw[0]) << 32) | (u64)bswap32(hw[1])) + 1u;
                *reinterpret_cast<v4u_ua *>(row0 + pos + (total - 64u * q)) =
                    v4u_t{HDR0, HDR1, bswap32((u32)(nx >> 32)), bswap32((u32)nx)};
            }
        }
        const bool done = (t & 64u) != 0u;
        if (mixed) {
            flush<FL_MIXED>(q);
        } else if (__builtin_amdgcn_readfirstlane(done ? 1u : 0u)) {
            flush<FL_PHASE>(q);
        } else {
            last_q = q;
            return;
        }
        if (__builtin_amdgcn_ballot_w64(done && pos + 64u + b > 128u) != 0 && done)
            shift_row(pos + 64u + b);
        last_q = q;
    }
    __device__ __forceinline__ void emit_full(u32 q, const u32 D[16]) { emit(q, D); }
    __device__ __forceinline__ void tag(const u32 t[4])
    {
        if (WHOLE && (te & 0x10000000u)) {
            // the 16-byte units of the output that overlap its tag slot (body bytes 16..31), whole:
            // unit A = body [s, s + 16) at pA = (mine + 16) rounded down to 16, s = pA - mine in
            // 1..16, and for s < 16 unit B = body [s + 16, s + 32); from body dwords 0..11
            const u32 H[12] = {HDR0, HDR1, hw[0], hw[1], t[0], t[1], t[2], t[3], hw[2], hw[3], hw[4], hw[5]};
            uint8_t *pA = reinterpret_cast<uint8_t *>(((uintptr_t)mine + 16u) & ~(uintptr_t)15);
            const u32 sft = (u32)(pA - mine), si = sft >> 2, sb = sft & 3u;
            u32 Hs[9];
#pragma unroll
            for (int k = 0; k < 9; k++)
                Hs[k] = si == 0u ? H[k] : si == 1u ? H[k + 1] : si == 2u ? H[k + 2] : si == 3u ? H[k + 3] : (k < 8 ? H[k + 4] : 0u);
            u32 O[8];
#pragma unroll
            for (int k = 0; k < 8; k++)
                O[k] = funnel(Hs[k + 1], Hs[k], sb);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // after any line store that covered these units
            const uint4 oa = make_uint4(O[0], O[1], O[2], O[3]);
            CZ_DIAG_STORE_GUARD(oa)
            *reinterpret_cast<uint4 *>(pA) = oa;
            const uint4 ob = make_uint4(O[4], O[5], O[6], O[7]);
            CZ_DIAG_STORE_GUARD(ob)
            if (sft < 16u)
                *reinterpret_cast<uint4 *>(pA + 16) = ob;
        } else {
            const uint4 tv = make_uint4(t[0], t[1], t[2], t[3]);
            CZ_DIAG_STORE_GUARD(tv)
            reinterpret_cast<U16ua *>(mine + 16)->v = tv;
        }
    }
    __device__ __forceinline__ void finish()
    {
        // bytes past an output are clipped by its count; the line after the last completed one
        // still holds output bytes unless the output ends on it
        const u32 t = ((u32)(uintptr_t)mine & 127u) + 64u * (last_q + 1u);
        if (__builtin_amdgcn_ballot_w64(((u32)(uintptr_t)mine & 127u) + total > 128u * (t >> 7)) != 0)
            flush<FL_FINAL>(last_q);
    }
    __device__ __forceinline__ void close(bool bad)
    {
        finish();
        if (bad)
            poison();
    }
    __device__ void poison()
    {
        __threadfence_block();  // land after the other lanes' stores of this lane's lines
        zero_bytes(mine, total);
    }
};
using EmitShiftLines = EmitShiftLinesT<false>;
using EmitShiftLinesUni = EmitShiftLinesT<true>;
using EmitShiftLinesSeal = EmitShiftLinesT<false, CZ_SEAL_STORE_CPOL>;
using EmitShiftLinesUniSeal = EmitShiftLinesT<true, CZ_SEAL_STORE_CPOL, true>;

// EmitShiftLinesUni for a wave of ONE line class, the class fixed at compile time (round 5).
// The generic emitter decides at every chunk, at run time, whether a line completes (its class),
// whether the line is interior (fast store path) and which rows spill into the next line.  Each of
// those branches splits the seal's pair loop into separate basic blocks, and at the join after a
// flush whose store count differs per path the compiler can only wait vmcnt(0): the next block's
// first load wait then also waits for the 8 line stores just issued (class-A waves flush in the
// middle of the pair).  Here a wave of class PAR_ODD = 1 (d < 64) completes line q / 2 after every
// odd chunk q, a wave of class 0 (d >= 64) after every even chunk, with no run-time test:
//  - emit_steady(q, D) is the pair loop's emit (q >= 2, a full chunk): byte-address chunk writes,
//    then at its parity the fast whole-line flush and an unconditional row shift.  Every line the
//    pair loop completes is whole inside every output of the wave (the chunk that completes it is a
//    full block); the one exception is line 1 of a class-0 output with d > 96, which holds tag
//    bytes [128 - d, 32): it leaves with the zeros chunk 0 put there, and tag() writes the tag
//    after a vmcnt(0) wait, so the tag lands after that line;
//  - everything else (chunks 0 and 1 with line 0, the tail, the last line) takes the generic
//    emitter's paths.
// Shifting every row is harmless: the bytes moved past a row's carry are overwritten by the next
// chunk before the next flush reads them.
template <int PAR_ODD, int CP>
struct EmitShiftLinesUniClassT : EmitShiftLinesT<true, CP, true> {
    using Base = EmitShiftLinesT<true, CP, true>;
    __device__ __forceinline__ void emit_steady(u32 q, const u32 D[16])
    {
        const u32 pos = (((u32)(uintptr_t)this->mine & 127u) + 64u * q) & 127u;
        uint8_t *row0 = this->rows + this->lane * SROW + SHEAD;
#pragma unroll
        for (u32 c = 0; c < 4; c++)
            *reinterpret_cast<v4u_ua *>(row0 + pos + 16u * c) = v4u_t{D[4 * c], D[4 * c + 1], D[4 * c + 2], D[4 * c + 3]};
        this->last_q = q;
        if ((q & 1u) != (u32)PAR_ODD)
            return;
        const u32 c = this->lane & 7u, r = this->lane >> 3;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the other lanes' ds_writes of this line
        const u64 lb = this->ubase + (u32)__builtin_amdgcn_readfirstlane(128u * (q >> 1));
#pragma unroll
        for (u32 j = 0; j < 8; j++) {
            const u32 F = 8u * j + r;
            const uint4 v = *reinterpret_cast<const uint4 *>(this->rows + F * SROW + SHEAD + 16u * c);
            buf_store16<CP>(lb, this->loff[j], v);
        }
        asm volatile("" ::: "memory");
        uint4 *row = reinterpret_cast<uint4 *>(row0);
        uint4 t[4];
#pragma unroll
        for (u32 u = 0; u < 4; u++)
            t[u] = row[8u + u];
#pragma unroll
        for (u32 u = 0; u < 4; u++)
            row[u] = t[u];
        asm volatile("" ::: "memory");
    }
    __device__ __forceinline__ void tag(const u32 t[4])
    {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every line store of the wave has landed
        Base::tag(t);
    }
};
template <int PAR_ODD>
using EmitShiftLinesUniClassSeal = EmitShiftLinesUniClassT<PAR_ODD, CZ_SEAL_STORE_CPOL>;

// the pair loops' emit: emitters that have a steady-state form (emit_steady) take it
template <class EM, class = void>
struct has_emit_steady : std::false_type {};
template <class EM>
struct has_emit_steady<EM, std::void_t<decltype(&EM::emit_steady)>> : std::true_type {};
template <class EM>
__device__ __forceinline__ void emit_steady(EM &em, u32 q, const u32 D[16])
{
    if constexpr (has_emit_steady<EM>::value)
        em.emit_steady(q, D);
    else
        em.emit_full(q, D);
}

// Line staging for a wave of segments at arbitrary 16-byte aligned bases.  Like
// EmitLines, 8 lanes write one 128-byte output line per store instruction, but
// each frame's base and byte count are fetched from its owner lane with
// ds_bpermute (no LDS table: 8 KiB per wave keeps 5 workgroups per CU), and
// stores are clipped to the segment's bytes (ragged frames are packed, nothing
// is padding).  emit/finish/close must be reached by all 64 lanes together:
// ds_bpermute from an inactive lane returns garbage, not its base.
constexpr u32 SEG_LDS_BYTES = LINE_LDS_BYTES;  // EmitSegLines: 64 x 128-byte line buffer per wave
template <int CP>
struct EmitSegLinesT {
    static constexpr bool cooperative = true;
    uint4 *lds;      // this wave's 64 x 8 chunks
    uint8_t *mine;
    u32 lane, total, last_q;
    u32 tt;          // total | bit 31: leave bytes 16..31 of line 0 to tag()
    WaveRel wr;      // every output of the wave within 2^30 bytes of lane 0's: 32-bit offsets

    __device__ __forceinline__ void init(bool tag_slot)
    {
        tt = total | (tag_slot ? 0x80000000u : 0u);
        wr.init(mine);
    }
    __device__ __forceinline__ void flush(u32 line)
    {
        const u32 c = lane & 7u;
        const u32 r = lane >> 3;
        const u32 off = 128u * line + 16u * c;
        const u64 mb = (u64)(uintptr_t)mine;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        // Interior line of every segment in the wave (whole, no tag bytes): one ds_bpermute of the
        // owner's 32-bit offset and one add per store, base + line in the buffer resource (the
        // general path below fetches a 64-bit base and a count per store and
        // clips: ~12 VALU and a branch per store).
        const bool inner = 128u * line + 128u <= total && !((tt >> 31) && line == 0u);
        if (wr.ok && __builtin_amdgcn_ballot_w64(!inner) == 0) {
            const u64 lb = wr.base + (u32)__builtin_amdgcn_readfirstlane(128u * line);
#pragma unroll
            for (u32 j = 0; j < 8; j++) {
                const u32 F = 8u * j + r;
                const uint4 v = lds[F * 8u + (c ^ (F & 7u))];
                buf_store16<CP>(lb, (u32)__builtin_amdgcn_ds_bpermute((int)(F << 2), (int)wr.rel) + 16u * c, v);
            }
            return;
        }
#pragma unroll
        for (u32 j = 0; j < 8; j++) {
            const u32 F = 8u * j + r;
            const uint4 v = lds[F * 8u + (c ^ (F & 7u))];
            const int sel = (int)(F << 2);
            const u32 blo = (u32)__builtin_amdgcn_ds_bpermute(sel, (int)(u32)mb);
            const u32 bhi = (u32)__builtin_amdgcn_ds_bpermute(sel, (int)(u32)(mb >> 32));
            const u32 ft = (u32)__builtin_amdgcn_ds_bpermute(sel, (int)tt);
            const u32 tot = ft & 0x7fffffffu;
            uint8_t *p = reinterpret_cast<uint8_t *>((uintptr_t)(((u64)bhi << 32) | blo)) + off;
            const bool skip = (ft >> 31) && line == 0 && c == 1;
            if (!skip) {
                if (off + 16u <= tot)
                    *reinterpret_cast<uint4 *>(p) = v;
                else if (off < tot)
                    st_bytes(p, v.x, v.y, v.z, v.w, tot - off);
            }
        }
    }
    __device__ __forceinline__ void emit(u32 q, const u32 D[16])
    {
        const u32 h = q & 1u;
        const u32 sw = lane & 7u;
#pragma unroll
        for (u32 c = 0; c < 4; c++)
            lds[lane * 8u + ((4u * h + c) ^ sw)] = make_uint4(D[4 * c], D[4 * c + 1], D[4 * c + 2], D[4 * c + 3]);
        if (h)
            flush(q >> 1);
        last_q = q;
    }
    __device__ __forceinline__ void emit_full(u32 q, const u32 D[16]) { emit(q, D); }
    __device__ __forceinline__ void tag(const u32 t[4])
    {
        *reinterpret_cast<uint4 *>(mine + 16) = make_uint4(t[0], t[1], t[2], t[3]);
    }
    __device__ __forceinline__ void finish()
    {
        if ((last_q & 1u) == 0)
            flush(last_q >> 1);  // bytes past the segment are clipped by the table's count
    }
    __device__ __forceinline__ void close(bool bad)
    {
        finish();
        if (bad)
            poison();
    }
    __device__ void poison()
    {
        __threadfence_block();  // land after the other lanes' stores of this lane's lines
        for (u32 o = 0; o < total; o += 16) {
            if (o + 16u <= total)
                *reinterpret_cast<uint4 *>(mine + o) = make_uint4(0u, 0u, 0u, 0u);
            else
                st_bytes(mine + o, 0u, 0u, 0u, 0u, total - o);
        }
    }
};
using EmitSegLines = EmitSegLinesT<CZ_OPEN_STORE_CPOL>;
using EmitSegLinesSeal = EmitSegLinesT<CZ_SEAL_STORE_CPOL>;

// Reorder the work items of one full workgroup so that each wave holds outputs of one
// EmitShiftLines class (bit 6 of the output address): such a wave flushes once per chunk pair
// instead of at every chunk.  `cls` is the class of this thread's own item; returns the
// workgroup-relative index of the item this thread takes instead.  Deterministic (a
// stable partition), so kernels that split waves between them agree on the layout.
// perm: BLOCK + WAVES words of scratch LDS, free again on return.  The kernels pass the start of
// their dynamic LDS (the emitter rows, not in use yet): a static array of its own would add
// 1040 bytes per workgroup, and 3 x (52 KiB rows + that) no longer fit a CU's 160 KiB -- the
// dense seal then ran 2 waves per SIMD instead of 3.
__device__ __forceinline__ u32 class_permute(bool cls, u32 *__restrict__ perm)
{
    const u32 tid = threadIdx.x, w = tid >> 6;
    const uint64_t m = __builtin_amdgcn_ballot_w64(cls);
    const u32 below1 = __builtin_amdgcn_mbcnt_hi((u32)(m >> 32), __builtin_amdgcn_mbcnt_lo((u32)m, 0u));
    const u32 below0 = (tid & 63u) - below1;
    if ((tid & 63u) == 0)
        perm[BLOCK + w] = (u32)__builtin_popcountll(m);
    __syncthreads();
    u32 pre1 = 0, tot1 = 0;
#pragma unroll
    for (u32 i = 0; i < (u32)WAVES; i++) {
        const u32 v = perm[BLOCK + i];
        tot1 += v;
        pre1 += i < w ? v : 0u;
    }
    const u32 pos = cls ? (BLOCK - tot1) + pre1 + below1 : (64u * w - pre1) + below0;
    perm[pos] = tid;
    __syncthreads();
    const u32 mine = perm[tid];
    __syncthreads();
    return mine;
}

// Bytes of box blocks [b0, bend) that go to the output of a seal segment.
__device__ __forceinline__ u32 seal_seg_bytes(u32 mlen, u32 b0, u32 bend)
{
    const u32 e = 64u * bend < mlen ? 64u * bend : mlen;
    return e - 64u * b0;
}

// Seal box blocks [b0, b1) of one MESSAGE.  Output chunk q is box block b0 + q
// at em's base (body + 64*b0).  rec == nullptr: the whole frame, the tag goes
// to bytes 16..31; otherwise the Poly1305 partial goes to rec.
// PAIR (16-byte aligned input): block 2k's window is P[32k-9 .. 32k+7] and
// block 2k+1's is P[32k+7 .. 32k+23], so each iteration reads payload line k
// whole (8 back-to-back loads) and seals two blocks from it, carrying the
// line's last 9 dwords.  Lane-wise 16-byte loads one block apart made L2 fetch
// most lines twice (2.6x the payload on the Zipf batch).
// INA: as seal_frame's (16: 16-byte aligned payload; 8 / 1 with AL true: payload at an 8-byte /
// any byte offset, read from the dword boundary at or above it with the funnel shift sh).
template <bool AL, class EM, bool PAIR = false, int INA = 16>
__device__ __forceinline__ void seal_segment(const uint8_t *__restrict__ in0, u32 n, u32 flags, u64 counter, const u32 key[8], u32 b0,
                             u32 b1, u32 *__restrict__ rec, EM &em, u32 nrun = 0)
{
    static_assert(INA == 16 || AL, "INA 8/1 take the AL code paths");
    const u32 ina_a = INA == 1 ? (u32)(uintptr_t)in0 & 3u : 0u;
    const u32 ina_d = (4u - ina_a) & 3u;
    const uint8_t *__restrict__ in = in0 + ina_d;
    const u32 sh = ina_a ? ina_a - 1u : 3u;
    u32 pm1 = flags << 24;  // P[-1]
    if constexpr (INA == 1) {
        if (ina_a) {
            const u32 r = *reinterpret_cast<const u32 *>(in0 - ina_a);
            pm1 = (r & ~(0xffu << (8u * sh))) | (flags << (8u * sh));
        }
    }
    auto ldF = [&](const uint8_t *p) -> V4 {
        if constexpr (INA == 16) {
            return ld16f_in<AL>(p);
        } else {
            const uint4 r = *reinterpret_cast<const u4_a4 *>(p);
            return V4{r.x, r.y, r.z, r.w};
        }
    };
    auto ldP = [&](const uint8_t *p, u64 avail) -> V4 {
        if constexpr (INA == 16)
            return ld16<AL>(p, avail);
        else
            return avail >= 16u ? ldF(p) : ld16<false>(p, avail);
    };
    const u32 mlen = n + 33u;
    const u32 nblk = (mlen + 63u) >> 6;
    const u32 nfull = mlen >> 6;
    const u32 bend = b1 < nblk ? b1 : nblk;
    const u32 nch = bend - b0;
    // bytes from `in`.  A payload of 0..2 bytes at an odd offset is shorter than d = -in0 & 3 and
    // lies wholly in P[-1] (pm1): no load may read past it (n - d would wrap to ~2^64, and the pair
    // loop would then read up to 128 bytes past the payload).
    const u64 inlen = n > ina_d ? (u64)(n - ina_d) : 0ull;
    u32 n0, n1;
    counter_nonce(counter, n0, n1);
    u32 x[16], C[16];
    salsa20_block(x, key, n0, n1, 0u, 0u);
    Poly P;
    poly_init(P, x[0], x[1], x[2], x[3], x[4], x[5], x[6], x[7]);
    u32 mpoly = 0;

    // box block blk from its 17-dword window W = P[16blk-9 .. 16blk+7] (P[-1] = flags << 24);
    // own = false: a block past this lane's segment, run only to keep the wave in step
    // (PAIR with nrun > nch): not absorbed, and its stores are clipped by the emitter
    auto block = [&](u32 blk, const u32 *W, bool own = true) {
        salsa20_block(x, key, n0, n1, blk, 0u);
#pragma unroll
        for (int k = 0; k < 16; k++)
            C[k] = funnel(W[k + 1], W[k], sh) ^ x[k];
        if (blk == 0) {
            C[0] = HDR0; C[1] = HDR1; C[2] = n0; C[3] = n1;
            C[4] = C[5] = C[6] = C[7] = 0u;  // tag slot
        }
        if (!own) {
        } else if (blk != 0 && blk < nfull) {
            poly_block(P, C[0], C[1], C[2], C[3], 1u);
            poly_block(P, C[4], C[5], C[6], C[7], 1u);
            poly_block(P, C[8], C[9], C[10], C[11], 1u);
            poly_block(P, C[12], C[13], C[14], C[15], 1u);
            mpoly += 4;
        } else {
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const u32 s = 64u * blk + 16u * j;
                if (s >= 32u && s < mlen) {
                    const u32 nb = mlen - s;
                    if (nb >= 16)
                        poly_block(P, C[4 * j], C[4 * j + 1], C[4 * j + 2], C[4 * j + 3], 1u);
                    else
                        poly_block_partial(P, C[4 * j], C[4 * j + 1], C[4 * j + 2], C[4 * j + 3], nb);
                    mpoly++;
                }
            }
        }
    };

    if constexpr (PAIR) {
        static_assert(AL, "PAIR needs 16-byte aligned input");
        u32 cy[9];  // P[16*(b0+q0) - 9 .. 16*(b0+q0) - 1]
        // nrun (cooperative emitters): the wave's longest segment; shorter ones run along
        const u32 run = nrun > nch ? nrun : nch;
        // Line phase.  Pair k reads payload [64(b0 + 2k), +128): a whole 128-byte line only when
        // in + 64*b0 is line-aligned.  Otherwise ("odd", half of a 64-byte packed ragged batch)
        // every pair load straddles two lines and each line is fetched twice, one pair apart
        // (FETCH 1.47x the payload).  A wave whose segments are all odd (the planner sorts
        // segments by phase within a length) seals block b0 alone from the line that ends
        // 64 bytes into it, then pairs (b0+1, b0+2), ... from whole lines.
        const bool odd = (((uintptr_t)(in + 64u * b0)) & 64u) != 0u;
        u32 q0 = 0;
        if (__builtin_amdgcn_ballot_w64(!odd) == 0) {
            // line [64*b0 - 64, 64*b0 + 64): aligned, so on a mapped page even where it starts
            // before the payload (bytes outside the frame are never used)
            const uint8_t *ln = in + 64u * b0 - 64;
            u32 L[32];
#pragma unroll
            for (int c = 0; c < 8; c++) {
                const long o = (long)(64u * b0) - 64 + 16 * c;
                V4 v = (o < 0) ? zero4() : ldP(ln + 16 * c, (u64)o < inlen ? inlen - (u64)o : 0);
                L[4 * c] = v.x; L[4 * c + 1] = v.y; L[4 * c + 2] = v.z; L[4 * c + 3] = v.w;
            }
            if (b0 == 0)
                L[15] = pm1;  // P[-1]
            block(b0, L + 7, 0u < nch);
            em.emit(0u, C);
#pragma unroll
            for (int k = 0; k < 9; k++)
                cy[k] = L[23 + k];
            q0 = 1;
        } else if (b0 == 0) {
#pragma unroll
            for (int k = 0; k < 8; k++)
                cy[k] = 0u;
            cy[8] = pm1;
        } else {
            const uint8_t *p = in + 64u * b0 - 48u;
            V4 a = ldF(p), b = ldF(p + 16), c = ldF(p + 32);
            cy[0] = a.w; cy[1] = b.x; cy[2] = b.y; cy[3] = b.z; cy[4] = b.w;
            cy[5] = c.x; cy[6] = c.y; cy[7] = c.z; cy[8] = c.w;
        }
        for (u32 q = q0; q < run; q += 2u) {
            const u32 blk = b0 + q;
            const uint8_t *src = in + 64u * blk;
            const u64 o = 64ull * blk;
            u32 L[32];
            if (o + 128u <= inlen) {
#pragma unroll
                for (int c = 0; c < 8; c++) {
                    V4 v = ldF(src + 16 * c);
                    L[4 * c] = v.x; L[4 * c + 1] = v.y; L[4 * c + 2] = v.z; L[4 * c + 3] = v.w;
                }
            } else {
#pragma unroll
                for (int c = 0; c < 8; c++) {
                    V4 v = ldP(src + 16 * c, inlen > o + 16u * c ? inlen - o - 16u * c : 0);
                    L[4 * c] = v.x; L[4 * c + 1] = v.y; L[4 * c + 2] = v.z; L[4 * c + 3] = v.w;
                }
            }
            u32 W[17];
#pragma unroll
            for (int k = 0; k < 9; k++)
                W[k] = cy[k];
#pragma unroll
            for (int k = 0; k < 8; k++)
                W[9 + k] = L[k];
            block(blk, W, q < nch);
            em.emit(q, C);
            if (q + 1u < run) {
                block(blk + 1u, L + 7, q + 1u < nch);
                em.emit(q + 1u, C);
            }
#pragma unroll
            for (int k = 0; k < 9; k++)
                cy[k] = L[23 + k];
        }
    } else {
        u32 carry = b0 == 0 ? pm1 : (INA == 16 ? ld32<AL>(in + 64u * b0 - 36u) : *reinterpret_cast<const u32 *>(in + 64u * b0 - 36u));  // P[16*b0 - 9]
        for (u32 q = 0; q < nch; q++) {
            const u32 blk = b0 + q;
            u32 W[17];
            W[0] = carry;
            if (blk == 0) {
                V4 a = ldP(in, inlen);
                V4 b = ldP(in + 16, inlen > 16 ? inlen - 16 : 0);
                // block 0 only uses W[8..16] = P[-1 .. 7]
                W[8] = carry;
                W[9] = a.x; W[10] = a.y; W[11] = a.z; W[12] = a.w;
                W[13] = b.x; W[14] = b.y; W[15] = b.z; W[16] = b.w;
#pragma unroll
                for (int k = 1; k < 8; k++)
                    W[k] = 0u;
            } else {
                const uint8_t *src = in + 64u * blk - 32u;
                V4 q0, q1, q2, q3;
                if (blk < nfull) {
                    q0 = ldF(src); q1 = ldF(src + 16); q2 = ldF(src + 32);
                    q3 = ldP(src + 48, inlen - (64u * blk + 16u));
                } else {
                    const u64 o = 64u * blk - 32u;
                    q0 = ldP(src, o < inlen ? inlen - o : 0);
                    q1 = ldP(src + 16, o + 16 < inlen ? inlen - o - 16 : 0);
                    q2 = ldP(src + 32, o + 32 < inlen ? inlen - o - 32 : 0);
                    q3 = ldP(src + 48, o + 48 < inlen ? inlen - o - 48 : 0);
                }
                W[1] = q0.x; W[2] = q0.y; W[3] = q0.z; W[4] = q0.w;
                W[5] = q1.x; W[6] = q1.y; W[7] = q1.z; W[8] = q1.w;
                W[9] = q2.x; W[10] = q2.y; W[11] = q2.z; W[12] = q2.w;
                W[13] = q3.x; W[14] = q3.y; W[15] = q3.z; W[16] = q3.w;
            }
            block(blk, W);
            carry = W[16];
            em.emit(q, C);
        }
    }
    if (!rec) {
        u32 tag[4];
        poly_finish(P, tag);
        em.tag(tag);
    }
    em.close(false);  // convergent: a cooperative flush must see every lane of the wave
    if (rec) {
        rec[0] = P.h0; rec[1] = P.h1; rec[2] = P.h2; rec[3] = P.h3; rec[4] = P.h4; rec[5] = mpoly;
        if (b0 == 0) {
            rec[8] = P.r0; rec[9] = P.r1; rec[10] = P.r2; rec[11] = P.r3;
            rec[12] = P.p0; rec[13] = P.p1; rec[14] = P.p2; rec[15] = P.p3;
        }
    }
}

// MESSAGE header checks of ZmqCurveMechanism.decode (order: command, malformed,
// sequence); on OK returns the nonce words.  See open_frame for the citations.
__device__ __forceinline__ u32 open_header(const uint8_t *__restrict__ in, u32 size, bool check_floor,
                                           long long floor, u32 &n0, u32 &n1, u64 &nonce)
{
    if (size < 8u)
        return CZ_STATUS_COMMAND;
    V4 h = ld16<false>(in, size);
    if (h.x != HDR0 || (h.y & 0x00ffffffu) != (HDR1 & 0x00ffffffu))
        return CZ_STATUS_COMMAND;
    if (size < 33u)
        return CZ_STATUS_MALFORMED;
    n0 = h.z;
    n1 = h.w;
    nonce = ((u64)bswap32(n0) << 32) | (u64)bswap32(n1);
    if (check_floor && (long long)nonce <= floor)
        return CZ_STATUS_SEQUENCE;
    return CZ_STATUS_OK;
}

// Open segment geometry.  Segment 0 MACs box blocks [0, b1); segment s >= 1
// starts at block b0 = s*SEG + 1 and MACs [b0, b1).  Payload chunk g (bytes
// 64g..64g+63) needs box blocks g and g+1, so the segment emits chunks
// [cb, ce) with cb = b0 ? b0 - 1 : 0 and ce = b1 - 1, or every remaining chunk
// when b1 reaches the end of the box.
struct OpenSeg {
    u32 nblk, nout, cb, ce, bend;
};
__device__ __forceinline__ OpenSeg open_seg_geom(u32 size, u32 b0, u32 b1)
{
    OpenSeg g;
    g.nblk = (size + 63u) >> 6;
    g.nout = size - 33u;
    g.bend = b1 < g.nblk ? b1 : g.nblk;
    g.cb = b0 ? b0 - 1u : 0u;
    g.ce = g.bend == g.nblk ? (g.nout + 63u) >> 6 : g.bend - 1u;
    return g;
}

// Open box blocks [b0, b1) of one MESSAGE body whose header passed open_header.
// Returns CZ_STATUS_OK or (whole frame, bad tag) CZ_STATUS_CRYPTO.
template <bool AL, class EM, bool AL8 = false, bool ANY = false>
__device__ __forceinline__ u32 open_segment(const uint8_t *__restrict__ in, u32 size, const u32 key[8], u32 n0, u32 n1, u32 b0,
                            u32 b1, u32 *__restrict__ rec, u32 &flags_out, EM &em)
{
    // AL: input 16-byte aligned; AL8: 8-byte aligned (two 8-byte loads per chunk); ANY: any byte
    // offset (16-byte loads from the dword at or below, funnelled as open_frame's INA 1); else
    // lane-wise unaligned loads
    const u32 ina = ANY ? (u32)(uintptr_t)in & 3u : 0u;
    const uint8_t *in4 = in - ina;
    auto ldf = [&](const uint8_t *p) -> V4 {  // all 16 bytes inside the body
        if constexpr (ANY) {
            const uint8_t *q = in4 + (p - in);
            const uint4 r = *reinterpret_cast<const u4_a4 *>(q);
            const u32 r4 = ina ? *reinterpret_cast<const u32 *>(q + 16) : 0u;
            return V4{funnel(r.y, r.x, ina), funnel(r.z, r.y, ina), funnel(r.w, r.z, ina), funnel(r4, r.w, ina)};
        } else if constexpr (AL8) {
            return ld16f_8(p);
        } else {
            return ld16f<AL>(p);
        }
    };
    auto ldp = [&](const uint8_t *p, u64 avail) -> V4 {
        if constexpr (ANY)
            return avail >= 16u ? ldf(p) : ld16<false>(p, avail);
        else if constexpr (AL8)
            return ld16_8(p, avail);
        else
            return ld16<AL>(p, avail);
    };
    const OpenSeg g = open_seg_geom(size, b0, b1);
    const u32 mlen = size;
    const u32 nfull = mlen >> 6;
    u32 x[16], X[16], K[8];
    salsa20_block(x, key, n0, n1, 0u, 0u);
    Poly P;
    poly_init(P, x[0], x[1], x[2], x[3], x[4], x[5], x[6], x[7]);
    u32 mpoly = 0;
    // prologue: plaintext dwords 8..15 of block cb (MACed here only for segment 0)
    if (b0 == 0) {
        V4 a = ldp(in + 32, size > 32 ? size - 32u : 0);
        V4 b = ldp(in + 48, size > 48 ? size - 48u : 0);
        const u32 nb = (mlen < 64u ? mlen : 64u) - 32u;
        if (nb >= 16u) {
            poly_block(P, a.x, a.y, a.z, a.w, 1u);
            mpoly++;
            if (nb >= 32u) {
                poly_block(P, b.x, b.y, b.z, b.w, 1u);
                mpoly++;
            } else if (nb > 16u) {
                poly_block_partial(P, b.x, b.y, b.z, b.w, nb - 16u);
                mpoly++;
            }
        } else if (nb > 0u) {
            poly_block_partial(P, a.x, a.y, a.z, a.w, nb);
            mpoly++;
        }
        K[0] = a.x ^ x[8]; K[1] = a.y ^ x[9]; K[2] = a.z ^ x[10]; K[3] = a.w ^ x[11];
        K[4] = b.x ^ x[12]; K[5] = b.y ^ x[13]; K[6] = b.z ^ x[14]; K[7] = b.w ^ x[15];
        flags_out = K[0] & 0xffu;
    } else {
        salsa20_block(X, key, n0, n1, g.cb, 0u);
        const uint8_t *src = in + 64u * g.cb + 32u;
        V4 a = ldf(src), b = ldf(src + 16);
        K[0] = a.x ^ X[8]; K[1] = a.y ^ X[9]; K[2] = a.z ^ X[10]; K[3] = a.w ^ X[11];
        K[4] = b.x ^ X[12]; K[5] = b.y ^ X[13]; K[6] = b.z ^ X[14]; K[7] = b.w ^ X[15];
    }
    for (u32 q = 0; q < g.ce - g.cb; q++) {
        const u32 blk = g.cb + q + 1u;  // chunk cb+q needs box block cb+q+1
        if (blk < g.nblk) {
            const uint8_t *src = in + 64u * blk;
            V4 q0, q1, q2, q3;
            const bool full = blk < nfull;
            if (full) {
                q0 = ldf(src); q1 = ldf(src + 16); q2 = ldf(src + 32); q3 = ldf(src + 48);
            } else {
                const u32 o = 64u * blk;
                q0 = ldp(src, size - o);
                q1 = ldp(src + 16, o + 16u < size ? size - o - 16u : 0);
                q2 = ldp(src + 32, o + 32u < size ? size - o - 32u : 0);
                q3 = ldp(src + 48, o + 48u < size ? size - o - 48u : 0);
            }
            u32 C[16] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w,
                         q2.x, q2.y, q2.z, q2.w, q3.x, q3.y, q3.z, q3.w};
            salsa20_block(x, key, n0, n1, blk, 0u);
            if (full) {
                poly_block(P, C[0], C[1], C[2], C[3], 1u);
                poly_block(P, C[4], C[5], C[6], C[7], 1u);
                poly_block(P, C[8], C[9], C[10], C[11], 1u);
                poly_block(P, C[12], C[13], C[14], C[15], 1u);
                mpoly += 4;
            } else {
                const u32 tailv = mlen - 64u * blk;
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const u32 s = 16u * j;
                    if (s < tailv) {
                        const u32 nb = tailv - s;
                        if (nb >= 16)
                            poly_block(P, C[4 * j], C[4 * j + 1], C[4 * j + 2], C[4 * j + 3], 1u);
                        else
                            poly_block_partial(P, C[4 * j], C[4 * j + 1], C[4 * j + 2], C[4 * j + 3], nb);
                        mpoly++;
                    }
                }
            }
#pragma unroll
            for (int k = 0; k < 16; k++)
                X[k] = C[k] ^ x[k];
        } else {
#pragma unroll
            for (int k = 0; k < 16; k++)
                X[k] = 0u;
        }
        u32 O[16];
        u32 E[17] = {K[0], K[1], K[2], K[3], K[4], K[5], K[6], K[7], X[0], X[1], X[2], X[3], X[4], X[5], X[6], X[7],
                     X[8]};
#pragma unroll
        for (int t = 0; t < 16; t++)
            O[t] = funnel(E[t + 1], E[t], 1);
        em.emit(q, O);
#pragma unroll
        for (int k = 0; k < 8; k++)
            K[k] = X[8 + k];
    }
    bool bad = false;
    if (!rec) {
        u32 tag[4];
        poly_finish(P, tag);
        V4 tin = ld16<AL>(in + 16, size - 16u);
        bad = ((tag[0] ^ tin.x) | (tag[1] ^ tin.y) | (tag[2] ^ tin.z) | (tag[3] ^ tin.w)) != 0;
    }
    em.close(bad);  // convergent: a cooperative flush must see every lane of the wave
    if (!rec)
        return bad ? CZ_STATUS_CRYPTO : CZ_STATUS_OK;
    rec[0] = P.h0; rec[1] = P.h1; rec[2] = P.h2; rec[3] = P.h3; rec[4] = P.h4; rec[5] = mpoly;
    if (b0 == 0) {
        rec[6] = flags_out;
        rec[8] = P.r0; rec[9] = P.r1; rec[10] = P.r2; rec[11] = P.r3;
        rec[12] = P.p0; rec[13] = P.p1; rec[14] = P.p2; rec[15] = P.p3;
    }
    return CZ_STATUS_OK;
}

// Join a frame's segment records: H = Horner over segments with multipliers r^m.
// The planner cuts every segment but a frame's last to the same length, so a lane needs two
// powers, r^m_mid and r^m_last. One square-and-multiply chain over the bits yields both, its
// loop bound wave-uniform; a multiply runs where any lane of the wave has that bit set. (Caching
// r^m at each change of m instead ran one divergent exponentiation per distinct segment count
// in the wave: ~45 us per Zipf batch, one latency-bound lane per split frame.) A middle segment
// of another length, which no plan makes, still gets its own power.
__device__ __forceinline__ void combine_tag(const u32 *__restrict__ R0, u32 nseg, u32 tag[4])
{
    const F26 r = f26_from32(R0[8], R0[9], R0[10], R0[11], 0u);
    F26 H = f26_from32(R0[0], R0[1], R0[2], R0[3], R0[4]);
    if (nseg > 1u) {
        const u32 *RL = R0 + 16u * (nseg - 1u);
        const u32 m_last = RL[5];
        const u32 m_mid = nseg > 2u ? R0[16 + 5] : m_last;
        const F26 hl = f26_from32(RL[0], RL[1], RL[2], RL[3], RL[4]);
        F26 hn = nseg > 2u ? f26_from32(R0[16], R0[17], R0[18], R0[19], R0[20]) : hl;
        F26 base = r, pm = {{1u, 0u, 0u, 0u, 0u}}, pl = pm;
        for (u32 bit = 0; __builtin_amdgcn_ballot_w64(((m_mid | m_last) >> bit) != 0u) != 0; bit++) {
            if (bit)
                base = f26_mul(base, base);
            if ((m_mid >> bit) & 1u)
                pm = f26_mul(pm, base);
            if ((m_last >> bit) & 1u)
                pl = f26_mul(pl, base);
        }
        for (u32 s = 1; s + 1u < nseg; s++) {
            const u32 *R = R0 + 16u * s;
            const F26 h = hn;
            const u32 m = R[5];
            if (s + 2u < nseg)  // next record's loads in flight under this multiply
                hn = f26_from32(R[16], R[17], R[18], R[19], R[20]);
            F26 pw = pm;
            if (m != m_mid)
                pw = f26_pow(r, m);
            H = f26_add(f26_mul(H, pw), h);
        }
        H = f26_add(f26_mul(H, pl), hl);
    }
    Poly Q;
    f26_to32(H, Q.h0, Q.h1, Q.h2, Q.h3, Q.h4);
    Q.p0 = R0[12]; Q.p1 = R0[13]; Q.p2 = R0[14]; Q.p3 = R0[15];
    poly_finish(Q, tag);
}

// ---- kernels -------------------------------------------------------------

enum Staging { ST_DIRECT = 0, ST_LINES = 1, ST_REGION = 2, ST_SHIFT = 3 };

// Uniform batch of one connection direction: frame i = in[i*in_stride .. +len)
// -> slot out[i*out_stride .. +out_stride), nonce counter0 + i, flags8[i] (or 0).
// ST_LINES / ST_REGION need the launcher's preconditions (see czk_seal_uniform);
// a wave with fewer than 64 frames always stores directly.
// MODE_BOX (cz_seal_uniform_box): frame i = the box at in + i*in_stride (len = payload bytes),
// flags from box byte 32, flags8 unused.
// INA (seal_frame, MODE_ZMQ): 16 for 16-byte aligned payload slots; 8 / 1 for payloads at 8-byte /
// any byte offsets (messages packed back to back), staged kernels only
template <int ST, bool PAIR, int MODE, int INA>
__device__ __forceinline__ void seal_uniform_body(const uint8_t *__restrict__ in, uint64_t in_stride,
                                                  uint8_t *__restrict__ out, uint64_t out_stride, uint32_t count,
                                                  uint32_t len, const uint8_t *__restrict__ subkey, uint64_t counter0,
                                                  const uint8_t *__restrict__ flags8, int allow_un0)
{
    extern __shared__ uint4 smem[];
    uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if constexpr (ST == ST_SHIFT) {
        // waves of one line phase (EmitShiftLines): a full workgroup's frames sorted by class
        if (blockIdx.x * BLOCK + BLOCK <= count)
            i = blockIdx.x * BLOCK + class_permute(((uintptr_t)(out + (uint64_t)i * out_stride) & 64u) != 0,
                                                   reinterpret_cast<u32 *>(smem));
    }
    const uint32_t wave_first = (blockIdx.x * BLOCK + threadIdx.x) & ~63u;
    if (wave_first >= count)
        return;
    u32 key[8];
    load_key(subkey, key);
    const bool full_wave = wave_first + 64u <= count;
    const uint8_t *src = in + (uint64_t)i * in_stride;
    uint8_t *dst = out + (uint64_t)i * out_stride;
    const u32 mlen = len + 33u;
    // high nonce word uniform over the wave (true unless the counters cross a 2^32 boundary)
    const bool un0 = allow_un0 && wave_uniform((u32)((counter0 + i) >> 32));
    if (ST != ST_DIRECT && full_wave) {
        const u32 fl = (MODE == MODE_ZMQ && flags8) ? flags8[i] : 0u;
        const u32 lane = threadIdx.x & 63u;
        if constexpr (ST == ST_LINES) {
            using EmL = EmitLinesSeal;
            EmL em{smem + (threadIdx.x >> 6) * (LINE_LDS_BYTES / 16), out + (uint64_t)wave_first * out_stride,
                   dst, out_stride, lane, mlen, 0u, true,
                   smem + (WAVES * LINE_LDS_BYTES + (threadIdx.x >> 6) * HOLD_LDS_BYTES) / 16};
            if (un0)
                seal_frame<MODE, true, EmL, PAIR, true, true, INA>(src, len, fl, counter0 + i, key, em);
            else
                seal_frame<MODE, true, EmL, PAIR, false, true, INA>(src, len, fl, counter0 + i, key, em);
        } else if constexpr (ST == ST_SHIFT) {
            // bodies at any byte offset (dense packing, wire layout): byte-shifted line staging
            EmitShiftLinesUniSeal em{reinterpret_cast<uint8_t *>(smem) + (threadIdx.x >> 6) * SHIFT_LDS_BYTES, dst, lane,
                                 mlen, 0u, 0u};
            em.init(true, true);
            em.init_uniform(i - blockIdx.x * BLOCK, (u32)out_stride, out + (uint64_t)blockIdx.x * BLOCK * out_stride);
            // bodies back to back (the V2 wire layout) whose last chunk is a tail chunk (emit, not
            // the pair loop's emit_steady): edge units shared with the neighbours leave whole
            const bool b2b = out_stride == (uint64_t)mlen && (mlen & 63u) != 0u;
            em.init_ext(b2b && i > 0u, b2b && i + 1u < count);
            if (un0 && !em.mixed) {
                // one line class per wave (class_permute): the class-static emitter
                if (__builtin_amdgcn_readfirstlane((((u32)(uintptr_t)dst & 64u) == 0u) ? 1u : 0u)) {
                    EmitShiftLinesUniClassSeal<1> ec{em};
                    seal_frame<MODE, true, EmitShiftLinesUniClassSeal<1>, PAIR, true, true, INA>(src, len, fl,
                                                                                               counter0 + i, key, ec);
                } else {
                    EmitShiftLinesUniClassSeal<0> ec{em};
                    seal_frame<MODE, true, EmitShiftLinesUniClassSeal<0>, PAIR, true, true, INA>(src, len, fl,
                                                                                               counter0 + i, key, ec);
                }
            } else if (un0)
                seal_frame<MODE, true, EmitShiftLinesUniSeal, PAIR, true, true, INA>(src, len, fl, counter0 + i, key, em);
            else
                seal_frame<MODE, true, EmitShiftLinesUniSeal, PAIR, false, true, INA>(src, len, fl, counter0 + i, key, em);
        } else {
            const u32 st = (u32)out_stride;
            EmitRegionSeal em{smem + (threadIdx.x >> 6) * ((64u * st) >> 4), out + (uint64_t)wave_first * out_stride, st,
                          lane, mlen};
            if (un0)
                seal_frame<MODE, true, EmitRegionSeal, PAIR, true, true, INA>(src, len, fl, counter0 + i, key, em);
            else
                seal_frame<MODE, true, EmitRegionSeal, PAIR, false, true, INA>(src, len, fl, counter0 + i, key, em);
        }
        return;
    }
    if (i >= count)
        return;
    const u32 fl = (MODE == MODE_ZMQ && flags8) ? flags8[i] : 0u;
    if (aligned16(src, dst)) {
        EmitDirect<true> em{dst, mlen};
        seal_frame<MODE, true, EmitDirect<true>, PAIR>(src, len, fl, counter0 + i, key, em);
    } else if ((((uintptr_t)src) & 15u) == 0) {
        EmitDirect<false> em{dst, mlen};
        seal_frame<MODE, true, EmitDirect<false>, PAIR>(src, len, fl, counter0 + i, key, em);
    } else {
        EmitDirect<false> em{dst, mlen};
        seal_frame<MODE, false>(src, len, fl, counter0 + i, key, em);
    }
    // the partial last wave of a batch that owns its slots: zeros past the body, as the staged waves
    if constexpr (ST == ST_LINES || ST == ST_REGION)
        if (out_stride > mlen)
            zero_bytes(dst + mlen, (u32)(out_stride - mlen));
}

#ifdef CZ_DIAG_CLOCK
// Clock diagnostic (tools/build_variant.sh NAME -DCZ_DIAG_CLOCK, tools/clock_stamp.py): every wave of
// k_seal_uniform, k_open_uniform and k_seal_segments_lines stamps the shader clock counter (s_memtime) and the 100 MHz constant counter
// (s_memrealtime) when it starts and when it leaves; lane 0 writes the four values with a vector
// store.  Wave clock = d(memtime) / d(realtime) * 100 MHz, unprofiled.  Output bytes are unchanged.
constexpr u32 DIAG_CLOCK_WAVES = 1u << 16;
static __device__ uint64_t g_diag_clock[DIAG_CLOCK_WAVES * 4u];
#define CZ_DIAG_CLOCK_BEGIN                                                                                   \
    const uint64_t dc_t0 = __builtin_amdgcn_s_memtime(), dc_r0 = __builtin_amdgcn_s_memrealtime();
#define CZ_DIAG_CLOCK_END                                                                                     \
    {                                                                                                         \
        const uint64_t dc_t1 = __builtin_amdgcn_s_memtime(), dc_r1 = __builtin_amdgcn_s_memrealtime();       \
        const u32 w = blockIdx.x * WAVES + (threadIdx.x >> 6);                                                \
        if ((threadIdx.x & 63u) == 0u && w < DIAG_CLOCK_WAVES) {                                              \
            volatile uint64_t *g = g_diag_clock + 4u * w;                                                     \
            g[0] = dc_t0; g[1] = dc_r0; g[2] = dc_t1; g[3] = dc_r1;                                           \
        }                                                                                                     \
    }
#else
#define CZ_DIAG_CLOCK_BEGIN
#define CZ_DIAG_CLOCK_END
#endif

template <int ST, bool PAIR, int MODE = MODE_ZMQ>
__global__ __launch_bounds__(BLOCK) CZ_OCC CZ_OPEN_UNI_OCC void k_seal_uniform(const uint8_t *__restrict__ in, uint64_t in_stride,
                                                         uint8_t *__restrict__ out, uint64_t out_stride,
                                                         uint32_t count, uint32_t len,
                                                         const uint8_t *__restrict__ subkey, uint64_t counter0,
                                                         const uint8_t *__restrict__ flags8, int allow_un0)
{
    CZ_DIAG_CLOCK_BEGIN
    seal_uniform_body<ST, PAIR, MODE, 16>(in, in_stride, out, out_stride, count, len, subkey, counter0, flags8,
                                          allow_un0);
    CZ_DIAG_CLOCK_END
}

// payloads off 16-byte alignment (INA 8 / 1): at least 3 waves per SIMD (uncapped, the funnelled
// loads take the line kernels to 169-186 VGPRs, 2 waves)
template <int ST, bool PAIR, int INA>
__global__ __launch_bounds__(BLOCK) CZ_OCC CZ_OPEN_UNI_OCC void k_seal_uniform_ina(
    const uint8_t *__restrict__ in, uint64_t in_stride, uint8_t *__restrict__ out, uint64_t out_stride, uint32_t count,
    uint32_t len, const uint8_t *__restrict__ subkey, uint64_t counter0, const uint8_t *__restrict__ flags8,
    int allow_un0)
{
    seal_uniform_body<ST, PAIR, MODE_ZMQ, INA>(in, in_stride, out, out_stride, count, len, subkey, counter0, flags8,
                                               allow_un0);
}

#if CZ_KPART_HAS(3)
__global__ __launch_bounds__(BLOCK) void k_seal_desc(const cz_frame_desc *__restrict__ desc,
                                                      const uint32_t *__restrict__ order, uint32_t count,
                                                      const uint8_t *__restrict__ in, uint8_t *__restrict__ out,
                                                      const uint8_t *__restrict__ subkeys)
{
    const uint32_t t = blockIdx.x * BLOCK + threadIdx.x;
    if (t >= count)
        return;
    const uint32_t i = order ? order[t] : t;
    const cz_frame_desc d = desc[i];
    u32 key[8];
    load_key(subkeys + 32ull * d.key_idx, key);
    const uint8_t *src = in + d.in_off;
    uint8_t *dst = out + d.out_off;
    if (aligned16(src, dst)) {
        EmitDirect<true> em{dst, d.len + 33u};
        seal_frame<MODE_ZMQ, true, EmitDirect<true>, false, false, false>(src, d.len, d.flags & 0xffu, d.counter, key, em);
    } else {
        EmitDirect<false> em{dst, d.len + 33u};
        seal_frame<MODE_ZMQ, false, EmitDirect<false>, false, false, false>(src, d.len, d.flags & 0xffu, d.counter, key, em);
    }
}

// status[i] = CZ_STATUS_* | (flags byte << 8)
__global__ __launch_bounds__(BLOCK) void k_open_desc(const cz_frame_desc *__restrict__ desc,
                                                      const uint32_t *__restrict__ order, uint32_t count,
                                                      const uint8_t *__restrict__ in, uint8_t *__restrict__ out,
                                                      const uint8_t *__restrict__ subkeys,
                                                      uint16_t *__restrict__ status, uint64_t *__restrict__ nonces)
{
    const uint32_t t = blockIdx.x * BLOCK + threadIdx.x;
    if (t >= count)
        return;
    const uint32_t i = order ? order[t] : t;
    const cz_frame_desc d = desc[i];
    u32 key[8];
    load_key(subkeys + 32ull * d.key_idx, key);
    long long floor = (long long)d.counter;
    if (d.prev >= 0) {
        // replay floor = nonce of the previous frame of this connection in the batch
        const cz_frame_desc p = desc[d.prev];
        floor = (long long)read_be64(in + p.in_off + 8);
    }
    const bool check = (d.flags & CZ_DESC_CHECK_NONCE) != 0;
    const uint8_t *src = in + d.in_off;
    uint8_t *dst = out + d.out_off;
    u32 fl = 0;
    u64 nonce = 0;
    u32 st;
    const u32 nout = d.len >= 33u ? d.len - 33u : 0u;
    if (aligned16(src, dst)) {
        EmitDirect<true> em{dst, nout};
        st = open_frame<MODE_ZMQ, true, EmitDirect<true>, false, false, false>(src, d.len, key, check, floor, &fl, &nonce, 0, em);
    } else {
        EmitDirect<false> em{dst, nout};
        st = open_frame<MODE_ZMQ, false, EmitDirect<false>, false, false, false>(src, d.len, key, check, floor, &fl, &nonce, 0, em);
    }
    status[i] = (uint16_t)(st | (st == CZ_STATUS_OK ? (fl << 8) : 0u));
    if (nonces)
        nonces[i] = nonce;
}

#endif  // CZ_KPART_HAS(3)

// Uniform open of one connection's bodies in order: frame i must beat frame
// i-1's nonce, frame 0 must beat floor0 (when check != 0).
// INA (open_frame): 16 for 16-byte aligned bodies; 8 / 1 for bodies at 8-byte / any byte offsets
// (the dense wire layout), line-staged (ST_LINES) plaintext only
// (at least 3 waves per SIMD: the byte-shifted plaintext staging needs 170-179 VGPRs uncapped)
#ifdef CZ_DIAG_CLOCK
// the clock build stamps every wave around the body (k_open_uniform below); the product kernel is
// the body itself, so its machine code does not change with the diagnostic
template <int ST, bool PAIR, int INA>
__device__ __forceinline__ void open_uniform_body(const uint8_t *__restrict__ in, uint64_t in_stride,
                                                  uint8_t *__restrict__ out, uint64_t out_stride, uint32_t count,
                                                  uint32_t size, const uint8_t *__restrict__ subkey, uint64_t floor0,
                                                  int check, uint16_t *__restrict__ status, int allow_un0, int prev0)
#else
template <int ST, bool PAIR, int INA = 16>
__global__ __launch_bounds__(BLOCK) CZ_OCC CZ_OPEN_UNI_OCC void k_open_uniform(const uint8_t *__restrict__ in, uint64_t in_stride,
                                                         uint8_t *__restrict__ out, uint64_t out_stride,
                                                         uint32_t count, uint32_t size,
                                                         const uint8_t *__restrict__ subkey, uint64_t floor0,
                                                         int check, uint16_t *__restrict__ status, int allow_un0,
                                                         int prev0 = 0)
#endif
{
    // prev0: frame 0's floor is the nonce of the body in_stride bytes before it (a tail launched
    // behind the phase-sorted carry kernel), not floor0
    static_assert(INA == 16 || ST != ST_DIRECT, "unaligned bodies: staged plaintext only");
    extern __shared__ uint4 smem[];
    uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if constexpr (ST == ST_SHIFT) {
        // plaintext at any byte offset: a full workgroup's frames sorted by line class, as the seal
        if (blockIdx.x * BLOCK + BLOCK <= count)
            i = blockIdx.x * BLOCK + class_permute(((uintptr_t)(out + (uint64_t)i * out_stride) & 64u) != 0,
                                                   reinterpret_cast<u32 *>(smem));
    }
    const uint32_t wave_first = (blockIdx.x * BLOCK + threadIdx.x) & ~63u;
    if (wave_first >= count)
        return;
    u32 key[8];
    load_key(subkey, key);
    const bool full_wave = wave_first + 64u <= count;
    const uint8_t *src = in + (uint64_t)i * in_stride;
    uint8_t *dst = out + (uint64_t)i * out_stride;
    const u32 nout = size >= 33u ? size - 33u : 0u;
    u32 fl = 0;
    u64 nonce = 0;
    u32 st;
    if (ST != ST_DIRECT && full_wave) {
        // (16-byte aligned slots here: the previous body's nonce is one 8-byte load, not 8 byte loads)
        long long floor = (long long)floor0;
        if (i > 0 || prev0) {
            if constexpr (INA >= 8) {
                const uint2 pn = *reinterpret_cast<const uint2 *>(src - in_stride + 8);
                floor = (long long)(((u64)bswap32(pn.x) << 32) | (u64)bswap32(pn.y));
            } else {
                floor = (long long)read_be64(src - in_stride + 8);
            }
        }
        const u32 lane = threadIdx.x & 63u;
        const bool un0 = allow_un0 && wave_uniform(INA >= 8 ? *reinterpret_cast<const u32 *>(src + 8) : ld32<false>(src + 8));
        if constexpr (ST == ST_LINES) {
            // bodies off 16-byte alignment (the dense wire layout) store non-temporal
            using EmL = EmitLinesT<INA == 16 ? CZ_OPEN_STORE_CPOL : CZ_OPEN_ANY_STORE_CPOL>;
            EmL em{smem + (threadIdx.x >> 6) * (LINE_LDS_BYTES / 16), out + (uint64_t)wave_first * out_stride,
                   dst, out_stride, lane, nout, 0u, false};
            if (un0)
                st = open_frame<MODE_ZMQ, true, EmL, PAIR, true, true, INA>(src, size, key, check != 0, floor, &fl,
                                                                           &nonce, 0, em);
            else
                st = open_frame<MODE_ZMQ, true, EmL, PAIR, false, true, INA>(src, size, key, check != 0, floor, &fl,
                                                                            &nonce, 0, em);
        } else if constexpr (ST == ST_SHIFT) {
            using EmS = EmitShiftLinesT<true, CZ_OPEN_ANY_STORE_CPOL>;  // plaintext at any byte offset
            EmS em{reinterpret_cast<uint8_t *>(smem) + (threadIdx.x >> 6) * SHIFT_LDS_BYTES, dst, lane, nout, 0u, 0u};
            em.init(false);
            em.init_uniform(i - blockIdx.x * BLOCK, (u32)out_stride, out + (uint64_t)blockIdx.x * BLOCK * out_stride);
            if (un0)
                st = open_frame<MODE_ZMQ, true, EmS, PAIR, true, true, INA>(src, size, key, check != 0, floor, &fl,
                                                                           &nonce, 0, em);
            else
                st = open_frame<MODE_ZMQ, true, EmS, PAIR, false, true, INA>(src, size, key, check != 0, floor, &fl,
                                                                            &nonce, 0, em);
        } else {
            const u32 ost = (u32)out_stride;
            EmitRegion em{smem + (threadIdx.x >> 6) * ((64u * ost) >> 4), out + (uint64_t)wave_first * out_stride,
                          ost, lane, nout};
            if (un0)
                st = open_frame<MODE_ZMQ, true, EmitRegion, PAIR, true, true, INA>(src, size, key, check != 0, floor,
                                                                                  &fl, &nonce, 0, em);
            else
                st = open_frame<MODE_ZMQ, true, EmitRegion, PAIR, false, true, INA>(src, size, key, check != 0, floor,
                                                                                   &fl, &nonce, 0, em);
        }
        // rejected frames ran the loop as dead lanes: their slots hold zeros
        status[i] = (uint16_t)(st | (st == CZ_STATUS_OK ? (fl << 8) : 0u));
        return;
    }
    if (i >= count)
        return;
    long long floor = (i > 0 || prev0) ? (long long)read_be64(src - in_stride + 8) : (long long)floor0;
    if (aligned16(src, dst)) {
        EmitDirect<true> em{dst, nout};
        st = open_frame<MODE_ZMQ, true>(src, size, key, check != 0, floor, &fl, &nonce, 0, em);
    } else {
        EmitDirect<false> em{dst, nout};
        st = open_frame<MODE_ZMQ, false>(src, size, key, check != 0, floor, &fl, &nonce, 0, em);
    }
    // lane-wise frames (a partial last wave, or a batch the staged emitters do not take) keep the
    // staged waves' contract: zeros in the payload of a frame rejected before decryption, which
    // emitted nothing (a bad tag's plaintext was already zeroed by poison()), and, in a batch that
    // owns its slots, zeros past the payload
    if (st != CZ_STATUS_OK && st != CZ_STATUS_CRYPTO)
        zero_bytes(dst, nout);
    if constexpr (ST == ST_LINES || ST == ST_REGION)
        if (out_stride > nout)
            zero_bytes(dst + nout, (u32)(out_stride - nout));
    status[i] = (uint16_t)(st | (st == CZ_STATUS_OK ? (fl << 8) : 0u));
}

#ifdef CZ_DIAG_CLOCK
template <int ST, bool PAIR, int INA = 16>
__global__ __launch_bounds__(BLOCK) CZ_OCC CZ_OPEN_UNI_OCC void k_open_uniform(const uint8_t *__restrict__ in, uint64_t in_stride,
                                                         uint8_t *__restrict__ out, uint64_t out_stride,
                                                         uint32_t count, uint32_t size,
                                                         const uint8_t *__restrict__ subkey, uint64_t floor0,
                                                         int check, uint16_t *__restrict__ status, int allow_un0,
                                                         int prev0 = 0)
{
    CZ_DIAG_CLOCK_BEGIN
    open_uniform_body<ST, PAIR, INA>(in, in_stride, out, out_stride, count, size, subkey, floor0, check, status,
                                     allow_un0, prev0);
    CZ_DIAG_CLOCK_END
}
#endif

// Phase-sorted open of bodies off 16-byte alignment into line-aligned plaintext slots (the dense
// wire layout: V2Decoder leaves bodies back to back, zmq/io/coder/v2/V2Decoder.java:67-105).
// Frame i's body starts (in + i * in_stride) & 127 bytes into a cache line; that phase repeats
// every P = 128 / gcd(in_stride mod 128, 128) frames.  Within each block of 64 P frames, wave c
// takes frames c, c + P, ..., c + 63 P: one phase per wave, so open_frame<CARRY> loads every
// aligned line of a body once and carries it into the next pair.  Plaintext slot j of the wave is
// out + (first + P j) * out_stride, EmitLines with a lane stride of P * out_stride.  nwaves = the
// number of whole blocks x P; the frames after them go to k_open_uniform (prev0 = 1).
template <int INA>
__global__ __launch_bounds__(BLOCK) CZ_OPEN_CARRY_OCC void k_open_uniform_carry(
    const uint8_t *__restrict__ in, uint64_t in_stride, uint8_t *__restrict__ out, uint64_t out_stride, uint32_t nwaves,
    uint32_t P, uint32_t size, const uint8_t *__restrict__ subkey, uint64_t floor0, int check,
    uint16_t *__restrict__ status, int allow_un0)
{
    extern __shared__ uint4 smem[];
    const uint32_t w = (blockIdx.x * BLOCK + threadIdx.x) >> 6;
    if (w >= nwaves)
        return;
    const u32 lane = threadIdx.x & 63u;
    const uint32_t first = (w / P) * 64u * P + w % P;
    const uint32_t i = first + P * lane;
    u32 key[8];
    load_key(subkey, key);
    const uint8_t *src = in + (uint64_t)i * in_stride;
    uint8_t *dst = out + (uint64_t)i * out_stride;
    const u32 nout = size - 33u;
    long long floor = (long long)floor0;
    if (i > 0) {
        if constexpr (INA >= 8) {
            const uint2 pn = *reinterpret_cast<const uint2 *>(src - in_stride + 8);
            floor = (long long)(((u64)bswap32(pn.x) << 32) | (u64)bswap32(pn.y));
        } else {
            floor = (long long)read_be64(src - in_stride + 8);
        }
    }
    const bool un0 = allow_un0 && wave_uniform(INA >= 8 ? *reinterpret_cast<const u32 *>(src + 8) : ld32<false>(src + 8));
    using EmL = EmitLinesT<INA == 8 ? CZ_OPEN_STORE_CPOL : CZ_OPEN_ANY_STORE_CPOL>;
    EmL em{smem + (threadIdx.x >> 6) * (LINE_LDS_BYTES / 16), out + (uint64_t)first * out_stride, dst,
           (uint64_t)P * out_stride, lane, nout, 0u, false};
    u32 fl = 0;
    u64 nonce = 0;
    u32 st;
    if (un0)
        st = open_frame<MODE_ZMQ, true, EmL, true, true, true, INA, true>(src, size, key, check != 0, floor, &fl,
                                                                            &nonce, 0, em);
    else
        st = open_frame<MODE_ZMQ, true, EmL, true, false, true, INA, true>(src, size, key, check != 0, floor, &fl,
                                                                             &nonce, 0, em);
    status[i] = (uint16_t)(st | (st == CZ_STATUS_OK ? (fl << 8) : 0u));
}

#if CZ_KPART_HAS(3)
// ---- segmented (ragged) batches ------------------------------------------
constexpr int SEGMODE_LINES = 1;  // line-staged stores for waves of equal-length segments
constexpr int SEGMODE_PAIR = 2;   // whole-line input loads (seal)

// A wave takes the line emitter when all 64 lanes hold segments with the same
// chunk count and 16-byte aligned input/output; otherwise each lane stores directly.
// Seal, whole-line loads: a full wave of aligned segments may mix chunk counts; shorter
// segments run along to the wave's longest (wave_max) with their extra blocks discarded.
__device__ __forceinline__ bool wave_lines_ragged_ok(bool full_wave, bool al)
{
    return full_wave && __builtin_amdgcn_ballot_w64(!al) == 0;
}
__device__ __forceinline__ u32 wave_max(u32 v)
{
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const u32 w = (u32)__shfl_xor((int)v, o);
        v = w > v ? w : v;
    }
    return v;
}

__device__ __forceinline__ bool wave_lines_ok(bool full_wave, u32 nchunks, bool al)
{
    if (!full_wave)
        return false;
    return wave_uniform(nchunks) && __builtin_amdgcn_ballot_w64(!al) == 0;
}

constexpr int SEGMODE_REST = 4;   // k_seal_segments: only the waves k_seal_segments_lines leaves
constexpr int SEGMODE_SHIFT16 = 8;  // 16-byte aligned outputs not all on 128-byte lines: EmitShiftLines
constexpr int SEGMODE_ANYIN = 16;   // inputs at any byte offset on the line paths (dword-aligned loads)

// Segment kernels.  With line staging and whole-line loads enabled the launcher runs two
// kernels over the same segment list: k_seal_segments_lines takes every full wave of aligned
// segments (wave_lines_ragged_ok) and is built for 3 waves per SIMD (168 VGPRs; its single
// path fits them, while the general kernel needs ~190 and runs 2); k_seal_segments with
// SEGMODE_REST then takes exactly the other waves (same predicate, inverted: the partial last
// wave and unaligned buffers).  Without those modes k_seal_segments alone runs every wave.
enum { SEGPART_ALL = 0, SEGPART_LINES = 1, SEGPART_REST = 2 };

template <int PART>
__device__ __forceinline__ void seal_segments_body(const cz_frame_desc *__restrict__ desc,
                                                   const cz_segment *__restrict__ segs, uint32_t nseg,
                                                   const uint8_t *__restrict__ in, uint8_t *__restrict__ out,
                                                   const uint8_t *__restrict__ subkeys, u32 *__restrict__ work,
                                                   int mode, uint4 *smem)
{
    const uint32_t t = blockIdx.x * BLOCK + threadIdx.x;
    const uint32_t wave_first = t & ~63u;
    const bool allow_lines = mode & SEGMODE_LINES, pair = mode & SEGMODE_PAIR;
    if (wave_first >= nseg)
        return;
    const bool live = t < nseg;
    const cz_segment sg = segs[live ? t : wave_first];
    const cz_frame_desc d = desc[sg.frame];
    u32 *rec = sg.part == 0xffffffffu ? nullptr : work + 16ull * sg.part;
    const uint8_t *src = in + d.in_off;
    uint8_t *dst = out + d.out_off + 64ull * sg.first_block;
    const u32 b1 = sg.first_block + sg.nblocks;
    const u32 mlen = d.len + 33u;
    const u32 nblk = (mlen + 63u) >> 6;
    const u32 nch = (b1 < nblk ? b1 : nblk) - sg.first_block;
    const u32 total = seal_seg_bytes(mlen, sg.first_block, b1 < nblk ? b1 : nblk);
    const bool al = aligned16(src, dst);
    // whole-line loads: a full wave of 16-byte aligned inputs takes a line emitter, EmitSegLines
    // when every output is 16-byte aligned too, EmitShiftLines (any byte offset) otherwise
    const bool in_al = (((uintptr_t)src) & 15u) == 0;
    const bool full_wave = wave_first + 64u <= nseg;
    const bool lines = allow_lines && (pair ? wave_lines_ragged_ok(full_wave, in_al) : wave_lines_ok(full_wave, nch, al));
    if constexpr (PART == SEGPART_LINES) {
        if (!lines)
            return;
    }
    if constexpr (PART == SEGPART_REST) {
        if (lines)
            return;
    }
    u32 key[8];
    load_key(subkeys + 32ull * d.key_idx, key);
    if constexpr (PART != SEGPART_REST) {
        if (lines) {
            const u32 lane = threadIdx.x & 63u;
            uint8_t *wl = reinterpret_cast<uint8_t *>(smem) + (threadIdx.x >> 6) * SHIFT_LDS_BYTES;
            if (PART == SEGPART_LINES || pair) {
                // EmitSegLines stores 128-byte groups at each output's own base, which straddle two
                // cache lines unless the base is line-aligned; EmitShiftLines stores whole cache
                // lines at any base (SEGMODE_SHIFT16 sends it the 16-byte aligned waves too)
                const bool line_al = (((uintptr_t)dst) & 127u) == 0;
                if (__builtin_amdgcn_ballot_w64(!al) == 0 &&
                    (!(mode & SEGMODE_SHIFT16) || __builtin_amdgcn_ballot_w64(!line_al) == 0)) {
                    EmitSegLinesSeal em{reinterpret_cast<uint4 *>(wl), dst, lane, total, 0u, 0u};
                    em.init(sg.first_block == 0);
                    seal_segment<true, EmitSegLinesSeal, true>(src, d.len, d.flags & 0xffu, d.counter, key,
                                                           sg.first_block, b1, rec, em, wave_max(nch));
                } else {
                    EmitShiftLinesSeal em{wl, dst, lane, total, 0u, 0u};
                    em.init(sg.first_block == 0);
                    seal_segment<true, EmitShiftLinesSeal, true>(src, d.len, d.flags & 0xffu, d.counter, key,
                                                             sg.first_block, b1, rec, em, wave_max(nch));
                }
            } else {
                EmitSegLinesSeal em{reinterpret_cast<uint4 *>(wl), dst, lane, total, 0u, 0u};
                em.init(sg.first_block == 0);
                seal_segment<true>(src, d.len, d.flags & 0xffu, d.counter, key, sg.first_block, b1, rec, em);
            }
            return;
        }
    }
    if constexpr (PART == SEGPART_REST) {
        // full waves left here because some payload is off 16-byte alignment: line-staged stores
        // with dword-aligned loads (seal_segment INA 8 / 1) instead of lane-wise paths
        if (allow_lines && pair && full_wave && (mode & SEGMODE_ANYIN)) {
            const u32 lane = threadIdx.x & 63u;
            uint8_t *wl = reinterpret_cast<uint8_t *>(smem) + (threadIdx.x >> 6) * SHIFT_LDS_BYTES;
            EmitShiftLinesSeal em{wl, dst, lane, total, 0u, 0u};
            em.init(sg.first_block == 0);
            if (__builtin_amdgcn_ballot_w64((((uintptr_t)src) & 7u) != 0u) == 0)
                seal_segment<true, EmitShiftLinesSeal, true, 8>(src, d.len, d.flags & 0xffu, d.counter, key,
                                                            sg.first_block, b1, rec, em, wave_max(nch));
            else
                seal_segment<true, EmitShiftLinesSeal, true, 1>(src, d.len, d.flags & 0xffu, d.counter, key,
                                                            sg.first_block, b1, rec, em, wave_max(nch));
            return;
        }
    }
    if constexpr (PART != SEGPART_LINES) {
        if (!live)
            return;
        if (al) {
            EmitDirect<true> em{dst, total};
            if (pair)
                seal_segment<true, EmitDirect<true>, true>(src, d.len, d.flags & 0xffu, d.counter, key,
                                                           sg.first_block, b1, rec, em);
            else
                seal_segment<true>(src, d.len, d.flags & 0xffu, d.counter, key, sg.first_block, b1, rec, em);
        } else {
            EmitDirect<false> em{dst, total};
            seal_segment<false>(src, d.len, d.flags & 0xffu, d.counter, key, sg.first_block, b1, rec, em);
        }
    }
}

__global__ __launch_bounds__(BLOCK) CZ_SEG_OCC void k_seal_segments(const cz_frame_desc *__restrict__ desc,
                                                          const cz_segment *__restrict__ segs, uint32_t nseg,
                                                          const uint8_t *__restrict__ in, uint8_t *__restrict__ out,
                                                          const uint8_t *__restrict__ subkeys,
                                                          u32 *__restrict__ work, int mode)
{
    extern __shared__ uint4 smem[];
    if (mode & SEGMODE_REST)
        seal_segments_body<SEGPART_REST>(desc, segs, nseg, in, out, subkeys, work, mode, smem);
    else
        seal_segments_body<SEGPART_ALL>(desc, segs, nseg, in, out, subkeys, work, mode, smem);
}

// mode must hold SEGMODE_LINES | SEGMODE_PAIR
__global__ __launch_bounds__(BLOCK) CZ_SEG_LINES_OCC void k_seal_segments_lines(
    const cz_frame_desc *__restrict__ desc, const cz_segment *__restrict__ segs, uint32_t nseg,
    const uint8_t *__restrict__ in, uint8_t *__restrict__ out, const uint8_t *__restrict__ subkeys,
    u32 *__restrict__ work, int mode)
{
    extern __shared__ uint4 smem[];
    CZ_DIAG_CLOCK_BEGIN
    seal_segments_body<SEGPART_LINES>(desc, segs, nseg, in, out, subkeys, work, mode, smem);
    CZ_DIAG_CLOCK_END
}

__global__ __launch_bounds__(BLOCK) void k_seal_combine(const cz_frame_desc *__restrict__ desc,
                                                         const cz_combine *__restrict__ comb, uint32_t ncomb,
                                                         uint8_t *__restrict__ out, const u32 *__restrict__ work)
{
    const uint32_t t = blockIdx.x * BLOCK + threadIdx.x;
    if (t >= ncomb)
        return;
    const cz_combine cb = comb[t];
    const cz_frame_desc d = desc[cb.frame];
    u32 tag[4];
    combine_tag(work + 16ull * cb.part0, cb.nseg, tag);
    uint8_t *dst = out + d.out_off + 16;
    if ((((uintptr_t)dst) & 15u) == 0)
        st16<true>(dst, tag[0], tag[1], tag[2], tag[3]);
    else
        st16<false>(dst, tag[0], tag[1], tag[2], tag[3]);
}

__global__ __launch_bounds__(BLOCK) CZ_OPEN_SEG_OCC void k_open_segments(const cz_frame_desc *__restrict__ desc,
                                                          const cz_segment *__restrict__ segs, uint32_t nseg,
                                                          const uint8_t *__restrict__ in, uint8_t *__restrict__ out,
                                                          const uint8_t *__restrict__ subkeys,
                                                          u32 *__restrict__ work, uint16_t *__restrict__ status,
                                                          uint64_t *__restrict__ nonces, int mode)
{
    const bool allow_lines = mode & SEGMODE_LINES;
    extern __shared__ uint4 smem[];
    uint32_t t = blockIdx.x * BLOCK + threadIdx.x;
    const uint32_t wave_first = t & ~63u;
    if (wave_first >= nseg)
        return;
    const bool live = t < nseg;
    const cz_segment sg = segs[live ? t : wave_first];
    const cz_frame_desc d = desc[sg.frame];
    long long floor = (long long)d.counter;
    if (d.prev >= 0)
        floor = (long long)read_be64(in + desc[d.prev].in_off + 8);
    const bool check = (d.flags & CZ_DESC_CHECK_NONCE) != 0;
    const uint8_t *src = in + d.in_off;
    u32 n0 = 0, n1 = 0;
    u64 nonce = 0;
    const u32 early = open_header(src, d.len, check, floor, n0, n1, nonce);
    u32 *rec = sg.part == 0xffffffffu ? nullptr : work + 16ull * sg.part;
    const bool seg0 = sg.first_block == 0;
    if (live && seg0) {
        if (nonces)
            nonces[sg.frame] = nonce;
        if (rec)
            rec[7] = early;  // the combine kernel finishes frames whose header passed
        if (early != CZ_STATUS_OK)
            status[sg.frame] = (uint16_t)early;
    }
    u32 key[8];
    load_key(subkeys + 32ull * d.key_idx, key);
    const u32 b1 = sg.first_block + sg.nblocks;
    OpenSeg g{};
    u32 nch = 0;
    if (early == CZ_STATUS_OK) {
        g = open_seg_geom(d.len, sg.first_block, b1);
        nch = g.ce - g.cb;
    }
    uint8_t *dst = out + d.out_off + 64ull * g.cb;
    const u32 total = early == CZ_STATUS_OK ? (g.bend == g.nblk ? g.nout : 64u * g.ce) - 64u * g.cb : 0u;
    const bool al = aligned16(src, dst);
    const bool in_al = (((uintptr_t)src) & 15u) == 0;  // the line emitter takes outputs at any byte offset
    // bodies at 8-byte offsets take the line emitters too, reading with 8-byte loads (lane-wise
    // byte-exact stores ran them at ~1030 GiB/s on the Zipf batch)
    const bool in_al8 = (((uintptr_t)src) & 7u) == 0;
    const bool any_in = (mode & SEGMODE_ANYIN) != 0;  // bodies at any byte offset: funnelled loads
    u32 fl = 0;
    if (allow_lines && wave_lines_ok(wave_first + 64u <= nseg, nch, in_al8 || any_in) &&
        __builtin_amdgcn_ballot_w64(early != CZ_STATUS_OK) == 0) {
        const u32 lane = threadIdx.x & 63u;
        uint8_t *wl = reinterpret_cast<uint8_t *>(smem) + (threadIdx.x >> 6) * SHIFT_LDS_BYTES;
        u32 st;
        const bool line_al = (((uintptr_t)dst) & 127u) == 0;  // as in seal_segments_body
        if (__builtin_amdgcn_ballot_w64(!al) == 0 &&
            (!(mode & SEGMODE_SHIFT16) || __builtin_amdgcn_ballot_w64(!line_al) == 0)) {
            EmitSegLinesT<CZ_OPEN_ANY_STORE_CPOL> em{reinterpret_cast<uint4 *>(wl), dst, lane, total, 0u, 0u};
            em.init(false);
            st = open_segment<true>(src, d.len, key, n0, n1, sg.first_block, b1, rec, fl, em);
        } else {  // plaintext at any byte offset
            using EmS = EmitShiftLinesT<false, CZ_OPEN_ANY_STORE_CPOL>;
            EmS em{wl, dst, lane, total, 0u, 0u};
            em.init(false);
            if (__builtin_amdgcn_ballot_w64(!in_al) == 0)
                st = open_segment<true>(src, d.len, key, n0, n1, sg.first_block, b1, rec, fl, em);
            else if (__builtin_amdgcn_ballot_w64(!in_al8) == 0)
                st = open_segment<false, EmS, true>(src, d.len, key, n0, n1, sg.first_block, b1, rec, fl, em);
            else
                st = open_segment<false, EmS, false, true>(src, d.len, key, n0, n1, sg.first_block, b1, rec, fl, em);
        }
        if (!rec)
            status[sg.frame] = (uint16_t)(st | (st == CZ_STATUS_OK ? (fl << 8) : 0u));
        return;
    }
    if (!live || early != CZ_STATUS_OK)
        return;
    u32 st;
    if (al) {
        EmitDirect<true> em{dst, total};
        st = open_segment<true>(src, d.len, key, n0, n1, sg.first_block, b1, rec, fl, em);
    } else {
        EmitDirect<false> em{dst, total};
        st = open_segment<false>(src, d.len, key, n0, n1, sg.first_block, b1, rec, fl, em);
    }
    if (!rec)
        status[sg.frame] = (uint16_t)(st | (st == CZ_STATUS_OK ? (fl << 8) : 0u));
}

__global__ __launch_bounds__(BLOCK) void k_open_combine(const cz_frame_desc *__restrict__ desc,
                                                         const cz_combine *__restrict__ comb, uint32_t ncomb,
                                                         const uint8_t *__restrict__ in, uint8_t *__restrict__ out,
                                                         const u32 *__restrict__ work,
                                                         uint16_t *__restrict__ status)
{
    const uint32_t t = blockIdx.x * BLOCK + threadIdx.x;
    if (t >= ncomb)
        return;
    const cz_combine cb = comb[t];
    const u32 *R0 = work + 16ull * cb.part0;
    if (R0[7] != CZ_STATUS_OK)
        return;
    const cz_frame_desc d = desc[cb.frame];
    u32 tag[4];
    combine_tag(R0, cb.nseg, tag);
    const uint8_t *tp = in + d.in_off + 16;
    u32 tin[4];
    for (int w = 0; w < 4; w++)
        tin[w] = (u32)tp[4 * w] | ((u32)tp[4 * w + 1] << 8) | ((u32)tp[4 * w + 2] << 16) |
                 ((u32)tp[4 * w + 3] << 24);
    if ((tag[0] ^ tin[0]) | (tag[1] ^ tin[1]) | (tag[2] ^ tin[2]) | (tag[3] ^ tin[3])) {
        // never release unauthenticated plaintext: zero what the segments wrote
        // (16-byte stores over the aligned interior, bytes only at the edges: a tampered 64 KiB frame
        // costs ~4K stores, not 64K serial byte stores)
        uint8_t *dst = out + d.out_off;
        const u32 nout = d.len - 33u;
        const u32 head = (u32)((16u - ((uintptr_t)dst & 15u)) & 15u);
        u32 o = 0;
        for (; o < head && o < nout; o++)
            dst[o] = 0;
        for (; o + 16u <= nout; o += 16u)
            *reinterpret_cast<uint4 *>(dst + o) = make_uint4(0u, 0u, 0u, 0u);
        for (; o < nout; o++)
            dst[o] = 0;
        status[cb.frame] = CZ_STATUS_CRYPTO;
    } else {
        status[cb.frame] = (uint16_t)(CZ_STATUS_OK | (R0[6] << 8));
    }
}


// ---- ZMTP v2 framing (V2Encoder / V2Decoder) -------------------------------
// One wave per item copies `size` bytes between arbitrary byte offsets: lane w
// owns 16-byte aligned destination word w (lanes coalesce on consecutive words),
// reads the 5 source dwords that cover it with clamped aligned loads and
// funnels them by the item's constant byte shift; partially covered edge words
// are stored byte by byte (adjacent items and headers own the other bytes).
// With CZ_V2_ITEM_HEADER, the V2Encoder header (V2Encoder.java:31-55: flags byte
// with LARGE for size > 255, then a 1-byte size or a BE64 size) is written at
// dst_off and the body after it.
__device__ __forceinline__ u32 ld_dw_clamped(const uint8_t *__restrict__ base, intptr_t lo, intptr_t hi, intptr_t a)
{
    a = a < lo ? lo : (a > hi ? hi : a);
    return *reinterpret_cast<const u32 *>(base + a);
}

__global__ __launch_bounds__(BLOCK) void k_v2_copy(const cz_v2_item *__restrict__ items, uint32_t count,
                                                    const uint8_t *__restrict__ src, uint8_t *__restrict__ dst)
{
    const uint32_t wave = __builtin_amdgcn_readfirstlane((blockIdx.x * BLOCK + threadIdx.x) >> 6);
    const u32 lane = threadIdx.x & 63u;
    if (wave >= count)
        return;
    const cz_v2_item it = items[wave];
    uint64_t d = it.dst_off;
    if (it.flags & CZ_V2_ITEM_HEADER) {
        const bool large = it.size > 255u;
        const u32 h = large ? 9u : 2u;
        if (lane < h) {
            u32 b;
            if (lane == 0)
                b = (it.flags & 0xffu & ~(u32)CZ_V2_LARGE) | (large ? (u32)CZ_V2_LARGE : 0u);
            else if (!large)
                b = it.size;
            else
                b = (u32)((uint64_t)it.size >> (8u * (8u - lane)));  // BE64, Wire.putUInt64
            dst[d + lane] = (uint8_t)b;
        }
        d += h;
    }
    const u32 n = it.size;
    if (n == 0)
        return;
    const uintptr_t t0 = (uintptr_t)(dst + d);
    const uintptr_t s0 = (uintptr_t)(src + it.src_off);
    const uintptr_t a0 = t0 & ~(uintptr_t)15;
    const uintptr_t tend = t0 + n;
    const uint64_t nw = (tend - a0 + 15u) >> 4;
    // source byte for destination byte x is s0 + (x - t0): constant shift r within aligned dwords
    const intptr_t sdelta = (intptr_t)s0 - (intptr_t)t0;
    const u32 r = (u32)(sdelta & 3);
    const uint8_t *sbase = reinterpret_cast<const uint8_t *>(s0 & ~(uintptr_t)3);
    const intptr_t lo = 0, hi = (intptr_t)(((s0 + n - 1u) & ~(uintptr_t)3) - (s0 & ~(uintptr_t)3));
    for (uint64_t w = lane; w < nw; w += 64u) {
        const uintptr_t D = a0 + 16u * w;
        // aligned source dword holding the source byte of destination byte D
        const intptr_t j0 = (intptr_t)((D + sdelta) & ~(uintptr_t)3) - (intptr_t)(s0 & ~(uintptr_t)3);
        u32 S[5];
#pragma unroll
        for (int k = 0; k < 5; k++)
            S[k] = ld_dw_clamped(sbase, lo, hi, j0 + 4 * k);
        u32 o[4];
#pragma unroll
        for (int k = 0; k < 4; k++)
            o[k] = r ? funnel(S[k + 1], S[k], r) : S[k];
        uint8_t *p = reinterpret_cast<uint8_t *>(D);
        if (D >= t0 && D + 16u <= tend) {
            *reinterpret_cast<uint4 *>(p) = make_uint4(o[0], o[1], o[2], o[3]);
        } else {
            for (u32 b = 0; b < 16u; b++) {
                const uintptr_t x = D + b;
                if (x >= t0 && x < tend)
                    p[b] = (uint8_t)(o[b >> 2] >> (8u * (b & 3u)));
            }
        }
    }
}

// ---- one NaCl box per launch (the jnacl crypto_box_afternm / open_afternm drop-ins) ----------
// One call used to be a chain of copies and launches (subkey, segments, combine, wipe): ~50 us at
// 4 KiB against ~11 us for a bare launch + sync (tools/diag/latency_ub.hip).  This kernel does the
// whole call in ONE launch of one 256-thread workgroup, reading its input from and writing its
// output to the caller thread's pinned staging (host memory the device addresses directly):
//   - the subkey HSalsa20(k, n[0:16]) comes from the thread's device cache, or is derived here and
//     cached (CurveZMQ uses one (k, "CurveZMQMESSAGE?") pair per connection direction);
//   - thread t owns box blocks [t*w, t*w + w), walked in passes of NACL_ONE_W blocks (one pass for
//     boxes up to 80 KiB): loads them, XORs its keystream, writes the output and runs Horner over
//     the pass's ciphertext;
//   - the MAC key is NaCl's: crypto_secretbox keys Poly1305 with c[0:32] = keystream ^ m[0:32], so a
//     seal whose m[0:32] is not zero (jnacl and libsodium accept it; Curve.box, Curve.java:184-193,
//     reaches it) gets the same tag as theirs; crypto_secretbox_open keys it with the keystream;
//   - Poly1305 over c[32:len) in parallel: each thread's Horner value over its own 16-byte blocks
//     (box block b >= 1 holds MAC blocks 4b-2 .. 4b+1); the full threads 0..L-1 are joined by a
//     pairwise tree with multipliers r^(Q*2^l), Q = 4w MAC blocks per thread (radix 2^26), and the
//     thread L holding the last block finishes H = G * r^(n_L) + A_L.
// k and n come in the kernel arguments; staging layout (bytes): [56,60) rc (written here),
// [128, 128 + len) input, [out_off, out_off + len) output.  Seal: the output holds c[16:len) at
// out_off + 16; open: the output holds m[32:len) at out_off + 32, released by the host only when
// rc == 0.
constexpr int NACL_ONE_T = 256;
constexpr int NACL_ONE_W = 5;  // blocks per thread and pass: one pass covers 256 * 5 * 64 = 80 KiB
// k and n travel in the kernel arguments (the dispatch packet), not through host memory: the only
// PCIe read on the critical path is the message itself, issued first
struct NaclOneArgs {
    u32 k[8];   // precom (used on a subkey-cache miss)
    u32 n[6];   // the 24-byte nonce, little-endian words
};
__global__ __launch_bounds__(NACL_ONE_T) void k_nacl_one(uint8_t *st, uint32_t len, int open, uint8_t *subcache,
                                                         int miss, uint32_t out_off, NaclOneArgs args)
{
    __shared__ u32 s_key[8];       // subkey
    __shared__ u32 s_rs[8];        // Poly1305 r (clamped) and s
    __shared__ u32 s_tree[NACL_ONE_T * 5];
    const u32 t = threadIdx.x;
    const u32 nblk = (len + 63u) >> 6;
    const u32 w = (nblk + NACL_ONE_T - 1) / NACL_ONE_T;  // blocks per thread
    const u32 npass = (w + NACL_ONE_W - 1) / NACL_ONE_W;  // the same in every thread
    const u32 n0 = args.n[4], n1 = args.n[5];
    const u32 b0 = t * w;
    const u32 bend = b0 + w < nblk ? b0 + w : nblk;      // <= b0 for the threads past the box
    const uint8_t *in = st + 128;
    uint8_t *out = st + out_off;
    u32 Cb[NACL_ONE_W][16];
    // the pass's message blocks (host memory, over PCIe); the seal reads m[0:32] too (the MAC key)
    auto load_pass = [&](u32 pb) {
#pragma unroll
        for (int j = 0; j < NACL_ONE_W; j++) {
            const u32 b = pb + (u32)j;
            if (b >= bend)
                continue;
#pragma unroll
            for (int c = 0; c < 4; c++) {
                const u32 oc = 64u * b + 16u * c;
                V4 v = (oc >= 32u || !open) ? ld16<true>(in + oc, oc < len ? len - oc : 0) : zero4();
                Cb[j][4 * c] = v.x; Cb[j][4 * c + 1] = v.y; Cb[j][4 * c + 2] = v.z; Cb[j][4 * c + 3] = v.w;
            }
        }
    };
    // keystream, XOR, output; Cb keeps the ciphertext for the MAC
    auto xor_pass = [&](u32 pb, const u32 key[8]) {
#pragma unroll
        for (int j = 0; j < NACL_ONE_W; j++) {
            const u32 b = pb + (u32)j;
            if (b >= bend)
                continue;
            u32 x[16];
            salsa20_block<false>(x, key, n0, n1, b, 0u);
            const u32 o = 64u * b;
            u32 M[16];
#pragma unroll
            for (int k = 0; k < 16; k++) {
                M[k] = Cb[j][k] ^ x[k];  // output: c (seal) or m (open)
                if (!open)
                    Cb[j][k] = M[k];     // the MAC runs over the ciphertext
            }
            if (b == 0) {  // MAC key: c[0:32] (seal), the keystream (open)
#pragma unroll
                for (int i = 0; i < 8; i++) {
                    const u32 kw = open ? x[i] : M[i];
                    s_rs[i] = i >= 4 ? kw : kw & (i == 0 ? 0x0fffffffu : 0x0ffffffcu);
                }
            }
            // output bytes [max(o, 32), min(o + 64, len)) (seal: bytes 16..31 are the tag, written below)
#pragma unroll
            for (int c = 0; c < 4; c++) {
                const u32 oc = o + 16u * c;
                if (oc >= 32u && oc < len) {
                    const u32 cnt = len - oc < 16u ? len - oc : 16u;
                    if (cnt == 16u)
                        *reinterpret_cast<uint4 *>(out + oc) = make_uint4(M[4 * c], M[4 * c + 1], M[4 * c + 2], M[4 * c + 3]);
                    else
                        st_bytes(out + oc, M[4 * c], M[4 * c + 1], M[4 * c + 2], M[4 * c + 3], cnt);
                }
            }
        }
    };
    Poly P;
    // Horner over the pass's MAC blocks: p covers c[32 + 16p, 48 + 16p), the last one possibly partial
    auto horner_pass = [&](u32 pb) {
#pragma unroll
        for (int j = 0; j < NACL_ONE_W; j++) {
            const u32 b = pb + (u32)j;
            if (b >= bend)
                continue;
#pragma unroll
            for (int c = 0; c < 4; c++) {
                const u32 oc = 64u * b + 16u * c;
                if (oc < 32u || oc >= len)
                    continue;
                const u32 cnt = len - oc;
                if (cnt >= 16u)
                    poly_block(P, Cb[j][4 * c], Cb[j][4 * c + 1], Cb[j][4 * c + 2], Cb[j][4 * c + 3], 1u);
                else
                    poly_block_partial(P, Cb[j][4 * c], Cb[j][4 * c + 1], Cb[j][4 * c + 2], Cb[j][4 * c + 3], cnt);
            }
        }
    };
    // 1. the first pass's loads, issued before anything else
    load_pass(b0);
    // 2. the subkey: wave 0 derives it (every lane the same HSalsa20; lane 0 caches it) or loads it
    if (t < 64) {
        u32 key[8];
        if (miss) {
            const u32 in4[4] = {args.n[0], args.n[1], args.n[2], args.n[3]};
            hsalsa20(key, args.k, in4);
            if (t == 0) {
                *reinterpret_cast<uint4 *>(subcache) = make_uint4(key[0], key[1], key[2], key[3]);
                *reinterpret_cast<uint4 *>(subcache + 16) = make_uint4(key[4], key[5], key[6], key[7]);
            }
        } else {
            load_key(subcache, key);
        }
        if (t < 8)
            s_key[t] = key[t];
    }
    __syncthreads();
    u32 key[8];
#pragma unroll
    for (int i = 0; i < 8; i++)
        key[i] = s_key[i];
    // 3. the first pass (block 0 gives the MAC key), then the rest with their MAC on the way
    xor_pass(b0, key);
    __syncthreads();
    poly_init(P, s_rs[0], s_rs[1], s_rs[2], s_rs[3], s_rs[4], s_rs[5], s_rs[6], s_rs[7]);
    horner_pass(b0);
    for (u32 p = 1; p < npass; p++) {
        const u32 pb = b0 + p * (u32)NACL_ONE_W;
        load_pass(pb);
        xor_pass(pb, key);
        horner_pass(pb);
    }
    // 4. join the full threads 0..L-1: G = sum_u A_u R^u, u = L-1-t, by pairs with R_l = r^(Q 2^l)
    const u32 L = (nblk - 1u) / w;  // the thread holding the last box block
    const F26 r26 = f26_from32(P.r0, P.r1, P.r2, P.r3, 0u);
    F26 R = f26_pow(r26, 4u * w);
    const u32 u = L - 1u - t;  // (meaningful for t < L)
    F26 A = f26_from32(P.h0, P.h1, P.h2, P.h3, P.h4);
    if (t < L) {
#pragma unroll
        for (int i = 0; i < 5; i++)
            s_tree[u * 5 + i] = A.l[i];
    }
    for (u32 step = 1; step < L; step <<= 1) {
        __syncthreads();
        const bool act = t < L && (u % (2u * step)) == 0u && u + step < L;
        F26 B;
        if (act) {
#pragma unroll
            for (int i = 0; i < 5; i++)
                B.l[i] = s_tree[(u + step) * 5 + i];
            A = f26_add(A, f26_mul(B, R));
        }
        __syncthreads();
        if (act) {
#pragma unroll
            for (int i = 0; i < 5; i++)
                s_tree[u * 5 + i] = A.l[i];
        }
        R = f26_mul(R, R);
    }
    __syncthreads();
    if (t == L) {
        if (L > 0) {  // H = G r^(n_L) + A_L, n_L = thread L's MAC blocks (>= 1: its last block is not empty)
            F26 G;
#pragma unroll
            for (int i = 0; i < 5; i++)
                G.l[i] = s_tree[i];  // u = 0
            const u32 lo = 64u * b0, hi = len;
            const u32 nL = (hi - lo + 15u) >> 4;
            A = f26_add(f26_mul(G, f26_pow(r26, nL)), A);
            f26_to32(A, P.h0, P.h1, P.h2, P.h3, P.h4);
        }
        u32 tag[4];
        poly_finish(P, tag);
        int rc = 0;
        if (!open) {
            *reinterpret_cast<uint4 *>(out + 16) = make_uint4(tag[0], tag[1], tag[2], tag[3]);
        } else {
            const uint4 tin = *reinterpret_cast<const uint4 *>(in + 16);
            rc = ((tag[0] ^ tin.x) | (tag[1] ^ tin.y) | (tag[2] ^ tin.z) | (tag[3] ^ tin.w)) ? -1 : 0;
        }
        *reinterpret_cast<int *>(st + 56) = rc;
    }
}

// subkeys[i] = HSalsa20(precom[i], prefix16)
__global__ __launch_bounds__(BLOCK) void k_subkeys(const uint8_t *__restrict__ precom, uint8_t *__restrict__ out,
                                                    uint32_t nkeys, uint32_t p0, uint32_t p1, uint32_t p2, uint32_t p3)
{
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= nkeys)
        return;
    u32 k[8], o[8];
    const uint8_t *kp = precom + 32ull * i;
    for (int w = 0; w < 8; w++)
        k[w] = (u32)kp[4 * w] | ((u32)kp[4 * w + 1] << 8) | ((u32)kp[4 * w + 2] << 16) | ((u32)kp[4 * w + 3] << 24);
    const u32 in4[4] = {p0, p1, p2, p3};
    hsalsa20(o, k, in4);
    uint8_t *op = out + 32ull * i;
    for (int w = 0; w < 8; w++)
        for (int b = 0; b < 4; b++)
            op[4 * w + b] = (uint8_t)(o[w] >> (8 * b));
}

// Synthetic payload generator: counter-based SplitMix64 words (tests/cz_testlib.py splitmix_words).
__device__ __forceinline__ u64 splitmix(u64 seed, u64 idx)
{
    u64 z = seed + (idx + 1ull) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(BLOCK) void k_fill(uint8_t *__restrict__ buf, uint64_t nbytes, uint64_t seed)
{
    const uint64_t w = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;  // 16-byte chunk index
    const uint64_t off = w * 16;
    if (off >= nbytes)
        return;
    u64 a = splitmix(seed, 2 * w), b = splitmix(seed, 2 * w + 1);
    if (off + 16 <= nbytes) {
        *reinterpret_cast<uint4 *>(buf + off) = make_uint4((u32)a, (u32)(a >> 32), (u32)b, (u32)(b >> 32));
    } else {
        for (uint64_t i = 0; off + i < nbytes; i++)
            buf[off + i] = (uint8_t)((i < 8 ? a >> (8 * i) : b >> (8 * (i - 8))));
    }
}

// Device-to-device copy (bench.py's HBM copy ceiling, the guide's float4 copy): each workgroup
// copies one contiguous 16 KiB tile, 4 x 16-byte loads in flight per thread, every wave
// instruction 1 KiB contiguous.  tools/diag/copy_ub.hip on MI355X: this form 5.6 TB/s (read +
// write), grid-stride loops 4.4-4.7, hipMemcpy D2D 4.9, torch copy_ 4.7-4.9.
__global__ __launch_bounds__(BLOCK) void k_copy16(uint4 *__restrict__ dst, const uint4 *__restrict__ src, uint64_t n16)
{
    const uint64_t base = (uint64_t)blockIdx.x * BLOCK * 4;
    uint4 v[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const uint64_t i = base + u * BLOCK + threadIdx.x;
        if (i < n16)
            v[u] = src[i];
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const uint64_t i = base + u * BLOCK + threadIdx.x;
        if (i < n16)
            dst[i] = v[u];
    }
}

#endif  // CZ_KPART_HAS(3)

// Staging choice for a uniform batch (all pointers 16-byte aligned assumed by the caller check).
int pick_staging(uint64_t stride, uint32_t out_bytes, bool aligned)
{
    if (!aligned)
        return ST_DIRECT;
    // (EmitLines' buffer-store offsets, up to 64 * stride, stay below 2^31)
    if (stride % 128 == 0 && out_bytes >= 256 && stride < (1ull << 25))
        return ST_LINES;
    if (stride % 16 == 0 && 64 * stride <= REGION_MAX)
        return ST_REGION;
    return ST_DIRECT;
}

}  // namespace

// run-time tuning knobs (one definition, in part 3; hidden: not part of the library's ABI)
namespace czk_knobs {
#define CZ_KNOB __attribute__((visibility("hidden")))
#if CZ_KPART_HAS(3)
// g_pair: whole-line input loads for the uniform kernels
CZ_KNOB int g_pair = 1;
CZ_KNOB int g_un0 = 1;  // scalar first Salsa round when the high nonce word is wave-uniform
CZ_KNOB int g_seglines = 1;  // line-staged stores for waves of equal-length segments
CZ_KNOB int g_shift = 1;     // uniform seal: shifted line staging for bodies at any byte offset
CZ_KNOB int g_open_ina = 1;  // uniform open: line path for bodies off 16-byte alignment (dword-aligned loads)
CZ_KNOB int g_seal_ina = 1;  // seal: staged / line paths for payloads off 16-byte alignment
#ifndef CZ_OPEN_CARRY_DEFAULT
#define CZ_OPEN_CARRY_DEFAULT 1
#endif
CZ_KNOB int g_open_carry = CZ_OPEN_CARRY_DEFAULT;  // uniform open off 16-byte alignment: phase-sorted waves, carried lines
// segment kernels: waves of 16-byte aligned outputs that are not all on 128-byte lines go through
// EmitShiftLines (whole cache lines) instead of EmitSegLines (128-byte groups at each output's
// base, two partial cache lines per group): Zipf seal with 16-byte output slots 1250 -> 1629 GiB/s
#ifndef CZ_SHIFT16_DEFAULT
#define CZ_SHIFT16_DEFAULT 1
#endif
CZ_KNOB int g_shift16 = CZ_SHIFT16_DEFAULT;
#else
extern CZ_KNOB int g_pair;
extern CZ_KNOB int g_un0;
extern CZ_KNOB int g_seglines;
extern CZ_KNOB int g_shift;
extern CZ_KNOB int g_open_ina;
extern CZ_KNOB int g_seal_ina;
extern CZ_KNOB int g_open_carry;
extern CZ_KNOB int g_shift16;
#endif
}  // namespace czk_knobs
using namespace czk_knobs;

// ---------------------------------------------------------------------------
// Launchers (called from cz_host.cpp).  No allocation, no synchronisation:
// safe to capture in a hipGraph.
// ---------------------------------------------------------------------------
extern "C" {

#if CZ_KPART_HAS(1)
hipError_t czk_seal_uniform(const void *in, uint64_t in_stride, void *out, uint64_t out_stride, uint32_t count,
                            uint32_t len, const void *subkey, uint64_t counter0, const uint8_t *flags8,
                            hipStream_t s)
{
    if (count == 0)
        return hipSuccess;
    dim3 grid((count + BLOCK - 1) / BLOCK);
    const bool in_al = ((((uintptr_t)in | in_stride) & 15u) == 0);
    const bool al = in_al && ((((uintptr_t)out | out_stride) & 15u) == 0);
#define CZ_SEAL_LAUNCH(ST, PR, LDS)                                                                        \
    hipLaunchKernelGGL((k_seal_uniform<ST, PR>), grid, dim3(BLOCK), (LDS), s, (const uint8_t *)in, in_stride,   \
                       (uint8_t *)out, out_stride, count, len, (const uint8_t *)subkey, counter0, flags8, g_un0)
    // payloads off 16-byte alignment (messages packed back to back): the staged kernels with
    // dword-aligned loads (INA 8 / 1) instead of lane-wise unaligned loads and byte-exact stores
    if (!in_al && g_pair && g_seal_ina && len >= 64u) {
        const bool out_al = ((((uintptr_t)out | out_stride) & 15u) == 0);
        int so = pick_staging(out_stride, len + 33u, out_al);
        if (so == ST_DIRECT && len + 33u >= 256u && out_stride < (1ull << 22) && len <= SHIFT_TOTAL_MAX - 33u && g_shift)
            so = ST_SHIFT;
        const bool i8 = (((uintptr_t)in | in_stride) & 7u) == 0;
#define CZ_SEAL_LAUNCH_INA(ST, PR, INA, LDS)                                                                  \
    hipLaunchKernelGGL((k_seal_uniform_ina<ST, PR, INA>), grid, dim3(BLOCK), (LDS), s, (const uint8_t *)in,        \
                       in_stride, (uint8_t *)out, out_stride, count, len, (const uint8_t *)subkey, counter0,       \
                       flags8, g_un0)
        const unsigned lds_l = WAVES * (LINE_LDS_BYTES + HOLD_LDS_BYTES), lds_s = SEAL_SHIFT_LDS_BYTES;
        const unsigned lds_r = (unsigned)(WAVES * 64 * out_stride);
        if (so == ST_LINES) {
            if (i8) CZ_SEAL_LAUNCH_INA(ST_LINES, true, 8, lds_l);
            else CZ_SEAL_LAUNCH_INA(ST_LINES, true, 1, lds_l);
            return hipGetLastError();
        }
        if (so == ST_SHIFT) {
            if (i8) CZ_SEAL_LAUNCH_INA(ST_SHIFT, true, 8, lds_s);
            else CZ_SEAL_LAUNCH_INA(ST_SHIFT, true, 1, lds_s);
            return hipGetLastError();
        }
        if (so == ST_REGION) {
            if (i8) CZ_SEAL_LAUNCH_INA(ST_REGION, false, 8, lds_r);
            else CZ_SEAL_LAUNCH_INA(ST_REGION, false, 1, lds_r);
            return hipGetLastError();
        }
#undef CZ_SEAL_LAUNCH_INA
    }
    int st = pick_staging(out_stride, len + 33u, al);
    // bodies at any byte offset (dense slots, wire layout) from aligned payloads: shifted line staging
    // (EmitShiftLinesUni's buffer-store offsets, below 256 * stride + len + 160, stay below 2^31)
    if (st == ST_DIRECT && in_al && len + 33u >= 256u && out_stride < (1ull << 22) && len <= SHIFT_TOTAL_MAX - 33u && g_shift)
        st = ST_SHIFT;
    const unsigned lds = st == ST_LINES ? WAVES * (LINE_LDS_BYTES + HOLD_LDS_BYTES)
                                        : st == ST_SHIFT ? SEAL_SHIFT_LDS_BYTES
                                        : (st == ST_REGION ? (unsigned)(WAVES * 64 * out_stride) : 0u);
    // whole-line input pays for large frames (A/B: 4 KiB seal 2.34 vs 2.51 ms) but
    // not for the small frames of the region stager (100 B: 0.119 vs 0.114 ms)
    if (g_pair && st != ST_REGION) {
        if (st == ST_LINES) CZ_SEAL_LAUNCH(ST_LINES, true, lds);
        else if (st == ST_SHIFT) CZ_SEAL_LAUNCH(ST_SHIFT, true, lds);
        else CZ_SEAL_LAUNCH(ST_DIRECT, true, 0);
    } else {
        if (st == ST_LINES) CZ_SEAL_LAUNCH(ST_LINES, false, lds);
        else if (st == ST_REGION) CZ_SEAL_LAUNCH(ST_REGION, false, lds);
        else if (st == ST_SHIFT) CZ_SEAL_LAUNCH(ST_SHIFT, false, lds);
        else CZ_SEAL_LAUNCH(ST_DIRECT, false, 0);
    }
#undef CZ_SEAL_LAUNCH
    return hipGetLastError();
}

// Box-layout input (MODE_BOX): whole-line staging for 128-byte multiple output slots, direct
// stores otherwise; whole-line input loads always (the box is read where it lies).
hipError_t czk_seal_uniform_box(const void *in, uint64_t in_stride, void *out, uint64_t out_stride, uint32_t count,
                                uint32_t len, const void *subkey, uint64_t counter0, hipStream_t s)
{
    if (count == 0)
        return hipSuccess;
    dim3 grid((count + BLOCK - 1) / BLOCK);
    const bool al = ((((uintptr_t)in | in_stride | (uintptr_t)out | out_stride) & 15u) == 0);
    const int st = pick_staging(out_stride, len + 33u, al);
    if (st == ST_LINES)
        hipLaunchKernelGGL((k_seal_uniform<ST_LINES, true, MODE_BOX>), grid, dim3(BLOCK),
                           WAVES * (LINE_LDS_BYTES + HOLD_LDS_BYTES), s, (const uint8_t *)in, in_stride, (uint8_t *)out,
                           out_stride, count, len, (const uint8_t *)subkey, counter0, nullptr, g_un0);
    else
        hipLaunchKernelGGL((k_seal_uniform<ST_DIRECT, true, MODE_BOX>), grid, dim3(BLOCK), 0, s, (const uint8_t *)in,
                           in_stride, (uint8_t *)out, out_stride, count, len, (const uint8_t *)subkey, counter0, nullptr,
                           g_un0);
    return hipGetLastError();
}

#ifdef CZ_DIAG_CLOCK
// diagnostic builds only: copy the last k_seal_uniform launch's wave stamps (4 x u64 per wave) out
extern "C" __attribute__((visibility("default"))) int cz_diag_clock_read(uint64_t *host, uint64_t waves)
{
    if (waves > DIAG_CLOCK_WAVES)
        waves = DIAG_CLOCK_WAVES;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_diag_clock), waves * 32u, 0, hipMemcpyDeviceToHost) == hipSuccess
               ? (int)waves
               : -1;
}
#endif

#endif  // CZ_KPART_HAS(1)

#if CZ_KPART_HAS(3)
hipError_t czk_seal_desc(const cz_frame_desc *desc, const uint32_t *order, uint32_t count, const void *in, void *out,
                         const void *subkeys, hipStream_t s)
{
    if (count == 0)
        return hipSuccess;
    dim3 grid((count + BLOCK - 1) / BLOCK);
    hipLaunchKernelGGL(k_seal_desc, grid, dim3(BLOCK), 0, s, desc, order, count, (const uint8_t *)in,
                       (uint8_t *)out, (const uint8_t *)subkeys);
    return hipGetLastError();
}

hipError_t czk_open_desc(const cz_frame_desc *desc, const uint32_t *order, uint32_t count, const void *in, void *out,
                         const void *subkeys, uint16_t *status, uint64_t *nonces, hipStream_t s)
{
    if (count == 0)
        return hipSuccess;
    dim3 grid((count + BLOCK - 1) / BLOCK);
    hipLaunchKernelGGL(k_open_desc, grid, dim3(BLOCK), 0, s, desc, order, count, (const uint8_t *)in,
                       (uint8_t *)out, (const uint8_t *)subkeys, status, nonces);
    return hipGetLastError();
}

#endif  // CZ_KPART_HAS(3)

#if CZ_KPART_HAS(2)
hipError_t czk_open_uniform(const void *in, uint64_t in_stride, void *out, uint64_t out_stride, uint32_t count,
                            uint32_t size, const void *subkey, uint64_t floor0, int check, uint16_t *status,
                            hipStream_t s)
{
    if (count == 0)
        return hipSuccess;
    dim3 grid((count + BLOCK - 1) / BLOCK);
    const bool al = ((((uintptr_t)in | (uintptr_t)out | in_stride | out_stride) & 15u) == 0);
    const uint32_t nout = size >= 33u ? size - 33u : 0u;
#define CZ_OPEN_LAUNCH(ST, PR, LDS)                                                                        \
    hipLaunchKernelGGL((k_open_uniform<ST, PR>), grid, dim3(BLOCK), (LDS), s, (const uint8_t *)in, in_stride,   \
                       (uint8_t *)out, out_stride, count, size, (const uint8_t *)subkey, floor0, check, status, g_un0, 0)
#define CZ_OPEN_LAUNCH_INA(ST, INA, LDS)                                                                     \
    hipLaunchKernelGGL((k_open_uniform<ST, true, INA>), grid, dim3(BLOCK), (LDS), s, (const uint8_t *)in,          \
                       in_stride, (uint8_t *)out, out_stride, count, size, (const uint8_t *)subkey, floor0, check, \
                       status, g_un0, 0)
    const int st = size >= 33u ? pick_staging(out_stride, nout, al) : (int)ST_DIRECT;
    const unsigned lds = st == ST_LINES ? WAVES * LINE_LDS_BYTES : (st == ST_REGION ? (unsigned)(WAVES * 64 * out_stride) : 0u);
    // bodies off 16-byte alignment (the dense wire layout) into line-aligned plaintext slots: the
    // line path with dword-aligned loads (INA 8 / 1) instead of lane-wise byte-exact stores
    const bool out_al = ((((uintptr_t)out | out_stride) & 15u) == 0);
    int st_out = size >= 33u ? pick_staging(out_stride, nout, out_al) : (int)ST_DIRECT;
    // plaintext at any byte offset (slots that are not 128-byte multiples): byte-shifted line
    // staging, as the seal's bodies (EmitShiftLinesUni; its buffer-store offsets stay below 2^31)
    if (st_out == ST_DIRECT && size >= 33u && nout >= 256u && nout <= SHIFT_TOTAL_MAX && out_stride < (1ull << 22) &&
        g_shift)
        st_out = ST_SHIFT;
    const uint64_t ia = (uintptr_t)in | in_stride;
    const int ina = (ia & 15u) == 0 ? 16 : (ia & 7u) == 0 ? 8 : 1;
    const unsigned lds_out_region = (unsigned)(WAVES * 64 * out_stride);
    if (ina != 16 && st_out == ST_REGION && g_open_ina) {
        // small bodies (64 plaintext slots <= 16 KiB) off 16-byte alignment: region staging
        if (ina == 8)
            hipLaunchKernelGGL((k_open_uniform<ST_REGION, false, 8>), grid, dim3(BLOCK), lds_out_region, s,
                               (const uint8_t *)in, in_stride, (uint8_t *)out, out_stride, count, size,
                               (const uint8_t *)subkey, floor0, check, status, g_un0, 0);
        else
            hipLaunchKernelGGL((k_open_uniform<ST_REGION, false, 1>), grid, dim3(BLOCK), lds_out_region, s,
                               (const uint8_t *)in, in_stride, (uint8_t *)out, out_stride, count, size,
                               (const uint8_t *)subkey, floor0, check, status, g_un0, 0);
        return hipGetLastError();
    }
    // (INA 1 -- any byte offset -- measured 1.3% slower with carried lines at 2 waves per SIMD than
    // the straddling loads at 3, so only 8-byte aligned bodies take it: +2.6%)
    // (cz_tune("open_carry", 2): INA 1 too, A/B only)
    if (g_pair && st_out == ST_LINES && (ina == 8 || (ina == 1 && g_open_carry == 2)) && g_open_ina && g_open_carry &&
        nout >= 256u) {
        // phase-sorted waves with carried aligned lines (k_open_uniform_carry): whole blocks of 64 P
        // frames, P = the period of the bodies' line phase; the rest through k_open_uniform
        uint64_t g = in_stride & 127u, m = 128u;
        while (g) {  // gcd(in_stride mod 128, 128)
            const uint64_t t = m % g;
            m = g;
            g = t;
        }
        const uint32_t P = (uint32_t)(128u / m);
        const uint64_t blocks = count / (64ull * P);
        if (blocks > 0 && 64ull * P * out_stride < (1ull << 31)) {
            const uint32_t nwaves = (uint32_t)(blocks * P);
            const dim3 cgrid((nwaves + WAVES - 1) / WAVES);
            if (ina == 8)
                hipLaunchKernelGGL((k_open_uniform_carry<8>), cgrid, dim3(BLOCK), WAVES * LINE_LDS_BYTES, s,
                                   (const uint8_t *)in, in_stride, (uint8_t *)out, out_stride, nwaves, P, size,
                                   (const uint8_t *)subkey, floor0, check, status, g_un0);
            else
                hipLaunchKernelGGL((k_open_uniform_carry<1>), cgrid, dim3(BLOCK), WAVES * LINE_LDS_BYTES, s,
                                   (const uint8_t *)in, in_stride, (uint8_t *)out, out_stride, nwaves, P, size,
                                   (const uint8_t *)subkey, floor0, check, status, g_un0);
            const uint64_t done = blocks * 64ull * P;
            if (done < count) {
                hipError_t e = hipGetLastError();
                if (e != hipSuccess)
                    return e;
                const uint32_t rest = count - (uint32_t)done;
                const dim3 tgrid((rest + BLOCK - 1) / BLOCK);
                const uint8_t *tin = (const uint8_t *)in + done * in_stride;
                uint8_t *tout = (uint8_t *)out + done * out_stride;
                if (ina == 8)
                    hipLaunchKernelGGL((k_open_uniform<ST_LINES, true, 8>), tgrid, dim3(BLOCK), WAVES * LINE_LDS_BYTES,
                                       s, tin, in_stride, tout, out_stride, rest, size, (const uint8_t *)subkey, floor0,
                                       check, status + done, g_un0, 1);
                else
                    hipLaunchKernelGGL((k_open_uniform<ST_LINES, true, 1>), tgrid, dim3(BLOCK), WAVES * LINE_LDS_BYTES,
                                       s, tin, in_stride, tout, out_stride, rest, size, (const uint8_t *)subkey, floor0,
                                       check, status + done, g_un0, 1);
            }
            return hipGetLastError();
        }
    }
    if (g_pair && (st_out == ST_SHIFT || (st_out == ST_LINES && ina != 16)) && (ina == 16 || g_open_ina)) {
        if (st_out == ST_LINES) {
            if (ina == 8)
                CZ_OPEN_LAUNCH_INA(ST_LINES, 8, WAVES * LINE_LDS_BYTES);
            else
                CZ_OPEN_LAUNCH_INA(ST_LINES, 1, WAVES * LINE_LDS_BYTES);
        } else if (ina == 16) {
            CZ_OPEN_LAUNCH_INA(ST_SHIFT, 16, WAVES * SHIFT_LDS_BYTES);
        } else if (ina == 8) {
            CZ_OPEN_LAUNCH_INA(ST_SHIFT, 8, WAVES * SHIFT_LDS_BYTES);
        } else {
            CZ_OPEN_LAUNCH_INA(ST_SHIFT, 1, WAVES * SHIFT_LDS_BYTES);
        }
        return hipGetLastError();
    }
    if (g_pair && st != ST_REGION) {
        if (st == ST_LINES) CZ_OPEN_LAUNCH(ST_LINES, true, lds);
        else CZ_OPEN_LAUNCH(ST_DIRECT, true, 0);
    } else {
        if (st == ST_LINES) CZ_OPEN_LAUNCH(ST_LINES, false, lds);
        else if (st == ST_REGION) CZ_OPEN_LAUNCH(ST_REGION, false, lds);
        else CZ_OPEN_LAUNCH(ST_DIRECT, false, 0);
    }
#undef CZ_OPEN_LAUNCH
#undef CZ_OPEN_LAUNCH_INA
    return hipGetLastError();
}

#ifdef CZ_DIAG_CLOCK
// diagnostic builds only: the last k_open_uniform launch's wave stamps (this part's g_diag_clock)
extern "C" __attribute__((visibility("default"))) int cz_diag_clock_read_open(uint64_t *host, uint64_t waves)
{
    if (waves > DIAG_CLOCK_WAVES)
        waves = DIAG_CLOCK_WAVES;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_diag_clock), waves * 32u, 0, hipMemcpyDeviceToHost) == hipSuccess
               ? (int)waves
               : -1;
}
#endif

#endif  // CZ_KPART_HAS(2)

#if CZ_KPART_HAS(3)
uint32_t czk_nacl_one_limit(void);

hipError_t czk_nacl_one(void *st, uint32_t len, int open, void *subcache, int miss, uint32_t out_off,
                        const uint8_t k[32], const uint8_t n[24], hipStream_t s)
{
    if (len < 32u || len > czk_nacl_one_limit() || out_off < 128u + len || out_off > 0xffffffffu - len)
        return hipErrorInvalidValue;
    NaclOneArgs a;
    __builtin_memcpy(a.k, k, 32);
    __builtin_memcpy(a.n, n, 24);
    hipLaunchKernelGGL(k_nacl_one, dim3(1), dim3(NACL_ONE_T), 0, s, (uint8_t *)st, len, open, (uint8_t *)subcache, miss,
                       out_off, a);
    volatile u32 *vk = a.k;  // the launch copied the arguments: no key left on this stack frame
    for (int i = 0; i < 8; i++)
        vk[i] = 0u;
    return hipGetLastError();
}

// one pass of k_nacl_one (80 KiB): the size up to which one launch beats the segment kernels
uint32_t czk_nacl_one_max(void) { return (uint32_t)(NACL_ONE_T * NACL_ONE_W * 64); }
// the largest box k_nacl_one takes (jnacl's byte[] bound; 64 * block index and out_off + len fit u32)
uint32_t czk_nacl_one_limit(void) { return 0x7fffff00u; }

hipError_t czk_subkeys(const void *precom, void *out, uint32_t nkeys, const uint8_t prefix[16], hipStream_t s)
{
    if (nkeys == 0)
        return hipSuccess;
    u32 p[4];
    for (int w = 0; w < 4; w++)
        p[w] = (u32)prefix[4 * w] | ((u32)prefix[4 * w + 1] << 8) | ((u32)prefix[4 * w + 2] << 16) |
               ((u32)prefix[4 * w + 3] << 24);
    dim3 grid((nkeys + BLOCK - 1) / BLOCK);
    hipLaunchKernelGGL(k_subkeys, grid, dim3(BLOCK), 0, s, (const uint8_t *)precom, (uint8_t *)out, nkeys, p[0], p[1],
                       p[2], p[3]);
    return hipGetLastError();
}

hipError_t czk_seal_segments(const cz_frame_desc *desc, const cz_segment *segs, uint32_t nseg, const cz_combine *comb,
                             uint32_t ncomb, const void *in, void *out, const void *subkeys, void *work, hipStream_t s)
{
    const dim3 grid((nseg + BLOCK - 1) / BLOCK);
    if (nseg && g_seglines && g_pair) {
        const int mode = SEGMODE_LINES | SEGMODE_PAIR | (g_shift16 ? SEGMODE_SHIFT16 : 0) | (g_seal_ina ? SEGMODE_ANYIN : 0);
        hipLaunchKernelGGL(k_seal_segments_lines, grid, dim3(BLOCK), WAVES * SHIFT_LDS_BYTES, s, desc, segs, nseg,
                           (const uint8_t *)in, (uint8_t *)out, (const uint8_t *)subkeys, (u32 *)work, mode);
        hipLaunchKernelGGL(k_seal_segments, grid, dim3(BLOCK), g_seal_ina ? WAVES * SHIFT_LDS_BYTES : 0, s, desc, segs,
                           nseg, (const uint8_t *)in, (uint8_t *)out, (const uint8_t *)subkeys, (u32 *)work,
                           mode | SEGMODE_REST);
    } else if (nseg) {
        hipLaunchKernelGGL(k_seal_segments, grid, dim3(BLOCK), WAVES * SHIFT_LDS_BYTES, s, desc, segs, nseg,
                           (const uint8_t *)in, (uint8_t *)out, (const uint8_t *)subkeys, (u32 *)work,
                           (g_seglines ? SEGMODE_LINES : 0) | (g_pair ? SEGMODE_PAIR : 0));
    }
    if (ncomb)
        hipLaunchKernelGGL(k_seal_combine, dim3((ncomb + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, desc, comb, ncomb,
                           (uint8_t *)out, (const u32 *)work);
    return hipGetLastError();
}

hipError_t czk_open_segments(const cz_frame_desc *desc, const cz_segment *segs, uint32_t nseg, const cz_combine *comb,
                             uint32_t ncomb, const void *in, void *out, const void *subkeys, void *work,
                             uint16_t *status, uint64_t *nonces, hipStream_t s)
{
    if (nseg)
        hipLaunchKernelGGL(k_open_segments, dim3((nseg + BLOCK - 1) / BLOCK), dim3(BLOCK), WAVES * SHIFT_LDS_BYTES, s,
                           desc, segs, nseg, (const uint8_t *)in, (uint8_t *)out, (const uint8_t *)subkeys,
                           (u32 *)work, status, nonces,
                           (g_seglines ? SEGMODE_LINES : 0) | (g_pair ? SEGMODE_PAIR : 0) | (g_shift16 ? SEGMODE_SHIFT16 : 0) |
                               (g_open_ina ? SEGMODE_ANYIN : 0));
    if (ncomb)
        hipLaunchKernelGGL(k_open_combine, dim3((ncomb + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, desc, comb, ncomb,
                           (const uint8_t *)in, (uint8_t *)out, (const u32 *)work, status);
    return hipGetLastError();
}

hipError_t czk_v2_copy(const cz_v2_item *items, uint32_t count, const void *src, void *dst, hipStream_t s)
{
    if (count == 0)
        return hipSuccess;
    const uint32_t per_block = BLOCK / 64;
    hipLaunchKernelGGL(k_v2_copy, dim3((count + per_block - 1) / per_block), dim3(BLOCK), 0, s, items, count,
                       (const uint8_t *)src, (uint8_t *)dst);
    return hipGetLastError();
}

int czk_tune(const char *key, int value)
{
    if (!key)
        return -1;
    if (key[0] == 'p' && key[1] == 'a' && key[2] == 'i' && key[3] == 'r' && key[4] == 0) {
        int old = g_pair;
        g_pair = value != 0;
        return old;
    }
    if (key[0] == 'u' && key[1] == 'n' && key[2] == '0' && key[3] == 0) {
        int old = g_un0;
        g_un0 = value != 0;
        return old;
    }
    if (__builtin_strcmp(key, "seglines") == 0) {
        int old = g_seglines;
        g_seglines = value != 0;
        return old;
    }
    if (__builtin_strcmp(key, "seal_ina") == 0) {
        int old = g_seal_ina;
        g_seal_ina = value != 0;
        return old;
    }
    if (__builtin_strcmp(key, "open_ina") == 0) {
        int old = g_open_ina;
        g_open_ina = value != 0;
        return old;
    }
    if (__builtin_strcmp(key, "open_carry") == 0) {
        int old = g_open_carry;
        g_open_carry = value < 0 ? 0 : value > 2 ? 2 : value;
        return old;
    }
    if (__builtin_strcmp(key, "shift16") == 0) {
        int old = g_shift16;
        g_shift16 = value != 0;
        return old;
    }
    if (__builtin_strcmp(key, "shift") == 0) {
        int old = g_shift;
        g_shift = value != 0;
        return old;
    }
    return -1;
}

hipError_t czk_copy16(void *dst, const void *src, uint64_t nbytes, hipStream_t s)
{
    const uint64_t n16 = nbytes / 16;
    if (n16 == 0)
        return hipSuccess;
    const uint64_t blocks = (n16 + 4 * BLOCK - 1) / (4 * BLOCK);
    if (blocks > 0x7fffffffull)
        return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_copy16, dim3((unsigned)blocks), dim3(BLOCK), 0, s, (uint4 *)dst, (const uint4 *)src, n16);
    return hipGetLastError();
}

hipError_t czk_fill(void *buf, uint64_t nbytes, uint64_t seed, hipStream_t s)
{
    if (nbytes == 0)
        return hipSuccess;
    uint64_t chunks = (nbytes + 15) / 16;
    dim3 grid((unsigned)((chunks + BLOCK - 1) / BLOCK));
    hipLaunchKernelGGL(k_fill, grid, dim3(BLOCK), 0, s, (uint8_t *)buf, nbytes, seed);
    return hipGetLastError();
}

#ifdef CZ_DIAG_CLOCK
// diagnostic builds only: the last k_seal_segments_lines launch's wave stamps (this part's g_diag_clock)
extern "C" __attribute__((visibility("default"))) int cz_diag_clock_read_seg(uint64_t *host, uint64_t waves)
{
    if (waves > DIAG_CLOCK_WAVES)
        waves = DIAG_CLOCK_WAVES;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_diag_clock), waves * 32u, 0, hipMemcpyDeviceToHost) == hipSuccess
               ? (int)waves
               : -1;
}
#endif

#endif  // CZ_KPART_HAS(3)

}  // extern "C"
