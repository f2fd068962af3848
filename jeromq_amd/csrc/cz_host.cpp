// cz_host.cpp -- host side of the C-ABI (include/curvezmq_mi355x.h):
// argument checking, error reporting, per-thread device context for the jnacl
// drop-ins, host-staged batch contexts.  Every cryptographic byte is computed
// by the gfx950 kernels in cz_kernels.hip; there is no CPU crypto fallback:
// without a usable device every entry point fails with CZ_EHIP.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <numeric>
#include <string>
#include <unordered_set>
#include <vector>

#include "../../include/curvezmq_mi355x.h"
#include "cz_internal.h"

extern "C" {
hipError_t czk_seal_uniform_box(const void *, uint64_t, void *, uint64_t, uint32_t, uint32_t, const void *, uint64_t,
                                hipStream_t);
hipError_t czk_seal_uniform(const void *, uint64_t, void *, uint64_t, uint32_t, uint32_t, const void *, uint64_t,
                            const uint8_t *, hipStream_t);
hipError_t czk_seal_desc(const cz_frame_desc *, const uint32_t *, uint32_t, const void *, void *, const void *,
                         hipStream_t);
hipError_t czk_open_desc(const cz_frame_desc *, const uint32_t *, uint32_t, const void *, void *, const void *,
                         uint16_t *, uint64_t *, hipStream_t);
hipError_t czk_open_uniform(const void *, uint64_t, void *, uint64_t, uint32_t, uint32_t, const void *, uint64_t, int,
                            uint16_t *, hipStream_t);
hipError_t czk_fill(void *, uint64_t, uint64_t, hipStream_t);
hipError_t czk_copy16(void *, const void *, uint64_t, hipStream_t);
int czk_tune(const char *, int);
}

namespace czi {

static thread_local std::string g_err;

int fail(int code, const char *fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

int hip_fail(hipError_t e, const char *where)
{
    return fail(CZ_EHIP, "%s: %s", where, hipGetErrorString(e));
}

const uint8_t *prefix_for(int direction)
{
    return (const uint8_t *)(direction == CZ_DIR_S2C ? "CurveZMQMESSAGES" : "CurveZMQMESSAGEC");
}

// ---- DevBuf ----------------------------------------------------------------
hipError_t DevBuf::reserve(uint64_t bytes)
{
    if (bytes <= cap)
        return hipSuccess;
    if (ptr)
        (void)hipFree(ptr);
    ptr = nullptr;
    cap = 0;
    uint64_t want = std::max<uint64_t>(bytes, 4096);
    hipError_t e = hipMalloc(&ptr, want);
    if (e == hipSuccess)
        cap = want;
    return e;
}

void DevBuf::release()
{
    if (ptr)
        (void)hipFree(ptr);
    ptr = nullptr;
    cap = 0;
}

hipError_t HostBuf::reserve(uint64_t bytes)
{
    if (bytes <= cap)
        return hipSuccess;
    if (ptr)
        (void)hipHostFree(ptr);
    ptr = nullptr;
    cap = 0;
    uint64_t want = std::max<uint64_t>(bytes, 4096);
    hipError_t e = hipHostMalloc(&ptr, want, hipHostMallocDefault);
    if (e == hipSuccess)
        cap = want;
    return e;
}

void HostBuf::release()
{
    if (ptr)
        (void)hipHostFree(ptr);
    ptr = nullptr;
    cap = 0;
}

// ---- per-thread single-shot context ----------------------------------------
// One message per call (the jnacl drop-ins).  Boxes above 80 KiB run through the segment planner
// and kernels, so a long box spreads over many workgroups: everything the device needs -- key,
// descriptor, segment and combine lists, the message -- goes over in ONE pinned H2D copy, and the
// result in one D2H copy.
// One-launch path (k_nacl_one): the staging is pinned host memory the kernel reads and writes
// directly, and the subkey HSalsa20(k, n[0:16]) of the last NCACHE (k, n[0:16]) pairs this thread
// used stays in device memory (CurveZMQ: one pair per connection direction).  cz_nacl_forget()
// wipes both.
struct Single {
    static constexpr int NCACHE = 8;
    bool ready = false;
    hipStream_t stream = nullptr;
    DevBuf dev, rc, subcache;
    HostBuf stage, one;
    uint8_t ckey[NCACHE][48] = {};  // k || n[0:16] of each cached subkey
    bool cvalid[NCACHE] = {};
    int cnext = 0;
    // (the destructor touches no HIP memory: at process exit the runtime may be gone first)
    ~Single() { forget_host(false); }
    void forget_host(bool staging)
    {
        explicit_bzero(ckey, sizeof ckey);
        for (bool &v : cvalid)
            v = false;
        if (staging && one.ptr)
            explicit_bzero(one.ptr, one.cap);
    }
};

static thread_local Single t_single;

// base addresses cz_host_alloc handed out and cz_host_free has not released
static std::mutex g_host_mu;
static std::unordered_set<void *> g_host_bases;

static int single_init()
{
    if (t_single.ready)
        return CZ_OK;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n == 0)
        return fail(CZ_EHIP, "no HIP device available (the CURVE path runs only on the GPU)");
    e = hipStreamCreateWithFlags(&t_single.stream, hipStreamNonBlocking);
    if (e != hipSuccess)
        return hip_fail(e, "hipStreamCreate");
    if ((e = t_single.rc.reserve(64)) != hipSuccess || (e = t_single.subcache.reserve(32 * Single::NCACHE)) != hipSuccess)
        return hip_fail(e, "hipMalloc");
    t_single.ready = true;
    return CZ_OK;
}

static uint64_t up128(uint64_t v) { return (v + 127) & ~127ull; }

// Bytes a uniform batch spans from its base, (count - 1) * stride + last, if that fits in 2^47 (a
// canonical user address range: no stride makes frame i's address wrap, and count * stride sums of
// the staging sizes stay far from 2^64); false otherwise.
static bool uniform_span(uint32_t count, uint64_t stride, uint64_t last, uint64_t *bytes)
{
    uint64_t v = 0;
    if (count && (__builtin_mul_overflow((uint64_t)(count - 1), stride, &v) || __builtin_add_overflow(v, last, &v)))
        return false;
    if (v > (1ull << 47))
        return false;
    if (bytes)
        *bytes = v;
    return true;
}

// NaCl box/open of one message in ONE launch (k_nacl_one): input staged into pinned host memory
// the kernel reads directly, output read back from it after the launch.  -1 on a bad tag (dst
// untouched).  The seal is NaCl's for every m: the MAC key is c[0:32] = keystream ^ m[0:32].
static int nacl_one_launch(uint8_t *dst, const uint8_t *src, uint64_t len, const uint8_t n[24], const uint8_t k[32],
                           int open)
{
    Single &s = t_single;
    const uint64_t out_off = 128 + ((len + 127) & ~127ull);
    hipError_t e;
    if ((e = s.one.reserve(out_off + len + 128)) != hipSuccess) {
        hip_fail(e, "hipHostMalloc");
        return -1;
    }
    uint8_t *st = (uint8_t *)s.one.ptr;
    // subkey cache: (k, n[0:16]) -> device slot
    int slot = -1;
    for (int i = 0; i < Single::NCACHE; i++)
        if (s.cvalid[i] && memcmp(s.ckey[i], k, 32) == 0 && memcmp(s.ckey[i] + 32, n, 16) == 0) {
            slot = i;
            break;
        }
    const int miss = slot < 0;
    if (miss) {
        slot = s.cnext;
        s.cnext = (s.cnext + 1) % Single::NCACHE;
        memcpy(s.ckey[slot], k, 32);
        memcpy(s.ckey[slot] + 32, n, 16);
        s.cvalid[slot] = false;  // valid once the launch that derives it has completed
    }
    memcpy(st + 128, src, len);
    *(volatile int *)(st + 56) = -2;
    if ((e = czk_nacl_one(st, (uint32_t)len, open, (uint8_t *)s.subcache.ptr + 32 * slot, miss, (uint32_t)out_off, k, n,
                          s.stream)) != hipSuccess ||
        (e = hipStreamSynchronize(s.stream)) != hipSuccess) {
        // no plaintext left in the pinned staging on a failed call: the staged box (seal) or
        // whatever part of m the kernel wrote before the failure (open)
        explicit_bzero(open ? st + out_off : st + 128, len);
        hip_fail(e, "cz_box (one launch)");
        return -1;
    }
    if (miss)
        s.cvalid[slot] = true;
    const int rc = *(volatile int *)(st + 56);
    if (!open) {
        explicit_bzero(st + 128, len);  // no plaintext left in the pinned staging after the call
        if (rc != 0)
            return fail(CZ_EHIP, "cz_box (one launch): the kernel did not complete"), -1;
        memset(dst, 0, 16);
        memcpy(dst + 16, st + out_off + 16, len - 16);
        return 0;
    }
    if (rc != 0) {
        explicit_bzero(st + out_off, len);  // never leave unauthenticated plaintext behind
        return -1;
    }
    memset(dst, 0, 32);
    memcpy(dst + 32, st + out_off + 32, len - 32);
    explicit_bzero(st + out_off, len);
    return 0;
}

// Boxes above this many bytes whose MAC key is the keystream alone (every open, and every seal
// with m[0:32] == 0, i.e. every CurveZMQ box) run on the segment kernels, which spread a long box
// over many workgroups; smaller boxes, and seals whose m[0:32] is not zero (the MAC key is then
// keystream ^ m[0:32], which only k_nacl_one derives), take one launch.  Measured on MI355X
// (bench.py --config nacl, "large_boxes"; profiles/r05/nacl_large_boxes.json): one launch / segments
// seal 57 / 166 us at 96 KiB, 114 / 254 at 256 KiB, 380 / 471 at 1 MiB, 1330 / 1174 at 4 MiB.
// cz_tune("nacl_one_max") moves the edge; the Mechanism mirror uses the same one.
// written by cz_tune while IO threads read it: relaxed atomic (a knob, no ordering needed)
static std::atomic<uint64_t> g_nacl_one_bytes{2ull << 20};

uint64_t nacl_one_bytes()
{
    return std::max<uint64_t>(g_nacl_one_bytes.load(std::memory_order_relaxed), czk_nacl_one_max());
}

// NaCl box/open of one message on the device.  A MESSAGE is the NaCl box of
// 0^32 || flags || payload, so m[32] rides as the flags byte and m[33:] as the payload; for open
// the 16 bytes ahead of the tag are rebuilt as "\x07MESSAGE" || n[16:24] and the nonce check is off.
static int nacl_one(uint8_t *dst, const uint8_t *src, uint64_t len, const uint8_t n[24], const uint8_t k[32],
                    int open)
{
    if (!dst || !src || !n || !k)
        return -1;
    if (len < 32 || len > 0xffffffffull)
        return -1;
    if (single_init() != CZ_OK)
        return -1;
    bool one = len <= nacl_one_bytes();
    if (!one && !open) {
        uint8_t z = 0;
        for (int i = 0; i < 32; i++)
            z |= src[i];
        one = z != 0;
    }
    if (one) {
        if (len > czk_nacl_one_limit())
            return fail(CZ_EINVAL, "cz_box_afternm: a box with m[0:32] != 0 is limited to %u bytes",
                        czk_nacl_one_limit()), -1;
        return nacl_one_launch(dst, src, len, n, k, open);
    }
    Single &s = t_single;
    uint64_t counter = 0;
    for (int i = 0; i < 8; i++)
        counter = (counter << 8) | n[16 + i];
    hipError_t e;
    // one descriptor, its segments and combine record
    cz_frame_desc d{};
    d.key_idx = 0;
    d.prev = -1;
    if (!open) {
        d.len = (uint32_t)(len - CZ_MESSAGE_OVERHEAD);
        d.counter = counter;
        d.flags = src[32];
    } else {
        d.len = (uint32_t)len;
        d.counter = 0;
        d.flags = 0;  // no replay check: a NaCl nonce is opaque
    }
    const uint32_t nblk = (uint32_t)((len + 63) / 64);
    const uint32_t seg_blocks = single_seg_blocks(nblk);
    uint32_t nseg = 0, ncomb = 0, npart = 0;
    cz_plan_segments(&d, 1, open, seg_blocks, nullptr, 0, &nseg, nullptr, 0, &ncomb, &npart);
    std::vector<cz_segment> seg(std::max<uint32_t>(nseg, 1));
    std::vector<cz_combine> comb(std::max<uint32_t>(ncomb, 1));
    if (cz_plan_segments(&d, 1, open, seg_blocks, seg.data(), (uint32_t)seg.size(), &nseg, comb.data(),
                         (uint32_t)comb.size(), &ncomb, &npart) != CZ_OK)
        return -1;
    // device / staging layout: [0,32) precom [32,64) subkey [64,104) desc [128,130) status
    // [136,144) nonce [256, ..) segments, combines | in | out | work
    const uint64_t o_seg = 256, o_comb = o_seg + 16ull * nseg, o_in = up128(o_comb + 16ull * ncomb + 1);
    const uint64_t in_bytes = open ? len : len - CZ_MESSAGE_OVERHEAD;
    const uint64_t o_out = o_in + up128(in_bytes + 1), out_bytes = open ? len - CZ_MESSAGE_OVERHEAD : len;
    const uint64_t o_work = o_out + up128(out_bytes + 1), total = o_work + 64ull * std::max<uint32_t>(npart, 1);
    if ((e = s.dev.reserve(total)) != hipSuccess || (e = s.stage.reserve(total)) != hipSuccess) {
        hip_fail(e, "alloc");
        return -1;
    }
    uint8_t *st = (uint8_t *)s.stage.ptr, *dv = (uint8_t *)s.dev.ptr;
    memcpy(st, k, 32);
    d.in_off = o_in;
    d.out_off = o_out;
    memcpy(st + 64, &d, sizeof d);
    memcpy(st + o_seg, seg.data(), 16ull * nseg);
    memcpy(st + o_comb, comb.data(), 16ull * ncomb);
    if (!open) {
        memcpy(st + o_in, src + CZ_MESSAGE_OVERHEAD, in_bytes);
    } else {
        static const uint8_t hdr[8] = {7, 'M', 'E', 'S', 'S', 'A', 'G', 'E'};
        memcpy(st + o_in, hdr, 8);
        memcpy(st + o_in + 8, n + 16, 8);
        memcpy(st + o_in + 16, src + 16, len - 16);
    }
    const cz_frame_desc *dd = (const cz_frame_desc *)(dv + 64);
    const cz_segment *ds = (const cz_segment *)(dv + o_seg);
    const cz_combine *dc = (const cz_combine *)(dv + o_comb);
    if ((e = hipMemcpyAsync(dv, st, o_in + in_bytes, hipMemcpyHostToDevice, s.stream)) != hipSuccess ||
        (e = czk_subkeys(dv, dv + 32, 1, n, s.stream)) != hipSuccess ||
        (e = open ? czk_open_segments(dd, ds, nseg, dc, ncomb, dv, dv, dv + 32, dv + o_work, (uint16_t *)(dv + 128),
                                      (uint64_t *)(dv + 136), s.stream)
                  : czk_seal_segments(dd, ds, nseg, dc, ncomb, dv, dv, dv + 32, dv + o_work, s.stream)) !=
            hipSuccess ||
        (e = hipMemsetAsync(dv, 0, 64, s.stream)) != hipSuccess ||  // no key material left behind
        (e = hipMemcpyAsync(st + 128, dv + 128, 2, hipMemcpyDeviceToHost, s.stream)) != hipSuccess ||
        (e = hipMemcpyAsync(st + o_out, dv + o_out, out_bytes, hipMemcpyDeviceToHost, s.stream)) != hipSuccess ||
        // nor plaintext: the staged payload (seal) or the opened one (open), on the device
        (e = hipMemsetAsync(dv + (open ? o_out : o_in), 0, open ? out_bytes : in_bytes, s.stream)) != hipSuccess ||
        (e = hipStreamSynchronize(s.stream)) != hipSuccess) {
        (void)hipStreamSynchronize(s.stream);
        explicit_bzero(st, 32);
        explicit_bzero(st + o_in, in_bytes);
        explicit_bzero(st + o_out, out_bytes);
        hip_fail(e, "box");
        return -1;
    }
    explicit_bzero(st, 32);
    if (!open) {
        explicit_bzero(st + o_in, in_bytes);
        memset(dst, 0, 16);
        memcpy(dst + 16, st + o_out + 16, len - 16);
        return 0;
    }
    uint16_t status;
    memcpy(&status, st + 128, 2);
    if ((status & 0xff) != CZ_STATUS_OK) {
        explicit_bzero(st + o_out, out_bytes);
        return -1;  // tag mismatch: dst untouched (as NaCl)
    }
    memset(dst, 0, 32);
    dst[32] = (uint8_t)(status >> 8);
    memcpy(dst + 33, st + o_out, out_bytes);
    explicit_bzero(st + o_out, out_bytes);
    return 0;
}

}  // namespace czi

namespace czi {

// The segment planner (cz_plan_segments) in one pass, into vectors: the engine plans each
// pipeline group while the copies of the previous one run.
void plan_segments(const cz_frame_desc *h_desc, uint32_t count, int open, uint32_t seg_blocks,
                   std::vector<cz_segment> &segs, std::vector<cz_combine> &combs, uint32_t &npart)
{
    segs.clear();
    combs.clear();
    // (split threshold 1.0 / 1.25 / 1.5 / 2.0 x seg_blocks measured within noise on the Zipf batch,
    // profiles/r03/zipf_order_split_s7_s8.log)
    const uint32_t split_above = seg_blocks + seg_blocks / 2;
    segs.reserve(count);
    uint32_t parts = 0;
    for (uint32_t i = 0; i < count; i++) {
        const uint64_t mlen = open ? (uint64_t)h_desc[i].len : (uint64_t)h_desc[i].len + CZ_MESSAGE_OVERHEAD;
        uint32_t nblk = (uint32_t)((mlen + 63) / 64);
        if (nblk == 0)
            nblk = 1;
        if (nblk <= split_above) {
            segs.push_back({i, 0u, nblk, 0xffffffffu});
            continue;
        }
        // Seal segment s covers box blocks [s*seg, (s+1)*seg).  Open segments s >= 1 start one
        // block later, at s*seg + 1, so each one's payload chunks start at s*seg: the 33-byte
        // shift puts payload chunk g across box blocks g and g+1.  Last segment: the remainder.
        const uint32_t lead = open ? 1u : 0u;
        const uint32_t ns = (nblk - lead + seg_blocks - 1) / seg_blocks;
        combs.push_back({i, parts, ns, 0u});
        for (uint32_t s = 0; s < ns; s++) {
            const uint32_t b0 = s ? s * seg_blocks + lead : 0u;
            const uint32_t b1 = s + 1 < ns ? (s + 1) * seg_blocks + lead : nblk;
            segs.push_back({i, b0, b1 - b0, parts + s});
        }
        parts += ns;
    }
    // longest first, keyed on the kernel's loop count (output chunks), so that waves hold
    // equal-length segments and can take the line-staged store path
    auto chunks = [&](const cz_segment &g) -> uint32_t {
        if (!open)
            return g.nblocks;
        const uint32_t len = h_desc[g.frame].len;
        if (len < CZ_MESSAGE_OVERHEAD)
            return 0u;
        const uint32_t nblk = (len + 63) / 64, bend = g.first_block + g.nblocks;
        const uint32_t cb = g.first_block ? g.first_block - 1 : 0u;
        const uint32_t ce = bend == nblk ? (len - CZ_MESSAGE_OVERHEAD + 63) / 64 : bend - 1;
        return ce - cb;
    };
    // Seal, within one length: segments whose input starts on a 128-byte line first, then the
    // ones starting 64 bytes into a line, so that waves hold one line phase and the odd ones
    // can read whole lines (seal_segment in cz_kernels.hip).
    auto phase = [&](const cz_segment &g) -> uint32_t {
        return open ? 0u : (uint32_t)(((h_desc[g.frame].in_off + 64ull * g.first_block) >> 6) & 1u);
    };
    // Then, within one (length, input phase), by the output's line class (bit 6 of the output
    // offset: the half of a 128-byte line it starts in).  Outputs at any byte offset go through
    // EmitShiftLines, which flushes once per chunk pair for a wave of one class and at every
    // chunk (each lane's store masked half the time) for a mixed wave: with 8-byte packed output
    // offsets, sorting by length alone left most Zipf waves mixed (3.8x the SALU, +17% VALU of
    // the 128-byte-slot layout).  128-byte aligned outputs are all class 0: no change for them.
    // Key: chunks * 4 + (1 - phase) * 2 + (1 - class).
    auto oclass = [&](const cz_segment &g) -> uint32_t {
        const uint64_t first_out = open ? (g.first_block ? 64ull * (g.first_block - 1) : 0ull) : 64ull * g.first_block;
        return (uint32_t)(((h_desc[g.frame].out_off + first_out) >> 6) & 1u);
    };
    std::vector<std::pair<uint64_t, uint32_t>> key(segs.size());
    for (size_t k = 0; k < segs.size(); k++)
        key[k] = {4ull * chunks(segs[k]) + 2u * (1u - phase(segs[k])) + (1u - oclass(segs[k])), (uint32_t)k};
    std::stable_sort(key.begin(), key.end(), [](const std::pair<uint64_t, uint32_t> &a,
                                                 const std::pair<uint64_t, uint32_t> &b) { return a.first > b.first; });
    std::vector<cz_segment> sorted(segs.size());
    for (size_t k = 0; k < segs.size(); k++)
        sorted[k] = segs[key[k].second];
    segs.swap(sorted);
    npart = parts;
}

}  // namespace czi

using namespace czi;

// ---- cz_ctx ----------------------------------------------------------------
// host-staged uniform batches up to this many bytes (in + out slots) run on one stream
constexpr uint64_t SMALL_BATCH_BYTES = 4ull << 20;
// single-chunk host-staged uniform batches of multi-block frames up to this many bytes: segment kernels
constexpr uint64_t SEG_BATCH_BYTES = 64ull << 20;

struct cz_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    DevBuf desc, in, out, status, keys, subkeys, work;
    HostBuf hdesc;
    uint32_t nkeys = 0;
    // pipelined uniform batches: one stream per role (H2D, kernels, D2H) and NB chunk buffer sets
    // used round robin; events order the reuse of each set across the three streams
    static constexpr int PIPE = 3, NB = 4;
    hipStream_t ps[PIPE] = {nullptr, nullptr, nullptr};
    hipEvent_t ev_in[NB] = {}, ev_kern[NB] = {}, ev_out[NB] = {};
    DevBuf pin[NB], pout[NB], pflags[NB], pstatus[NB];
};

extern "C" {

const char *cz_last_error(void) { return g_err.c_str(); }

const char *cz_version(void) { return "curvezmq-mi355x 0.1 (gfx950)"; }

int cz_tune(const char *key, int value)
{
    if (key && strcmp(key, "nacl_one_max") == 0) {  // bytes; at least one pass of k_nacl_one
        const int old = (int)g_nacl_one_bytes.load(std::memory_order_relaxed);
        g_nacl_one_bytes.store(std::min<uint64_t>(std::max<int64_t>(value, 0), czk_nacl_one_limit()),
                               std::memory_order_relaxed);
        return old;
    }
    int old = czk_tune(key, value);
    if (old < 0)
        return fail(CZ_EINVAL, "cz_tune: unknown key");
    return old;
}

int cz_device_ok(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0)
        return 0;
    return 1;
}

int cz_box_afternm(uint8_t *c, const uint8_t *m, uint64_t mlen, const uint8_t n[24], const uint8_t k[32])
{
    return nacl_one(c, m, mlen, n, k, 0);
}

int cz_nacl_forget(void)
{
    Single &s = t_single;
    s.forget_host(true);
    if (s.ready && s.subcache.ptr) {
        hipError_t e = hipMemsetAsync(s.subcache.ptr, 0, s.subcache.cap, s.stream);
        if (e == hipSuccess)
            e = hipStreamSynchronize(s.stream);
        if (e != hipSuccess)
            return hip_fail(e, "cz_nacl_forget");
    }
    return CZ_OK;
}

int cz_box_open_afternm(uint8_t *m, const uint8_t *c, uint64_t clen, const uint8_t n[24], const uint8_t k[32])
{
    return nacl_one(m, c, clen, n, k, 1);
}

int cz_secretbox(uint8_t *c, const uint8_t *m, uint64_t mlen, const uint8_t n[24], const uint8_t k[32])
{
    return nacl_one(c, m, mlen, n, k, 0);
}

int cz_secretbox_open(uint8_t *m, const uint8_t *c, uint64_t clen, const uint8_t n[24], const uint8_t k[32])
{
    return nacl_one(m, c, clen, n, k, 1);
}

int cz_subkeys(void *d_subkeys, const void *d_precom, uint32_t nkeys, int direction, void *stream)
{
    if (!d_subkeys || !d_precom)
        return fail(CZ_EINVAL, "cz_subkeys: null pointer");
    if (direction != CZ_DIR_C2S && direction != CZ_DIR_S2C)
        return fail(CZ_EINVAL, "cz_subkeys: bad direction %d", direction);
    hipError_t e = czk_subkeys(d_precom, d_subkeys, nkeys, prefix_for(direction), (hipStream_t)stream);
    return e == hipSuccess ? CZ_OK : hip_fail(e, "cz_subkeys");
}

int cz_subkey(uint8_t out[32], const uint8_t k[32], int direction)
{
    if (!out || !k)
        return fail(CZ_EINVAL, "cz_subkey: null pointer");
    if (direction != CZ_DIR_C2S && direction != CZ_DIR_S2C)
        return fail(CZ_EINVAL, "cz_subkey: bad direction %d", direction);
    int rc = single_init();
    if (rc != CZ_OK)
        return rc;
    Single &s = t_single;
    hipError_t e;
    if ((e = s.dev.reserve(256)) != hipSuccess)
        return hip_fail(e, "hipMalloc");
    uint8_t *d = (uint8_t *)s.dev.ptr;
    if ((e = hipMemcpyAsync(d, k, 32, hipMemcpyHostToDevice, s.stream)) != hipSuccess ||
        (e = czk_subkeys(d, d + 32, 1, prefix_for(direction), s.stream)) != hipSuccess ||
        (e = hipMemcpyAsync(out, d + 32, 32, hipMemcpyDeviceToHost, s.stream)) != hipSuccess) {
        (void)hipMemsetAsync(d, 0, 64, s.stream);
        (void)hipStreamSynchronize(s.stream);
        return hip_fail(e, "cz_subkey");
    }
    if ((e = hipMemsetAsync(d, 0, 64, s.stream)) != hipSuccess || (e = hipStreamSynchronize(s.stream)) != hipSuccess)
        return hip_fail(e, "cz_subkey");
    return CZ_OK;
}

int cz_seal_batch(const cz_frame_desc *d_desc, const uint32_t *d_order, uint32_t count, const void *d_in,
                  void *d_out, const void *d_subkeys, void *stream)
{
    if (count && (!d_desc || !d_in || !d_out || !d_subkeys))
        return fail(CZ_EINVAL, "cz_seal_batch: null pointer");
    hipError_t e = czk_seal_desc(d_desc, d_order, count, d_in, d_out, d_subkeys, (hipStream_t)stream);
    return e == hipSuccess ? CZ_OK : hip_fail(e, "cz_seal_batch");
}

int cz_open_batch(const cz_frame_desc *d_desc, const uint32_t *d_order, uint32_t count, const void *d_in,
                  void *d_out, const void *d_subkeys, uint16_t *d_status, uint64_t *d_nonces, void *stream)
{
    if (count && (!d_desc || !d_in || !d_out || !d_subkeys || !d_status))
        return fail(CZ_EINVAL, "cz_open_batch: null pointer");
    hipError_t e =
        czk_open_desc(d_desc, d_order, count, d_in, d_out, d_subkeys, d_status, d_nonces, (hipStream_t)stream);
    return e == hipSuccess ? CZ_OK : hip_fail(e, "cz_open_batch");
}

int cz_seal_uniform(uint32_t count, uint32_t len, const void *d_in, uint64_t in_stride, void *d_out,
                    uint64_t out_stride, const void *d_subkey, uint64_t counter0, const uint8_t *d_flags8,
                    void *stream)
{
    if (count && (!d_in || !d_out || !d_subkey))
        return fail(CZ_EINVAL, "cz_seal_uniform: null pointer");
    if (count > 1 && (in_stride < len || out_stride < (uint64_t)len + CZ_MESSAGE_OVERHEAD))
        return fail(CZ_EINVAL, "cz_seal_uniform: stride smaller than the frame");
    if ((uint64_t)len + CZ_MESSAGE_OVERHEAD > 0xffffffffull)
        return fail(CZ_EINVAL, "cz_seal_uniform: frame too large");
    if (!uniform_span(count, in_stride, len, nullptr) ||
        !uniform_span(count, out_stride, (uint64_t)len + CZ_MESSAGE_OVERHEAD, nullptr))
        return fail(CZ_EINVAL, "cz_seal_uniform: count x stride overflows the address space");
    hipError_t e = czk_seal_uniform(d_in, in_stride, d_out, out_stride, count, len, d_subkey, counter0, d_flags8,
                                    (hipStream_t)stream);
    return e == hipSuccess ? CZ_OK : hip_fail(e, "cz_seal_uniform");
}

int cz_seal_uniform_box(uint32_t count, uint32_t len, const void *d_box, uint64_t box_stride, void *d_out,
                        uint64_t out_stride, const void *d_subkey, uint64_t counter0, void *stream)
{
    if (count && (!d_box || !d_out || !d_subkey))
        return fail(CZ_EINVAL, "cz_seal_uniform_box: null pointer");
    if ((uint64_t)len + CZ_MESSAGE_OVERHEAD > 0xffffffffull)
        return fail(CZ_EINVAL, "cz_seal_uniform_box: frame too large");
    if (count > 1 && (box_stride < (uint64_t)len + CZ_MESSAGE_OVERHEAD || out_stride < (uint64_t)len + CZ_MESSAGE_OVERHEAD))
        return fail(CZ_EINVAL, "cz_seal_uniform_box: stride smaller than the frame");
    if (!uniform_span(count, box_stride, (uint64_t)len + CZ_MESSAGE_OVERHEAD, nullptr) ||
        !uniform_span(count, out_stride, (uint64_t)len + CZ_MESSAGE_OVERHEAD, nullptr))
        return fail(CZ_EINVAL, "cz_seal_uniform_box: count x stride overflows the address space");
    hipError_t e = czk_seal_uniform_box(d_box, box_stride, d_out, out_stride, count, len, d_subkey, counter0,
                                        (hipStream_t)stream);
    return e == hipSuccess ? CZ_OK : hip_fail(e, "cz_seal_uniform_box");
}

int cz_open_uniform(uint32_t count, uint32_t size, const void *d_in, uint64_t in_stride, void *d_out,
                    uint64_t out_stride, const void *d_subkey, uint64_t floor0, int check, uint16_t *d_status,
                    void *stream)
{
    if (count && (!d_in || !d_out || !d_subkey || !d_status))
        return fail(CZ_EINVAL, "cz_open_uniform: null pointer");
    if (count > 1 && (in_stride < size || (size >= 33 && out_stride < size - 33u)))
        return fail(CZ_EINVAL, "cz_open_uniform: stride smaller than the frame");
    if (!uniform_span(count, in_stride, size, nullptr) ||
        !uniform_span(count, out_stride, size >= 33 ? size - 33u : 0u, nullptr))
        return fail(CZ_EINVAL, "cz_open_uniform: count x stride overflows the address space");
    hipError_t e = czk_open_uniform(d_in, in_stride, d_out, out_stride, count, size, d_subkey, floor0, check,
                                    d_status, (hipStream_t)stream);
    return e == hipSuccess ? CZ_OK : hip_fail(e, "cz_open_uniform");
}

int cz_plan_order(const cz_frame_desc *h_desc, uint32_t count, uint32_t *h_order)
{
    if (count && (!h_desc || !h_order))
        return fail(CZ_EINVAL, "cz_plan_order: null pointer");
    std::iota(h_order, h_order + count, 0u);
    std::stable_sort(h_order, h_order + count,
                     [h_desc](uint32_t a, uint32_t b) { return h_desc[a].len > h_desc[b].len; });
    return CZ_OK;
}

int cz_plan_segments(const cz_frame_desc *h_desc, uint32_t count, int open, uint32_t seg_blocks, cz_segment *h_seg,
                     uint32_t seg_cap, uint32_t *nseg, cz_combine *h_comb, uint32_t comb_cap, uint32_t *ncomb,
                     uint32_t *npart)
{
    if ((count && !h_desc) || !nseg || !ncomb || !npart)
        return fail(CZ_EINVAL, "cz_plan_segments: null pointer");
    if (seg_blocks < 2)
        return fail(CZ_EINVAL, "cz_plan_segments: seg_blocks must be >= 2");
    std::vector<cz_segment> segs;
    std::vector<cz_combine> combs;
    uint32_t parts = 0;
    plan_segments(h_desc, count, open, seg_blocks, segs, combs, parts);
    *nseg = (uint32_t)segs.size();
    *ncomb = (uint32_t)combs.size();
    *npart = parts;
    if (segs.size() > seg_cap || combs.size() > comb_cap || (segs.size() && !h_seg) || (combs.size() && !h_comb))
        return fail(CZ_EINVAL, "cz_plan_segments: capacity too small (need %u segments, %u combines)", *nseg,
                    *ncomb);
    std::copy(segs.begin(), segs.end(), h_seg);
    std::copy(combs.begin(), combs.end(), h_comb);
    return CZ_OK;
}

int cz_seal_segments(const cz_frame_desc *d_desc, const cz_segment *d_seg, uint32_t nseg, const cz_combine *d_comb,
                     uint32_t ncomb, const void *d_in, void *d_out, const void *d_subkeys, void *d_work,
                     void *stream)
{
    if (nseg && (!d_desc || !d_seg || !d_in || !d_out || !d_subkeys))
        return fail(CZ_EINVAL, "cz_seal_segments: null pointer");
    if (ncomb && (!d_comb || !d_work))
        return fail(CZ_EINVAL, "cz_seal_segments: null combine list / workspace");
    hipError_t e = czk_seal_segments(d_desc, d_seg, nseg, d_comb, ncomb, d_in, d_out, d_subkeys, d_work,
                                     (hipStream_t)stream);
    return e == hipSuccess ? CZ_OK : hip_fail(e, "cz_seal_segments");
}

int cz_open_segments(const cz_frame_desc *d_desc, const cz_segment *d_seg, uint32_t nseg, const cz_combine *d_comb,
                     uint32_t ncomb, const void *d_in, void *d_out, const void *d_subkeys, void *d_work,
                     uint16_t *d_status, uint64_t *d_nonces, void *stream)
{
    if (nseg && (!d_desc || !d_seg || !d_in || !d_out || !d_subkeys || !d_status))
        return fail(CZ_EINVAL, "cz_open_segments: null pointer");
    if (ncomb && (!d_comb || !d_work))
        return fail(CZ_EINVAL, "cz_open_segments: null combine list / workspace");
    hipError_t e = czk_open_segments(d_desc, d_seg, nseg, d_comb, ncomb, d_in, d_out, d_subkeys, d_work, d_status,
                                     d_nonces, (hipStream_t)stream);
    return e == hipSuccess ? CZ_OK : hip_fail(e, "cz_open_segments");
}

int cz_fill(void *d_buf, uint64_t nbytes, uint64_t seed, void *stream)
{
    if (nbytes && !d_buf)
        return fail(CZ_EINVAL, "cz_fill: null pointer");
    hipError_t e = czk_fill(d_buf, nbytes, seed, (hipStream_t)stream);
    return e == hipSuccess ? CZ_OK : hip_fail(e, "cz_fill");
}

int cz_dev_copy(void *d_dst, const void *d_src, uint64_t nbytes, void *stream)
{
    if (nbytes && (!d_dst || !d_src))
        return fail(CZ_EINVAL, "cz_dev_copy: null pointer");
    if ((nbytes | (uintptr_t)d_dst | (uintptr_t)d_src) & 15u)
        return fail(CZ_EINVAL, "cz_dev_copy: pointers and size must be 16-byte multiples");
    hipError_t e = czk_copy16(d_dst, d_src, nbytes, (hipStream_t)stream);
    return e == hipSuccess ? CZ_OK : hip_fail(e, "cz_dev_copy");
}

// ---- host-staged contexts ----------------------------------------------------
int cz_ctx_create(cz_ctx **out, int device)
{
    if (!out)
        return fail(CZ_EINVAL, "cz_ctx_create: null");
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0)
        return fail(CZ_EHIP, "no HIP device available (the CURVE path runs only on the GPU)");
    if (device < 0 || device >= n)
        return fail(CZ_EINVAL, "cz_ctx_create: device %d of %d", device, n);
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess)
        return hip_fail(e, "hipSetDevice");
    cz_ctx *c = new cz_ctx();
    c->device = device;
    e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete c;
        return hip_fail(e, "hipStreamCreate");
    }
    *out = c;
    return CZ_OK;
}

void cz_ctx_destroy(cz_ctx *c)
{
    if (!c)
        return;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    c->desc.release();
    c->in.release();
    c->out.release();
    c->status.release();
    c->keys.release();
    c->subkeys.release();
    c->work.release();
    c->hdesc.release();
    for (int k = 0; k < cz_ctx::PIPE; k++)
        if (c->ps[k]) {
            (void)hipStreamSynchronize(c->ps[k]);
            (void)hipStreamDestroy(c->ps[k]);
        }
    for (int k = 0; k < cz_ctx::NB; k++) {
        for (hipEvent_t ev : {c->ev_in[k], c->ev_kern[k], c->ev_out[k]})
            if (ev)
                (void)hipEventDestroy(ev);
        c->pin[k].release();
        c->pout[k].release();
        c->pflags[k].release();
        c->pstatus[k].release();
    }
    (void)hipStreamDestroy(c->stream);
    delete c;
}

int cz_ctx_set_keys(cz_ctx *c, const uint8_t *h_precom, uint32_t nkeys, int direction)
{
    if (!c || (nkeys && !h_precom))
        return fail(CZ_EINVAL, "cz_ctx_set_keys: null");
    if (direction != CZ_DIR_C2S && direction != CZ_DIR_S2C)
        return fail(CZ_EINVAL, "cz_ctx_set_keys: bad direction %d", direction);
    hipError_t e;
    (void)hipSetDevice(c->device);
    if ((e = c->keys.reserve(32ull * nkeys)) != hipSuccess || (e = c->subkeys.reserve(32ull * nkeys)) != hipSuccess)
        return hip_fail(e, "hipMalloc");
    if ((e = hipMemcpyAsync(c->keys.ptr, h_precom, 32ull * nkeys, hipMemcpyHostToDevice, c->stream)) != hipSuccess ||
        (e = czk_subkeys(c->keys.ptr, c->subkeys.ptr, nkeys, prefix_for(direction), c->stream)) != hipSuccess ||
        (e = hipStreamSynchronize(c->stream)) != hipSuccess)
        return hip_fail(e, "cz_ctx_set_keys");
    c->nkeys = nkeys;
    return CZ_OK;
}

static int ctx_check_desc(const cz_ctx *c, const cz_frame_desc *d, uint32_t count, uint64_t in_bytes,
                          uint64_t out_bytes, bool seal)
{
    for (uint32_t i = 0; i < count; i++) {
        uint64_t ilen = d[i].len;
        uint64_t olen = seal ? ilen + CZ_MESSAGE_OVERHEAD : (ilen >= 33 ? ilen - 33 : 0);
        if (d[i].in_off + ilen > in_bytes || d[i].out_off + olen > out_bytes)
            return fail(CZ_EINVAL, "frame %u out of the buffer bounds", i);
        if (d[i].key_idx >= c->nkeys)
            return fail(CZ_EINVAL, "frame %u: key_idx %u >= %u keys", i, d[i].key_idx, c->nkeys);
        if (!seal && d[i].prev >= (int32_t)count)
            return fail(CZ_EINVAL, "frame %u: prev %d out of range", i, d[i].prev);
    }
    return CZ_OK;
}

static int ctx_run(cz_ctx *c, const cz_frame_desc *h_desc, uint32_t count, const void *h_in, uint64_t in_bytes,
                   void *h_out, uint64_t out_bytes, uint16_t *h_status, bool seal)
{
    if (!c || (count && (!h_desc || !h_in || !h_out)))
        return fail(CZ_EINVAL, "cz_ctx: null pointer");
    if (!seal && count && !h_status)
        return fail(CZ_EINVAL, "cz_ctx_open: null status");
    int rc = ctx_check_desc(c, h_desc, count, in_bytes, out_bytes, seal);
    if (rc != CZ_OK)
        return rc;
    if (count == 0)
        return CZ_OK;
    // segment kernels, the segment length scaled to the batch (batch_seg_blocks): a batch of a few
    // long frames spreads over many lanes instead of walking each frame on one
    uint64_t tb = 0, longest = 0;
    for (uint32_t i = 0; i < count; i++) {
        const uint64_t nb = ((seal ? (uint64_t)h_desc[i].len + CZ_MESSAGE_OVERHEAD : (uint64_t)h_desc[i].len) + 63) / 64;
        tb += nb;
        longest = std::max<uint64_t>(longest, nb);
    }
    std::vector<cz_segment> segs;
    std::vector<cz_combine> combs;
    uint32_t npart = 0;
    plan_segments(h_desc, count, seal ? 0 : 1, batch_seg_blocks(tb, longest), segs, combs, npart);
    const uint64_t m_seg = sizeof(cz_frame_desc) * (uint64_t)count, m_comb = m_seg + sizeof(cz_segment) * segs.size(),
                   m_end = m_comb + sizeof(cz_combine) * combs.size();
    hipError_t e;
    (void)hipSetDevice(c->device);
    if ((e = c->desc.reserve(m_end)) != hipSuccess || (e = c->hdesc.reserve(m_end)) != hipSuccess ||
        (e = c->in.reserve(in_bytes + 16)) != hipSuccess || (e = c->out.reserve(out_bytes + 16)) != hipSuccess ||
        (e = c->status.reserve(sizeof(uint16_t) * (uint64_t)count)) != hipSuccess ||
        (e = c->work.reserve(64ull * std::max<uint32_t>(npart, 1))) != hipSuccess)
        return hip_fail(e, "hipMalloc");
    uint8_t *hm = (uint8_t *)c->hdesc.ptr;
    memcpy(hm, h_desc, m_seg);
    memcpy(hm + m_seg, segs.data(), m_comb - m_seg);
    memcpy(hm + m_comb, combs.data(), m_end - m_comb);
    const uint8_t *dm = (const uint8_t *)c->desc.ptr;
    if ((e = hipMemcpyAsync(c->desc.ptr, hm, m_end, hipMemcpyHostToDevice, c->stream)) != hipSuccess ||
        (e = hipMemcpyAsync(c->in.ptr, h_in, in_bytes, hipMemcpyHostToDevice, c->stream)) != hipSuccess)
        return hip_fail(e, "H2D");
    const cz_frame_desc *dd = (const cz_frame_desc *)dm;
    const cz_segment *ds = (const cz_segment *)(dm + m_seg);
    const cz_combine *dc = (const cz_combine *)(dm + m_comb);
    if (seal) {
        e = czk_seal_segments(dd, ds, (uint32_t)segs.size(), dc, (uint32_t)combs.size(), c->in.ptr, c->out.ptr,
                              c->subkeys.ptr, c->work.ptr, c->stream);
    } else {
        if (out_bytes && (e = hipMemsetAsync(c->out.ptr, 0, out_bytes, c->stream)) != hipSuccess)
            return hip_fail(e, "memset");
        e = czk_open_segments(dd, ds, (uint32_t)segs.size(), dc, (uint32_t)combs.size(), c->in.ptr, c->out.ptr,
                              c->subkeys.ptr, c->work.ptr, (uint16_t *)c->status.ptr, nullptr, c->stream);
    }
    if (e != hipSuccess)
        return hip_fail(e, "launch");
    if ((e = hipMemcpyAsync(h_out, c->out.ptr, out_bytes, hipMemcpyDeviceToHost, c->stream)) != hipSuccess)
        return hip_fail(e, "D2H");
    if (!seal &&
        (e = hipMemcpyAsync(h_status, c->status.ptr, sizeof(uint16_t) * (uint64_t)count, hipMemcpyDeviceToHost,
                            c->stream)) != hipSuccess)
        return hip_fail(e, "D2H");
    if ((e = hipStreamSynchronize(c->stream)) != hipSuccess)
        return hip_fail(e, "sync");
    return CZ_OK;
}

int cz_ctx_seal(cz_ctx *c, const cz_frame_desc *h_desc, uint32_t count, const void *h_in, uint64_t in_bytes,
                void *h_out, uint64_t out_bytes)
{
    return ctx_run(c, h_desc, count, h_in, in_bytes, h_out, out_bytes, nullptr, true);
}

int cz_ctx_open(cz_ctx *c, const cz_frame_desc *h_desc, uint32_t count, const void *h_in, uint64_t in_bytes,
                void *h_out, uint64_t out_bytes, uint16_t *h_status)
{
    return ctx_run(c, h_desc, count, h_in, in_bytes, h_out, out_bytes, h_status, false);
}

// Host-staged uniform batch of one chunk (<= SEG_BATCH_BYTES) through the segment kernels.
// The uniform kernel walks a frame's blocks on one lane, so a batch of a few frames costs one
// lane's whole walk (~150 us at 4 KiB); segments of a few blocks spread each frame over many lanes.
// Uniform frames need no sort: segments go out segment-major (segment s of every frame, then s + 1),
// which keeps equal lengths together.
static int ctx_uniform_segments(cz_ctx *c, bool seal, uint32_t count, uint32_t len, const void *h_in,
                                uint64_t in_stride, void *h_out, uint64_t out_stride, uint64_t counter0,
                                const uint8_t *h_flags8, uint16_t *h_status, int check, uint32_t nblk)
{
    const uint32_t seg = batch_seg_blocks((uint64_t)count * nblk, nblk);
    const uint32_t lead = seal ? 0u : 1u;
    const bool split = nblk > seg + seg / 2;
    const uint32_t ns = split ? (nblk - lead + seg - 1) / seg : 1u;
    const uint64_t nseg = (uint64_t)count * ns, ncomb = split ? count : 0;
    const uint64_t m_desc = 0, m_seg = (uint64_t)count * sizeof(cz_frame_desc),
                   m_comb = m_seg + nseg * sizeof(cz_segment), m_end = m_comb + ncomb * sizeof(cz_combine);
    const uint64_t in_bytes = (uint64_t)(count - 1) * in_stride + len, out_bytes = (uint64_t)count * out_stride;
    hipError_t e;
    if ((e = c->hdesc.reserve(m_end)) != hipSuccess || (e = c->desc.reserve(m_end)) != hipSuccess ||
        (e = c->in.reserve(in_bytes + 16)) != hipSuccess || (e = c->out.reserve(out_bytes + 16)) != hipSuccess ||
        (e = c->status.reserve(2ull * count)) != hipSuccess ||
        (e = c->work.reserve(64ull * std::max<uint64_t>(ncomb * ns, 1))) != hipSuccess)
        return hip_fail(e, "alloc");
    uint8_t *hm = (uint8_t *)c->hdesc.ptr;
    cz_frame_desc *hd = (cz_frame_desc *)(hm + m_desc);
    cz_segment *hs = (cz_segment *)(hm + m_seg);
    cz_combine *hc = (cz_combine *)(hm + m_comb);
    for (uint32_t i = 0; i < count; i++) {
        if (seal)
            hd[i] = {(uint64_t)i * in_stride, (uint64_t)i * out_stride, len, 0u, counter0 + i,
                     h_flags8 ? (uint32_t)h_flags8[i] : 0u, -1};
        else
            hd[i] = {(uint64_t)i * in_stride, (uint64_t)i * out_stride, len, 0u, counter0,
                     check ? (uint32_t)CZ_DESC_CHECK_NONCE : 0u, i ? (int32_t)(i - 1) : -1};
    }
    for (uint32_t s = 0; s < ns; s++) {
        const uint32_t b0 = s ? s * seg + lead : 0u, b1 = s + 1 < ns ? (s + 1) * seg + lead : nblk;
        for (uint32_t i = 0; i < count; i++)
            hs[(uint64_t)s * count + i] = {i, b0, b1 - b0, split ? i * ns + s : 0xffffffffu};
    }
    for (uint64_t i = 0; i < ncomb; i++)
        hc[i] = {(uint32_t)i, (uint32_t)i * ns, ns, 0u};
    hipStream_t q = c->ps[1];
    uint8_t *dm = (uint8_t *)c->desc.ptr;
    const cz_frame_desc *dd = (const cz_frame_desc *)(dm + m_desc);
    const cz_segment *ds = (const cz_segment *)(dm + m_seg);
    const cz_combine *dc = (const cz_combine *)(dm + m_comb);
    if ((e = hipMemcpyAsync(dm, hm, m_end, hipMemcpyHostToDevice, q)) != hipSuccess ||
        (e = hipMemcpyAsync(c->in.ptr, h_in, in_bytes, hipMemcpyHostToDevice, q)) != hipSuccess)
        return hip_fail(e, "H2D");
    // whole slots, as the pipelined path returns them: the body, then zeros to the slot's end (and
    // zeros in a rejected open's slot)
    if ((e = hipMemsetAsync(c->out.ptr, 0, out_bytes, q)) == hipSuccess) {
        if (seal)
            e = czk_seal_segments(dd, ds, (uint32_t)nseg, dc, (uint32_t)ncomb, c->in.ptr, c->out.ptr, c->subkeys.ptr,
                                  c->work.ptr, q);
        else
            e = czk_open_segments(dd, ds, (uint32_t)nseg, dc, (uint32_t)ncomb, c->in.ptr, c->out.ptr, c->subkeys.ptr,
                                  c->work.ptr, (uint16_t *)c->status.ptr, nullptr, q);
    }
    if (e != hipSuccess)
        return hip_fail(e, "launch");
    if ((e = hipMemcpyAsync(h_out, c->out.ptr, out_bytes, hipMemcpyDeviceToHost, q)) != hipSuccess ||
        (!seal && (e = hipMemcpyAsync(h_status, c->status.ptr, 2ull * count, hipMemcpyDeviceToHost, q)) != hipSuccess) ||
        (e = hipStreamSynchronize(q)) != hipSuccess)
        return hip_fail(e, "D2H");
    return CZ_OK;
}

// Pipelined host-staged uniform batch.  Chunk k of `chunk` frames uses buffer set k % NB:
//   stream 0: H2D of chunk k (after the kernel of chunk k - NB released the set's input)
//   stream 1: kernel of chunk k (after its H2D, and after the D2H of chunk k - NB released the
//             set's output)
//   stream 2: D2H of chunk k (after its kernel)
// One stream per direction keeps each DMA direction's queue in chunk order, so H2D and D2H run
// concurrently (full duplex) instead of queueing behind each other on shared streams.
static int ctx_uniform(cz_ctx *c, bool seal, uint32_t count, uint32_t len, const void *h_in, uint64_t in_stride,
                       void *h_out, uint64_t out_stride, uint64_t counter0, const uint8_t *h_flags8,
                       uint16_t *h_status, int check, uint32_t chunk)
{
    if (!c || (count && (!h_in || !h_out)))
        return fail(CZ_EINVAL, "cz_ctx_*_uniform: null pointer");
    if (c->nkeys < 1)
        return fail(CZ_EINVAL, "cz_ctx_*_uniform: no key (cz_ctx_set_keys)");
    if (!seal && count && !h_status)
        return fail(CZ_EINVAL, "cz_ctx_open_uniform: null status");
    const uint64_t olen = seal ? (uint64_t)len + CZ_MESSAGE_OVERHEAD : (len >= 33 ? len - 33u : 0u);
    if (count > 1 && (in_stride < len || out_stride < olen))
        return fail(CZ_EINVAL, "cz_ctx_*_uniform: stride smaller than a frame");
    // the staging sizes below are count * stride products: refuse strides they would wrap
    if (count > 1 && (!uniform_span(count, in_stride, len, nullptr) || !uniform_span(count, out_stride, olen, nullptr)))
        return fail(CZ_EINVAL, "cz_ctx_*_uniform: count x stride overflows the address space");
    if (count == 0)
        return CZ_OK;
    if (count == 1) {  // strides are not checked for one frame: its slot is the frame itself
        in_stride = len;
        out_stride = std::max<uint64_t>(olen, 1);
    }
    // a single-chunk batch of multi-block frames: the segment kernels (one stream)
    const uint64_t nblk = ((seal ? (uint64_t)len + CZ_MESSAGE_OVERHEAD : (uint64_t)len) + 63) / 64;
    const bool seg_path = nblk >= 8 && (chunk == 0 || chunk >= count) &&
                          (uint64_t)count * (in_stride + out_stride) <= SEG_BATCH_BYTES;
    // (default chunks of count / 8 within 2048 .. 16384 frames were slower than 16384 for every
    // batch of 8192 .. 65536 x 4 KiB: profiles/r03/ctx_small_batch.log)
    if (chunk == 0)
        chunk = 16384;
    hipError_t e;
    (void)hipSetDevice(c->device);
    const uint32_t per = chunk < count ? chunk : count;
    for (int k = 0; k < cz_ctx::PIPE; k++)
        if (!c->ps[k] && (e = hipStreamCreateWithFlags(&c->ps[k], hipStreamNonBlocking)) != hipSuccess)
            return hip_fail(e, "hipStreamCreate");
    if (seg_path)
        return ctx_uniform_segments(c, seal, count, len, h_in, in_stride, h_out, out_stride, counter0, h_flags8,
                                    h_status, check, (uint32_t)nblk);
    for (int k = 0; k < cz_ctx::NB; k++) {
        for (hipEvent_t *ev : {&c->ev_in[k], &c->ev_kern[k], &c->ev_out[k]})
            if (!*ev && (e = hipEventCreateWithFlags(ev, hipEventDisableTiming)) != hipSuccess)
                return hip_fail(e, "hipEventCreate");
        if ((e = c->pin[k].reserve((uint64_t)per * in_stride + 16)) != hipSuccess ||
            (e = c->pout[k].reserve((uint64_t)per * out_stride + 16)) != hipSuccess ||
            (e = c->pflags[k].reserve(per)) != hipSuccess || (e = c->pstatus[k].reserve(2ull * per)) != hipSuccess)
            return hip_fail(e, "hipMalloc");
    }
    const uint8_t *hin = (const uint8_t *)h_in;
    uint8_t *hout = (uint8_t *)h_out;
    hipStream_t s_in = c->ps[0], s_k = c->ps[1], s_out = c->ps[2];
    // A small batch runs H2D, kernel and D2H on one stream: each cross-stream event wait costs
    // tens of us, which dominates below a few MiB (host-resident paths).
    if (count == per && (uint64_t)count * (in_stride + out_stride) <= SMALL_BATCH_BYTES)
        s_in = s_out = s_k;
    uint32_t k = 0;
    for (uint32_t f0 = 0; f0 < count; f0 += per, k++) {
        const uint32_t nc = count - f0 < per ? count - f0 : per;
        const int q = k % cz_ctx::NB;
        const bool reuse = k >= (uint32_t)cz_ctx::NB;
        const uint64_t ib = (uint64_t)(nc - 1) * in_stride + len;
        if ((reuse && (e = hipStreamWaitEvent(s_in, c->ev_kern[q], 0)) != hipSuccess) ||
            (e = hipMemcpyAsync(c->pin[q].ptr, hin + (uint64_t)f0 * in_stride, ib, hipMemcpyHostToDevice, s_in)) !=
                hipSuccess)
            return hip_fail(e, "H2D");
        const uint8_t *dfl = nullptr;
        if (seal && h_flags8) {
            if ((e = hipMemcpyAsync(c->pflags[q].ptr, h_flags8 + f0, nc, hipMemcpyHostToDevice, s_in)) != hipSuccess)
                return hip_fail(e, "H2D flags");
            dfl = (const uint8_t *)c->pflags[q].ptr;
        }
        if (s_in != s_k && ((e = hipEventRecord(c->ev_in[q], s_in)) != hipSuccess ||
                            (e = hipStreamWaitEvent(s_k, c->ev_in[q], 0)) != hipSuccess ||
                            (reuse && (e = hipStreamWaitEvent(s_k, c->ev_out[q], 0)) != hipSuccess)))
            return hip_fail(e, "event");
        if (seal) {
            // a slot stride off the 128-byte lines leaves the bytes between bodies to the caller
            // (cz_seal_uniform): zero them, so the host gets whole slots on every path
            e = out_stride % 128 ? hipMemsetAsync(c->pout[q].ptr, 0, (uint64_t)nc * out_stride, s_k) : hipSuccess;
            if (e == hipSuccess)
                e = czk_seal_uniform(c->pin[q].ptr, in_stride, c->pout[q].ptr, out_stride, nc, len, c->subkeys.ptr,
                                     counter0 + f0, dfl, s_k);
        } else {
            // the chunk's first frame must beat the previous chunk's last nonce: read it from the host copy
            uint64_t floor0 = counter0;
            if (f0 > 0) {
                const uint8_t *pb = hin + (uint64_t)(f0 - 1) * in_stride + 8;
                floor0 = 0;
                for (int b = 0; b < 8; b++)
                    floor0 = (floor0 << 8) | pb[b];
            }
            // zeros in rejected frames' slots, never an earlier chunk's plaintext
            e = hipMemsetAsync(c->pout[q].ptr, 0, (uint64_t)nc * out_stride, s_k);
            if (e == hipSuccess)
                e = czk_open_uniform(c->pin[q].ptr, in_stride, c->pout[q].ptr, out_stride, nc, len, c->subkeys.ptr,
                                     floor0, check, (uint16_t *)c->pstatus[q].ptr, s_k);
        }
        if (e != hipSuccess)
            return hip_fail(e, "launch");
        if (s_out != s_k && ((e = hipEventRecord(c->ev_kern[q], s_k)) != hipSuccess ||
                             (e = hipStreamWaitEvent(s_out, c->ev_kern[q], 0)) != hipSuccess))
            return hip_fail(e, "event");
        if ((e = hipMemcpyAsync(hout + (uint64_t)f0 * out_stride, c->pout[q].ptr, (uint64_t)nc * out_stride,
                                hipMemcpyDeviceToHost, s_out)) != hipSuccess)
            return hip_fail(e, "D2H");
        if (!seal && (e = hipMemcpyAsync(h_status + f0, c->pstatus[q].ptr, 2ull * nc, hipMemcpyDeviceToHost, s_out)) !=
                         hipSuccess)
            return hip_fail(e, "D2H status");
        if (s_out != s_k && (e = hipEventRecord(c->ev_out[q], s_out)) != hipSuccess)
            return hip_fail(e, "event");
    }
    for (int q = 0; q < cz_ctx::PIPE; q++)
        if ((s_in != s_k || q == 1) && (e = hipStreamSynchronize(c->ps[q])) != hipSuccess)
            return hip_fail(e, "sync");
    return CZ_OK;
}

int cz_ctx_seal_uniform(cz_ctx *c, uint32_t count, uint32_t len, const void *h_in, uint64_t in_stride, void *h_out,
                        uint64_t out_stride, uint64_t counter0, const uint8_t *h_flags8, uint32_t chunk_frames)
{
    return ctx_uniform(c, true, count, len, h_in, in_stride, h_out, out_stride, counter0, h_flags8, nullptr, 0,
                       chunk_frames);
}

int cz_ctx_open_uniform(cz_ctx *c, uint32_t count, uint32_t size, const void *h_in, uint64_t in_stride, void *h_out,
                        uint64_t out_stride, uint64_t floor0, int check, uint16_t *h_status, uint32_t chunk_frames)
{
    return ctx_uniform(c, false, count, size, h_in, in_stride, h_out, out_stride, floor0, nullptr, h_status, check,
                       chunk_frames);
}

void *cz_host_alloc(uint64_t bytes)
{
    void *p = nullptr;
    if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) {
        fail(CZ_ENOMEM, "hipHostMalloc(%llu) failed", (unsigned long long)bytes);
        return nullptr;
    }
    std::lock_guard<std::mutex> g(g_host_mu);
    g_host_bases.insert(p);
    return p;
}

int cz_host_free(void *p)
{
    if (!p)
        return CZ_OK;
    {
        std::lock_guard<std::mutex> g(g_host_mu);
        if (g_host_bases.erase(p) == 0)
            return fail(CZ_EINVAL, "cz_host_free: %p is not a live cz_host_alloc base address", p);
    }
    hipError_t e = hipHostFree(p);
    return e == hipSuccess ? CZ_OK : hip_fail(e, "cz_host_free");
}

int cz_nacl_thread_init(void)
{
    int rc = single_init();
    if (rc == CZ_OK)
        rc = hs_thread_init();
    return rc;
}

}  // extern "C"
