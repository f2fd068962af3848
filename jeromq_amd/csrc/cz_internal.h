// cz_internal.h -- shared host-side helpers of libcurvezmq_mi355x (not part of the C-ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdint.h>

#include <vector>

#include "../../include/curvezmq_mi355x.h"

extern "C" {
hipError_t czk_seal_desc(const cz_frame_desc *, const uint32_t *, uint32_t, const void *, void *, const void *,
                         hipStream_t);
hipError_t czk_open_desc(const cz_frame_desc *, const uint32_t *, uint32_t, const void *, void *, const void *,
                         uint16_t *, uint64_t *, hipStream_t);
hipError_t czk_subkeys(const void *, void *, uint32_t, const uint8_t *, hipStream_t);
hipError_t czk_seal_segments(const cz_frame_desc *, const cz_segment *, uint32_t, const cz_combine *, uint32_t,
                             const void *, void *, const void *, void *, hipStream_t);
hipError_t czk_open_segments(const cz_frame_desc *, const cz_segment *, uint32_t, const cz_combine *, uint32_t,
                             const void *, void *, const void *, void *, uint16_t *, uint64_t *, hipStream_t);
hipError_t czk_v2_copy(const cz_v2_item *, uint32_t, const void *, void *, hipStream_t);
hipError_t czk_nacl_one(void *, uint32_t, int, void *, int, uint32_t, const uint8_t *, const uint8_t *, hipStream_t);
uint32_t czk_nacl_one_max(void);
uint32_t czk_nacl_one_limit(void);
}

namespace czi {

int fail(int code, const char *fmt, ...);
int hs_thread_init();  // the calling thread's handshake context (cz_handshake.cpp)
uint64_t nacl_one_bytes();  // boxes up to this size take k_nacl_one (cz_tune "nacl_one_max")
int hip_fail(hipError_t e, const char *where);
const uint8_t *prefix_for(int direction);
void plan_segments(const cz_frame_desc *h_desc, uint32_t count, int open, uint32_t seg_blocks,
                   std::vector<cz_segment> &segs, std::vector<cz_combine> &combs, uint32_t &npart);

// segments, combine records and partial records the planner makes for one frame of `len` (payload for seal, body
// for open) -- lets a caller size its buffers before planning
inline void plan_counts(uint64_t len, int open, uint32_t seg_blocks, uint64_t &nseg, uint64_t &ncomb, uint64_t &npart)
{
    const uint64_t mlen = open ? len : len + CZ_MESSAGE_OVERHEAD;
    uint64_t nblk = (mlen + 63) / 64;
    if (nblk == 0)
        nblk = 1;
    if (nblk <= seg_blocks + seg_blocks / 2) {
        nseg += 1;
        return;
    }
    const uint64_t lead = open ? 1u : 0u;
    const uint64_t ns = (nblk - lead + seg_blocks - 1) / seg_blocks;
    nseg += ns;
    npart += ns;
    ncomb += 1;
}

// Segment length for ONE frame of nblk blocks on its own: a lane walks seg + 1 blocks (block 0
// gives its Poly1305 key) and the combine lane walks the nblk / seg segments serially, so the
// latency is ~ (seg + 1) * T_block + (nblk / seg) * T_combine, T_block / T_combine ~ 18
// (DESIGN.md section 4).
inline uint32_t single_seg_blocks(uint64_t nblk)
{
    uint32_t s = 2;
    while ((uint64_t)(s + 1) * (s + 1) * 18 <= nblk)
        s++;
    return s;
}

// Segment length for a batch of `total` blocks whose longest frame has `longest` blocks: 128
// (SEG_BLOCKS, the throughput setting) once the batch has 64K lanes' worth, shorter below that, so
// a small batch spreads its frames over many lanes; never shorter than the one-frame optimum.
inline uint32_t batch_seg_blocks(uint64_t total, uint64_t longest)
{
    uint64_t s = (total + 65535) / 65536;
    s = s > single_seg_blocks(longest) ? s : single_seg_blocks(longest);
    return (uint32_t)(s < 128 ? s : 128);
}

// device buffer that grows on demand (never shrinks)
struct DevBuf {
    void *ptr = nullptr;
    uint64_t cap = 0;
    hipError_t reserve(uint64_t bytes);
    void release();
};

// pinned host buffer that grows on demand
struct HostBuf {
    void *ptr = nullptr;
    uint64_t cap = 0;
    hipError_t reserve(uint64_t bytes);
    void release();
};

}  // namespace czi
