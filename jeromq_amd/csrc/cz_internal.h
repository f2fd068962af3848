// cz_internal.h -- shared host-side helpers of libcurvezmq_mi355x (not part of the C-ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdint.h>

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
}

namespace czi {

int fail(int code, const char *fmt, ...);
int hip_fail(hipError_t e, const char *where);
const uint8_t *prefix_for(int direction);

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
