// cz_wire.cpp -- ZMTP v2 framing: host parser (V2Decoder rules) and the device pack/unpack launcher.
//
// Reference: zmq/io/coder/v2/V2Encoder.java:31-55 (flags byte, 1-byte or BE64 size),
// V2Decoder.java:37-105 (flagsReady / oneByteSizeReady / eightByteSizeReady), and the size
// checks of zmq/io/coder/Decoder.java:76-98.  Parsing stays on the host: it is a sequential walk
// over one header per frame (the bodies are never touched here), while the byte movement
// (packing sealed bodies behind their headers, unpacking received bodies into aligned slots)
// runs on the device in k_v2_copy.
#include <stdint.h>
#include <string.h>

#include "cz_internal.h"

using namespace czi;

extern "C" {

uint32_t cz_v2_header_size(uint64_t size) { return size > 255u ? 9u : 2u; }

int cz_v2_parse(const uint8_t *wire, uint64_t len, int64_t maxmsgsize, cz_v2_frame *frames, uint32_t cap,
                uint32_t *nframes, uint64_t *consumed)
{
    if (!nframes || !consumed || (len && !wire) || (cap && !frames))
        return fail(CZ_EINVAL, "cz_v2_parse: null pointer");
    uint64_t p = 0;
    uint32_t nf = 0;
    int rc = CZ_OK;
    while (nf < cap && p < len) {
        const uint8_t f = wire[p];
        uint64_t size, h;
        if (f & CZ_V2_LARGE) {
            if (len - p < 9)
                break;
            size = 0;
            for (int b = 1; b <= 8; b++)
                size = (size << 8) | wire[p + b];  // Wire.getUInt64: big-endian
            h = 9;
            if ((int64_t)size <= 0) {  // V2Decoder.eightByteSizeReady: `size <= 0` on a Java long
                rc = fail(CZ_EPROTO, "cz_v2_parse: 8-byte frame size %lld at offset %llu",
                          (long long)(int64_t)size, (unsigned long long)p);
                break;
            }
        } else {
            if (len - p < 2)
                break;
            size = wire[p + 1];
            h = 2;
        }
        // Decoder.sizeReady: maxmsgsize, then the int range of a Java array
        if ((maxmsgsize >= 0 && size > (uint64_t)maxmsgsize) || size > 0x7fffffffull) {
            rc = fail(CZ_EMSGSIZE, "cz_v2_parse: frame size %llu at offset %llu exceeds the limit",
                      (unsigned long long)size, (unsigned long long)p);
            break;
        }
        if (len - p - h < size)
            break;  // body not complete yet: keep the bytes for the next read
        uint32_t mf = 0;
        if (f & CZ_V2_MORE)
            mf |= CZ_MSG_MORE;
        if (f & CZ_V2_COMMAND)
            mf |= CZ_MSG_COMMAND;
        frames[nf++] = {p + h, (uint32_t)size, mf};
        p += h + size;
    }
    *nframes = nf;
    *consumed = p;
    return rc;
}

int cz_v2_copy(const cz_v2_item *d_items, uint32_t count, const void *d_src, void *d_dst, void *stream)
{
    if (count && (!d_items || !d_src || !d_dst))
        return fail(CZ_EINVAL, "cz_v2_copy: null pointer");
    hipError_t e = czk_v2_copy(d_items, count, d_src, d_dst, (hipStream_t)stream);
    return e == hipSuccess ? CZ_OK : hip_fail(e, "cz_v2_copy");
}

}  // extern "C"
