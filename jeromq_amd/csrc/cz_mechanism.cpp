// cz_mechanism.cpp -- host-side mirror of JeroMQ's CURVE Mechanism plugin for
// MESSAGE traffic, with the crypto on the GPU.
//
// Mirrors (names, argument meaning and error behaviour):
//   abstract class Mechanism: Msg encode(Msg) / Msg decode(Msg)     Mechanism.java:202-210
//   CurveClientMechanism.encode / decode (CONNECTED state)          CurveClientMechanism.java:126-224
//   CurveServerMechanism.encode / decode (CONNECTED state)          CurveServerMechanism.java:127-224
// The handshake (HELLO / WELCOME / INITIATE / READY, per connection) is out of
// scope for this tier: a mechanism is created in the CONNECTED state from the
// handshake's outputs (cnPrecom, cnNonce, cnPeerNonce).
//
// Error behaviour: encode cannot fail (the reference asserts rc == 0,
// CurveClientMechanism.java:153-154).  decode returns "null" (here CZ_EPROTO)
// with errno EPROTO and the monitor event the reference raises:
//   not "\x07MESSAGE"          -> ZMTP_UNEXPECTED_COMMAND            (:168-172)
//   size < 33                  -> ZMTP_MALFORMED_COMMAND_MESSAGE     (:174-178)
//   nonce <= cnPeerNonce       -> client: ZMTP_CRYPTOGRAPHIC (:188-191),
//                                 server: ZMTP_INVALID_SEQUENCE (CurveServerMechanism.java:188-191)
//   bad tag                    -> ZMTP_CRYPTOGRAPHIC                 (:219-223)
// cnPeerNonce is updated before the crypto check, as the reference does (:193).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "cz_internal.h"

using namespace czi;

namespace jeromq_amd {

class CurveMechanism {
public:
    CurveMechanism(bool as_server, const uint8_t precom[32], uint64_t cn_nonce, uint64_t cn_peer_nonce, int device)
        : as_server_(as_server), cn_nonce_(cn_nonce), cn_peer_nonce_(cn_peer_nonce), device_(device)
    {
        memcpy(precom_, precom, 32);
    }

    ~CurveMechanism()
    {
        if (stream_) {
            (void)hipSetDevice(device_);
            (void)hipStreamSynchronize(stream_);
            (void)hipStreamDestroy(stream_);
        }
        for (DevBuf *b : {&keys_, &desc_, &in_, &out_, &status_, &nonces_, &work_})
            b->release();
        if (one_.ptr)
            explicit_bzero(one_.ptr, one_.cap);
        for (HostBuf *b : {&hdesc_, &hstatus_, &hnonces_, &hin_, &hout_, &one_})
            b->release();
    }

    int init()
    {
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess || n == 0)
            return fail(CZ_EHIP, "no HIP device available (the CURVE path runs only on the GPU)");
        hipError_t e;
        if ((e = hipSetDevice(device_)) != hipSuccess)
            return hip_fail(e, "hipSetDevice");
        if ((e = hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking)) != hipSuccess)
            return hip_fail(e, "hipStreamCreate");
        // subkey table: [0] = ours (encode), [1] = peer's (decode); [2..3] precom staging
        if ((e = keys_.reserve(128)) != hipSuccess)
            return hip_fail(e, "hipMalloc");
        uint8_t *k = (uint8_t *)keys_.ptr;
        const int tx = as_server_ ? CZ_DIR_S2C : CZ_DIR_C2S;
        const int rx = as_server_ ? CZ_DIR_C2S : CZ_DIR_S2C;
        if ((e = hipMemcpyAsync(k + 64, precom_, 32, hipMemcpyHostToDevice, stream_)) != hipSuccess ||
            (e = czk_subkeys(k + 64, k + 0, 1, prefix_for(tx), stream_)) != hipSuccess ||
            (e = czk_subkeys(k + 64, k + 32, 1, prefix_for(rx), stream_)) != hipSuccess ||
            (e = hipMemsetAsync(k + 64, 0, 32, stream_)) != hipSuccess ||
            (e = hipStreamSynchronize(stream_)) != hipSuccess)
            return hip_fail(e, "subkeys");
        return CZ_OK;
    }

    // Mechanism.encode(Msg) for one MESSAGE
    int64_t encode(const uint8_t *payload, uint64_t n, int msg_flags, uint8_t *out)
    {
        if (n > (uint64_t)CZ_MESSAGE_MAX)
            return fail(CZ_EMSGSIZE, "encode: %llu-byte payload exceeds CZ_MESSAGE_MAX", (unsigned long long)n);
        uint64_t in_off = 0, out_off = 0;
        uint32_t len = (uint32_t)n;
        uint8_t fl = (uint8_t)msg_flags;
        int rc = encode_batch(1, payload, &in_off, &len, &fl, out, &out_off);
        return rc == CZ_OK ? (int64_t)(n + CZ_MESSAGE_OVERHEAD) : rc;
    }

    int encode_batch(uint32_t count, const uint8_t *h_in, const uint64_t *in_off, const uint32_t *len,
                     const uint8_t *msg_flags, uint8_t *h_out, const uint64_t *out_off)
    {
        if (count == 0)
            return CZ_OK;
        if (!h_in || !in_off || !len || !h_out || !out_off)
            return fail(CZ_EINVAL, "encode_batch: null pointer");
        for (uint32_t i = 0; i < count; i++)
            if (len[i] > (uint32_t)CZ_MESSAGE_MAX)
                return fail(CZ_EMSGSIZE, "encode_batch: frame %u (%u bytes) exceeds CZ_MESSAGE_MAX", i, len[i]);
        if (count == 1 && (uint64_t)len[0] + 33 <= nacl_one_bytes())
            return seal_one(h_in + in_off[0], len[0], msg_flags ? msg_flags[0] : 0u, h_out + out_off[0]);
        // device layout: 16-byte aligned frames, packed; segments of batch_seg_blocks blocks
        std::vector<cz_frame_desc> d(count);
        uint64_t ib = 0, ob = 0, tb = 0, longest = 0;
        for (uint32_t i = 0; i < count; i++) {
            d[i].in_off = ib;
            d[i].out_off = ob;
            d[i].len = len[i];
            d[i].key_idx = 0;
            d[i].counter = cn_nonce_ + i;  // cnNonce++ per message (CurveClientMechanism.java:161)
            uint32_t f = msg_flags ? msg_flags[i] : 0u;
            d[i].flags = f & (CZ_MSG_MORE | CZ_MSG_COMMAND);
            d[i].prev = -1;
            ib += (len[i] + 15ull) & ~15ull;
            ob += (len[i] + CZ_MESSAGE_OVERHEAD + 15ull) & ~15ull;
            const uint64_t nb = (len[i] + (uint64_t)CZ_MESSAGE_OVERHEAD + 63) / 64;
            tb += nb;
            longest = std::max<uint64_t>(longest, nb);
        }
        hipError_t e;
        (void)hipSetDevice(device_);
        if ((e = stage_plan(d, 0, batch_seg_blocks(tb, longest))) != hipSuccess ||
            (e = in_.reserve(ib + 16)) != hipSuccess || (e = out_.reserve(ob + 16)) != hipSuccess ||
            (e = hin_.reserve(ib + 16)) != hipSuccess || (e = hout_.reserve(ob + 16)) != hipSuccess)
            return hip_fail(e, "hipMalloc");
        // the frames gathered into pinned staging, one H2D; one D2H back, scattered on the host
        uint8_t *hs = (uint8_t *)hin_.ptr;
        for (uint32_t i = 0; i < count; i++)
            if (len[i])
                memcpy(hs + d[i].in_off, h_in + in_off[i], len[i]);
        const uint8_t *dm = (const uint8_t *)desc_.ptr;
        if ((e = hipMemcpyAsync(in_.ptr, hs, ib, hipMemcpyHostToDevice, stream_)) != hipSuccess ||
            (e = hipMemcpyAsync(desc_.ptr, hdesc_.ptr, plan_bytes_, hipMemcpyHostToDevice, stream_)) != hipSuccess ||
            (e = czk_seal_segments((const cz_frame_desc *)dm, (const cz_segment *)(dm + seg_off_), (uint32_t)segs_.size(),
                                   (const cz_combine *)(dm + comb_off_), (uint32_t)combs_.size(), in_.ptr, out_.ptr,
                                   keys_.ptr, work_.ptr, stream_)) != hipSuccess ||
            (e = hipMemcpyAsync(hout_.ptr, out_.ptr, ob, hipMemcpyDeviceToHost, stream_)) != hipSuccess ||
            (e = hipStreamSynchronize(stream_)) != hipSuccess)
            return hip_fail(e, "seal");
        const uint8_t *ho = (const uint8_t *)hout_.ptr;
        for (uint32_t i = 0; i < count; i++)
            memcpy(h_out + out_off[i], ho + d[i].out_off, len[i] + (uint64_t)CZ_MESSAGE_OVERHEAD);
        cn_nonce_ += count;
        return CZ_OK;
    }

    // Mechanism.decode(Msg) for one MESSAGE body
    int64_t decode(const uint8_t *body, uint64_t size, uint8_t *out, int *msg_flags, int *event)
    {
        uint64_t in_off = 0, out_off = 0;
        uint32_t sz = (uint32_t)size;
        uint8_t fl = 0;
        int32_t failed = -1;
        if (size > 0xffffffffull)
            return fail(CZ_EINVAL, "decode: body too large");
        int rc = decode_batch(1, body, &in_off, &sz, out, &out_off, &fl, &failed, event);
        if (rc != CZ_OK)
            return rc;
        if (failed >= 0)
            return CZ_EPROTO;
        if (msg_flags)
            *msg_flags = fl;
        return (int64_t)(size - CZ_MESSAGE_OVERHEAD);
    }

    int decode_batch(uint32_t count, const uint8_t *h_in, const uint64_t *in_off, const uint32_t *size,
                     uint8_t *h_out, const uint64_t *out_off, uint8_t *msg_flags, int32_t *failed, int *event)
    {
        if (failed)
            *failed = -1;
        if (event)
            *event = 0;
        if (count == 0)
            return CZ_OK;
        if (!h_in || !in_off || !size || !h_out || !out_off)
            return fail(CZ_EINVAL, "decode_batch: null pointer");
        if (count == 1 && size[0] <= nacl_one_bytes())
            return open_one(h_in + in_off[0], size[0], h_out + out_off[0], msg_flags, failed, event);
        std::vector<cz_frame_desc> d(count);
        uint64_t ib = 0, ob = 0, tb = 0, longest = 0;
        for (uint32_t i = 0; i < count; i++) {
            d[i].in_off = ib;
            d[i].out_off = ob;
            d[i].len = size[i];
            d[i].key_idx = 1;
            d[i].counter = cn_peer_nonce_;
            d[i].flags = CZ_DESC_CHECK_NONCE;
            d[i].prev = (int32_t)i - 1;  // frames of this connection, in order
            ib += (size[i] + 15ull) & ~15ull;
            uint64_t plen = size[i] >= CZ_MESSAGE_OVERHEAD ? size[i] - CZ_MESSAGE_OVERHEAD : 0;
            ob += (plen + 15ull) & ~15ull;
            const uint64_t nb = (size[i] + 63ull) / 64;
            tb += nb;
            longest = std::max<uint64_t>(longest, nb);
        }
        hipError_t e;
        (void)hipSetDevice(device_);
        if ((e = stage_plan(d, 1, batch_seg_blocks(tb, longest))) != hipSuccess ||
            (e = in_.reserve(ib + 16)) != hipSuccess || (e = out_.reserve(ob + 16)) != hipSuccess ||
            (e = status_.reserve(2ull * count)) != hipSuccess || (e = nonces_.reserve(8ull * count)) != hipSuccess ||
            (e = hstatus_.reserve(2ull * count)) != hipSuccess || (e = hnonces_.reserve(8ull * count)) != hipSuccess ||
            (e = hin_.reserve(ib + 16)) != hipSuccess || (e = hout_.reserve(ob + 16)) != hipSuccess)
            return hip_fail(e, "alloc");
        uint8_t *hs = (uint8_t *)hin_.ptr;
        for (uint32_t i = 0; i < count; i++)
            if (size[i])
                memcpy(hs + d[i].in_off, h_in + in_off[i], size[i]);
        const uint8_t *dm = (const uint8_t *)desc_.ptr;
        if ((e = hipMemcpyAsync(in_.ptr, hs, ib, hipMemcpyHostToDevice, stream_)) != hipSuccess ||
            (e = hipMemcpyAsync(desc_.ptr, hdesc_.ptr, plan_bytes_, hipMemcpyHostToDevice, stream_)) != hipSuccess ||
            (e = czk_open_segments((const cz_frame_desc *)dm, (const cz_segment *)(dm + seg_off_), (uint32_t)segs_.size(),
                                   (const cz_combine *)(dm + comb_off_), (uint32_t)combs_.size(), in_.ptr, out_.ptr,
                                   keys_.ptr, work_.ptr, (uint16_t *)status_.ptr, (uint64_t *)nonces_.ptr, stream_)) !=
                hipSuccess ||
            (e = hipMemcpyAsync(hstatus_.ptr, status_.ptr, 2ull * count, hipMemcpyDeviceToHost, stream_)) !=
                hipSuccess ||
            (e = hipMemcpyAsync(hnonces_.ptr, nonces_.ptr, 8ull * count, hipMemcpyDeviceToHost, stream_)) !=
                hipSuccess ||
            (e = hipStreamSynchronize(stream_)) != hipSuccess)
            return hip_fail(e, "open");
        const uint16_t *st = (const uint16_t *)hstatus_.ptr;
        const uint64_t *nn = (const uint64_t *)hnonces_.ptr;
        // deliver in order; the first failure ends the batch (StreamEngine.java:1072-1073 tears the pipe down)
        uint32_t ok = 0;
        for (; ok < count; ok++)
            if ((st[ok] & 0xff) != CZ_STATUS_OK)
                break;
        // the accepted frames' plaintext: one D2H of their slots, scattered on the host
        const uint64_t okb = ok ? d[ok - 1].out_off + ((size[ok - 1] - CZ_MESSAGE_OVERHEAD + 15ull) & ~15ull) : 0;
        if (okb && ((e = hipMemcpyAsync(hout_.ptr, out_.ptr, okb, hipMemcpyDeviceToHost, stream_)) != hipSuccess ||
                    (e = hipStreamSynchronize(stream_)) != hipSuccess))
            return hip_fail(e, "D2H");
        const uint8_t *ho = (const uint8_t *)hout_.ptr;
        for (uint32_t i = 0; i < ok; i++) {
            uint64_t plen = size[i] - CZ_MESSAGE_OVERHEAD;
            if (plen)
                memcpy(h_out + out_off[i], ho + d[i].out_off, plen);
            if (msg_flags)  // only MORE and COMMAND reach the Msg (CurveClientMechanism.java:207-213)
                msg_flags[i] = (uint8_t)(((st[i] >> 8) & 0x01 ? CZ_MSG_MORE : 0) | ((st[i] >> 8) & 0x02 ? CZ_MSG_COMMAND : 0));
        }
        if ((e = hipStreamSynchronize(stream_)) != hipSuccess)
            return hip_fail(e, "sync");
        if (ok)
            cn_peer_nonce_ = nn[ok - 1];
        if (ok < count) {
            int s = st[ok] & 0xff;
            int ev = 0;
            switch (s) {
            case CZ_STATUS_COMMAND: ev = CZ_ZMTP_UNEXPECTED_COMMAND; break;
            case CZ_STATUS_MALFORMED: ev = CZ_ZMTP_MALFORMED_COMMAND_MESSAGE; break;
            case CZ_STATUS_SEQUENCE: ev = as_server_ ? CZ_ZMTP_INVALID_SEQUENCE : CZ_ZMTP_CRYPTOGRAPHIC; break;
            default:
                ev = CZ_ZMTP_CRYPTOGRAPHIC;
                cn_peer_nonce_ = nn[ok];  // the nonce passed the replay check before the tag failed
                break;
            }
            if (failed)
                *failed = (int32_t)ok;
            if (event)
                *event = ev;
        }
        return CZ_OK;
    }

    // descriptors, segments and combine records of a batch into pinned staging [desc | seg | comb]
    // (one H2D into desc_), and the partial-record buffer sized
    hipError_t stage_plan(const std::vector<cz_frame_desc> &d, int open, uint32_t seg_blocks)
    {
        uint32_t npart = 0;
        plan_segments(d.data(), (uint32_t)d.size(), open, seg_blocks, segs_, combs_, npart);
        seg_off_ = sizeof(cz_frame_desc) * d.size();
        comb_off_ = seg_off_ + sizeof(cz_segment) * segs_.size();
        plan_bytes_ = comb_off_ + sizeof(cz_combine) * combs_.size();
        hipError_t e;
        if ((e = hdesc_.reserve(plan_bytes_)) != hipSuccess || (e = desc_.reserve(plan_bytes_)) != hipSuccess ||
            (e = work_.reserve(64ull * std::max<uint32_t>(npart, 1))) != hipSuccess)
            return e;
        uint8_t *h = (uint8_t *)hdesc_.ptr;
        memcpy(h, d.data(), seg_off_);
        memcpy(h + seg_off_, segs_.data(), comb_off_ - seg_off_);
        memcpy(h + comb_off_, combs_.data(), plan_bytes_ - comb_off_);
        return hipSuccess;
    }

    static void put_be64(uint8_t *p, uint64_t v)
    {
        for (int i = 7; i >= 0; i--, v >>= 8)
            p[i] = (uint8_t)v;
    }

    // One MESSAGE in ONE launch (k_nacl_one, as the jnacl drop-ins): the box
    // 0^32 || flags || payload staged in pinned host memory the kernel reads and writes in place,
    // the subkey read from this mechanism's table (nothing derived per call).
    int seal_one(const uint8_t *payload, uint32_t n, uint32_t flags, uint8_t *out)
    {
        const uint64_t len = 33ull + n, out_off = 128 + ((len + 127) & ~127ull);
        hipError_t e;
        (void)hipSetDevice(device_);
        if ((e = one_.reserve(out_off + len + 128)) != hipSuccess)
            return hip_fail(e, "hipHostMalloc");
        uint8_t *st = (uint8_t *)one_.ptr;
        memset(st + 128, 0, 32);
        st[160] = (uint8_t)(flags & (CZ_MSG_MORE | CZ_MSG_COMMAND));
        if (n)
            memcpy(st + 161, payload, n);
        uint8_t nonce[24];
        memcpy(nonce, prefix_for(as_server_ ? CZ_DIR_S2C : CZ_DIR_C2S), 16);
        put_be64(nonce + 16, cn_nonce_);
        static const uint8_t kz[32] = {};
        *(volatile int *)(st + 56) = -2;
        e = czk_nacl_one(st, (uint32_t)len, 0, keys_.ptr, 0, (uint32_t)out_off, kz, nonce, stream_);
        if (e == hipSuccess)
            e = hipStreamSynchronize(stream_);
        explicit_bzero(st + 128, len);  // the plaintext
        if (e != hipSuccess)
            return hip_fail(e, "seal");
        if (*(volatile int *)(st + 56) != 0)
            return fail(CZ_EHIP, "seal: the kernel did not complete");
        // "\x07MESSAGE" || nonce || tag || ciphertext (CurveClientMechanism.java:144-160)
        memcpy(out, "\x07MESSAGE", 8);
        memcpy(out + 8, nonce + 16, 8);
        memcpy(out + 16, st + out_off + 16, 17ull + n);
        cn_nonce_++;
        return CZ_OK;
    }

    int open_status_event(int status) const
    {
        switch (status) {
        case CZ_STATUS_COMMAND: return CZ_ZMTP_UNEXPECTED_COMMAND;
        case CZ_STATUS_MALFORMED: return CZ_ZMTP_MALFORMED_COMMAND_MESSAGE;
        case CZ_STATUS_SEQUENCE: return as_server_ ? CZ_ZMTP_INVALID_SEQUENCE : CZ_ZMTP_CRYPTOGRAPHIC;
        default: return CZ_ZMTP_CRYPTOGRAPHIC;
        }
    }

    // One MESSAGE body opened in ONE launch: the header checks on the host, in the kernels' order
    // (open_header in cz_kernels.hip: command name, size, replay), then 0^16 || tag || ciphertext
    // opened in place in pinned host memory.
    int open_one(const uint8_t *body, uint32_t size, uint8_t *out, uint8_t *msg_flags, int32_t *failed, int *event)
    {
        int status = CZ_STATUS_OK;
        uint64_t nonce = 0;
        if (size < 8 || memcmp(body, "\x07MESSAG", 7) != 0)  // byte 7 is never compared (Msgs.java:31)
            status = CZ_STATUS_COMMAND;
        else if (size < CZ_MESSAGE_OVERHEAD)
            status = CZ_STATUS_MALFORMED;
        else {
            for (int i = 0; i < 8; i++)
                nonce = (nonce << 8) | body[8 + i];
            if ((int64_t)nonce <= (int64_t)cn_peer_nonce_)
                status = CZ_STATUS_SEQUENCE;
        }
        if (status == CZ_STATUS_OK) {
            const uint64_t out_off = 128 + ((size + 127ull) & ~127ull);
            hipError_t e;
            (void)hipSetDevice(device_);
            if ((e = one_.reserve(out_off + size + 128)) != hipSuccess)
                return hip_fail(e, "hipHostMalloc");
            uint8_t *st = (uint8_t *)one_.ptr;
            memset(st + 128, 0, 16);
            memcpy(st + 144, body + 16, size - 16ull);
            uint8_t n24[24];
            memcpy(n24, prefix_for(as_server_ ? CZ_DIR_C2S : CZ_DIR_S2C), 16);
            memcpy(n24 + 16, body + 8, 8);
            static const uint8_t kz[32] = {};
            *(volatile int *)(st + 56) = -2;
            e = czk_nacl_one(st, size, 1, (uint8_t *)keys_.ptr + 32, 0, (uint32_t)out_off, kz, n24, stream_);
            if (e == hipSuccess)
                e = hipStreamSynchronize(stream_);
            if (e != hipSuccess)
                return hip_fail(e, "open");
            cn_peer_nonce_ = nonce;  // before the crypto check, as the reference (:193)
            if (*(volatile int *)(st + 56) != 0) {
                status = CZ_STATUS_CRYPTO;
            } else {
                const uint8_t fl = st[out_off + 32];
                if (size > CZ_MESSAGE_OVERHEAD)
                    memcpy(out, st + out_off + 33, size - (uint64_t)CZ_MESSAGE_OVERHEAD);
                if (msg_flags)
                    *msg_flags = (uint8_t)((fl & 0x01 ? CZ_MSG_MORE : 0) | (fl & 0x02 ? CZ_MSG_COMMAND : 0));
            }
            explicit_bzero(st + out_off, size);  // plaintext, authenticated or not
        }
        if (status != CZ_STATUS_OK) {
            if (failed)
                *failed = 0;
            if (event)
                *event = open_status_event(status);
        }
        return CZ_OK;
    }

    uint64_t nonce() const { return cn_nonce_; }
    uint64_t peer_nonce() const { return cn_peer_nonce_; }

private:
    bool as_server_;
    uint8_t precom_[32];
    uint64_t cn_nonce_, cn_peer_nonce_;
    int device_;
    hipStream_t stream_ = nullptr;
    DevBuf keys_, desc_, in_, out_, status_, nonces_, work_;
    HostBuf hdesc_, hstatus_, hnonces_;
    HostBuf hin_, hout_;  // pinned staging: one H2D and one D2H per batch, not one per frame
    HostBuf one_;         // one-launch staging, read and written by the kernel in place
    uint64_t seg_off_ = 0, comb_off_ = 0, plan_bytes_ = 0;
    std::vector<cz_segment> segs_;
    std::vector<cz_combine> combs_;
};

}  // namespace jeromq_amd

struct cz_mech {
    jeromq_amd::CurveMechanism *impl;
};

extern "C" {

cz_mech *cz_mech_create(int as_server, const uint8_t precom[32], uint64_t cn_nonce, uint64_t cn_peer_nonce, int device)
{
    if (!precom) {
        fail(CZ_EINVAL, "cz_mech_create: null key");
        return nullptr;
    }
    auto *impl = new jeromq_amd::CurveMechanism(as_server != 0, precom, cn_nonce, cn_peer_nonce, device);
    if (impl->init() != CZ_OK) {
        delete impl;
        return nullptr;
    }
    return new cz_mech{impl};
}

void cz_mech_destroy(cz_mech *m)
{
    if (!m)
        return;
    delete m->impl;
    delete m;
}

int64_t cz_mech_encode(cz_mech *m, const uint8_t *payload, uint64_t n, int msg_flags, uint8_t *out)
{
    if (!m || (!payload && n) || !out)
        return fail(CZ_EINVAL, "cz_mech_encode: null pointer");
    static const uint8_t empty[16] = {0};
    return m->impl->encode(payload ? payload : empty, n, msg_flags, out);
}

int64_t cz_mech_decode(cz_mech *m, const uint8_t *body, uint64_t size, uint8_t *out, int *msg_flags, int *event)
{
    if (!m || !body || !out)
        return fail(CZ_EINVAL, "cz_mech_decode: null pointer");
    return m->impl->decode(body, size, out, msg_flags, event);
}

int cz_mech_encode_batch(cz_mech *m, uint32_t count, const uint8_t *h_in, const uint64_t *in_off, const uint32_t *len,
                         const uint8_t *msg_flags, uint8_t *h_out, const uint64_t *out_off)
{
    if (!m)
        return fail(CZ_EINVAL, "cz_mech_encode_batch: null mech");
    return m->impl->encode_batch(count, h_in, in_off, len, msg_flags, h_out, out_off);
}

int cz_mech_decode_batch(cz_mech *m, uint32_t count, const uint8_t *h_in, const uint64_t *in_off,
                         const uint32_t *size, uint8_t *h_out, const uint64_t *out_off, uint8_t *msg_flags,
                         int32_t *failed, int *event)
{
    if (!m)
        return fail(CZ_EINVAL, "cz_mech_decode_batch: null mech");
    return m->impl->decode_batch(count, h_in, in_off, size, h_out, out_off, msg_flags, failed, event);
}

uint64_t cz_mech_nonce(const cz_mech *m) { return m ? m->impl->nonce() : 0; }

uint64_t cz_mech_peer_nonce(const cz_mech *m) { return m ? m->impl->peer_nonce() : 0; }

}  // extern "C"
