// cz_engine.cpp -- batching engine: many CURVE connections, one device batch per flush.
//
// The reference encrypts one message at a time on each connection's IO thread:
//   outEvent  (StreamEngine.java:467-535) pulls Msgs, mechanism.encode()s each one
//             (CurveClientMechanism.java:126-163) and V2Encoder-frames it
//             (V2Encoder.java:31-55) into an OUT_BATCH_SIZE buffer for the socket;
//   inEvent   (StreamEngine.java:379-465) V2Decoder-parses the received bytes
//             (V2Decoder.java:37-105) and decodeAndPush (:1067-1098) mechanism.decode()s
//             each frame (CurveClientMechanism.java:165-224), tearing the connection down at
//             the first failure.
// Here the messages of ALL connections are queued in a pinned arena (the ZMQ_MSG_ALLOCATOR
// role, zmq/msg/MsgAllocator.java:5-8) and handled per flush with one device batch:
//   flush_out: descriptors with each connection's next nonces -> H2D -> segmented seal into
//              128-byte aligned body slots -> k_v2_copy packs every connection's frames, in send
//              order, behind their V2 headers into one contiguous wire stream per connection ->
//              D2H into pinned memory, ready for the socket write.
//   flush_in:  host V2 parse of each connection's received bytes (one header per frame; a
//              partial frame waits for more bytes) -> H2D of the whole frames -> k_v2_copy unpacks
//              bodies into aligned slots -> segmented open with the nonce floor chained frame to
//              frame inside each connection (desc.prev) -> D2H -> per-connection delivery up to the
//              first failing frame, whose status becomes the connection's error event.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <thread>
#include <vector>

#include "cz_internal.h"

// pipeline depth of a large flush: groups of >= 8 MiB of wire bytes, at most this many.  At 1 GiB
// per flush, 16 against 8: out 39.0 -> 40.9, in 38.0 -> 40.0 GiB/s (shorter pipeline fill and
// drain); 24 and 32 drop flush_out to 28 / 20 GiB/s (profiles/r03/engine_groups_ab_s9/s10.log).
#ifndef CZ_ENGINE_GROUPS
#define CZ_ENGINE_GROUPS 16
#endif

using namespace czi;

namespace {

constexpr uint64_t SLOT_ALIGN = 128;  // body / payload slots: line-staged stores, whole-line loads
constexpr uint32_t SEG_BLOCKS = 128;  // as jeromq_amd.batch.SEG_BLOCKS

// Segment length for a received flush of `blocks` 64-byte blocks in all (frame sizes are known
// only after the parse): SEG_BLOCKS once there are 64K lanes' worth, shorter below that (down to
// 4) so that a small flush spreads each frame over many lanes instead of walking it on one (a
// 4 KiB frame alone: 65 blocks on one lane, ~150 us).  flush_out knows its lengths up front and
// uses batch_seg_blocks.
uint32_t flush_seg_blocks(uint64_t blocks)
{
    return (uint32_t)std::min<uint64_t>(SEG_BLOCKS, std::max<uint64_t>(4, (blocks + 65535) / 65536));
}

uint64_t round_up(uint64_t v, uint64_t a) { return (v + a - 1) / a * a; }

// CZ_ENGINE_TRACE=1: per-phase wall times of each flush on stderr (profiling aid)
struct PhaseTimer {
    bool on;
    const char *what;
    std::chrono::steady_clock::time_point t0, last;
    char buf[512];
    int len = 0;
    explicit PhaseTimer(const char *w) : on(getenv("CZ_ENGINE_TRACE") != nullptr), what(w)
    {
        t0 = last = std::chrono::steady_clock::now();
    }
    void mark(const char *phase)
    {
        if (!on)
            return;
        auto now = std::chrono::steady_clock::now();
        len += snprintf(buf + len, sizeof(buf) - len, " %s=%.2fms", phase,
                        std::chrono::duration<double, std::milli>(now - last).count());
        last = now;
    }
    ~PhaseTimer()
    {
        if (on)
            fprintf(stderr, "[cz_engine] %s%s total=%.2fms\n", what, buf,
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    }
};

struct Run {
    uint64_t off, len;
};

// A connection's receive buffer: a region of one of the engine's pinned receive blocks.
struct RxBuf {
    uint8_t *ptr = nullptr;
    uint64_t cap = 0;
    uint32_t blk = 0;
};

// Pinned receive blocks shared by every connection.  Regions are bump-allocated, so connections
// that receive together lie next to each other and flush_in moves a run of them with one DMA
// (each DMA costs a ~25 us gap on the SDMA queue, about the time of a 1 MiB copy).  A region that
// grows extends in place when it is the last one of its block; otherwise it moves and its old
// space goes to a first-fit free list.
struct RxPool {
    struct Block {
        uint8_t *base;
        uint64_t cap, used;
    };
    std::vector<Block> blocks;
    std::vector<RxBuf> free_list;
    uint64_t total = 0;

    ~RxPool()
    {
        for (Block &b : blocks)
            (void)hipHostFree(b.base);
    }
    // grow r to hold `want` bytes, keeping its first `used` bytes
    hipError_t grow(RxBuf &r, uint64_t used, uint64_t want)
    {
        if (want <= r.cap)
            return hipSuccess;
        const uint64_t cap = (std::max<uint64_t>({want, 2 * r.cap, 65536}) + 255) & ~255ull;
        if (r.ptr) {
            Block &b = blocks[r.blk];
            if (r.ptr + r.cap == b.base + b.used && b.used - r.cap + cap <= b.cap) {
                b.used += cap - r.cap;
                r.cap = cap;
                return hipSuccess;
            }
        }
        RxBuf n;
        size_t fi = 0;
        for (; fi < free_list.size() && free_list[fi].cap < cap; fi++) {
        }
        if (fi < free_list.size()) {
            n = free_list[fi];
            free_list.erase(free_list.begin() + (long)fi);
        } else {
            if (blocks.empty() || blocks.back().cap - blocks.back().used < cap) {
                // blocks grow with the pool: 1 MiB .. 256 MiB, or one region's size
                const uint64_t bcap = std::max<uint64_t>(cap, std::min<uint64_t>(256ull << 20,
                                                                                std::max<uint64_t>(1ull << 20, total)));
                void *p = nullptr;
                hipError_t e = hipHostMalloc(&p, bcap, hipHostMallocDefault);
                if (e != hipSuccess)
                    return e;
                blocks.push_back({(uint8_t *)p, bcap, 0});
                total += bcap;
            }
            Block &b = blocks.back();
            n = {b.base + b.used, cap, (uint32_t)(blocks.size() - 1)};
            b.used += cap;
        }
        if (used)
            memcpy(n.ptr, r.ptr, used);
        if (r.ptr)
            free_list.push_back(r);
        r = n;
        return hipSuccess;
    }
};

struct Conn {
    bool server = false;
    uint32_t tx_key = 0, rx_key = 0;  // subkey table indices
    uint64_t nonce = 0;               // cnNonce: next MESSAGE nonce to send
    uint64_t peer_nonce = 0;          // cnPeerNonce: last accepted peer nonce
    int error = 0;                    // CZ_EPROTO / CZ_EMSGSIZE once torn down
    int event = 0;                    // ZMTP protocol-error event of the failure
    RxBuf rx;                         // received bytes not yet parsed, pinned (DMA'd as they lie)
    uint64_t rx_len = 0;
    std::vector<Run> runs;            // wire stream of the last flush_out: pieces of h_wire, in send order
    std::vector<uint8_t> gathered;    // contiguous copy for cz_engine_wire_out when runs > 1
    std::vector<uint32_t> in_msgs;    // indices into Engine::in_msgs of the last flush_in
    bool removed = false;             // cz_engine_remove_conn: the id and its key slots await reuse
};

struct OutMsg {
    uint32_t conn;
    uint64_t arena_off;
    uint32_t len;
    uint32_t flags;
};

struct InMsg {
    uint64_t plain_off;
    uint32_t len;
    int flags;
};

struct Segs {
    std::vector<cz_segment> seg;
    std::vector<cz_combine> comb;
    uint32_t nseg = 0, ncomb = 0, npart = 0;
};

// destroys a flush's events on every return path
struct EvGuard {
    std::vector<hipEvent_t> &v;
    ~EvGuard()
    {
        for (hipEvent_t x : v)
            if (x)
                (void)hipEventDestroy(x);
    }
};

}  // namespace

struct cz_engine {
    int device = 0;
    hipStream_t stream = nullptr;
    // flush pipelines: ps[0] carries every group's H2D in order; ps[1] waits for a group's copies
    // (event) and runs its kernels; ps[2] waits for those (event) and carries the group's D2H -- so
    // group g's D2H overlaps group g+1's H2D and kernels
    static constexpr int PIPE = 3;
    hipStream_t ps[PIPE] = {nullptr, nullptr, nullptr};
    std::vector<Conn> conns;
    std::vector<int> free_ids;  // removed connections, reused (with their subkey slots) by add_conn
    DevBuf subkeys;  // 32 B per (connection, direction)
    uint32_t nkeys = 0;
    // outbound
    HostBuf arena;
    uint64_t arena_cap = 0, arena_used = 0;
    std::vector<OutMsg> pend;
    HostBuf h_wire;
    uint64_t wire_total = 0;
    // inbound
    HostBuf h_plain;
    std::vector<InMsg> in_msgs;
    // device staging (grows, never shrinks)
    DevBuf d_in, d_body, d_wire, d_desc, d_seg, d_comb, d_work, d_items, d_status, d_nonces, d_plain;
    HostBuf h_status, h_nonces;
    HostBuf h_meta;  // pinned staging of descriptors / items / segment lists (async H2D)
    RxPool rxpool;   // every connection's receive buffer

    // wait for everything issued on every stream (error paths of the flushes: the next recv /
    // flush may write or regrow the pinned buffers those copies still read or write)
    void drain()
    {
        if (stream)
            (void)hipStreamSynchronize(stream);
        for (hipStream_t q : ps)
            if (q)
                (void)hipStreamSynchronize(q);
    }

    ~cz_engine()
    {
        if (stream) {
            (void)hipSetDevice(device);
            (void)hipStreamSynchronize(stream);
            (void)hipStreamDestroy(stream);
        }
        for (hipStream_t &q : ps)
            if (q) {
                (void)hipStreamSynchronize(q);
                (void)hipStreamDestroy(q);
            }
        for (DevBuf *b : {&subkeys, &d_in, &d_body, &d_wire, &d_desc, &d_seg, &d_comb, &d_work, &d_items, &d_status,
                          &d_nonces, &d_plain})
            b->release();
        for (HostBuf *b : {&arena, &h_wire, &h_plain, &h_status, &h_nonces, &h_meta})
            b->release();
    }

    Conn *conn(int c)
    {
        if (c < 0 || (size_t)c >= conns.size() || conns[(size_t)c].removed) {
            fail(CZ_EINVAL, "cz_engine: unknown connection %d", c);
            return nullptr;
        }
        return &conns[(size_t)c];
    }

    // grow the device subkey table to hold `want` keys, keeping its contents
    hipError_t grow_keys(uint32_t want)
    {
        if ((uint64_t)want * 32 <= subkeys.cap)
            return hipSuccess;
        void *p = nullptr;
        const uint64_t bytes = std::max<uint64_t>(4096, (uint64_t)want * 64);
        hipError_t e = hipMalloc(&p, bytes);
        if (e != hipSuccess)
            return e;
        if (nkeys && (e = hipMemcpyAsync(p, subkeys.ptr, (uint64_t)nkeys * 32, hipMemcpyDeviceToDevice, stream)) !=
                         hipSuccess)
            return e;
        if ((e = hipStreamSynchronize(stream)) != hipSuccess)
            return e;
        subkeys.release();
        subkeys.ptr = p;
        subkeys.cap = bytes;
        return hipSuccess;
    }

    // Outbound pipeline.  The wire output is in SEND order: message i's V2 frame (header + body)
    // sits at wpos[i], and each connection's stream is the list of its runs of consecutive frames
    // (one run when the caller queued a connection's messages together, as StreamEngine.outEvent
    // pulls one pipe at a time).  Send order lets the flush run in G groups of ~equal bytes:
    // ps[0] copies group g's arena range and metadata while ps[1] seals + packs group g-1 and
    // copies its wire bytes back, so H2D and D2H overlap instead of running back to back.
    int flush_out()
    {
        PhaseTimer pt("flush_out");
        for (Conn &c : conns) {
            c.runs.clear();
            c.gathered.clear();
        }
        wire_total = 0;
        const uint32_t n = (uint32_t)pend.size();
        if (n == 0) {
            arena_used = 0;  // buffers allocated but never sent are released too
            return CZ_OK;
        }
        // 1. send-order wire positions and each connection's runs
        std::vector<uint64_t> wpos(n + 1);
        uint64_t w = 0, longest = 0;
        for (uint32_t i = 0; i < n; i++) {
            const OutMsg &m = pend[i];
            Conn &c = conns[m.conn];
            const uint64_t body = (uint64_t)m.len + CZ_MESSAGE_OVERHEAD;
            longest = std::max<uint64_t>(longest, body);
            const uint64_t fb = cz_v2_header_size(body) + body;
            wpos[i] = w;
            if (!c.runs.empty() && c.runs.back().off + c.runs.back().len == w)
                c.runs.back().len += fb;
            else
                c.runs.push_back({w, fb});
            w += fb;
        }
        wpos[n] = w;
        wire_total = w;
        const uint32_t seg = batch_seg_blocks(w / 64, (longest + 63) / 64);
        // 2. groups of ~equal wire bytes: [fa, fb) in send order, body slots contiguous per group;
        //    per group the arena prefix it needs, its body-slot base and its segment / combine
        //    counts (plan_counts) -- enough to size every buffer and start the arena copy before
        //    any descriptor exists
        struct Group {
            uint32_t fa, fb;
            uint64_t arena_hi;  // the arena prefix [0, arena_hi) holds every payload of groups <= this one
            uint64_t slot0;     // first body slot
        };
        std::vector<Group> groups;
        {
            const uint64_t G = std::min<uint64_t>(CZ_ENGINE_GROUPS, std::max<uint64_t>(1, w / (8ull << 20)));
            uint32_t fa = 0;
            for (uint32_t i = 0; i < n; i++)
                if (i + 1 == n || wpos[i + 1] * G >= w * (groups.size() + 1)) {
                    groups.push_back({fa, i + 1, 0, 0});
                    fa = i + 1;
                }
        }
        std::vector<uint64_t> soff(groups.size() + 1, 0), coff(groups.size() + 1, 0), woff(groups.size() + 1, 0);
        uint64_t slot = 0, hi = 0;
        for (size_t gi = 0; gi < groups.size(); gi++) {
            Group &g = groups[gi];
            g.slot0 = slot;
            uint64_t ns = 0, nc = 0, np = 0;
            for (uint32_t i = g.fa; i < g.fb; i++) {
                const OutMsg &m = pend[i];
                slot += round_up((uint64_t)m.len + CZ_MESSAGE_OVERHEAD, SLOT_ALIGN);
                hi = std::max<uint64_t>(hi, m.arena_off + m.len);
                plan_counts(m.len, 0, seg, ns, nc, np);
            }
            g.arena_hi = hi;
            soff[gi + 1] = soff[gi] + ns;
            coff[gi + 1] = coff[gi] + nc;
            woff[gi + 1] = woff[gi] + np;
        }
        const uint64_t nseg = soff[groups.size()], ncomb = coff[groups.size()], npart = woff[groups.size()];
        const uint64_t m_items = 0, m_desc = (uint64_t)n * sizeof(cz_v2_item),
                       m_seg = m_desc + (uint64_t)n * sizeof(cz_frame_desc), m_comb = m_seg + nseg * sizeof(cz_segment),
                       m_end = m_comb + ncomb * sizeof(cz_combine);
        hipError_t e;
        if ((e = d_in.reserve(std::max<uint64_t>(arena_used, 16))) != hipSuccess ||
            (e = d_body.reserve(slot)) != hipSuccess || (e = d_wire.reserve(wire_total)) != hipSuccess ||
            (e = d_items.reserve((uint64_t)n * sizeof(cz_v2_item))) != hipSuccess ||
            (e = d_desc.reserve((uint64_t)n * sizeof(cz_frame_desc))) != hipSuccess ||
            (e = d_seg.reserve(std::max<uint64_t>(nseg, 1) * sizeof(cz_segment))) != hipSuccess ||
            (e = d_comb.reserve(std::max<uint64_t>(ncomb, 1) * sizeof(cz_combine))) != hipSuccess ||
            (e = d_work.reserve(std::max<uint64_t>(npart, 1) * 64)) != hipSuccess ||
            (e = h_wire.reserve(wire_total)) != hipSuccess || (e = h_meta.reserve(m_end)) != hipSuccess)
            return hip_fail(e, "cz_engine: alloc");
        // descriptors and items are built straight into pinned staging (pageable sources would
        // make each H2D synchronous), one group at a time while the copies issued before run
        uint8_t *hm = (uint8_t *)h_meta.ptr;
        cz_v2_item *h_items = (cz_v2_item *)(hm + m_items);
        cz_frame_desc *h_desc = (cz_frame_desc *)(hm + m_desc);
        pt.mark("plan");
        std::vector<hipEvent_t> ev(groups.size(), nullptr), evk(groups.size(), nullptr);
        EvGuard evguard{ev}, evkguard{evk};
        for (size_t gi = 0; gi < groups.size(); gi++)
            if ((e = hipEventCreateWithFlags(&ev[gi], hipEventDisableTiming)) != hipSuccess ||
                (e = hipEventCreateWithFlags(&evk[gi], hipEventDisableTiming)) != hipSuccess)
                return hip_fail(e, "hipEventCreate");
        // one group: no overlap to gain, so one stream and no cross-stream events (each costs
        // tens of us, the bulk of a small flush's latency)
        hipStream_t qh = ps[0], qk = ps[1], qo = ps[2];
        if (groups.size() == 1)
            qh = qo = qk;
        uint64_t copied = 0;
        // the arena bytes not copied yet up to group g's last payload
        auto copy_arena = [&](size_t gi) -> hipError_t {
            if (gi >= groups.size() || groups[gi].arena_hi <= copied)
                return hipSuccess;
            hipError_t r = hipMemcpyAsync((uint8_t *)d_in.ptr + copied, (const uint8_t *)arena.ptr + copied,
                                          groups[gi].arena_hi - copied, hipMemcpyHostToDevice, qh);
            copied = groups[gi].arena_hi;
            return r;
        };
        if ((e = copy_arena(0)) != hipSuccess)
            return hip_fail(e, "cz_engine: H2D");
        Segs sg;
        for (size_t gi = 0; gi < groups.size(); gi++) {
            const Group &g = groups[gi];
            const uint32_t gn = g.fb - g.fa;
            uint64_t bs = g.slot0;
            for (uint32_t i = g.fa; i < g.fb; i++) {
                const OutMsg &m = pend[i];
                Conn &c = conns[m.conn];
                const uint64_t body = (uint64_t)m.len + CZ_MESSAGE_OVERHEAD;
                h_desc[i] = {m.arena_off, bs, m.len, c.tx_key, c.nonce++, m.flags & 0xffu, -1};
                h_items[i] = {bs, wpos[i], (uint32_t)body, (uint32_t)CZ_V2_ITEM_HEADER};
                bs += round_up(body, SLOT_ALIGN);
            }
            plan_segments(h_desc + g.fa, gn, 0, seg, sg.seg, sg.comb, sg.npart);
            const uint32_t gseg = (uint32_t)sg.seg.size(), gcomb = (uint32_t)sg.comb.size();
            if (gseg != soff[gi + 1] - soff[gi] || gcomb != coff[gi + 1] - coff[gi] || sg.npart != woff[gi + 1] - woff[gi])
                return fail(CZ_EINVAL, "cz_engine: segment plan disagrees with its count");
            memcpy(hm + m_seg + soff[gi] * sizeof(cz_segment), sg.seg.data(), (uint64_t)gseg * sizeof(cz_segment));
            memcpy(hm + m_comb + coff[gi] * sizeof(cz_combine), sg.comb.data(), (uint64_t)gcomb * sizeof(cz_combine));
            cz_frame_desc *dd = (cz_frame_desc *)d_desc.ptr + g.fa;
            cz_segment *dsg = (cz_segment *)d_seg.ptr + soff[gi];
            cz_combine *dcb = (cz_combine *)d_comb.ptr + coff[gi];
            // (a) copy stream: the group's metadata, then the next group's arena bytes (copied while
            //     the host builds that group)
            if ((e = hipMemcpyAsync((cz_v2_item *)d_items.ptr + g.fa, h_items + g.fa, (uint64_t)gn * sizeof(cz_v2_item),
                                    hipMemcpyHostToDevice, qh)) != hipSuccess ||
                (e = hipMemcpyAsync(dd, h_desc + g.fa, (uint64_t)gn * sizeof(cz_frame_desc), hipMemcpyHostToDevice,
                                    qh)) != hipSuccess ||
                (gseg && (e = hipMemcpyAsync(dsg, (const cz_segment *)(hm + m_seg) + soff[gi],
                                             (uint64_t)gseg * sizeof(cz_segment), hipMemcpyHostToDevice, qh)) !=
                             hipSuccess) ||
                (gcomb && (e = hipMemcpyAsync(dcb, (const cz_combine *)(hm + m_comb) + coff[gi],
                                              (uint64_t)gcomb * sizeof(cz_combine), hipMemcpyHostToDevice, qh)) !=
                              hipSuccess) ||
                (qh != qk && (e = hipEventRecord(ev[gi], qh)) != hipSuccess) ||
                (e = copy_arena(gi + 1)) != hipSuccess)
                return hip_fail(e, "cz_engine: flush_out H2D");
            // (b) compute stream: seal into body slots, pack behind V2 headers at the send-order
            //     wire positions; (c) D2H stream: the group's wire bytes back
            if ((qh != qk && (e = hipStreamWaitEvent(qk, ev[gi], 0)) != hipSuccess) ||
                (e = czk_seal_segments(dd, dsg, gseg, dcb, gcomb, d_in.ptr, d_body.ptr, subkeys.ptr,
                                       (uint8_t *)d_work.ptr + 64 * woff[gi], qk)) != hipSuccess ||
                (e = czk_v2_copy((const cz_v2_item *)d_items.ptr + g.fa, gn, d_body.ptr, d_wire.ptr, qk)) !=
                    hipSuccess ||
                (qo != qk && ((e = hipEventRecord(evk[gi], qk)) != hipSuccess ||
                              (e = hipStreamWaitEvent(qo, evk[gi], 0)) != hipSuccess)) ||
                (e = hipMemcpyAsync((uint8_t *)h_wire.ptr + wpos[g.fa], (uint8_t *)d_wire.ptr + wpos[g.fa],
                                    wpos[g.fb] - wpos[g.fa], hipMemcpyDeviceToHost, qo)) != hipSuccess)
                return hip_fail(e, "cz_engine: flush_out");
        }
        for (hipStream_t q : ps)
            if ((e = hipStreamSynchronize(q)) != hipSuccess)
                return hip_fail(e, "cz_engine: flush_out");
        pt.mark("h2d+kernels+d2h");
        pend.clear();
        arena_used = 0;
        return CZ_OK;
    }

    static int event_for(uint32_t status, bool server)
    {
        switch (status) {
        case CZ_STATUS_COMMAND: return CZ_ZMTP_UNEXPECTED_COMMAND;
        case CZ_STATUS_MALFORMED: return CZ_ZMTP_MALFORMED_COMMAND_MESSAGE;
        case CZ_STATUS_SEQUENCE: return server ? CZ_ZMTP_INVALID_SEQUENCE : CZ_ZMTP_CRYPTOGRAPHIC;
        default: return CZ_ZMTP_CRYPTOGRAPHIC;
        }
    }

    int flush_in()
    {
        PhaseTimer pt("flush_in");
        in_msgs.clear();
        for (Conn &c : conns)
            c.in_msgs.clear();
        // 0. the live connections, in groups of ~equal received bytes
        struct Parsed {
            uint32_t conn;
            uint32_t first, count;  // range in frames
            uint64_t rx_off;        // where the connection's received bytes start in d_wire
            uint64_t consumed;      // whole frames
            int perr;               // framing error after the parsed frames
        };
        std::vector<Parsed> parsed;
        uint64_t rx_total = 0;
        for (size_t ci = 0; ci < conns.size(); ci++) {
            Conn &c = conns[ci];
            if (c.error || c.rx_len == 0)
                continue;
            parsed.push_back({(uint32_t)ci, 0u, 0u, 0u, 0u, 0});
            rx_total += c.rx_len;
        }
        const uint32_t seg = flush_seg_blocks(rx_total / 64);
        struct Group {
            size_t pa, pb;        // parsed[pa, pb)
            uint32_t fa, fb;      // frames[fa, fb)
            uint64_t pl0, pl1;    // plaintext slot range
        };
        std::vector<Group> groups;
        {
            const int G = rx_total >= (64ull << 20) ? CZ_ENGINE_GROUPS : 1;
            size_t pa = 0;
            uint64_t acc = 0;
            for (size_t q = 0; q < parsed.size(); q++) {
                acc += conns[parsed[q].conn].rx_len;
                if (q + 1 == parsed.size() || acc * G >= rx_total * (groups.size() + 1)) {
                    groups.push_back({pa, q + 1, 0, 0, 0, 0});
                    pa = q + 1;
                }
            }
        }
        hipError_t e;
        std::vector<hipEvent_t> evm(groups.size(), nullptr), evk(groups.size(), nullptr);
        EvGuard evmguard{evm}, evkguard{evk};
        for (size_t gi = 0; gi < groups.size(); gi++)
            if ((e = hipEventCreateWithFlags(&evm[gi], hipEventDisableTiming)) != hipSuccess ||
                (e = hipEventCreateWithFlags(&evk[gi], hipEventDisableTiming)) != hipSuccess)
                return hip_fail(e, "hipEventCreate");
        // ps[0]: received bytes H2D straight from the pinned receive blocks, one DMA per run of
        // connections that lie next to each other there (RxPool), every group issued before any
        // parsing so the copies run while the host parses and plans; `stream`: metadata H2D;
        // ps[1]: unpack + open; ps[2]: D2H.  (A gather kernel reading the receive buffers over PCIe
        // instead of DMAs measured slower, and so did spreading the DMAs over two streams, gathering
        // each group into one pinned slab on 8 host threads (the memcpy is slower than the gaps it
        // removes) and hipMemcpyBatchAsync of the per-connection copies (the same gaps).)
        hipStream_t qh = ps[0], qk = ps[1], qo = ps[2], qm = stream;
        if (groups.size() <= 1)  // as flush_out: one group, one stream
            qh = qo = qm = qk;
        std::vector<hipEvent_t> ev(groups.size(), nullptr);
        EvGuard evguard{ev};
        for (size_t gi = 0; gi < groups.size(); gi++)
            if ((e = hipEventCreateWithFlags(&ev[gi], hipEventDisableTiming)) != hipSuccess)
                return hip_fail(e, "hipEventCreate");
        // spans: a group's connections in address order, merged while they share a receive block
        // and the bytes between them (other connections' spare capacity) are at most MERGE_GAP --
        // copying those costs less than another DMA's gap
        struct Span {
            const uint8_t *src;
            uint64_t dev, len;
        };
        std::vector<Span> spans;
        std::vector<size_t> span_end(groups.size());
        {
            constexpr uint64_t MERGE_GAP = 1ull << 20;
            uint64_t off = 0;
            std::vector<size_t> order;
            for (size_t gi = 0; gi < groups.size(); gi++) {
                order.clear();
                for (size_t pi = groups[gi].pa; pi < groups[gi].pb; pi++)
                    order.push_back(pi);
                std::sort(order.begin(), order.end(),
                          [&](size_t x, size_t y) { return conns[parsed[x].conn].rx.ptr < conns[parsed[y].conn].rx.ptr; });
                uint32_t blk = 0;
                for (size_t pi : order) {
                    Parsed &p = parsed[pi];
                    const Conn &c = conns[p.conn];
                    Span *last = spans.size() > (gi ? span_end[gi - 1] : 0) ? &spans.back() : nullptr;
                    if (last && c.rx.blk == blk && c.rx.ptr <= last->src + last->len + MERGE_GAP) {
                        p.rx_off = last->dev + (uint64_t)(c.rx.ptr - last->src);
                        const uint64_t end = (uint64_t)(c.rx.ptr + c.rx_len - last->src);
                        off += end - last->len;
                        last->len = end;
                    } else {
                        p.rx_off = off;
                        spans.push_back({c.rx.ptr, off, c.rx_len});
                        off += c.rx_len;
                        blk = c.rx.blk;
                    }
                }
                span_end[gi] = spans.size();
            }
            if (off && (e = d_wire.reserve(off)) != hipSuccess)
                return hip_fail(e, "cz_engine: alloc");
        }
        for (size_t gi = 0, si = 0; gi < groups.size(); gi++) {
            for (; si < span_end[gi]; si++)
                if ((e = hipMemcpyAsync((uint8_t *)d_wire.ptr + spans[si].dev, spans[si].src, spans[si].len,
                                        hipMemcpyHostToDevice, qh)) != hipSuccess)
                    return hip_fail(e, "cz_engine: H2D");
            if (qh != qk && (e = hipEventRecord(ev[gi], qh)) != hipSuccess)
                return hip_fail(e, "cz_engine: H2D");
        }
        pt.mark("h2d-issue");
        // 1. per group, on its own host thread: parse each connection's whole frames (V2Decoder; a
        //    partial frame waits for more bytes) and count the group's frames, body / plaintext slot
        //    bytes and segments (plan_counts) -- enough to place every group's arrays.
        struct GroupWork {
            std::vector<cz_v2_frame> frames;
            Segs sg;
            uint64_t bslot = 0, pslot = 0;   // slot bytes of the group
            uint64_t nseg = 0, ncomb = 0, npart = 0;
            uint64_t b0 = 0, soff = 0, coff = 0, woff = 0;  // where its arrays start
            bool bad_plan = false;
        };
        std::vector<GroupWork> gw(groups.size());
        auto parse = [&](size_t gi) {
            GroupWork &w = gw[gi];
            const Group &g = groups[gi];
            constexpr uint32_t CH = 4096;  // parse in chunks of CH frames
            for (size_t q = g.pa; q < g.pb; q++) {
                Parsed &p = parsed[q];
                const Conn &c = conns[p.conn];
                const size_t base = w.frames.size();
                uint64_t consumed = 0;
                int prc = CZ_OK;
                for (;;) {
                    const size_t at = w.frames.size();
                    w.frames.resize(at + CH);
                    uint32_t nf = 0;
                    uint64_t used = 0;
                    prc = cz_v2_parse((const uint8_t *)c.rx.ptr + consumed, c.rx_len - consumed, -1,
                                      w.frames.data() + at, CH, &nf, &used);
                    w.frames.resize(at + nf);
                    for (uint32_t k = 0; k < nf; k++)
                        w.frames[at + k].body_off += consumed;
                    consumed += used;
                    if (prc != CZ_OK || nf < CH)
                        break;
                }
                p.first = (uint32_t)base;  // group-relative until step 2
                p.count = (uint32_t)(w.frames.size() - base);
                p.consumed = consumed;
                p.perr = prc == CZ_OK ? 0 : prc;
            }
            for (const cz_v2_frame &f : w.frames) {
                const uint64_t plen = f.size > CZ_MESSAGE_OVERHEAD ? f.size - CZ_MESSAGE_OVERHEAD : 0;
                w.bslot += round_up(std::max<uint64_t>(f.size, 1), SLOT_ALIGN);
                w.pslot += round_up(std::max<uint64_t>(plen, 1), SLOT_ALIGN);
                plan_counts(f.size, 1, seg, w.nseg, w.ncomb, w.npart);
            }
        };
        {
            std::vector<std::thread> th;
            for (size_t gi = 1; gi < groups.size(); gi++)
                th.emplace_back(parse, gi);
            if (!groups.empty())
                parse(0);
            for (std::thread &t : th)
                t.join();
        }
        pt.mark("parse");
        // 2. place the groups: absolute frame indices, slot offsets, segment-list offsets; size
        //    every buffer once
        uint32_t n = 0;
        uint64_t bslot = 0, pslot = 0, nseg = 0, ncomb = 0, npart = 0;
        for (size_t gi = 0; gi < groups.size(); gi++) {
            Group &g = groups[gi];
            GroupWork &w = gw[gi];
            g.fa = n;
            for (size_t q = g.pa; q < g.pb; q++)
                parsed[q].first += n;
            n += (uint32_t)w.frames.size();
            g.fb = n;
            g.pl0 = pslot;
            w.b0 = bslot;
            w.soff = nseg;
            w.coff = ncomb;
            w.woff = npart;
            bslot += w.bslot;
            pslot += w.pslot;
            nseg += w.nseg;
            ncomb += w.ncomb;
            npart += w.npart;
            g.pl1 = pslot;
        }
        const uint64_t m_items = 0, m_desc = (uint64_t)n * sizeof(cz_v2_item),
                       m_seg = m_desc + (uint64_t)n * sizeof(cz_frame_desc),
                       m_comb = m_seg + nseg * sizeof(cz_segment), m_end = m_comb + ncomb * sizeof(cz_combine);
        // (a device buffer that has to grow is reallocated here, which waits for the copies in
        //  flight; steady-state flushes reuse their buffers)
        if (n && ((e = d_in.reserve(bslot)) != hipSuccess || (e = d_plain.reserve(pslot)) != hipSuccess ||
                  (e = d_items.reserve((uint64_t)n * sizeof(cz_v2_item))) != hipSuccess ||
                  (e = d_status.reserve((uint64_t)n * 2)) != hipSuccess ||
                  (e = d_nonces.reserve((uint64_t)n * 8)) != hipSuccess ||
                  (e = d_desc.reserve((uint64_t)n * sizeof(cz_frame_desc))) != hipSuccess ||
                  (e = d_seg.reserve(std::max<uint64_t>(nseg, 1) * sizeof(cz_segment))) != hipSuccess ||
                  (e = d_comb.reserve(std::max<uint64_t>(ncomb, 1) * sizeof(cz_combine))) != hipSuccess ||
                  (e = d_work.reserve(std::max<uint64_t>(npart, 1) * 64)) != hipSuccess ||
                  (e = h_plain.reserve(pslot)) != hipSuccess || (e = h_status.reserve((uint64_t)n * 2)) != hipSuccess ||
                  (e = h_nonces.reserve((uint64_t)n * 8)) != hipSuccess || (e = h_meta.reserve(m_end)) != hipSuccess))
            return hip_fail(e, "cz_engine: alloc");
        // the host-built arrays go straight into pinned staging (pageable sources would make each
        // H2D synchronous); descriptors stay there for the delivery step
        uint8_t *hm = (uint8_t *)h_meta.ptr;
        cz_v2_item *h_items = (cz_v2_item *)(hm + m_items);
        cz_frame_desc *h_desc = (cz_frame_desc *)(hm + m_desc);
        cz_segment *h_seg = (cz_segment *)(hm + m_seg);
        cz_combine *h_comb = (cz_combine *)(hm + m_comb);
        pt.mark("place");
        // 3. per group, on its own host thread: descriptors -- bodies unpacked into aligned slots,
        //    each connection's frames chained by prev (group-relative indices, as the kernels get
        //    the group's descriptor array) -- and the segment plan.  This thread issues group g's
        //    metadata H2D, kernels and D2H as soon as its worker is done, while later groups are
        //    still being built.
        auto build = [&](size_t gi) {
            GroupWork &w = gw[gi];
            const Group &g = groups[gi];
            cz_v2_item *items = h_items + g.fa;
            cz_frame_desc *desc = h_desc + g.fa;
            uint64_t bs = w.b0, ps = g.pl0;
            for (size_t q = g.pa; q < g.pb; q++) {
                const Parsed &p = parsed[q];
                const Conn &c = conns[p.conn];
                for (uint32_t k = 0; k < p.count; k++) {
                    const uint32_t i = p.first - g.fa + k;
                    const cz_v2_frame &f = w.frames[i];
                    const uint64_t plen = f.size > CZ_MESSAGE_OVERHEAD ? f.size - CZ_MESSAGE_OVERHEAD : 0;
                    items[i] = {p.rx_off + f.body_off, bs, f.size, 0u};
                    desc[i] = {bs, ps, f.size, c.rx_key, c.peer_nonce, CZ_DESC_CHECK_NONCE, k ? (int32_t)(i - 1) : -1};
                    bs += round_up(std::max<uint64_t>(f.size, 1), SLOT_ALIGN);
                    ps += round_up(std::max<uint64_t>(plen, 1), SLOT_ALIGN);
                }
            }
            const uint32_t gn = g.fb - g.fa;
            plan_segments(desc, gn, 1, seg, w.sg.seg, w.sg.comb, w.sg.npart);
            w.sg.nseg = (uint32_t)w.sg.seg.size();
            w.sg.ncomb = (uint32_t)w.sg.comb.size();
            if (w.sg.nseg != w.nseg || w.sg.ncomb != w.ncomb || w.sg.npart != w.npart) {
                w.bad_plan = true;
                return;
            }
            memcpy(h_seg + w.soff, w.sg.seg.data(), (uint64_t)w.sg.nseg * sizeof(cz_segment));
            memcpy(h_comb + w.coff, w.sg.comb.data(), (uint64_t)w.sg.ncomb * sizeof(cz_combine));
        };
        auto issue = [&](size_t gi) -> hipError_t {
            const Group &g = groups[gi];
            const GroupWork &w = gw[gi];
            const uint32_t gn = g.fb - g.fa;
            if (gn == 0)
                return hipSuccess;
            cz_frame_desc *dd = (cz_frame_desc *)d_desc.ptr + g.fa;
            cz_segment *dsg = (cz_segment *)d_seg.ptr + w.soff;
            cz_combine *dcb = (cz_combine *)d_comb.ptr + w.coff;
            hipError_t r;
            // (a) metadata stream: the group's descriptors / items / segment lists
            if ((r = hipMemcpyAsync((cz_v2_item *)d_items.ptr + g.fa, h_items + g.fa, (uint64_t)gn * sizeof(cz_v2_item),
                                    hipMemcpyHostToDevice, qm)) != hipSuccess ||
                (r = hipMemcpyAsync(dd, h_desc + g.fa, (uint64_t)gn * sizeof(cz_frame_desc), hipMemcpyHostToDevice,
                                    qm)) != hipSuccess ||
                (w.sg.nseg && (r = hipMemcpyAsync(dsg, h_seg + w.soff, (uint64_t)w.sg.nseg * sizeof(cz_segment),
                                                  hipMemcpyHostToDevice, qm)) != hipSuccess) ||
                (w.sg.ncomb && (r = hipMemcpyAsync(dcb, h_comb + w.coff, (uint64_t)w.sg.ncomb * sizeof(cz_combine),
                                                   hipMemcpyHostToDevice, qm)) != hipSuccess) ||
                (qm != qk && (r = hipEventRecord(evm[gi], qm)) != hipSuccess))
                return r;
            // (b) compute stream: once the group's bytes and metadata landed, unpack + open;
            // (c) D2H stream
            if ((qh != qk && (r = hipStreamWaitEvent(qk, ev[gi], 0)) != hipSuccess) ||
                (qm != qk && (r = hipStreamWaitEvent(qk, evm[gi], 0)) != hipSuccess) ||
                (r = czk_v2_copy((const cz_v2_item *)d_items.ptr + g.fa, gn, d_wire.ptr, d_in.ptr, qk)) != hipSuccess ||
                (r = czk_open_segments(dd, dsg, w.sg.nseg, dcb, w.sg.ncomb, d_in.ptr, d_plain.ptr, subkeys.ptr,
                                       (uint8_t *)d_work.ptr + 64 * w.woff, (uint16_t *)d_status.ptr + g.fa,
                                       (uint64_t *)d_nonces.ptr + g.fa, qk)) != hipSuccess ||
                (qo != qk && ((r = hipEventRecord(evk[gi], qk)) != hipSuccess ||
                              (r = hipStreamWaitEvent(qo, evk[gi], 0)) != hipSuccess)) ||
                (r = hipMemcpyAsync((uint8_t *)h_plain.ptr + g.pl0, (uint8_t *)d_plain.ptr + g.pl0, g.pl1 - g.pl0,
                                    hipMemcpyDeviceToHost, qo)) != hipSuccess ||
                (r = hipMemcpyAsync((uint16_t *)h_status.ptr + g.fa, (uint16_t *)d_status.ptr + g.fa, (uint64_t)gn * 2,
                                    hipMemcpyDeviceToHost, qo)) != hipSuccess ||
                (r = hipMemcpyAsync((uint64_t *)h_nonces.ptr + g.fa, (uint64_t *)d_nonces.ptr + g.fa, (uint64_t)gn * 8,
                                    hipMemcpyDeviceToHost, qo)) != hipSuccess)
                return r;
            return hipSuccess;
        };
        if (n) {
            std::vector<std::thread> th;
            for (size_t gi = 1; gi < groups.size(); gi++)
                th.emplace_back(build, gi);
            build(0);
            e = hipSuccess;
            bool bad = false;
            for (size_t gi = 0; gi < groups.size(); gi++) {
                if (gi)
                    th[gi - 1].join();
                bad = bad || gw[gi].bad_plan;
                if (!bad && e == hipSuccess)
                    e = issue(gi);  // after a failure: join the rest, issue nothing more
            }
            if (bad)
                return fail(CZ_EINVAL, "cz_engine: internal error, segment plan differs from its count");
            if (e != hipSuccess)
                return hip_fail(e, "cz_engine: flush_in");
        }
        const hipStream_t used[4] = {qh, qk, qo, qm};
        for (int i = 0; i < 4; i++)
            if (std::find(used, used + i, used[i]) == used + i && (e = hipStreamSynchronize(used[i])) != hipSuccess)
                return hip_fail(e, "cz_engine: flush_in");
        pt.mark("h2d+kernels+d2h");
        // 3. deliver in order per connection, up to the first failure (decodeAndPush returns false)
        const uint16_t *st = (const uint16_t *)h_status.ptr;
        const uint64_t *nn = (const uint64_t *)h_nonces.ptr;
        for (const Parsed &p : parsed) {
            Conn &c = conns[p.conn];
            bool failed = false;
            for (uint32_t k = 0; k < p.count; k++) {
                const uint32_t i = p.first + k;
                const uint32_t status = st[i] & 0xffu;
                if (status != CZ_STATUS_OK) {
                    if (status == CZ_STATUS_CRYPTO)  // the nonce passed the replay check: cnPeerNonce = nonce
                        c.peer_nonce = nn[i];        // precedes openAfternm (CurveClientMechanism.java:193)
                    c.error = CZ_EPROTO;
                    c.event = event_for(status, c.server);
                    failed = true;
                    break;
                }
                c.peer_nonce = nn[i];
                const uint32_t fl = st[i] >> 8;
                int mf = 0;
                if (fl & 0x01)
                    mf |= CZ_MSG_MORE;
                if (fl & 0x02)
                    mf |= CZ_MSG_COMMAND;
                c.in_msgs.push_back((uint32_t)in_msgs.size());
                in_msgs.push_back({h_desc[i].out_off, h_desc[i].len - CZ_MESSAGE_OVERHEAD, mf});
            }
            if (failed) {
                c.rx_len = 0;
                continue;
            }
            // keep the partial frame for the next read
            if (p.consumed) {
                memmove(c.rx.ptr, (uint8_t *)c.rx.ptr + p.consumed, c.rx_len - p.consumed);
                c.rx_len -= p.consumed;
            }
            if (p.perr) {  // V2Decoder error after the good frames: StreamEngine error(PROTOCOL)
                c.error = p.perr;
                c.event = 0;
                c.rx_len = 0;
            }
        }
        pt.mark("deliver");
        return CZ_OK;
    }
};

extern "C" {

int cz_engine_create(cz_engine **out, uint64_t arena_bytes, int device)
{
    if (!out)
        return fail(CZ_EINVAL, "cz_engine_create: null pointer");
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0)
        return fail(CZ_EHIP, "no HIP device available (the CURVE path runs only on the GPU)");
    cz_engine *e = new cz_engine();
    e->device = device;
    hipError_t he;
    if ((he = hipSetDevice(device)) != hipSuccess ||
        (he = hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking)) != hipSuccess ||
        (he = hipStreamCreateWithFlags(&e->ps[0], hipStreamNonBlocking)) != hipSuccess ||
        (he = hipStreamCreateWithFlags(&e->ps[1], hipStreamNonBlocking)) != hipSuccess ||
        (he = hipStreamCreateWithFlags(&e->ps[2], hipStreamNonBlocking)) != hipSuccess ||
        (he = e->arena.reserve(std::max<uint64_t>(arena_bytes, 4096))) != hipSuccess) {
        delete e;
        return hip_fail(he, "cz_engine_create");
    }
    e->arena_cap = e->arena.cap;
    *out = e;
    return CZ_OK;
}

void cz_engine_destroy(cz_engine *e) { delete e; }

int cz_engine_add_conn(cz_engine *e, int as_server, const uint8_t precom[32], uint64_t cn_nonce,
                       uint64_t cn_peer_nonce)
{
    if (!e || !precom)
        return fail(CZ_EINVAL, "cz_engine_add_conn: null pointer");
    hipError_t he;
    // a removed connection's id and subkey slots first, else two new table slots
    const bool reuse = !e->free_ids.empty();
    if ((he = hipSetDevice(e->device)) != hipSuccess || (!reuse && (he = e->grow_keys(e->nkeys + 2)) != hipSuccess))
        return hip_fail(he, "cz_engine_add_conn");
    void *dk = nullptr;
    if ((he = hipMalloc(&dk, 32)) != hipSuccess)
        return hip_fail(he, "hipMalloc");
    Conn c;
    c.server = as_server != 0;
    c.tx_key = reuse ? e->conns[(size_t)e->free_ids.back()].tx_key : e->nkeys;
    c.rx_key = reuse ? e->conns[(size_t)e->free_ids.back()].rx_key : e->nkeys + 1;
    c.nonce = cn_nonce;
    c.peer_nonce = cn_peer_nonce;
    uint8_t *table = (uint8_t *)e->subkeys.ptr;
    const int tx = c.server ? CZ_DIR_S2C : CZ_DIR_C2S;
    const int rx = c.server ? CZ_DIR_C2S : CZ_DIR_S2C;
    if ((he = hipMemcpyAsync(dk, precom, 32, hipMemcpyHostToDevice, e->stream)) != hipSuccess ||
        (he = czk_subkeys(dk, table + 32ull * c.tx_key, 1, prefix_for(tx), e->stream)) != hipSuccess ||
        (he = czk_subkeys(dk, table + 32ull * c.rx_key, 1, prefix_for(rx), e->stream)) != hipSuccess ||
        (he = hipMemsetAsync(dk, 0, 32, e->stream)) != hipSuccess || (he = hipStreamSynchronize(e->stream)) != hipSuccess) {
        (void)hipFree(dk);
        return hip_fail(he, "cz_engine_add_conn: subkeys");
    }
    (void)hipFree(dk);
    if (reuse) {
        const int id = e->free_ids.back();
        e->free_ids.pop_back();
        e->conns[(size_t)id] = std::move(c);
        return id;
    }
    e->nkeys += 2;
    e->conns.push_back(std::move(c));
    return (int)e->conns.size() - 1;
}

// StreamEngine teardown (unplug / error, StreamEngine.java:334-370,1116-1131) of an attached
// connection: its queued messages leave the next flush, its received bytes and the payloads of the
// last flush_in are dropped, its subkeys are wiped on the device, and its id and key slots are
// reused by the next cz_engine_add_conn -- a long-lived IO thread with connection churn keeps a
// bounded engine.
int cz_engine_remove_conn(cz_engine *e, int conn)
{
    if (!e)
        return fail(CZ_EINVAL, "cz_engine_remove_conn: null pointer");
    Conn *c = e->conn(conn);
    if (!c)
        return CZ_EINVAL;
    hipError_t he;
    uint8_t *table = (uint8_t *)e->subkeys.ptr;
    if ((he = hipSetDevice(e->device)) != hipSuccess ||
        (he = hipMemsetAsync(table + 32ull * c->tx_key, 0, 32, e->stream)) != hipSuccess ||
        (he = hipMemsetAsync(table + 32ull * c->rx_key, 0, 32, e->stream)) != hipSuccess ||
        (he = hipStreamSynchronize(e->stream)) != hipSuccess)
        return hip_fail(he, "cz_engine_remove_conn");
    e->pend.erase(std::remove_if(e->pend.begin(), e->pend.end(), [conn](const OutMsg &m) { return (int)m.conn == conn; }),
                  e->pend.end());
    if (c->rx.ptr) {
        explicit_bzero(c->rx.ptr, c->rx_len);
        e->rxpool.free_list.push_back(c->rx);
    }
    Conn dead;
    dead.tx_key = c->tx_key;
    dead.rx_key = c->rx_key;
    dead.removed = true;
    *c = std::move(dead);
    e->free_ids.push_back(conn);
    return CZ_OK;
}

void *cz_engine_msg_alloc(cz_engine *e, uint32_t len)
{
    if (!e)
        return nullptr;
    const uint64_t off = round_up(e->arena_used, 16);
    if (off + len > e->arena_cap)
        return nullptr;
    e->arena_used = off + len;
    return (uint8_t *)e->arena.ptr + off;
}

int cz_engine_send(cz_engine *e, int conn, const void *payload, uint32_t len, int msg_flags)
{
    if (!e || (len && !payload))
        return fail(CZ_EINVAL, "cz_engine_send: null pointer");
    Conn *c = e->conn(conn);
    if (!c)
        return CZ_EINVAL;
    if (c->error)
        return fail(c->error, "cz_engine_send: connection %d has failed", conn);
    if (len > (uint32_t)CZ_MESSAGE_MAX)
        return fail(CZ_EMSGSIZE, "cz_engine_send: %u-byte payload exceeds CZ_MESSAGE_MAX", len);
    const uint8_t *base = (const uint8_t *)e->arena.ptr;
    const uint8_t *p = (const uint8_t *)payload;
    uint64_t off;
    if (len && p >= base && p + len <= base + e->arena_used) {
        off = (uint64_t)(p - base);  // allocated by cz_engine_msg_alloc: no copy
    } else {
        uint8_t *dst = (uint8_t *)cz_engine_msg_alloc(e, len);
        if (!dst)
            return fail(CZ_ENOMEM, "cz_engine_send: arena full (%llu bytes), flush first",
                        (unsigned long long)e->arena_cap);
        if (len)
            memcpy(dst, p, len);
        off = (uint64_t)(dst - base);
    }
    uint32_t fl = 0;
    if (msg_flags & CZ_MSG_MORE)
        fl |= 0x01;
    if (msg_flags & CZ_MSG_COMMAND)
        fl |= 0x02;
    e->pend.push_back({(uint32_t)conn, off, len, fl});
    return CZ_OK;
}

int cz_engine_flush_out(cz_engine *e)
{
    if (!e)
        return fail(CZ_EINVAL, "cz_engine_flush_out: null engine");
    hipError_t he = hipSetDevice(e->device);
    if (he != hipSuccess)
        return hip_fail(he, "hipSetDevice");
    const int rc = e->flush_out();
    if (rc != CZ_OK)
        e->drain();  // an error return may leave copies into/out of the pinned buffers in flight
    return rc;
}

int cz_engine_wire_out(cz_engine *e, int conn, const uint8_t **wire, uint64_t *len)
{
    if (!e || !wire || !len)
        return fail(CZ_EINVAL, "cz_engine_wire_out: null pointer");
    Conn *c = e->conn(conn);
    if (!c)
        return CZ_EINVAL;
    const uint8_t *base = (const uint8_t *)e->h_wire.ptr;
    if (c->runs.size() <= 1) {  // frames queued together: the stream lies in the flush output as is
        *wire = c->runs.empty() ? base : base + c->runs[0].off;
        *len = c->runs.empty() ? 0 : c->runs[0].len;
        return CZ_OK;
    }
    if (c->gathered.empty()) {  // interleaved with other connections: one host gather
        uint64_t t = 0;
        for (const Run &r : c->runs)
            t += r.len;
        c->gathered.resize(t);
        t = 0;
        for (const Run &r : c->runs) {
            memcpy(c->gathered.data() + t, base + r.off, r.len);
            t += r.len;
        }
    }
    *wire = c->gathered.data();
    *len = c->gathered.size();
    return CZ_OK;
}

int cz_engine_wire_iov(cz_engine *e, int conn, cz_iovec *iov, uint32_t cap, uint32_t *count)
{
    if (!e || !count || (cap && !iov))
        return fail(CZ_EINVAL, "cz_engine_wire_iov: null pointer");
    Conn *c = e->conn(conn);
    if (!c)
        return CZ_EINVAL;
    *count = (uint32_t)c->runs.size();
    if (cap < c->runs.size())
        return cap ? fail(CZ_EINVAL, "cz_engine_wire_iov: %u pieces, capacity %u", *count, cap) : CZ_OK;
    const uint8_t *base = (const uint8_t *)e->h_wire.ptr;
    for (size_t k = 0; k < c->runs.size(); k++)
        iov[k] = {base + c->runs[k].off, c->runs[k].len};
    return CZ_OK;
}

int cz_engine_recv(cz_engine *e, int conn, const void *wire, uint64_t len)
{
    if (!e || (len && !wire))
        return fail(CZ_EINVAL, "cz_engine_recv: null pointer");
    Conn *c = e->conn(conn);
    if (!c)
        return CZ_EINVAL;
    if (c->error)
        return fail(c->error, "cz_engine_recv: connection %d has failed", conn);
    hipError_t he = e->rxpool.grow(c->rx, c->rx_len, c->rx_len + len);
    if (he != hipSuccess)
        return hip_fail(he, "cz_engine_recv: hipHostMalloc");
    if (len)
        memcpy((uint8_t *)c->rx.ptr + c->rx_len, wire, len);
    c->rx_len += len;
    return CZ_OK;
}

int cz_engine_recv_buffer(cz_engine *e, int conn, uint64_t min_bytes, uint8_t **buf, uint64_t *avail)
{
    if (!e || !buf || !avail)
        return fail(CZ_EINVAL, "cz_engine_recv_buffer: null pointer");
    Conn *c = e->conn(conn);
    if (!c)
        return CZ_EINVAL;
    if (c->error)
        return fail(c->error, "cz_engine_recv_buffer: connection %d has failed", conn);
    hipError_t he = e->rxpool.grow(c->rx, c->rx_len, c->rx_len + std::max<uint64_t>(min_bytes, 1));
    if (he != hipSuccess)
        return hip_fail(he, "cz_engine_recv_buffer: hipHostMalloc");
    *buf = (uint8_t *)c->rx.ptr + c->rx_len;
    *avail = c->rx.cap - c->rx_len;
    return CZ_OK;
}

int cz_engine_recv_commit(cz_engine *e, int conn, uint64_t n)
{
    if (!e)
        return fail(CZ_EINVAL, "cz_engine_recv_commit: null engine");
    Conn *c = e->conn(conn);
    if (!c)
        return CZ_EINVAL;
    if (n > c->rx.cap - c->rx_len)
        return fail(CZ_EINVAL, "cz_engine_recv_commit: %llu bytes exceed the buffer", (unsigned long long)n);
    c->rx_len += n;
    return CZ_OK;
}

int cz_engine_flush_in(cz_engine *e)
{
    if (!e)
        return fail(CZ_EINVAL, "cz_engine_flush_in: null engine");
    hipError_t he = hipSetDevice(e->device);
    if (he != hipSuccess)
        return hip_fail(he, "hipSetDevice");
    const int rc = e->flush_in();
    if (rc != CZ_OK)
        e->drain();  // an error return may leave copies into/out of the pinned buffers in flight
    return rc;
}

int cz_engine_msgs_in(cz_engine *e, int conn, uint32_t *count)
{
    if (!e || !count)
        return fail(CZ_EINVAL, "cz_engine_msgs_in: null pointer");
    Conn *c = e->conn(conn);
    if (!c)
        return CZ_EINVAL;
    *count = (uint32_t)c->in_msgs.size();
    return CZ_OK;
}

int cz_engine_msg_in(cz_engine *e, int conn, uint32_t i, const uint8_t **payload, uint32_t *len, int *msg_flags)
{
    if (!e || !payload || !len || !msg_flags)
        return fail(CZ_EINVAL, "cz_engine_msg_in: null pointer");
    Conn *c = e->conn(conn);
    if (!c)
        return CZ_EINVAL;
    if (i >= c->in_msgs.size())
        return fail(CZ_EINVAL, "cz_engine_msg_in: index %u out of range", i);
    const InMsg &m = e->in_msgs[c->in_msgs[i]];
    *payload = (const uint8_t *)e->h_plain.ptr + m.plain_off;
    *len = m.len;
    *msg_flags = m.flags;
    return CZ_OK;
}

int cz_engine_conn_error(cz_engine *e, int conn, int *event)
{
    if (!e)
        return fail(CZ_EINVAL, "cz_engine_conn_error: null engine");
    Conn *c = e->conn(conn);
    if (!c)
        return CZ_EINVAL;
    if (event)
        *event = c->event;
    return c->error;
}

uint64_t cz_engine_nonce(cz_engine *e, int conn)
{
    Conn *c = e ? e->conn(conn) : nullptr;
    return c ? c->nonce : 0;
}

uint64_t cz_engine_peer_nonce(cz_engine *e, int conn)
{
    Conn *c = e ? e->conn(conn) : nullptr;
    return c ? c->peer_nonce : 0;
}

}  // extern "C"
