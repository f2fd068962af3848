/*
 * curvezmq_mi355x.h -- C-ABI of the MI355X CurveZMQ MESSAGE crypto path.
 *
 * This library replaces, for JeroMQ's CURVE sockets, the per-message NaCl calls
 * that JeroMQ makes through the third-party jnacl artefact
 * (eu.neilalexander:jnacl:1.0.0, jeromq-core/pom.xml:18-22; imported at
 * jeromq-core/src/main/java/zmq/io/mechanism/curve/Curve.java:5-6).
 * Every entry point is plain C: pointers, sizes, ints.  Device pointers are
 * HIP device addresses; `stream` is a hipStream_t passed as void* (NULL = the
 * null stream).  All batched launchers are asynchronous, allocate nothing and
 * never synchronise, so they may be captured into a hipGraph.
 *
 * Return conventions
 *   jnacl drop-ins (section 1): 0 on success, -1 on failure -- exactly the
 *   int contract of crypto_box_afternm / crypto_box_open_afternm that
 *   Curve.java:134-147 forwards to callers (encode asserts rc == 0,
 *   CurveClientMechanism.java:153-154; decode maps -1 to EPROTO,
 *   CurveClientMechanism.java:218-223).
 *   Everything else: CZ_OK (0) or a negative CZ_E* code; cz_last_error()
 *   returns a thread-local message.
 *
 * Thread safety: all functions are reentrant.  The single-shot calls use a
 * per-thread device context (JeroMQ runs one connection per IO thread,
 * StreamEngine.java:467-535); cz_ctx objects must not be shared between
 * threads without external locking.
 */
#ifndef CURVEZMQ_MI355X_H
#define CURVEZMQ_MI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Sizes: Curve.Size (Curve.java:14-67) / jnacl crypto_secretbox_* constants */
#define CZ_NONCEBYTES 24
#define CZ_ZEROBYTES 32
#define CZ_BOXZEROBYTES 16
#define CZ_KEYBYTES 32
#define CZ_BEFORENMBYTES 32
#define CZ_MACBYTES 16
/* MESSAGE body = "\x07MESSAGE"(8) + nonce8 + tag16 + flags(1) + payload */
#define CZ_MESSAGE_OVERHEAD 33
/* largest MESSAGE payload: the body (payload + 33) must fit a Java int, as every Msg size does
 * (Msg.java size(): int); encode / encode_batch / cz_engine_send return CZ_EMSGSIZE beyond it */
#define CZ_MESSAGE_MAX (0x7fffffff - CZ_MESSAGE_OVERHEAD)

/* Msg flags carried in the encrypted flags byte (Msg.java:96-100, CurveClientMechanism.java:131-137) */
#define CZ_MSG_MORE 0x01
#define CZ_MSG_COMMAND 0x02

/* direction of a connection-direction subkey (nonce prefix, CurveClientMechanism.java:141, :182) */
#define CZ_DIR_C2S 0 /* "CurveZMQMESSAGEC": sealed by the client, opened by the server */
#define CZ_DIR_S2C 1 /* "CurveZMQMESSAGES": sealed by the server, opened by the client */

/* Per-frame status of an open (low byte) -- what Mechanism.decode would have raised */
#define CZ_STATUS_OK 0
#define CZ_STATUS_CRYPTO 1    /* bad tag: ZMQ_PROTOCOL_ERROR_ZMTP_CRYPTOGRAPHIC (zmq/ZMQ.java:227) */
#define CZ_STATUS_MALFORMED 2 /* size < 33: ZMTP_MALFORMED_COMMAND_MESSAGE (CurveClientMechanism.java:174-178) */
#define CZ_STATUS_COMMAND 3   /* not "\x07MESSAGE": ZMTP_UNEXPECTED_COMMAND (CurveClientMechanism.java:168-172) */
#define CZ_STATUS_SEQUENCE 4  /* nonce <= previous: replay (CurveClientMechanism.java:186-193) */
/* bits 8..15 of an OK status hold the decrypted flags byte (CZ_MSG_MORE / CZ_MSG_COMMAND) */

/* Library error codes */
#define CZ_OK 0
#define CZ_EINVAL (-22)
#define CZ_EHIP (-5)
#define CZ_ENOMEM (-12)
#define CZ_EPROTO (-71)
#define CZ_EMSGSIZE (-90)
#define CZ_EAGAIN (-11)

/* cz_frame_desc.flags bits (seal: low byte = the MESSAGE flags byte) */
#define CZ_DESC_CHECK_NONCE 0x100 /* open: enforce nonce > floor (counter or prev frame's nonce) */

/*
 * One frame of a batch (40 bytes).  Offsets are byte offsets into the batch's
 * in / out buffers, any alignment.  The segment kernels store outputs at any byte offset
 * through line staging (whole 128-byte cache lines) and read payloads / bodies at any byte
 * offset with dword-aligned loads (16-byte aligned inputs are fastest).
 *   seal: in  = payload (len = n bytes)      out = MESSAGE body (n + 33 bytes)
 *         counter = the 8-byte nonce counter (cnNonce), flags low byte = MORE|COMMAND
 *   open: in  = MESSAGE body (len = size)    out = payload (size - 33 bytes)
 *         counter = replay floor (cnPeerNonce) used when prev < 0;
 *         prev >= 0: the floor is the nonce of frame `prev` of this batch (same connection)
 *   key_idx selects the 32-byte Salsa20 subkey in the batch's subkey table.
 */
typedef struct cz_frame_desc {
    uint64_t in_off;
    uint64_t out_off;
    uint32_t len;
    uint32_t key_idx;
    uint64_t counter;
    uint32_t flags;
    int32_t prev;
} cz_frame_desc;

/* ---- 1. jnacl drop-ins (host memory, NaCl ZEROBYTES layouts) -------------------
 * Replaces curve25519xsalsa20poly1305.crypto_box_afternm (called at Curve.java:136)
 * and crypto_box_open_afternm (Curve.java:146); crypto_secretbox[_open]
 * (xsalsa20poly1305, Curve.java:166,176) is the same primitive.
 * NaCl's crypto_secretbox for every m, as jnacl and libsodium: c = keystream ^ m over all mlen
 * bytes, the Poly1305 key is c[0:32] = keystream[0:32] ^ m[0:32] (so an m whose first 32 bytes
 * are not zero -- Curve.box, Curve.java:184-193, accepts any m -- gets NaCl's tag, not an error),
 * the tag lands at c[16:32] and c[0:16] is written as zero.  The open keys the MAC with the
 * keystream (crypto_secretbox_open), returns -1 on a bad tag with m untouched, and writes
 * m[0:32] as zero.  Runs on the GPU in one launch per call (every seal whose m[0:32] is not zero,
 * and boxes up to 80 KiB; larger CurveZMQ boxes through the segmented kernels): latency-bound,
 * ~11 us of launch + sync floor -- use the batched API for throughput. */
int cz_box_afternm(uint8_t *c, const uint8_t *m, uint64_t mlen, const uint8_t n[24], const uint8_t k[32]);
int cz_box_open_afternm(uint8_t *m, const uint8_t *c, uint64_t clen, const uint8_t n[24], const uint8_t k[32]);
/* The one-launch drop-ins above keep, per calling thread, the HSalsa20 subkeys of the last 8
 * (k, n[0:16]) pairs in device memory (CurveZMQ: one pair per connection direction), so repeated
 * calls on a connection skip the derivation.  Wipe this thread's cache (host copy of the keys and
 * the device subkeys). */
int cz_nacl_forget(void);
/* Create the calling thread's single-shot contexts (the drop-ins' HIP stream, device buffers and
 * pinned staging, and the handshake calls') now instead of on its first call.  Optional; the JNI
 * shim calls it once per thread before it pins any Java array, so HIP runtime initialisation never
 * runs while the JVM's GC is locked out (GetPrimitiveArrayCritical).  CZ_OK or CZ_EHIP. */
int cz_nacl_thread_init(void);
int cz_secretbox(uint8_t *c, const uint8_t *m, uint64_t mlen, const uint8_t n[24], const uint8_t k[32]);
int cz_secretbox_open(uint8_t *m, const uint8_t *c, uint64_t clen, const uint8_t n[24], const uint8_t k[32]);

/* ---- 2. key schedule ------------------------------------------------------------
 * Per-connection-direction Salsa20 subkey = HSalsa20(cnPrecom, "CurveZMQMESSAGE{C|S}").
 * The MESSAGE nonce is that constant 16-byte prefix + BE64(counter)
 * (CurveClientMechanism.java:139-142), so XSalsa20's HSalsa20 step is hoisted
 * out of the per-message path.  d_precom / d_subkeys: nkeys x 32 bytes (device). */
int cz_subkeys(void *d_subkeys, const void *d_precom, uint32_t nkeys, int direction, void *stream);
/* host convenience: one subkey (runs the same device kernel, synchronously) */
int cz_subkey(uint8_t out[32], const uint8_t k[32], int direction);

/* ---- 3. batched, device-resident -----------------------------------------------
 * Mechanism.encode / decode for `count` independent frames in one launch.
 * d_order (optional, count x u32) permutes the lane->frame assignment: pass the
 * frames sorted by decreasing length to balance ragged batches (cz_plan_order). */
int cz_seal_batch(const cz_frame_desc *d_desc, const uint32_t *d_order, uint32_t count, const void *d_in,
                  void *d_out, const void *d_subkeys, void *stream);
/* d_status[i] = CZ_STATUS_* | (flags << 8); d_nonces (optional) = the frame's nonce counter */
int cz_open_batch(const cz_frame_desc *d_desc, const uint32_t *d_order, uint32_t count, const void *d_in,
                  void *d_out, const void *d_subkeys, uint16_t *d_status, uint64_t *d_nonces, void *stream);

/* Uniform-length batch of ONE connection direction: frame i at in + i*in_stride,
 * body i at out + i*out_stride, nonce counter0 + i, flags d_flags8[i] (NULL = 0).
 * Any strides and base alignments: payloads packed at any byte offset are read with
 * dword-aligned loads; an out_stride that is a multiple of 128 (or 64 slots <= 16 KiB)
 * makes the batch own count * out_stride output bytes, and slot bytes past a body are
 * written as zero (whole 128-byte lines stored once); any other out_stride (e.g. bodies
 * back to back, 4129 bytes apart at 4 KiB) goes through byte-shifted line staging and
 * leaves the bytes between bodies as the caller wrote them. */
int cz_seal_uniform(uint32_t count, uint32_t len, const void *d_in, uint64_t in_stride, void *d_out,
                    uint64_t out_stride, const void *d_subkey, uint64_t counter0, const uint8_t *d_flags8,
                    void *stream);
/* The same batch from input already in the reference's NaCl box layout: slot i holds the box
 * m = 0^32 || flags || payload (len = payload bytes, so a box is len + 33 bytes), exactly the
 * buffer CurveClientMechanism.encode builds and hands to Curve.afternm (CurveClientMechanism.java:
 * 144-153, Curve.java:134-137).  The flags byte comes from box byte 32; box bytes 0..31 are not
 * read.  Output as cz_seal_uniform.  Input read where it lies: no byte shift on the device. */
int cz_seal_uniform_box(uint32_t count, uint32_t len, const void *d_box, uint64_t box_stride, void *d_out,
                        uint64_t out_stride, const void *d_subkey, uint64_t counter0, void *stream);
/* Open `count` bodies of `size` bytes of one connection in order; frame 0 must
 * beat floor0, frame i must beat frame i-1 (when check != 0).  Payload i goes to
 * out + i*out_stride.  Bodies at any byte offset (in_stride 4129: the dense wire
 * layout) are read with dword-aligned loads.  out_stride a multiple of 128: the batch
 * owns count * out_stride output bytes (slot bytes past a payload, and rejected frames'
 * slots, are written as zero); any other out_stride: byte-shifted line staging, bytes
 * between payloads untouched, rejected frames' payload bytes written as zero. */
int cz_open_uniform(uint32_t count, uint32_t size, const void *d_in, uint64_t in_stride, void *d_out,
                    uint64_t out_stride, const void *d_subkey, uint64_t floor0, int check, uint16_t *d_status,
                    void *stream);

/* Host-side planner: order[] = frame indices sorted by decreasing len (stable). */
int cz_plan_order(const cz_frame_desc *h_desc, uint32_t count, uint32_t *h_order);

/* ---- 3b. segmented (ragged) batches ---------------------------------------------
 * One lane per frame makes a long frame the batch's critical path (a 64 KiB frame is
 * 1025 sequential Salsa20 blocks on one lane).  cz_plan_segments splits frames longer
 * than 1.5 x seg_blocks 64-byte blocks into seg_blocks-block segments (the last one
 * takes the remainder; for open, segments s >= 1 start at block s*seg_blocks + 1),
 * sorts segments longest first (by output chunks), and lists the split frames for
 * the combine step, which joins the per-segment Poly1305 partials with r^m powers.
 * d_work must hold 64 bytes per part (*npart from the planner).  Output contract as
 * cz_seal_batch / cz_open_batch (statuses, nonces, zeroed plaintext on a bad tag).
 * A caller may also build its own plan: the segments of a split frame cover its box blocks
 * [0, nblk) contiguously, one or more blocks each (open: segments after the first start at
 * block 2 or later), with consecutive part indices from the frame's part0, in any order in
 * the list and of any lengths (tests/test_gpu_segments.py cuts frames at random points). */
typedef struct cz_segment {
    uint32_t frame;       /* index into the descriptor array */
    uint32_t first_block; /* first 64-byte box block of the segment */
    uint32_t nblocks;
    uint32_t part;        /* partial-record index, 0xffffffff for a frame in one segment */
} cz_segment;
typedef struct cz_combine {
    uint32_t frame;
    uint32_t part0; /* first partial record of the frame (its segments are consecutive) */
    uint32_t nseg;
    uint32_t reserved;
} cz_combine;
/* open = 0: desc.len is a payload length (seal); 1: a body size (open).  Returns CZ_EINVAL
 * with *nseg / *ncomb set to the sizes needed when a capacity is too small. */
int cz_plan_segments(const cz_frame_desc *h_desc, uint32_t count, int open, uint32_t seg_blocks, cz_segment *h_seg,
                     uint32_t seg_cap, uint32_t *nseg, cz_combine *h_comb, uint32_t comb_cap, uint32_t *ncomb,
                     uint32_t *npart);
int cz_seal_segments(const cz_frame_desc *d_desc, const cz_segment *d_seg, uint32_t nseg, const cz_combine *d_comb,
                     uint32_t ncomb, const void *d_in, void *d_out, const void *d_subkeys, void *d_work,
                     void *stream);
int cz_open_segments(const cz_frame_desc *d_desc, const cz_segment *d_seg, uint32_t nseg, const cz_combine *d_comb,
                     uint32_t ncomb, const void *d_in, void *d_out, const void *d_subkeys, void *d_work,
                     uint16_t *d_status, uint64_t *d_nonces, void *stream);

/* Synthetic data: fill d_buf with the counter-based SplitMix64 byte stream (seed). */
int cz_fill(void *d_buf, uint64_t nbytes, uint64_t seed, void *stream);
/* Measurement: device-to-device copy of nbytes (a multiple of 16) with 16-byte loads and stores,
 * the float4 copy the MI355X guide measures at 6.29 TB/s; bench.py's HBM copy ceiling. */
int cz_dev_copy(void *d_dst, const void *d_src, uint64_t nbytes, void *stream);

/* ---- 4. host-staged batches (the JNI path: Java byte[] / direct ByteBuffer) -------
 * A context owns a HIP stream, pinned host staging and device buffers that grow
 * on demand.  cz_ctx_seal/open copy host frames in, run the batch kernel and copy
 * the results out (synchronous).  These are what a JNI shim binds. */
typedef struct cz_ctx cz_ctx;
int cz_ctx_create(cz_ctx **out, int device);
void cz_ctx_destroy(cz_ctx *ctx);
/* upload `nkeys` 32-byte cnPrecom keys and derive their subkeys for `direction` */
int cz_ctx_set_keys(cz_ctx *ctx, const uint8_t *h_precom, uint32_t nkeys, int direction);
int cz_ctx_seal(cz_ctx *ctx, const cz_frame_desc *h_desc, uint32_t count, const void *h_in, uint64_t in_bytes,
                void *h_out, uint64_t out_bytes);
int cz_ctx_open(cz_ctx *ctx, const cz_frame_desc *h_desc, uint32_t count, const void *h_in, uint64_t in_bytes,
                void *h_out, uint64_t out_bytes, uint16_t *h_status);
/* Pipelined host-staged uniform batches (the end-to-end path at throughput): frames in
 * chunks of chunk_frames (0 = 16384); chunk k runs H2D -> kernel
 * -> D2H on one of three streams with its own device buffers, so PCIe copies in both
 * directions overlap each other and the kernels.  A batch that is one chunk of at most
 * 64 MiB (in + out slots) of frames of 8+ blocks runs on one stream through the segment
 * kernels instead, so a few frames cost tens of us rather than one lane's whole walk.  Both
 * paths write whole output slots: each body followed by zeros to the end of its slot, and
 * zeros in the payload slot of a rejected open, whatever the batch size or chunk_frames.
 * For count == 1 the strides are ignored and the slot is the body alone.  Host buffers
 * should be pinned (cz_host_alloc) for full PCIe rate; the output host buffer must span
 * count * out_stride bytes (whole slots).  Uses the
 * context's key 0 (cz_ctx_set_keys).  Synchronous. */
int cz_ctx_seal_uniform(cz_ctx *ctx, uint32_t count, uint32_t len, const void *h_in, uint64_t in_stride, void *h_out,
                        uint64_t out_stride, uint64_t counter0, const uint8_t *h_flags8, uint32_t chunk_frames);
int cz_ctx_open_uniform(cz_ctx *ctx, uint32_t count, uint32_t size, const void *h_in, uint64_t in_stride, void *h_out,
                        uint64_t out_stride, uint64_t floor0, int check, uint16_t *h_status, uint32_t chunk_frames);
/* pinned host buffers for zero-extra-copy callers (a pinned MsgAllocator, zmq/msg/MsgAllocator.java:5-8).
 * cz_host_free frees only a base address cz_host_alloc returned and not yet freed (CZ_OK); any
 * other pointer -- an interior address, foreign memory, a second free -- is CZ_EINVAL and left alone. */
void *cz_host_alloc(uint64_t bytes);
int cz_host_free(void *p);

/* ---- 5. CURVE mechanism objects (host mirror of CurveClientMechanism / CurveServerMechanism
 *         in the CONNECTED state: encode/decode of MESSAGE commands with nonce bookkeeping) ---- */
typedef struct cz_mech cz_mech;
/* as_server = 0: client (seals ...MESSAGEC, opens ...MESSAGES); 1: server.
 * cn_nonce / cn_peer_nonce: the handshake's final values (client
 * MESSAGEs start at 3, server at 2). */
cz_mech *cz_mech_create(int as_server, const uint8_t precom[32], uint64_t cn_nonce, uint64_t cn_peer_nonce,
                        int device);
void cz_mech_destroy(cz_mech *m);
/* encode one Msg: out must hold n + 33 bytes; returns the body length or a negative CZ_E* */
int64_t cz_mech_encode(cz_mech *m, const uint8_t *payload, uint64_t n, int msg_flags, uint8_t *out);
/* decode one body: returns the payload length (>= 0) and *msg_flags, or CZ_EPROTO with
 * *event = ZMQ_PROTOCOL_ERROR_* code (zmq/ZMQ.java:209-227) the reference would raise */
int64_t cz_mech_decode(cz_mech *m, const uint8_t *body, uint64_t size, uint8_t *out, int *msg_flags, int *event);
/* batched encode of count frames packed back to back: payloads at in_off[i] (len[i]),
 * bodies written at out_off[i].  One device launch for the whole batch. */
int cz_mech_encode_batch(cz_mech *m, uint32_t count, const uint8_t *h_in, const uint64_t *in_off,
                         const uint32_t *len, const uint8_t *msg_flags, uint8_t *h_out, const uint64_t *out_off);
/* batched decode: stops at the first failing frame like StreamEngine does (returns its index
 * in *failed, or -1); frames before it are delivered. */
int cz_mech_decode_batch(cz_mech *m, uint32_t count, const uint8_t *h_in, const uint64_t *in_off,
                         const uint32_t *size, uint8_t *h_out, const uint64_t *out_off, uint8_t *msg_flags,
                         int32_t *failed, int *event);
uint64_t cz_mech_nonce(const cz_mech *m);
uint64_t cz_mech_peer_nonce(const cz_mech *m);

/* ZMTP protocol-error event codes (zmq/ZMQ.java:214-227) */
#define CZ_ZMTP_UNEXPECTED_COMMAND 0x10000001
#define CZ_ZMTP_MALFORMED_COMMAND_MESSAGE 0x10000012
#define CZ_ZMTP_INVALID_SEQUENCE 0x10000002
#define CZ_ZMTP_CRYPTOGRAPHIC 0x11000001
#define CZ_ZMTP_UNSPECIFIED 0x10000000
#define CZ_ZMTP_KEY_EXCHANGE 0x10000003
#define CZ_ZMTP_MALFORMED_COMMAND_HELLO 0x10000013
#define CZ_ZMTP_MALFORMED_COMMAND_INITIATE 0x10000014
#define CZ_ZMTP_MALFORMED_COMMAND_ERROR 0x10000015
#define CZ_ZMTP_MALFORMED_COMMAND_READY 0x10000016
#define CZ_ZAP_MALFORMED_REPLY 0x20000001
#define CZ_ZAP_INVALID_STATUS_CODE 0x20000004

/* ---- 7. ZMTP v2 framing (zmq/io/coder/v2/V2Encoder.java, V2Decoder.java) ----------------
 * Wire frame = flags byte (MORE 1, LARGE 2, COMMAND 4: V1Protocol/V2Protocol) + size
 * (1 byte, or BE64 with LARGE when size > 255: V2Encoder.java:31-55) + body. */
#define CZ_V2_MORE 0x01
#define CZ_V2_LARGE 0x02
#define CZ_V2_COMMAND 0x04
/* header bytes V2Encoder writes before a body of `size` bytes: 2, or 9 when size > 255 */
uint32_t cz_v2_header_size(uint64_t size);
/* Host parser with V2Decoder's rules (V2Decoder.java:37-105, Decoder.java:76-98): parses whole
 * frames from wire[0:len) into frames[] (body offset, size, Msg flags MORE=CZ_MSG_MORE /
 * COMMAND=CZ_MSG_COMMAND), stopping at cap frames or at an incomplete frame.  *consumed = bytes
 * of the whole frames.  Returns CZ_OK, or CZ_EPROTO (LARGE size <= 0 as a signed long) /
 * CZ_EMSGSIZE (size > maxmsgsize >= 0, or > INT32_MAX) at the first bad header; the frames
 * before it are still reported.  No device needed. */
typedef struct cz_v2_frame {
    uint64_t body_off;
    uint32_t size;
    uint32_t msg_flags;
} cz_v2_frame;
int cz_v2_parse(const uint8_t *wire, uint64_t len, int64_t maxmsgsize, cz_v2_frame *frames, uint32_t cap,
                uint32_t *nframes, uint64_t *consumed);
/* Device: one copy per item, any byte alignment.  With CZ_V2_ITEM_HEADER in flags, the V2
 * header for `size` (wire flags = flags & 0xff, LARGE set by size) is written at dst_off and the
 * body after it: packing sealed MESSAGE bodies into socket-ready wire streams.  Without it a
 * plain copy: unpacking received bodies into aligned slots for the open kernels. */
#define CZ_V2_ITEM_HEADER 0x100
typedef struct cz_v2_item {
    uint64_t src_off;
    uint64_t dst_off;
    uint32_t size;
    uint32_t flags;
} cz_v2_item;
int cz_v2_copy(const cz_v2_item *d_items, uint32_t count, const void *d_src, void *d_dst, void *stream);

/* ---- 8. batching engine: many CURVE connections, one device batch per flush -----------------
 * The GPU form of StreamEngine's encode/decode loops (outEvent: pull + mechanism.encode +
 * V2Encoder up to OUT_BATCH_SIZE, StreamEngine.java:467-535; inEvent: V2Decoder +
 * mechanism.decode, :379-465, decodeAndPush :1067-1098) across connections: messages of all
 * connections are sealed in one segmented device batch and packed into per-connection wire
 * streams; received wire bytes of all connections are parsed, opened in one batch and checked
 * against each connection's nonce chain.  Payload buffers come from a pinned arena
 * (ZMQ_MSG_ALLOCATOR, zmq/msg/MsgAllocator.java:5-8).  Not thread-safe: one engine per thread. */
typedef struct cz_engine cz_engine;
/* arena_bytes: capacity of the pinned outbound payload arena (messages per flush) */
int cz_engine_create(cz_engine **e, uint64_t arena_bytes, int device);
void cz_engine_destroy(cz_engine *e);
/* returns a connection id >= 0; cn_nonce / cn_peer_nonce as cz_mech_create */
int cz_engine_add_conn(cz_engine *e, int as_server, const uint8_t precom[32], uint64_t cn_nonce,
                       uint64_t cn_peer_nonce);
/* the connection is gone (StreamEngine unplug / error, StreamEngine.java:334-370,1116-1131): its
 * queued messages are dropped from the next flush, its received bytes and last flush_in payloads
 * are discarded, its subkeys are wiped, and its id is reused by a later cz_engine_add_conn.
 * Every other call on the id fails with CZ_EINVAL until then. */
int cz_engine_remove_conn(cz_engine *e, int conn);
/* pinned payload buffer inside the arena (no copy at send); NULL when the arena is full */
void *cz_engine_msg_alloc(cz_engine *e, uint32_t len);
/* queue one Msg (payload from cz_engine_msg_alloc, or copied into the arena); CZ_ENOMEM when the
 * arena is full (flush first), CZ_EPROTO when the connection has failed */
int cz_engine_send(cz_engine *e, int conn, const void *payload, uint32_t len, int msg_flags);
/* seal every queued Msg on the device and V2-frame it into one pinned output in SEND order
 * (valid until the next cz_engine_flush_out).  The flush is pipelined in groups of ~8 MiB+:
 * H2D of a group overlaps the seal + D2H of the one before. */
int cz_engine_flush_out(cz_engine *e);
/* one connection's MESSAGE frames, in its send order, as contiguous bytes: a pointer into the
 * flush output when its messages were queued back to back, else a host-gathered copy */
int cz_engine_wire_out(cz_engine *e, int conn, const uint8_t **wire, uint64_t *len);
/* the same stream as gather-write pieces of the flush output (for writev / a GatheringByteChannel,
 * StreamEngine.java:509-535): *count = pieces; fills iov when cap >= *count (cap 0: count only) */
typedef struct cz_iovec {
    const uint8_t *base;
    uint64_t len;
} cz_iovec;
int cz_engine_wire_iov(cz_engine *e, int conn, cz_iovec *iov, uint32_t cap, uint32_t *count);
/* append bytes received on a connection (partial frames are kept for the next flush) */
int cz_engine_recv(cz_engine *e, int conn, const void *wire, uint64_t len);
/* zero-copy receive (the V2Decoder getBuffer() pattern, StreamEngine.java:403-410): a pinned
 * buffer of *avail >= min_bytes bytes at the end of the connection's received data; read from
 * the socket into it, then commit the bytes read.  Valid until the next engine call. */
int cz_engine_recv_buffer(cz_engine *e, int conn, uint64_t min_bytes, uint8_t **buf, uint64_t *avail);
int cz_engine_recv_commit(cz_engine *e, int conn, uint64_t n);
/* parse, open and sequence-check every whole frame received on every connection */
int cz_engine_flush_in(cz_engine *e);
/* decoded messages of the last cz_engine_flush_in (pinned memory, valid until the next one) */
int cz_engine_msgs_in(cz_engine *e, int conn, uint32_t *count);
int cz_engine_msg_in(cz_engine *e, int conn, uint32_t i, const uint8_t **payload, uint32_t *len, int *msg_flags);
/* 0 while the connection is healthy; after a failure CZ_EPROTO / CZ_EMSGSIZE and *event = the
 * ZMTP protocol-error event the reference raises (0 for a framing error) */
int cz_engine_conn_error(cz_engine *e, int conn, int *event);
uint64_t cz_engine_nonce(cz_engine *e, int conn);
uint64_t cz_engine_peer_nonce(cz_engine *e, int conn);

/* ---- 9. handshake public-key calls (Curve.java:84-193 -> jnacl) --------------------------
 * jnacl int contract (0 / -1).  X25519 per RFC 7748 on the device; box / box_open are
 * beforenm + the section-1 afternm calls.  The secret key of cz_box_keypair comes from the OS
 * CSPRNG (getrandom), the public key from X25519(sk, 9) on the device. */
int cz_scalarmult(uint8_t q[32], const uint8_t n[32], const uint8_t p[32]);             /* crypto_scalarmult */
int cz_box_keypair(uint8_t pk[32], uint8_t sk[32]);                                      /* Curve.java:100-115 */
int cz_box_beforenm(uint8_t k[32], const uint8_t pk[32], const uint8_t sk[32]);          /* Curve.java:124-127 */
int cz_box(uint8_t *c, const uint8_t *m, uint64_t mlen, const uint8_t n[24], const uint8_t pk[32],
           const uint8_t sk[32]);                                                        /* Curve.java:183-193 */
int cz_box_open(uint8_t *m, const uint8_t *c, uint64_t clen, const uint8_t n[24], const uint8_t pk[32],
                const uint8_t sk[32]);                                                   /* Curve.java:149-157 */
/* Device batches for connection churn (one lane per key agreement, 32-byte records):
 * out[i] = X25519(scalars[i], points[i]) (points NULL = base point 9);
 * k[i] = beforenm(pk[i], sk[i]) = HSalsa20(X25519(sk[i], pk[i]), 0^16). */
int cz_x25519_batch(const void *d_scalars, const void *d_points, void *d_out, uint32_t count, void *stream);
int cz_beforenm_batch(const void *d_pk, const void *d_sk, void *d_k, uint32_t count, void *stream);

/* ---- 10. CURVE handshake: HELLO / WELCOME / INITIATE / READY (+ ERROR) -----------------------------
 * The state machines of CurveClientMechanism (:80-124, :246-429) and CurveServerMechanism
 * (:77-126, :227-517) with every box / open / secretbox / beforenm / X25519 on the GPU (section 9).
 * A handshake object is created in the reference constructor's state (fresh short-term key pair,
 * cnNonce = cnPeerNonce = 1); the caller moves ZMTP command bodies between the peers:
 *   cz_hs_next_command   = Mechanism.nextHandshakeCommand: CZ_OK with a command to send,
 *                          CZ_EAGAIN when there is nothing to send in this state;
 *   cz_hs_process_command = Mechanism.processHandshakeCommand: CZ_OK, or CZ_EPROTO with
 *                          cz_hs_event() = the ZMQ_PROTOCOL_ERROR_* event the reference raises,
 *                          CZ_EINVAL for an incompatible peer Socket-Type (parseMetadata);
 *   cz_hs_status         = Mechanism.status: CZ_HS_HANDSHAKING / READY / ERROR.
 * Once READY, cz_hs_session yields cnPrecom and the nonce counters that cz_mech_create /
 * cz_engine_add_conn take; cz_hs_mechanism / cz_engine_add_session do both steps.
 * socket_type: ZMQ_PAIR = 0 ... ZMQ_GATHER = 20 (zmq/ZMQ.java:50-70); the Socket-Type property and,
 * for REQ / DEALER / ROUTER, the Identity property are sent in INITIATE / READY.
 * ephemeral_secret / entropy (tests only, NULL in production): a fixed short-term secret and the
 * bytes the reference's Curve.random() draws return, in order (client: the 16-byte vouch nonce;
 * server: cookie nonce 16, cookie key 32, WELCOME nonce 16).  ZAP (out of scope): with
 * cz_hs_set_zap(hs, 1) the server waits after INITIATE for cz_hs_zap_reply(hs, "200" | "4xx" ...). */
typedef struct cz_hs cz_hs;
#define CZ_HS_HANDSHAKING 0
#define CZ_HS_READY 1
#define CZ_HS_ERROR 2
int cz_hs_create(cz_hs **hs, int as_server, const uint8_t public_key[32], const uint8_t secret_key[32],
                 const uint8_t server_key[32], int socket_type, const uint8_t *identity, uint32_t identity_len,
                 const uint8_t *ephemeral_secret, const uint8_t *entropy, uint32_t entropy_len);
void cz_hs_destroy(cz_hs *hs);
int cz_hs_next_command(cz_hs *hs, uint8_t *out, uint32_t cap, uint32_t *len);
int cz_hs_process_command(cz_hs *hs, const uint8_t *cmd, uint64_t size);
int cz_hs_status(const cz_hs *hs);
int cz_hs_event(const cz_hs *hs);
/* client: the status code (300..500) of a well-formed ERROR from the server, else 0 */
int cz_hs_error_status(const cz_hs *hs);
int cz_hs_set_zap(cz_hs *hs, int on);
int cz_hs_zap_reply(cz_hs *hs, const char *status_code);
/* server, after INITIATE: the client's long-term public key C (what a ZAP request carries) */
int cz_hs_client_key(const cz_hs *hs, uint8_t key[32]);
int cz_hs_session(const cz_hs *hs, uint8_t precom[32], uint64_t *cn_nonce, uint64_t *cn_peer_nonce);
/* a property of the peer's metadata (INITIATE / READY), e.g. "Socket-Type", "Identity" */
int cz_hs_peer_property(const cz_hs *hs, const char *name, const uint8_t **value, uint32_t *len);
cz_mech *cz_hs_mechanism(const cz_hs *hs, int device);
int cz_engine_add_session(cz_engine *e, const cz_hs *hs);
/* host only: Metadata.read + parseMetadata's Socket-Type check (CZ_OK / CZ_EPROTO / CZ_EINVAL), and the
 * metadata block a socket of this type sends (returns its size; written when it fits in cap) */
int cz_zmtp_metadata_check(const uint8_t *buf, uint64_t len, int socket_type);
uint32_t cz_zmtp_metadata(int socket_type, const uint8_t *identity, uint32_t identity_len, uint8_t *out, uint32_t cap);

/* ---- 6. misc -------------------------------------------------------------- */
const char *cz_last_error(void);
const char *cz_version(void);
/* 1 if a HIP device is present and the gfx950 code object loaded */
int cz_device_ok(void);
/* Kernel-variant knob for A/B measurement; returns the previous value or CZ_EINVAL.
 *   "pair": 1 = seal kernels read whole 128-byte input lines per two blocks (default), 0 = per block
 *   "un0":  1 = scalar first Salsa round when the high nonce word is wave-uniform (default), 0 = off
 *   "seglines": 1 = line-staged stores in the segment kernels (default), 0 = direct stores
 *   "shift": 1 = byte-shifted line staging for uniform outputs off 128-byte slots (default)
 *   "shift16": 1 = segment outputs that are 16-byte but not 128-byte aligned through the
 *              byte-shifted line emitter (default), 0 = 128-byte groups at each output's base
 *   "open_ina" / "seal_ina": 1 = line paths for bodies / payloads off 16-byte alignment with
 *              dword-aligned loads (default), 0 = lane-wise unaligned paths */
int cz_tune(const char *key, int value);

#ifdef __cplusplus
}
#endif
#endif
