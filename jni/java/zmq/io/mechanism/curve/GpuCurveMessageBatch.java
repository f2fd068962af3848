// The MESSAGE-phase half of a batching CURVE Mechanism (SURVEY.md section 7 step 6): the
// Mechanism.encode / decode of CurveClientMechanism (:126-224) and CurveServerMechanism (:127-224)
// for a whole list of messages in one GpuCurveBatch call (cz_ctx_seal / cz_ctx_open, include/
// curvezmq_mi355x.h section 4), with the same nonce bookkeeping, checks and monitor events.
// GpuCurveClientMechanism / GpuCurveServerMechanism own one each, created once the handshake is
// complete (status() == READY), from the session keys the handshake left in the mechanism.
package zmq.io.mechanism.curve;

import java.lang.reflect.Field;
import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import java.util.ArrayList;
import java.util.List;

import zmq.Msg;
import zmq.ZError;
import zmq.ZMQ;
import zmq.io.SessionBase;
import zmq.util.Errno;

final class GpuCurveMessageBatch implements AutoCloseable
{
    // include/curvezmq_mi355x.h
    private static final int CZ_OK               = 0;
    private static final int CZ_DIR_C2S          = 0;
    private static final int CZ_DIR_S2C          = 1;
    private static final int CZ_STATUS_OK        = 0;
    private static final int CZ_STATUS_CRYPTO    = 1;
    private static final int CZ_STATUS_MALFORMED = 2;
    private static final int CZ_STATUS_COMMAND   = 3;
    private static final int CZ_DESC_CHECK_NONCE = 0x100;
    private static final int DESC_BYTES          = 40;   // sizeof(cz_frame_desc)
    private static final int OVERHEAD            = 33;   // "\x07MESSAGE" + nonce8 + tag16 + flags

    private final boolean     server;
    private final SessionBase session;
    private final Errno       errno;
    private final long        sealCtx;   // key 0: this side's sending direction
    private final long        openCtx;   // key 0: the peer's sending direction
    private long              cnNonce;
    private long              cnPeerNonce;
    private int               lastEvent;

    // pinned staging (GpuCurveBatch.hostAlloc), grown on demand
    private ByteBuffer descs;
    private ByteBuffer in;
    private ByteBuffer out;
    private ByteBuffer status;

    // `mechanism`: a CurveClientMechanism / CurveServerMechanism whose handshake is complete
    GpuCurveMessageBatch(Object mechanism, Class<?> curveClass, boolean server, SessionBase session, Errno errno)
    {
        this.server = server;
        this.session = session;
        this.errno = errno;
        byte[] precom = (byte[]) field(mechanism, curveClass, "cnPrecom");
        cnNonce = (Long) field(mechanism, curveClass, "cnNonce");
        cnPeerNonce = (Long) field(mechanism, curveClass, "cnPeerNonce");
        ByteBuffer k = GpuCurveBatch.hostAlloc(32);
        if (k == null) {
            throw new IllegalStateException("GpuCurveBatch.hostAlloc failed");
        }
        k.put(precom);
        sealCtx = GpuCurveBatch.create(0);
        openCtx = GpuCurveBatch.create(0);
        try {
            if (sealCtx == 0 || openCtx == 0
                    || GpuCurveBatch.setKeys(sealCtx, k, 1, server ? CZ_DIR_S2C : CZ_DIR_C2S) != CZ_OK
                    || GpuCurveBatch.setKeys(openCtx, k, 1, server ? CZ_DIR_C2S : CZ_DIR_S2C) != CZ_OK) {
                close();
                throw new IllegalStateException("GpuCurveBatch context (no MI355X visible?)");
            }
        }
        finally {
            k.clear();
            k.put(new byte[32]);   // no key left in the pinned buffer
            GpuCurveBatch.hostFree(k);
        }
    }

    // the handshake's session state is private to CurveClientMechanism / CurveServerMechanism
    // (CurveClientMechanism.java:46-49, CurveServerMechanism.java:34-47)
    private static Object field(Object m, Class<?> cls, String name)
    {
        try {
            Field f = cls.getDeclaredField(name);
            f.setAccessible(true);
            return f.get(m);
        }
        catch (ReflectiveOperationException e) {
            throw new IllegalStateException("CURVE mechanism field " + name, e);
        }
    }

    private static ByteBuffer grow(ByteBuffer b, long need)
    {
        if (b != null && b.capacity() >= need) {
            return b;
        }
        if (b != null) {
            GpuCurveBatch.hostFree(b);
        }
        long cap = Math.max(need, 1L << 16);
        ByteBuffer n = GpuCurveBatch.hostAlloc(Math.min(2 * cap, Integer.MAX_VALUE));
        if (n == null) {
            throw new OutOfMemoryError("GpuCurveBatch.hostAlloc(" + cap + ")");
        }
        return n.order(ByteOrder.LITTLE_ENDIAN);
    }

    private static long up16(long v)
    {
        return (v + 15) & ~15L;
    }

    private static final byte[] ZEROS = new byte[1 << 16];

    // plaintext must not outlive the call in pinned memory (the C paths explicit_bzero their
    // staging): zero the first n bytes of b
    private static void wipe(ByteBuffer b, long n)
    {
        if (b == null) {
            return;
        }
        ByteBuffer d = b.duplicate();
        d.clear();
        long left = Math.min(n, d.capacity());
        while (left > 0) {
            int k = (int) Math.min(left, ZEROS.length);
            d.put(ZEROS, 0, k);
            left -= k;
        }
    }

    private void desc(int i, long inOff, long outOff, int len, long counter, int flags, int prev)
    {
        int d = i * DESC_BYTES;
        descs.putLong(d, inOff);
        descs.putLong(d + 8, outOff);
        descs.putInt(d + 16, len);
        descs.putInt(d + 20, 0);        // key_idx
        descs.putLong(d + 24, counter);
        descs.putInt(d + 32, flags);
        descs.putInt(d + 36, prev);
    }

    // Mechanism.encode of every message, in order: "\x07MESSAGE" || BE64(cnNonce) || tag || box
    // (CurveClientMechanism.java:126-163), cnNonce post-incremented per message.
    List<Msg> encode(List<Msg> msgs)
    {
        final int count = msgs.size();
        long inBytes = 0;
        long outBytes = 0;
        for (Msg m : msgs) {
            inBytes = up16(inBytes) + m.size();
            outBytes = up16(outBytes) + m.size() + OVERHEAD;
        }
        descs = grow(descs, (long) count * DESC_BYTES);
        in = grow(in, inBytes + 16);
        out = grow(out, outBytes + 16);
        long io = 0;
        long oo = 0;
        for (int i = 0; i < count; i++) {
            Msg m = msgs.get(i);
            io = up16(io);
            oo = up16(oo);
            ByteBuffer src = m.buf().slice();    // from the Msg's own position (Msg.java:146-155)
            src.limit(m.size());
            ByteBuffer dst = in.duplicate();
            dst.position((int) io);
            dst.put(src);
            int flags = (m.hasMore() ? 0x01 : 0) | (m.isCommand() ? 0x02 : 0);
            desc(i, io, oo, m.size(), cnNonce + i, flags, -1);
            io += m.size();
            oo += m.size() + OVERHEAD;
        }
        if (GpuCurveBatch.seal(sealCtx, descs, count, in, out) != CZ_OK) {
            wipe(in, io);
            throw new IllegalStateException("GpuCurveBatch.seal failed");
        }
        wipe(in, io);   // the staged plaintext
        cnNonce += count;
        List<Msg> encoded = new ArrayList<>(count);
        for (int i = 0; i < count; i++) {
            int d = i * DESC_BYTES;
            int len = descs.getInt(d + 16) + OVERHEAD;
            Msg e = new Msg(len);
            e.put(out, (int) descs.getLong(d + 8), len);
            encoded.add(e);
        }
        return encoded;
    }

    // Mechanism.decode of every body, in order, up to the first failure (CurveClientMechanism.java:
    // 165-224): the decoded prefix.  On a failure the reference's event is raised, errno = EPROTO and
    // failed() is true -- what decode returning null does, after which StreamEngine tears the
    // connection down (:1072-1073).
    List<Msg> decode(List<Msg> bodies)
    {
        final int count = bodies.size();
        long inBytes = 0;
        long outBytes = 0;
        for (Msg m : bodies) {
            inBytes = up16(inBytes) + m.size();
            outBytes = up16(outBytes) + Math.max(m.size() - OVERHEAD, 0);
        }
        descs = grow(descs, (long) count * DESC_BYTES);
        in = grow(in, inBytes + 16);
        out = grow(out, outBytes + 16);
        status = grow(status, 2L * count);
        long io = 0;
        long oo = 0;
        for (int i = 0; i < count; i++) {
            Msg m = bodies.get(i);
            io = up16(io);
            oo = up16(oo);
            ByteBuffer src = m.buf().slice();
            src.limit(m.size());
            ByteBuffer dst = in.duplicate();
            dst.position((int) io);
            dst.put(src);
            desc(i, io, oo, m.size(), cnPeerNonce, CZ_DESC_CHECK_NONCE, i > 0 ? i - 1 : -1);
            io += m.size();
            oo += Math.max(m.size() - OVERHEAD, 0);
        }
        lastEvent = 0;
        if (GpuCurveBatch.open(openCtx, descs, count, in, out, status) != CZ_OK) {
            wipe(out, oo);
            throw new IllegalStateException("GpuCurveBatch.open failed");
        }
        List<Msg> decoded = new ArrayList<>(count);
        for (int i = 0; i < count; i++) {
            int st = status.getShort(2 * i) & 0xffff;
            int d = i * DESC_BYTES;
            int size = descs.getInt(d + 16);
            if ((st & 0xff) != CZ_STATUS_OK) {
                if ((st & 0xff) == CZ_STATUS_CRYPTO) {
                    cnPeerNonce = nonceOf(i);   // set before the tag check (CurveClientMechanism.java:193)
                }
                lastEvent = event(st & 0xff);
                session.getSocket().eventHandshakeFailedProtocol(session.getEndpoint(), lastEvent);
                errno.set(ZError.EPROTO);
                break;
            }
            cnPeerNonce = nonceOf(i);
            Msg p = new Msg(size - OVERHEAD);
            if (((st >> 8) & 0x01) != 0) {
                p.setFlags(Msg.MORE);
            }
            if (((st >> 8) & 0x02) != 0) {
                p.setFlags(Msg.COMMAND);
            }
            p.put(out, (int) descs.getLong(d + 8), size - OVERHEAD);
            decoded.add(p);
        }
        wipe(out, oo);   // every opened plaintext, including frames after a failure
        return decoded;
    }

    private long nonceOf(int i)
    {
        int at = (int) descs.getLong(i * DESC_BYTES);
        return in.duplicate().order(ByteOrder.BIG_ENDIAN).getLong(at + 8);   // Wire.getUInt64
    }

    // the monitor event CurveClientMechanism / CurveServerMechanism.decode raises per failure
    private int event(int st)
    {
        switch (st) {
        case CZ_STATUS_COMMAND:
            return ZMQ.ZMQ_PROTOCOL_ERROR_ZMTP_UNEXPECTED_COMMAND;
        case CZ_STATUS_MALFORMED:
            return ZMQ.ZMQ_PROTOCOL_ERROR_ZMTP_MALFORMED_COMMAND_MESSAGE;
        case CZ_STATUS_CRYPTO:
            return ZMQ.ZMQ_PROTOCOL_ERROR_ZMTP_CRYPTOGRAPHIC;
        default:   // CZ_STATUS_SEQUENCE: a replayed nonce
            return server ? ZMQ.ZMQ_PROTOCOL_ERROR_ZMTP_INVALID_SEQUENCE : ZMQ.ZMQ_PROTOCOL_ERROR_ZMTP_CRYPTOGRAPHIC;
        }
    }

    boolean failed()
    {
        return lastEvent != 0;
    }

    @Override
    public void close()
    {
        if (sealCtx != 0) {
            GpuCurveBatch.destroy(sealCtx);
        }
        if (openCtx != 0) {
            GpuCurveBatch.destroy(openCtx);
        }
        for (ByteBuffer b : new ByteBuffer[] {descs, in, out, status}) {
            if (b != null) {
                wipe(b, b.capacity());
                GpuCurveBatch.hostFree(b);
            }
        }
    }
}
