// The IO-thread side of the batching engine: what StreamEngine's outEvent / inEvent do for a CURVE
// connection in the CONNECTED state, with every connection of the IO thread sealed and opened in one
// device batch per poller loop (include/curvezmq_mi355x.h section 8, INTEGRATION.md section 5).
//
// Reference loops it replaces, per connection and per wake-up:
//   outEvent  (StreamEngine.java:467-535): pullAndEncode = session.pullMsg + mechanism.encode
//             (:1052-1063), V2Encoder, SocketChannel.write of at most OUT_BATCH_SIZE bytes;
//   inEvent   (StreamEngine.java:379-465): SocketChannel.read, V2Decoder, decodeAndPush =
//             mechanism.decode + session.pushMsg (:1067-1098), error(PROTOCOL) on a failed decode.
// Here outEvent(conn) only pulls and queues (GpuCurveEngine.send), inEvent(conn) only reads and
// queues (GpuCurveEngine.recv); the poller calls endOfLoop() once per iteration, which opens every
// received frame (flushIn) and delivers the payloads in order, then seals every queued message of
// every connection (flushOut) and writes each connection's wire bytes with one gathering write
// (wireIov).  A connection whose frame fails (bad tag, replay, malformed, framing) gets the reference's
// monitor event (connError -> eventHandshakeFailedProtocol) and is torn down, as decodeAndPush
// returning false tears it down; the other connections carry on.
//
// The wiring into the reference is jni/patches/jeromq-gpu-curve.patch (INTEGRATION.md section 5):
// Poller owns one hook per IO thread (fromSystemProperties, -Dzmq.curve.gpu=true) and calls
// endOfLoop() at the end of every loop iteration; StreamEngine attaches a CURVE connection when
// its mechanism reaches READY, hands over the bytes its decoder had already read, delegates
// outEvent / inEvent, and detaches on teardown.  StreamEngine keeps the rest of its role
// (handshake, heartbeats, metadata, back-pressure) through Sink.  Not thread-safe: one per IO thread.
package zmq.io;

import java.io.IOException;
import java.lang.reflect.Field;
import java.nio.ByteBuffer;
import java.nio.channels.GatheringByteChannel;
import java.nio.channels.ReadableByteChannel;
import java.util.ArrayDeque;
import java.util.ArrayList;
import java.util.List;

import zmq.Msg;
import zmq.io.mechanism.Mechanism;
import zmq.io.mechanism.curve.CurveClientMechanism;
import zmq.io.mechanism.curve.CurveServerMechanism;

public final class GpuCurveIoHook implements AutoCloseable
{
    // library codes (include/curvezmq_mi355x.h)
    private static final int CZ_OK     = 0;
    private static final int CZ_ENOMEM = -12;

    // -Dzmq.curve.gpu=true turns the hook on for every IO thread; the sizes and the device are
    // -Dzmq.curve.gpu.arena (pinned outbound payload bytes per loop), -Dzmq.curve.gpu.read (receive
    // buffer) and -Dzmq.curve.gpu.device
    public static final String PROPERTY = "zmq.curve.gpu";

    // The StreamEngine side of one connection.
    public interface Sink
    {
        // the next message to send, or null (StreamEngine.pullAndEncode without the encode:
        // session.pullMsg, :1052-1063; a heartbeat PING / PONG command when one is due)
        Msg pull();

        // a decoded message (StreamEngine.decodeAndPush after mechanism.decode, :1072-1097: commands
        // to processCommand, metadata, session.pushMsg); false: the session refused it (back-pressure,
        // the engine stops reading until restartInput) -- the hook keeps it and the rest for resume()
        boolean push(Msg msg);

        // the connection failed: the reference's monitor event (0 for a V2 framing error, which
        // raises none), then error(ErrorReason.PROTOCOL) (StreamEngine.java:452-456)
        void failed(int event);

        // the hook needs another outEvent for this connection (socket backlog, or a message held
        // back by a full arena): StreamEngine sets POLLOUT (ioObject.setPollOut)
        void wantOutput();

        // the end of one loop's deliveries to this connection: StreamEngine flushes the session
        // (inEvent's session.flush(), StreamEngine.java:463-464)
        void delivered();

        // false while StreamEngine still has bytes of its own to write (the last handshake command,
        // outsize > 0): the sealed frames wait behind them
        boolean writable();
    }

    private static final class Conn
    {
        final int                  id;
        final Sink                 sink;
        final GatheringByteChannel out;
        Msg                        held;        // pulled but not queued (arena full): sent first next loop
        boolean                    queued;      // has messages in the current flushOut
        boolean                    received;    // has bytes for the current flushIn
        ByteBuffer                 backlog;     // wire bytes a non-blocking write left over
        ArrayDeque<Msg>            undelivered; // decoded messages the session has not taken yet
        boolean                    failed;
        boolean                    outputDead;  // a socket write failed: no more output (StreamEngine.java:518-524)

        Conn(int id, Sink sink, GatheringByteChannel out)
        {
            this.id = id;
            this.sink = sink;
            this.out = out;
        }
    }

    private final long       engine;
    private final List<Conn> conns   = new ArrayList<>();
    private final ByteBuffer readBuf;
    private final int[]      scratch = new int[1];

    // arenaBytes: pinned outbound payload arena (messages per loop); readBytes: receive buffer
    public GpuCurveIoHook(long arenaBytes, int readBytes, int device)
    {
        engine = GpuCurveEngine.create(arenaBytes, device);
        if (engine == 0) {
            throw new IllegalStateException("GpuCurveEngine.create failed (no MI355X visible?)");
        }
        readBuf = ByteBuffer.allocateDirect(readBytes);
    }

    // the hook Poller creates for its IO thread, or null when -Dzmq.curve.gpu is not true
    public static GpuCurveIoHook fromSystemProperties()
    {
        if (!Boolean.getBoolean(PROPERTY)) {
            return null;
        }
        return new GpuCurveIoHook(Long.getLong(PROPERTY + ".arena", 256L << 20),
                                  Integer.getInteger(PROPERTY + ".read", 1 << 20),
                                  Integer.getInteger(PROPERTY + ".device", 0));
    }

    // A pinned payload for an application send on an attached connection: the application writes
    // its bytes into the Msg and sends it; the engine seals it in place (no staging copy).  The bytes
    // belong to the engine's outbound arena, which is reused after the flush that sends the Msg, so
    // the Msg must be sent, once, before the next endOfLoop and not touched after.  Null when the
    // arena is full (send a heap Msg instead: it is copied once).  This is NOT a ZMQ_MSG_ALLOCATOR:
    // the reference hands that option to its decoders, i.e. to INBOUND frames
    // (StreamEngine.java:735-805, Decoder.java:102), whose lifetime the application controls.
    public Msg pinnedMsg(int size)
    {
        ByteBuffer b = GpuCurveEngine.msgAlloc(engine, size);
        return b != null ? new Msg(b) : null;
    }

    // A CURVE connection whose handshake is complete (mechanism.status() == READY): its cnPrecom and
    // nonce counters move into the engine, which seals and opens every MESSAGE from now on.  The
    // mechanism must not encode or decode another message after this call.
    public int attach(Mechanism mechanism, Sink sink, GatheringByteChannel out)
    {
        final boolean server;
        if (mechanism instanceof CurveServerMechanism) {
            server = true;
        }
        else if (mechanism instanceof CurveClientMechanism) {
            server = false;
        }
        else {
            throw new IllegalArgumentException("not a CURVE mechanism: " + mechanism);
        }
        byte[] precom = (byte[]) field(mechanism, "cnPrecom");
        long cnNonce = (Long) field(mechanism, "cnNonce");
        long cnPeerNonce = (Long) field(mechanism, "cnPeerNonce");
        int id = GpuCurveEngine.addConn(engine, server, precom, cnNonce, cnPeerNonce);
        if (id < 0) {
            throw new IllegalStateException("GpuCurveEngine.addConn: " + id);
        }
        while (conns.size() <= id) {
            conns.add(null);
        }
        conns.set(id, new Conn(id, sink, out));
        return id;
    }

    // The connection is gone (StreamEngine unplug / error): its queued and received data are
    // dropped and its engine id is reused by a later attach.
    public void detach(int conn)
    {
        Conn c = conns.get(conn);
        if (c == null) {
            return;
        }
        conns.set(conn, null);
        GpuCurveEngine.removeConn(engine, conn);
    }

    // CurveClientMechanism / CurveServerMechanism keep the session keys private
    // (CurveClientMechanism.java:46-49, CurveServerMechanism.java:34-47)
    private static Object field(Mechanism m, String name)
    {
        try {
            Field f = m.getClass().getDeclaredField(name);
            f.setAccessible(true);
            return f.get(m);
        }
        catch (ReflectiveOperationException e) {
            throw new IllegalStateException("CURVE mechanism field " + name, e);
        }
    }

    // StreamEngine.outEvent for an attached connection: pull every message the session has and
    // queue it for this loop's flush.  Nothing is sealed or written here.  True when something is
    // queued or held for a later loop.
    public boolean outEvent(int conn)
    {
        Conn c = conns.get(conn);
        if (c == null || c.failed || c.outputDead) {
            return false;
        }
        Msg msg = c.held != null ? c.held : c.sink.pull();
        c.held = null;
        while (msg != null) {
            if (!queue(c, msg)) {
                c.held = msg;      // the arena is full: this one leads the next loop
                return true;
            }
            if (c.failed) {
                return false;      // queue() tore the connection down: pull nothing more
            }
            msg = c.sink.pull();
        }
        return c.queued;
    }

    private boolean queue(Conn c, Msg msg)
    {
        final int size = msg.size();
        final int flags = (msg.hasMore() ? Msg.MORE : 0) | (msg.isCommand() ? Msg.COMMAND : 0);
        // Msg.buf() is a duplicate at the Msg's own position (not always 0, Msg.java:146-155): slice it,
        // so that the direct address the engine takes is the payload's first byte
        ByteBuffer payload = msg.buf().slice();
        payload.limit(size);
        if (!payload.isDirect()) {
            // a heap payload (not from pinnedMsg()): one copy into the arena
            ByteBuffer pinned = GpuCurveEngine.msgAlloc(engine, size);
            if (pinned == null) {
                return false;
            }
            pinned.put(payload);
            pinned.flip();
            payload = pinned;
        }
        int rc = GpuCurveEngine.send(engine, c.id, payload, size, flags);
        if (rc == CZ_ENOMEM) {
            return false;
        }
        if (rc != CZ_OK) {
            fail(c);
            return true;
        }
        c.queued = true;
        return true;
    }

    // StreamEngine.inEvent for an attached connection: read what the socket has into the engine.
    // Returns the bytes read, -1 at end of stream (the caller's error(ErrorReason.CONNECTION)).
    public int inEvent(int conn, ReadableByteChannel in) throws IOException
    {
        Conn c = conns.get(conn);
        int total = 0;
        while (true) {
            readBuf.clear();
            int n = in.read(readBuf);
            if (n < 0) {
                return total > 0 ? total : -1;
            }
            if (n == 0) {
                return total;
            }
            total += n;
            if (c == null || c.failed) {
                continue;          // drain the socket; the bytes of a failed connection go nowhere
            }
            if (GpuCurveEngine.recv(engine, c.id, readBuf, n) != CZ_OK) {
                fail(c);           // tears the connection down (StreamEngine.error): stop reading
                return total;
            }
            c.received = true;
        }
    }

    // Wire bytes StreamEngine's decoder had read past the frame that completed the handshake (the
    // peer's first MESSAGEs can share a TCP read with its READY): they start at a frame boundary and
    // go to the engine ahead of anything read later.
    public void handOver(int conn, ByteBuffer data, int len)
    {
        Conn c = conns.get(conn);
        if (c == null || c.failed || len <= 0) {
            return;
        }
        ByteBuffer src = data.duplicate();
        src.limit(src.position() + len);
        while (src.hasRemaining()) {
            readBuf.clear();
            int n = Math.min(readBuf.capacity(), src.remaining());
            ByteBuffer part = src.duplicate();
            part.limit(part.position() + n);
            readBuf.put(part);
            src.position(src.position() + n);
            if (GpuCurveEngine.recv(engine, c.id, readBuf, n) != CZ_OK) {
                fail(c);
                return;
            }
        }
        c.received = true;
    }

    // Once per poller loop: open and deliver every connection's received frames, then seal and
    // write every connection's queued messages -- in that order, so a reply queued during delivery
    // (a heartbeat PONG, StreamEngine.java:1217-1246) leaves in the same loop.  Returns the
    // connections whose output is not fully written or that hold a message back; each of those has
    // been asked for another outEvent (Sink.wantOutput).
    public List<Integer> endOfLoop() throws IOException
    {
        boolean anyIn = false;
        for (Conn c : conns) {
            anyIn |= c != null && c.received;
        }
        if (anyIn) {
            if (GpuCurveEngine.flushIn(engine) != CZ_OK) {
                throw new IOException("GpuCurveEngine.flushIn failed");
            }
            for (int i = 0; i < conns.size(); i++) {
                Conn c = conns.get(i);
                if (c == null || !c.received) {
                    continue;
                }
                c.received = false;
                deliver(c);
                if (conns.get(i) == c) {
                    c.sink.delivered();
                }
            }
        }
        List<Integer> blocked = new ArrayList<>();
        boolean anyOut = false;
        for (Conn c : conns) {
            anyOut |= c != null && c.queued;
        }
        if (!anyOut) {
            return blocked;
        }
        if (GpuCurveEngine.flushOut(engine) != CZ_OK) {
            throw new IOException("GpuCurveEngine.flushOut failed");
        }
        for (Conn c : conns) {
            if (c == null || !c.queued) {
                continue;
            }
            c.queued = false;
            boolean done;
            try {
                done = write(c);
            }
            catch (IOException e) {
                // as StreamEngine.outEvent on a write error: stop output, keep reading, so the input
                // side sees the disconnect and no incoming message is lost (:518-524)
                c.outputDead = true;
                c.backlog = null;
                continue;
            }
            if (!done || c.held != null) {
                blocked.add(c.id);
                c.sink.wantOutput();
            }
        }
        return blocked;
    }

    // the connection's sealed V2 frames in one gathering write of direct views of the pinned flush
    // output (StreamEngine.java:509-535); what a non-blocking socket does not take is copied aside,
    // because the next flushOut reuses the output
    private boolean write(Conn c) throws IOException
    {
        ByteBuffer[] pieces = GpuCurveEngine.wireIov(engine, c.id);
        if (pieces == null) {
            throw new IOException("GpuCurveEngine.wireIov failed");
        }
        if (!c.sink.writable()) {
            appendBacklog(c, pieces);   // the engine's own bytes leave first
            return false;
        }
        if (!writeBacklog(c)) {
            // earlier bytes are still waiting: these go behind them
            appendBacklog(c, pieces);
            return false;
        }
        long left = 0;
        for (ByteBuffer p : pieces) {
            left += p.remaining();
        }
        while (left > 0) {
            long n = c.out.write(pieces);
            if (n <= 0) {
                appendBacklog(c, pieces);
                return false;
            }
            left -= n;
        }
        return true;
    }

    // write bytes left over by an earlier loop; true when none are left
    public boolean writeBacklog(int conn) throws IOException
    {
        Conn c = conns.get(conn);
        return c == null || c.outputDead || writeBacklog(c);
    }

    private boolean writeBacklog(Conn c) throws IOException
    {
        if (c.backlog == null) {
            return true;
        }
        while (c.backlog.hasRemaining()) {
            if (c.out.write(c.backlog) <= 0) {
                return false;
            }
        }
        c.backlog = null;
        return true;
    }

    private static void appendBacklog(Conn c, ByteBuffer[] pieces)
    {
        int more = 0;
        for (ByteBuffer p : pieces) {
            more += p.remaining();
        }
        int have = c.backlog == null ? 0 : c.backlog.remaining();
        ByteBuffer b = ByteBuffer.allocate(have + more);
        if (c.backlog != null) {
            b.put(c.backlog);
        }
        for (ByteBuffer p : pieces) {
            b.put(p);
        }
        b.flip();
        c.backlog = b;
    }

    // the frames of the last flushIn in order, then the connection's failure if it has one: every
    // frame before the failing one is delivered, none after it (decodeAndPush returning false).  The
    // payloads are pinned engine memory valid until the next flushIn, so each becomes a heap Msg
    // (the reference's decoder also allocates per message); what the session refuses waits in
    // `undelivered` for resume().
    private void deliver(Conn c)
    {
        int n = GpuCurveEngine.msgsIn(engine, c.id);
        for (int i = 0; i < n; i++) {
            ByteBuffer p = GpuCurveEngine.msgIn(engine, c.id, i, scratch);
            byte[] data = new byte[p.remaining()];
            p.get(data);
            Msg msg = new Msg(data);
            if ((scratch[0] & Msg.MORE) != 0) {
                msg.setFlags(Msg.MORE);
            }
            if ((scratch[0] & Msg.COMMAND) != 0) {
                msg.setFlags(Msg.COMMAND);
            }
            if (c.undelivered != null) {
                c.undelivered.add(msg);
            }
            else if (!c.sink.push(msg)) {
                if (conns.get(c.id) != c) {
                    return;        // the push tore the connection down (StreamEngine.error -> detach)
                }
                c.undelivered = new ArrayDeque<>();
                c.undelivered.add(msg);
            }
        }
        if (conns.get(c.id) != c) {
            return;
        }
        if (!c.failed && GpuCurveEngine.connError(engine, c.id, scratch) != CZ_OK) {
            c.failed = true;
            c.sink.failed(scratch[0]);
        }
    }

    // StreamEngine.restartInput for an attached connection: push what the session refused earlier.
    // True when everything is delivered (the engine may read again).
    public boolean resume(int conn)
    {
        Conn c = conns.get(conn);
        if (c == null || c.undelivered == null) {
            return true;
        }
        while (!c.undelivered.isEmpty()) {
            if (!c.sink.push(c.undelivered.peekFirst())) {
                return false;
            }
            c.undelivered.pollFirst();
        }
        c.undelivered = null;
        return true;
    }

    private void fail(Conn c)
    {
        if (c.failed) {
            return;
        }
        c.failed = true;
        GpuCurveEngine.connError(engine, c.id, scratch);
        c.sink.failed(scratch[0]);
    }

    @Override
    public void close()
    {
        GpuCurveEngine.destroy(engine);
    }
}
