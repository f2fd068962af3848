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
// queues (GpuCurveEngine.recv); the poller calls endOfLoop() once per iteration, which seals every
// queued message of every connection (flushOut), writes each connection's wire bytes with one
// gathering write (wireIov), opens every received frame (flushIn) and delivers the payloads in
// order.  A connection whose frame fails (bad tag, replay, malformed, framing) gets the reference's
// monitor event (connError -> eventHandshakeFailedProtocol) and is torn down, as decodeAndPush
// returning false tears it down; the other connections carry on.
//
// StreamEngine keeps the rest of its role (handshake, heartbeats, metadata): it hands a connection
// to attach() once mechanism.status() == READY and implements Sink with its own pullMsg / decodeAndPush
// tail.  One hook per IO thread (the engine is not thread-safe).
package zmq.io;

import java.io.IOException;
import java.nio.ByteBuffer;
import java.nio.channels.GatheringByteChannel;
import java.nio.channels.ReadableByteChannel;
import java.lang.reflect.Field;
import java.util.ArrayList;
import java.util.List;

import zmq.Msg;
import zmq.io.mechanism.Mechanism;
import zmq.io.mechanism.curve.CurveClientMechanism;
import zmq.io.mechanism.curve.CurveServerMechanism;
import zmq.io.mechanism.curve.PinnedMsgAllocator;
import zmq.msg.MsgAllocator;

public final class GpuCurveIoHook implements AutoCloseable
{
    // library codes (include/curvezmq_mi355x.h)
    private static final int CZ_OK     = 0;
    private static final int CZ_ENOMEM = -12;

    // The StreamEngine side of one connection.
    public interface Sink
    {
        // the next message to send, or null (StreamEngine.pullAndEncode without the encode:
        // session.pullMsg, :1052-1063)
        Msg pull();

        // a decoded message (StreamEngine.decodeAndPush after mechanism.decode, :1072-1097: commands
        // to processCommand, metadata, session.pushMsg); false stops delivery on this connection
        boolean push(Msg msg);

        // the connection failed: the reference's monitor event (0 for a V2 framing error, which
        // raises none), then error(ErrorReason.PROTOCOL) (StreamEngine.java:452-456)
        void failed(int event);
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
        boolean                    failed;

        Conn(int id, Sink sink, GatheringByteChannel out)
        {
            this.id = id;
            this.sink = sink;
            this.out = out;
        }
    }

    private final long               engine;
    private final PinnedMsgAllocator allocator;
    private final List<Conn>         conns   = new ArrayList<>();
    private final ByteBuffer         readBuf;
    private final int[]              scratch = new int[1];

    // arenaBytes: pinned outbound payload arena (messages per loop); readBytes: receive buffer
    public GpuCurveIoHook(long arenaBytes, int readBytes, int device)
    {
        engine = GpuCurveEngine.create(arenaBytes, device);
        if (engine == 0) {
            throw new IllegalStateException("GpuCurveEngine.create failed (no MI355X visible?)");
        }
        allocator = PinnedMsgAllocator.overEngine(engine);
        readBuf = ByteBuffer.allocateDirect(readBytes);
    }

    // ZMQ_MSG_ALLOCATOR for the sockets this IO thread serves: payloads written into these Msgs are
    // sealed straight from the pinned arena
    public MsgAllocator allocator()
    {
        return allocator;
    }

    // A CURVE connection whose handshake is complete (mechanism.status() == READY): its cnPrecom and
    // nonce counters move into the engine, which seals and opens every MESSAGE from now on.
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
    // queue it for this loop's flush.  Nothing is sealed or written here.
    public void outEvent(int conn)
    {
        Conn c = conns.get(conn);
        if (c.failed) {
            return;
        }
        Msg msg = c.held != null ? c.held : c.sink.pull();
        c.held = null;
        while (msg != null) {
            if (!queue(c, msg)) {
                c.held = msg;      // the arena is full: this one leads the next loop
                return;
            }
            msg = c.sink.pull();
        }
    }

    private boolean queue(Conn c, Msg msg)
    {
        final int size = msg.size();
        final int flags = (msg.hasMore() ? Msg.MORE : 0) | (msg.isCommand() ? Msg.COMMAND : 0);
        ByteBuffer payload = msg.buf();   // position 0: Msg never moves its buffer's position
        if (!payload.isDirect()) {
            // a heap payload (not from allocator()): one copy into the arena
            ByteBuffer pinned = GpuCurveEngine.msgAlloc(engine, size);
            if (pinned == null) {
                return false;
            }
            payload.limit(size);
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
            if (!c.failed && GpuCurveEngine.recv(engine, c.id, readBuf, n) != CZ_OK) {
                fail(c);
            }
            c.received = true;
            total += n;
        }
    }

    // Once per poller loop: seal and write every connection's queued messages, open and deliver
    // every connection's received frames.  Returns the connections whose output is not fully written
    // (the caller keeps POLLOUT on them and calls writeBacklog from their next outEvent).
    public List<Integer> endOfLoop() throws IOException
    {
        List<Integer> blocked = new ArrayList<>();
        boolean anyOut = false;
        boolean anyIn = false;
        for (Conn c : conns) {
            if (c != null) {
                anyOut |= c.queued;
                anyIn |= c.received;
            }
        }
        if (anyOut) {
            if (GpuCurveEngine.flushOut(engine) != CZ_OK) {
                throw new IOException("GpuCurveEngine.flushOut failed");
            }
            for (Conn c : conns) {
                if (c == null || !c.queued) {
                    continue;
                }
                c.queued = false;
                if (!write(c)) {
                    blocked.add(c.id);
                }
            }
        }
        if (anyIn) {
            if (GpuCurveEngine.flushIn(engine) != CZ_OK) {
                throw new IOException("GpuCurveEngine.flushIn failed");
            }
            for (Conn c : conns) {
                if (c == null || !c.received) {
                    continue;
                }
                c.received = false;
                deliver(c);
            }
        }
        return blocked;
    }

    // the connection's sealed V2 frames in one gathering write of direct views of the pinned flush
    // output (StreamEngine.java:509-535); what a non-blocking socket does not take is copied aside,
    // because the next flushOut reuses the output
    private boolean write(Conn c) throws IOException
    {
        if (!writeBacklog(c)) {
            // earlier bytes are still waiting: these go behind them
            appendBacklog(c, GpuCurveEngine.wireIov(engine, c.id));
            return false;
        }
        ByteBuffer[] pieces = GpuCurveEngine.wireIov(engine, c.id);
        if (pieces == null) {
            throw new IOException("GpuCurveEngine.wireIov failed");
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
        return writeBacklog(conns.get(conn));
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
    // frame before the failing one is delivered, none after it (decodeAndPush returning false)
    private void deliver(Conn c)
    {
        int n = GpuCurveEngine.msgsIn(engine, c.id);
        for (int i = 0; i < n; i++) {
            ByteBuffer p = GpuCurveEngine.msgIn(engine, c.id, i, scratch);
            // the payload is pinned engine memory, valid until the next flushIn: the pipe may hold
            // the Msg longer, so it takes a copy (the reference's decoder also allocates per message)
            byte[] data = new byte[p.remaining()];
            p.get(data);
            Msg msg = new Msg(data);
            if ((scratch[0] & Msg.MORE) != 0) {
                msg.setFlags(Msg.MORE);
            }
            if ((scratch[0] & Msg.COMMAND) != 0) {
                msg.setFlags(Msg.COMMAND);
            }
            if (!c.sink.push(msg)) {
                break;
            }
        }
        if (!c.failed && GpuCurveEngine.connError(engine, c.id, scratch) != CZ_OK) {
            c.failed = true;
            c.sink.failed(scratch[0]);
        }
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
        allocator.close();
        GpuCurveEngine.destroy(engine);
    }
}
