// A pinned MsgAllocator for CURVE sockets on the MI355X path (zmq/msg/MsgAllocator.java:5-8, set
// with the ZMQ_MSG_ALLOCATOR option, zmq/ZMQ.java:156, read by Options at zmq/Options.java:471-493).
// A payload the application writes into one of these Msgs is already in pinned host memory, so the
// batched seal reads it over PCIe with no staging copy:
//   - overEngine(e): payloads carved from a GpuCurveEngine's pinned arena (cz_engine_msg_alloc);
//     GpuCurveEngine.send of such a Msg copies nothing.  The arena is reused by the engine after
//     each flushOut.
//   - overHostSlabs(bytes): payloads carved from pinned slabs of GpuCurveBatch.hostAlloc
//     (cz_host_alloc), for a batching Mechanism that drives GpuCurveBatch.seal / sealUniform;
//     reset() hands the slabs out again once the batch that used them has been sealed.
// When the pinned memory is exhausted a Msg comes from the heap (MsgAllocatorHeap), as
// MsgAllocatorThreshold falls back (zmq/msg/MsgAllocatorThreshold.java:25-33); such a payload is
// copied once into the arena when it is sent.
package zmq.io.mechanism.curve;

import java.nio.ByteBuffer;
import java.util.ArrayList;
import java.util.List;

import zmq.Msg;
import zmq.io.GpuCurveEngine;
import zmq.msg.MsgAllocator;
import zmq.msg.MsgAllocatorHeap;

public final class PinnedMsgAllocator implements MsgAllocator, AutoCloseable
{
    public static final long DEFAULT_SLAB_BYTES = 64L << 20;

    private final long             engine;    // != 0: carve from this engine's arena
    private final long             slabBytes; // engine == 0: size of each pinned slab
    private final List<ByteBuffer> slabs = new ArrayList<>();
    private final List<ByteBuffer> large = new ArrayList<>(); // payloads above slabBytes, freed at reset()
    private final MsgAllocator     heap  = new MsgAllocatorHeap();
    private int                    slab;      // slab being carved
    private long                   carved;    // bytes of it handed out

    private PinnedMsgAllocator(long engine, long slabBytes)
    {
        this.engine = engine;
        this.slabBytes = slabBytes;
    }

    public static PinnedMsgAllocator overEngine(long engine)
    {
        if (engine == 0) {
            throw new IllegalArgumentException("no engine");
        }
        return new PinnedMsgAllocator(engine, 0);
    }

    public static PinnedMsgAllocator overHostSlabs(long slabBytes)
    {
        if (slabBytes <= 0 || slabBytes > Integer.MAX_VALUE) {
            throw new IllegalArgumentException("slab size " + slabBytes);
        }
        return new PinnedMsgAllocator(0, slabBytes);
    }

    @Override
    public Msg allocate(int size)
    {
        ByteBuffer b = engine != 0 ? GpuCurveEngine.msgAlloc(engine, size) : carve(size);
        return b != null ? new Msg(b) : heap.allocate(size);
    }

    // a direct view of `size` pinned bytes, 16-byte aligned within its slab (the batch kernels read
    // 16-byte aligned payloads fastest); null when no pinned memory is left
    private ByteBuffer carve(int size)
    {
        if (size > slabBytes) {
            ByteBuffer own = GpuCurveBatch.hostAlloc(size);
            if (own != null) {
                large.add(own);
            }
            return own;
        }
        long at = (carved + 15) & ~15L;
        if (slab < slabs.size() && at + size > slabBytes) {
            slab++;
            at = 0;
        }
        if (slab == slabs.size()) {
            ByteBuffer s = GpuCurveBatch.hostAlloc(slabBytes);
            if (s == null) {
                return null;
            }
            slabs.add(s);
            at = 0;
        }
        ByteBuffer v = slabs.get(slab).duplicate();
        v.position((int) at);
        v.limit((int) at + size);
        carved = at + size;
        return v.slice();
    }

    // Every Msg handed out since the last reset() has been sealed (GpuCurveBatch.seal / sealUniform
    // returned): its pinned bytes may be handed out again.  Over an engine the arena is the engine's
    // to recycle, so this only frees payloads that took their own pinned buffer.
    public void reset()
    {
        for (ByteBuffer b : large) {
            GpuCurveBatch.hostFree(b);
        }
        large.clear();
        slab = 0;
        carved = 0;
    }

    @Override
    public void close()
    {
        reset();
        for (ByteBuffer s : slabs) {
            GpuCurveBatch.hostFree(s);
        }
        slabs.clear();
    }
}
