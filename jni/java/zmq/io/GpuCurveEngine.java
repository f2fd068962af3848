// The multi-connection batching engine (include/curvezmq_mi355x.h section 8): one per IO thread,
// replacing StreamEngine's encode + V2Encoder and V2Decoder + decode loops
// (StreamEngine.java:379-535) for CURVE connections in the CONNECTED state.
package zmq.io;

import java.nio.ByteBuffer;

public final class GpuCurveEngine
{
    static {
        System.loadLibrary("curvezmq_jni");
    }

    private GpuCurveEngine()
    {
    }

    public static native long create(long arenaBytes, int device);

    public static native void destroy(long e);

    public static native int addConn(long e, boolean server, byte[] precom, long cnNonce, long cnPeerNonce);

    // the connection is gone (StreamEngine unplug / error): its id is reused by a later addConn
    public static native int removeConn(long e, int conn);

    public static native ByteBuffer msgAlloc(long e, int len);

    public static native int send(long e, int conn, ByteBuffer payload, int len, int flags);

    public static native int flushOut(long e);

    public static native ByteBuffer wireOut(long e, int conn);

    public static native ByteBuffer[] wireIov(long e, int conn);

    public static native int recv(long e, int conn, ByteBuffer wire, int len);

    public static native int flushIn(long e);

    public static native int msgsIn(long e, int conn);

    public static native ByteBuffer msgIn(long e, int conn, int i, int[] flags);

    public static native int connError(long e, int conn, int[] event);
}
