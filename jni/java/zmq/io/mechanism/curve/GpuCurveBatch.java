// Batched host-staged CURVE seal / open on the MI355X (include/curvezmq_mi355x.h section 4,
// INTEGRATION.md section 3): the throughput path a batching Mechanism drives.  Buffers are direct
// ByteBuffers, pinned when they come from hostAlloc.  Return values are the library's CZ_* codes.
package zmq.io.mechanism.curve;

import java.nio.ByteBuffer;

public final class GpuCurveBatch
{
    static {
        System.loadLibrary("curvezmq_jni");
    }

    private GpuCurveBatch()
    {
    }

    public static native long create(int device);

    public static native void destroy(long ctx);

    // precoms: nkeys x 32-byte cnPrecom; direction 0 = client-to-server nonces, 1 = server-to-client
    public static native int setKeys(long ctx, ByteBuffer precoms, int nkeys, int direction);

    // descs: count x 40-byte cz_frame_desc, little-endian
    public static native int seal(long ctx, ByteBuffer descs, int count, ByteBuffer in, ByteBuffer out);

    public static native int open(long ctx, ByteBuffer descs, int count, ByteBuffer in, ByteBuffer out,
                                  ByteBuffer status);

    public static native int sealUniform(long ctx, int count, int len, ByteBuffer in, long inStride, ByteBuffer out,
                                         long outStride, long counter0, ByteBuffer flags, int chunkFrames);

    public static native int openUniform(long ctx, int count, int size, ByteBuffer in, long inStride, ByteBuffer out,
                                         long outStride, long floor0, boolean check, ByteBuffer status,
                                         int chunkFrames);

    public static native ByteBuffer hostAlloc(long bytes);

    public static native void hostFree(ByteBuffer buf);
}
