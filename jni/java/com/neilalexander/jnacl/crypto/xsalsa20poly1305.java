// Replacement of jnacl's secretbox class, imported by zmq/io/mechanism/curve/Curve.java:6 (the
// handshake's cookie boxes, Curve.java:159-181).  Bodies in jni/curvezmq_jni.c.
package com.neilalexander.jnacl.crypto;

public final class xsalsa20poly1305
{
    static {
        System.loadLibrary("curvezmq_jni");
    }

    private xsalsa20poly1305()
    {
    }

    public static native int crypto_secretbox(byte[] c, byte[] m, int mlen, byte[] n, byte[] k);

    public static native int crypto_secretbox_open(byte[] m, byte[] c, int clen, byte[] n, byte[] k);
}
