// Replacement of jnacl's class (eu.neilalexander:jnacl:1.0.0), imported by
// zmq/io/mechanism/curve/Curve.java:5.  Same names and int contract (0 / -1); the bodies run on
// the MI355X through jni/curvezmq_jni.c -> libcurvezmq_mi355x.so.  Ship in a jar ahead of jnacl.
package com.neilalexander.jnacl.crypto;

public final class curve25519xsalsa20poly1305
{
    public static final int crypto_secretbox_NONCEBYTES = 24;
    public static final int crypto_secretbox_ZEROBYTES = 32;
    public static final int crypto_secretbox_BOXZEROBYTES = 16;
    public static final int crypto_secretbox_PUBLICKEYBYTES = 32;
    public static final int crypto_secretbox_SECRETKEYBYTES = 32;
    public static final int crypto_secretbox_BEFORENMBYTES = 32;

    static {
        System.loadLibrary("curvezmq_jni");
    }

    private curve25519xsalsa20poly1305()
    {
    }

    public static native int crypto_box_afternm(byte[] c, byte[] m, int mlen, byte[] n, byte[] k);

    public static native int crypto_box_open_afternm(byte[] m, byte[] c, int clen, byte[] n, byte[] k);

    public static native int crypto_box_beforenm(byte[] k, byte[] pk, byte[] sk);

    public static native int crypto_box(byte[] c, byte[] m, int mlen, byte[] n, byte[] pk, byte[] sk);

    public static native int crypto_box_open(byte[] m, byte[] c, int clen, byte[] n, byte[] pk, byte[] sk);

    public static native int crypto_box_keypair(byte[] pk, byte[] sk);
}
