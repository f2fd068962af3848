// cz_handshake.cpp -- the handshake's public-key calls of Curve.java on the device.
//
//   Curve.keypair / keypairZ85 -> crypto_box_keypair   Curve.java:84-115
//   Curve.beforenm             -> crypto_box_beforenm  Curve.java:124-127
//   Curve.box                  -> crypto_box           Curve.java:183-193
//   Curve.open                 -> crypto_box_open      Curve.java:149-157
// jnacl's int contract: 0 on success, -1 on failure (no exceptions).  X25519 runs in k_x25519
// (cz_x25519.hip); box / box_open are beforenm followed by the afternm drop-ins.  The secret
// key of a new key pair comes from the OS CSPRNG (getrandom), like jnacl's SecureRandom.
#include <string.h>
#include <sys/random.h>

#include "cz_internal.h"

using namespace czi;

extern "C" hipError_t czk_x25519(const void *, const void *, void *, uint32_t, int, hipStream_t);

namespace {

struct HsCtx {
    bool ready = false;
    hipStream_t stream = nullptr;
    DevBuf buf;  // [0,32) scalar  [32,64) point  [64,96) out
};

thread_local HsCtx t_hs;

int hs_init()
{
    if (t_hs.ready)
        return CZ_OK;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0)
        return fail(CZ_EHIP, "no HIP device available (the CURVE path runs only on the GPU)");
    hipError_t e;
    if ((e = hipStreamCreateWithFlags(&t_hs.stream, hipStreamNonBlocking)) != hipSuccess ||
        (e = t_hs.buf.reserve(96)) != hipSuccess)
        return hip_fail(e, "handshake context");
    t_hs.ready = true;
    return CZ_OK;
}

// out = X25519(scalar, point) (point NULL = base point 9), or beforenm when `beforenm`
int hs_one(uint8_t out[32], const uint8_t scalar[32], const uint8_t *point, int beforenm)
{
    int rc = hs_init();
    if (rc != CZ_OK)
        return rc;
    uint8_t *d = (uint8_t *)t_hs.buf.ptr;
    hipError_t e;
    if ((e = hipMemcpyAsync(d, scalar, 32, hipMemcpyHostToDevice, t_hs.stream)) != hipSuccess ||
        (point && (e = hipMemcpyAsync(d + 32, point, 32, hipMemcpyHostToDevice, t_hs.stream)) != hipSuccess) ||
        (e = czk_x25519(d, point ? d + 32 : nullptr, d + 64, 1, beforenm, t_hs.stream)) != hipSuccess ||
        (e = hipMemcpyAsync(out, d + 64, 32, hipMemcpyDeviceToHost, t_hs.stream)) != hipSuccess) {
        // do not leave key material behind, on the error path either
        (void)hipMemsetAsync(d, 0, 96, t_hs.stream);
        (void)hipStreamSynchronize(t_hs.stream);
        return hip_fail(e, "x25519");
    }
    if ((e = hipMemsetAsync(d, 0, 96, t_hs.stream)) != hipSuccess ||  // do not leave key material behind
        (e = hipStreamSynchronize(t_hs.stream)) != hipSuccess)
        return hip_fail(e, "x25519");
    return CZ_OK;
}

}  // namespace

int czi::hs_thread_init() { return hs_init(); }

extern "C" {

int cz_scalarmult(uint8_t q[32], const uint8_t n[32], const uint8_t p[32])
{
    if (!q || !n || !p)
        return -1;
    return hs_one(q, n, p, 0) == CZ_OK ? 0 : -1;
}

int cz_box_keypair(uint8_t pk[32], uint8_t sk[32])
{
    if (!pk || !sk)
        return -1;
    size_t got = 0;
    while (got < 32) {
        ssize_t r = getrandom(sk + got, 32 - got, 0);
        if (r < 0) {
            fail(CZ_EINVAL, "cz_box_keypair: getrandom failed");
            return -1;
        }
        got += (size_t)r;
    }
    return hs_one(pk, sk, nullptr, 0) == CZ_OK ? 0 : -1;
}

int cz_box_beforenm(uint8_t k[32], const uint8_t pk[32], const uint8_t sk[32])
{
    if (!k || !pk || !sk)
        return -1;
    return hs_one(k, sk, pk, 1) == CZ_OK ? 0 : -1;
}

int cz_box(uint8_t *c, const uint8_t *m, uint64_t mlen, const uint8_t n[24], const uint8_t pk[32],
           const uint8_t sk[32])
{
    uint8_t k[32];
    if (cz_box_beforenm(k, pk, sk) != 0)
        return -1;
    int rc = cz_box_afternm(c, m, mlen, n, k);
    explicit_bzero(k, sizeof(k));
    return rc;
}

int cz_box_open(uint8_t *m, const uint8_t *c, uint64_t clen, const uint8_t n[24], const uint8_t pk[32],
                const uint8_t sk[32])
{
    uint8_t k[32];
    if (cz_box_beforenm(k, pk, sk) != 0)
        return -1;
    int rc = cz_box_open_afternm(m, c, clen, n, k);
    explicit_bzero(k, sizeof(k));
    return rc;
}

int cz_x25519_batch(const void *d_scalars, const void *d_points, void *d_out, uint32_t count, void *stream)
{
    if (count && (!d_scalars || !d_out))
        return fail(CZ_EINVAL, "cz_x25519_batch: null pointer");
    hipError_t e = czk_x25519(d_scalars, d_points, d_out, count, 0, (hipStream_t)stream);
    return e == hipSuccess ? CZ_OK : hip_fail(e, "cz_x25519_batch");
}

int cz_beforenm_batch(const void *d_pk, const void *d_sk, void *d_k, uint32_t count, void *stream)
{
    if (count && (!d_pk || !d_sk || !d_k))
        return fail(CZ_EINVAL, "cz_beforenm_batch: null pointer");
    hipError_t e = czk_x25519(d_sk, d_pk, d_k, count, 1, (hipStream_t)stream);
    return e == hipSuccess ? CZ_OK : hip_fail(e, "cz_beforenm_batch");
}

}  // extern "C"
