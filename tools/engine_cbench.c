/* engine_cbench.c -- the batching-engine bench (bench.py --config engine) from C, without torch in
 * the process, so the library runs on the system HIP runtime (/opt/rocm) as a JNI deployment
 * would.  1024 connections x 256 MESSAGEs of 4 KiB: flush_out, then the wire streams fed to a
 * server engine and flush_in; prints the best of 3 rounds.
 *   gcc -O2 tools/engine_cbench.c -Iinclude -Ljeromq_amd -lcurvezmq_mi355x -Wl,-rpath,$PWD/jeromq_amd */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "curvezmq_mi355x.h"

static double now(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

#define CHECK(x)                                                        \
    do {                                                                \
        int rc_ = (x);                                                  \
        if (rc_ < 0) {                                                  \
            fprintf(stderr, "%s -> %d: %s\n", #x, rc_, cz_last_error()); \
            return 1;                                                   \
        }                                                               \
    } while (0)

int main(int argc, char **argv)
{
    const int nconn = argc > 1 ? atoi(argv[1]) : 1024, per = 256;
    const uint32_t n = 4096;
    const uint64_t total = (uint64_t)nconn * per * n;
    cz_engine *cli, *srv;
    CHECK(cz_engine_create(&cli, total + (1 << 20), 0));
    CHECK(cz_engine_create(&srv, 1 << 20, 0));
    int *cc = malloc(sizeof(int) * nconn), *sc = malloc(sizeof(int) * nconn);
    for (int c = 0; c < nconn; c++) {
        uint8_t key[32];
        for (int j = 0; j < 32; j++)
            key[j] = (uint8_t)(j * 7 + c);
        CHECK(cc[c] = cz_engine_add_conn(cli, 0, key, 3, 0));
        CHECK(sc[c] = cz_engine_add_conn(srv, 1, key, 3, 0));
    }
    uint8_t *payload = malloc(n);
    for (uint32_t i = 0; i < n; i++)
        payload[i] = (uint8_t)(i * 131 + 7);
    double best_out = 1e9, best_in = 1e9;
    for (int rep = 0; rep < 3; rep++) {
        for (int c = 0; c < nconn; c++)
            for (int k = 0; k < per; k++) {
                void *buf = cz_engine_msg_alloc(cli, n);
                if (!buf)
                    return fprintf(stderr, "arena full\n"), 1;
                memcpy(buf, payload, n);
                CHECK(cz_engine_send(cli, cc[c], buf, n, (k % 8 == 0) ? CZ_MSG_MORE : 0));
            }
        double t0 = now();
        CHECK(cz_engine_flush_out(cli));
        double t_out = now() - t0;
        for (int c = 0; c < nconn; c++) {
            const uint8_t *w;
            uint64_t len;
            CHECK(cz_engine_wire_out(cli, cc[c], &w, &len));
            CHECK(cz_engine_recv(srv, sc[c], w, len));
        }
        t0 = now();
        CHECK(cz_engine_flush_in(srv));
        double t_in = now() - t0;
        for (int c = 0; c < nconn; c++) {
            uint32_t cnt = 0;
            int ev = 0;
            CHECK(cz_engine_msgs_in(srv, sc[c], &cnt));
            if (cnt != (uint32_t)per || cz_engine_conn_error(srv, sc[c], &ev))
                return fprintf(stderr, "connection %d: %u messages, error\n", c, cnt), 1;
        }
        const uint8_t *p;
        uint32_t len;
        int fl;
        CHECK(cz_engine_msg_in(srv, sc[nconn - 1], per - 1, &p, &len, &fl));
        if (len != n || memcmp(p, payload, n))
            return fprintf(stderr, "payload mismatch\n"), 1;
        if (t_out < best_out)
            best_out = t_out;
        if (t_in < best_in)
            best_in = t_in;
    }
    printf("{\"flush_out_ms\": %.2f, \"out_GiBps\": %.2f, \"flush_in_ms\": %.2f, \"in_GiBps\": %.2f}\n",
           best_out * 1e3, total / best_out / 1073741824.0, best_in * 1e3, total / best_in / 1073741824.0);
    cz_engine_destroy(cli);
    cz_engine_destroy(srv);
    return 0;
}
