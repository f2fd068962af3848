// cz_diag.h -- the one timing-diagnostic hook of the kernels, and the guard that keeps it out of
// the product library.
//
// -DCZ_DIAG_NOSTORE_ALL (an A/B build: tools/build_variant.sh NAME -DCZ_DIAG_NOSTORE_ALL) drops
// every emitter's line store (kept for one impossible data value), so the clock and time of a
// kernel can be measured without its HBM writes.  Its output is WRONG by
// construction.  jeromq_amd/build.py compiles the product library with -DCZ_PRODUCT_BUILD and
// refuses any extra flags for it, and this header refuses a diagnostic flag in a product build.
// (The other diagnostic builds of rounds 1-4 -- NOLOAD, NOTAG, L2STORE, NOSTORE, NOSHIFTROW -- and
// the measured-and-rejected variants are in the git history, with their logs cited in DESIGN.md.)
#pragma once

#if defined(CZ_PRODUCT_BUILD) && defined(CZ_DIAG_NOSTORE_ALL)
#error "CZ_DIAG_NOSTORE_ALL writes wrong bytes: never in the product library (build with CZ_LIB_OUT=<A/B path>)"
#endif

// -DCZ_DIAG_CLOCK (round 6) stamps s_memtime / s_memrealtime per wave of k_seal_uniform into a
// device array (cz_diag_clock_read): correct output, but an extra store per wave, so A/B builds only.
#if defined(CZ_PRODUCT_BUILD) && defined(CZ_DIAG_CLOCK)
#error "CZ_DIAG_CLOCK is a measurement build: never in the product library"
#endif

#ifdef CZ_DIAG_NOSTORE_ALL
#define CZ_DIAG_STORE_GUARD(v) if ((v).x == 0x13579bdfu && (v).w == 0x2468ace0u)
#else
#define CZ_DIAG_STORE_GUARD(v)
#endif
