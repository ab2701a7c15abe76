/*
 * fgi_variants.h — options of the measurement build libfgi_variants.so (`make -C stl.fusion_amd/csrc
 * variant-all`). Each path below was built, tested parity-green and measured slower than the shipping
 * engine on MI355X, so the shipping libfgi.so leaves it out and returns FGI_ENOTSUP for
 * these options (any value but the default). The variant library exports the same C-ABI (include/fgi.h).
 * The cooperative launch of streaming cascades (environment FGI_COOP_LAUNCH=1) is in the variant build
 * only as well.
 */
#ifndef FGI_VARIANTS_H
#define FGI_VARIANTS_H
#include "fgi.h"

/* fgi_set_option:
 *   FGI_OPT_FUSED       [0]  VARIANT BUILD ONLY (libfgi_variants.so, `make variant-all`; the shipping
 *                            libfgi.so returns FGI_ENOTSUP for any value but 0).
 *                            1: waves whose directions are settled (pull lists ready, or push only)
 *                            run their roots and small push levels inside two persistent launches and
 *                            only the pull levels (and push levels over one round of the fused grid)
 *                            as separate launches, with one host synchronisation (DESIGN.md §3;
 *                            measured slower than the default level groups on MI355X). Tests add 2
 *                            (no prediction of the launches: extra rounds), 4 (every push level as its
 *                            own launch) or 8 (every push level in the fused grid); the environment's
 *                            FGI_FUSED=1 makes 1 the default
 *   FGI_OPT_PROBE_SUMMARY [-1] VARIANT BUILD ONLY (libfgi.so: FGI_ENOTSUP for any value but -1).
 *                            Before a pull level while few invalidated-bitmap words can be nonzero
 *                            (the invalidated count so far, by the levels' frontiers, under 1/8 of the
 *                            words), build a one-bit-per-64-bit-word summary and answer cold head /
 *                            tail probes of zero words from it, on graphs whose bitmap has at least
 *                            this many 64-bit words; 0 on any graph (tests), -1 never (the default:
 *                            measured slower on configs[2]; results never change)
 */
#define FGI_OPT_FUSED 12
#define FGI_OPT_PROBE_SUMMARY 15

#endif /* FGI_VARIANTS_H */
