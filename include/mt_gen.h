/*
 * mt_gen.h — synthetic conflict-farm op-log generator parameters (shared by the
 * GPU generator kernel and the test oracle's generator).
 *
 * The generator is the build's stand-in for the reference's farm harness
 * (merge-tree/src/test/mergeTreeOperationRunner.ts:97-179 + testServer.ts:108-121):
 * C writer clients issue ops against their own view (refSeq, clientId); the
 * sequencer stamps seq = 1..N and msn = min over clients of their last refSeq
 * (deli rule, server/routerlicious/packages/lambdas/src/deli/lambda.ts:448-453).
 * Positions are drawn from the issuer's view length getLength(refSeq, client),
 * computed by replaying the log as the passive observer does
 * (mergeTreeOperationRunner.ts:107-118: "client 0 ... is our baseline").
 *
 * The random-number stream and draw order are specified exactly in DESIGN.md
 * ("Synthetic op logs"); both implementations must produce identical logs.
 */
#ifndef MT_GEN_H
#define MT_GEN_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mt_gen_params {
    int32_t n_ops;       /* ops per document (seq = 1..n_ops)                       */
    int32_t n_clients;   /* writer clients, short ids 1..n_clients (long "A","B",..) */
    int32_t max_lag;     /* refSeq lag drawn uniformly from [0, max_lag]            */
    int32_t pct_insert;  /* op mix in percent; annotate = 100 - insert - remove      */
    int32_t pct_remove;
    int32_t min_len;     /* view length below this forces an insert (farm rule)     */
    int32_t max_insert;  /* insert text length drawn from [1, max_insert]           */
    int32_t pct_newline; /* per-character probability (%) of '\n'                   */
    uint64_t seed;
} mt_gen_params;

/* fixed interned tables used by generated logs */
#define MT_GEN_N_KEYS 4     /* 0 "bold", 1 "italic", 2 "color", 3 "size"              */
#define MT_GEN_N_VALUES 22  /* 0 null, 1 true, 2 "red", 3 "green", 4 "blue", 5..21 = 8..24 */

/* the same functions serve the gcc-built test oracle and the HIP kernels */
#ifdef __HIPCC__
#define MT_GEN_FN static inline __host__ __device__
#else
#define MT_GEN_FN static inline
#endif

MT_GEN_FN uint64_t mt_rng_next(uint64_t *x) {
    uint64_t z = (*x += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
/* uniform draw in [0, n), n >= 1 */
MT_GEN_FN uint32_t mt_rng_below(uint64_t *x, uint32_t n) {
    return (uint32_t)(((mt_rng_next(x) >> 32) * (uint64_t)n) >> 32);
}
MT_GEN_FN uint64_t mt_rng_seed(uint64_t seed, uint64_t doc) {
    return seed ^ (doc * 0xD1B54A32D192ED03ull) ^ 0x5851F42D4C957F2Dull;
}

#ifdef __cplusplus
}
#endif
#endif
