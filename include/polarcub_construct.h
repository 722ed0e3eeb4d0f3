/* polarcub_construct.h -- C ABI of the host-side polar code construction
 * (libpolarcub_construct.so, plain C++, no GPU).
 *
 * Replaces the reference's Tal-Vardy degrading/upgrading construction
 * (SURVEY.md section 8(f) rank 3):
 *   pcub_bmd_merge_equivalent  BinaryMemorylessDistribution.mergeEquivalentSymbols
 *                              (removeZeroProbOutput + sortProbs + merge + normalize)
 *                              ScalarDistributions/BinaryMemorylessDistribution.py:167-208
 *   pcub_bmd_degrade           BinaryMemorylessDistribution.degrade(L), after the merge  :287-346
 *   pcub_bmd_upgrade           BinaryMemorylessDistribution.upgrade(L), after the merge  :348-427
 *   pcub_bin_construct         calcFrozenSet_degradingUpgrading's TV / Pe vectors        :624-680
 *   pcub_qmd_* / pcub_qary_construct  the q-ary construction (below)
 * Letters are [n][2] doubles (p(y, x=0), p(y, x=1)), the reference's probs rows.
 * Results are bit-identical to the reference (tests/test_construct.py).
 *
 * Return codes: 0, PCUB_EINVAL (bad arguments), or the Python exception the
 * reference raises on the same input: PCUB_EASSERT (AssertionError),
 * PCUB_EZERODIV (ZeroDivisionError), PCUB_EINDEX (IndexError: no letter of
 * positive probability), PCUB_EATTR (AttributeError: no neighbour to merge into).
 */
#ifndef POLARCUB_CONSTRUCT_H
#define POLARCUB_CONSTRUCT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#ifndef PCUB_EINVAL
#define PCUB_EINVAL (-1)
#endif
#define PCUB_EASSERT (-10)
#define PCUB_EZERODIV (-11)
#define PCUB_EINDEX (-12)
#define PCUB_EATTR (-13)

/* probs[n][2] -> out[*out_n][2] (out holds n letters); group[n] (optional): the
 * output letter each input letter went into, -1 for dropped zero-probability letters. */
int pcub_bmd_merge_equivalent(const double* probs, int64_t n, double* out, int64_t* out_n, int64_t* group);

/* merged[n][2] (output of the merge) -> at most L letters; group[n] (optional):
 * the output letter each merged letter went into. */
int pcub_bmd_degrade(const double* merged, int64_t n, int64_t L, double* out, int64_t* out_n, int64_t* group);

/* merged[n][2] -> at most L letters (each removed letter's mass is split onto
 * its two neighbours). */
int pcub_bmd_upgrade(const double* merged, int64_t n, int64_t L, double* out, int64_t* out_n);

/* Pe[2^n] of the degraded xy tree and TV[2^n] of the upgraded x tree (0 when
 * xprobs is NULL), leaves in u order; `threads` workers (< 1: all cores). */
int pcub_bin_construct(int32_t n, int64_t L, const double* xprobs, int64_t nx, const double* xyprobs, int64_t nxy,
                       double* TV, double* Pe, int32_t threads);

/* q-ary (ScalarDistributions/QaryMemorylessDistribution.py).  Distributions are [n][q] doubles
 * (probs[y][x]), 2 <= q <= 64.
 *   pcub_qmd_degrade     degrade(L) = degrade_dynamic :218-260 (one-hot binary channels degraded
 *                        to M = floor(L^(1/(q-1))) letters each, product re-indexing, zero rows
 *                        removed, normalised)
 *   pcub_qmd_upgrade     upgrade(L) = upgrade_dynamic :329-475
 *   pcub_qmd_error_prob  errorProb :53-61 and totalVariation :87-96
 *   pcub_qary_construct  calcTVAndPe_degradingUpgrading's TV / Pe vectors :934-991 (x tree
 *                        upgraded, xy tree degraded; TV = 0 when xprobs is NULL)
 * out holds out_cap rows; *out_n receives the row count (PCUB_EINVAL when it exceeds out_cap;
 * at most M^(q-1) <= L rows). */
int pcub_qmd_degrade(int32_t q, const double* probs, int64_t n, int64_t L, double* out, int64_t out_cap,
                     int64_t* out_n);
int pcub_qmd_upgrade(int32_t q, const double* probs, int64_t n, int64_t L, double* out, int64_t out_cap,
                     int64_t* out_n);
int pcub_qmd_error_prob(int32_t q, const double* probs, int64_t n, double* pe, double* tv);
int pcub_qary_construct(int32_t q, int32_t n, int64_t L, const double* xprobs, int64_t nx, const double* xyprobs,
                        int64_t nxy, double* TV, double* Pe, int32_t threads);

#ifdef __cplusplus
}
#endif

#endif
