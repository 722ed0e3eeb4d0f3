/*
 * sc_oracle.c -- CPU restatement of the reference polar SC algorithm.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity oracle for the HIP
 * kernels in polarcub_amd/csrc.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it, and only as the checker or as the
 * timed CPU baseline -- never as a product code path.
 *
 * Pinned against golden vectors produced by the shimmed reference itself
 * (oracle/make_golden.py writes the tests/golden npz fixtures; tests/test_oracle.py).
 *
 * What it restates (paths relative to benjilieber/polarcub):
 *   binary SC recursion  BinaryPolarEncoderDecoder.py:223-325
 *   f / g butterflies     VectorDistributions/BinaryMemorylessVectorDistribution.py:15-47
 *   leaf marginal         VectorDistributions/BinaryMemorylessVectorDistribution.py:52-69
 *   max-normalisation     VectorDistributions/BinaryMemorylessVectorDistribution.py:71-87
 *   q-ary SC recursion    QaryPolarEncoderDecoder.py:318-401
 *   q-ary butterflies     VectorDistributions/QaryMemorylessVectorDistribution.py:26-64
 *   q-ary sum-normalise   VectorDistributions/QaryMemorylessVectorDistribution.py:69-118
 *
 * Arithmetic is IEEE binary64 evaluated in the reference's operation order.
 * It MUST be compiled with -ffp-contract=off (see oracle/Makefile): a fused
 * multiply-add changes the rounding of a0*b0 + a1*b1.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define PCUB_ORC_API __attribute__((visibility("default")))

/* ------------------------------------------------------------------------ */
/* binary memoryless vector distribution: probs[i][x] stored as p[2*i + x]   */
/* ------------------------------------------------------------------------ */

/* BinaryMemorylessVectorDistribution.py:15-29 */
static void bin_minus(const double* p, int len, double* out) {
    for (int h = 0; h < len / 2; ++h) {
        const double* a = p + 4 * h;
        const double* b = a + 2;
        out[2 * h + 0] = a[0] * b[0] + a[1] * b[1];
        out[2 * h + 1] = a[0] * b[1] + a[1] * b[0];
    }
}

/* BinaryMemorylessVectorDistribution.py:31-47 */
static void bin_plus(const double* p, int len, const uint8_t* u, double* out) {
    for (int h = 0; h < len / 2; ++h) {
        const double* a = p + 4 * h;
        const double* b = a + 2;
        if (u[h] == 0) {
            out[2 * h + 0] = a[0] * b[0];
            out[2 * h + 1] = a[1] * b[1];
        } else {
            out[2 * h + 0] = a[1] * b[0];
            out[2 * h + 1] = a[0] * b[1];
        }
    }
}

/* calcNormalizationVector :71-77 (np.maximum) then normalize :79-87 */
static void bin_normalize(double* p, int len) {
    for (int i = 0; i < len; ++i) {
        double t = p[2 * i] >= p[2 * i + 1] ? p[2 * i] : p[2 * i + 1];
        if (t == 0.0) t = 1.0;
        p[2 * i] /= t;
        p[2 * i + 1] /= t;
    }
}

/* calcMarginalizedProbabilities :52-69 */
static void bin_marginal(const double* p, double m[2]) {
    double s = 0.0;
    s += p[0];
    s += p[1];
    if (s > 0.0) {
        m[0] = p[0] / s;
        m[1] = p[1] / s;
    } else {
        m[0] = 0.5;
        m[1] = 0.5;
    }
}

typedef struct {
    const uint8_t* frozen; /* u8[N], 1 = frozen */
    const double* r;       /* common randomness r_i, or NULL (=> all frozen bits from uniform prior: 0.5 >= r_i) */
    const uint8_t* fval;   /* precomputed frozen values (used when r == NULL) */
    uint8_t* info;         /* decoded info bits (decode) / info bits to encode (encode) */
    double* leaf_m;        /* optional [N][2]: marginal used for the decision at each leaf */
    int u_index;
    int info_index;
    uint8_t* bits;         /* scratch for partial sums, 2N bytes */
} bin_ctx;

/* BinaryPolarEncoderDecoder.py:223-325.  x: a-priori tree (may be NULL = uniform
 * prior, every x-tree node is then exactly (1,1) after normalisation and the
 * leaf marginal is (0.5,0.5)); xy: a-posteriori tree (NULL = encoding). */
static void bin_rec(bin_ctx* c, const double* x, const double* xy, int len, uint8_t* enc, double* work,
                    uint8_t* bits) {
    if (len == 1) {
        int ui = c->u_index;
        if (!c->frozen[ui]) {
            double m[2];
            if (xy) {
                bin_marginal(xy, m);
                c->info[c->info_index] = (m[0] >= m[1]) ? 0 : 1;
                if (c->leaf_m) { c->leaf_m[2 * ui] = m[0]; c->leaf_m[2 * ui + 1] = m[1]; }
            }
            enc[0] = c->info[c->info_index];
            c->info_index++;
        } else {
            double m[2];
            if (x) bin_marginal(x, m); else { m[0] = 0.5; m[1] = 0.5; }
            if (c->r)
                enc[0] = (m[0] >= c->r[ui]) ? 0 : 1;
            else
                enc[0] = c->fval[ui];
            if (c->leaf_m) {
                if (xy) bin_marginal(xy, c->leaf_m + 2 * ui);
                else { c->leaf_m[2 * ui] = m[0]; c->leaf_m[2 * ui + 1] = m[1]; }
            }
        }
        c->u_index++;
        return;
    }
    int half = len / 2;
    double* xm = work;               /* half pairs */
    double* xym = work + 2 * half;   /* half pairs */
    double* sub = work + 4 * half;   /* child's scratch */
    uint8_t* um = bits;
    uint8_t* up = bits + half;

    if (x) { bin_minus(x, len, xm); bin_normalize(xm, half); }
    if (xy) { bin_minus(xy, len, xym); bin_normalize(xym, half); }
    bin_rec(c, x ? xm : NULL, xy ? xym : NULL, half, um, sub, bits + len);

    if (x) { bin_plus(x, len, um, xm); bin_normalize(xm, half); }
    if (xy) { bin_plus(xy, len, um, xym); bin_normalize(xym, half); }
    bin_rec(c, x ? xm : NULL, xy ? xym : NULL, half, up, sub, bits + len);

    for (int h = 0; h < half; ++h) {
        enc[2 * h] = (uint8_t)((um[h] + up[h]) % 2);
        enc[2 * h + 1] = up[h];
    }
}

static size_t bin_work_doubles(int n) { return (size_t)8 << n; }

/* Decode one codeword.  xy: [N][2] joint probabilities (never modified).
 * xprior: [N][2] a-priori distribution or NULL for a uniform prior.
 * r: common randomness [N] or NULL, in which case fval supplies the frozen
 * values directly (they must then equal (0.5 >= r_i) ? 0 : 1).
 * Returns the number of info bits written. */
PCUB_ORC_API int orc_sc_decode_bin(int log2N, const double* xy, const double* xprior,
                                    const uint8_t* frozen, const double* r, const uint8_t* fval,
                                    uint8_t* info, uint8_t* xhat, double* leaf_m) {
    int N = 1 << log2N;
    double* work = (double*)malloc(bin_work_doubles(log2N) * sizeof(double));
    uint8_t* bits = (uint8_t*)malloc(2 * (size_t)N);
    bin_ctx c = {frozen, r, fval, info, leaf_m, 0, 0, bits};
    bin_rec(&c, xprior, xy, N, xhat, work, bits);
    free(bits);
    free(work);
    return c.info_index;
}

/* Batch of B codewords, xy laid out [B][N][2]; info [B][K]; xhat [B][N]. */
PCUB_ORC_API void orc_sc_decode_bin_batch(int log2N, int64_t B, const double* xy, const uint8_t* frozen,
                                          const uint8_t* fval, int K, uint8_t* info, uint8_t* xhat,
                                          double* leaf_m) {
    int N = 1 << log2N;
    double* work = (double*)malloc(bin_work_doubles(log2N) * sizeof(double));
    uint8_t* bits = (uint8_t*)malloc(2 * (size_t)N);
    for (int64_t b = 0; b < B; ++b) {
        bin_ctx c = {frozen, NULL, fval, info + b * K, leaf_m ? leaf_m + b * 2 * N : NULL, 0, 0, bits};
        bin_rec(&c, NULL, xy + b * 2 * N, N, xhat + b * N, work, bits);
    }
    free(bits);
    free(work);
}

/* Encode (BinaryPolarEncoderDecoder.py:46-69): the same recursion with xy == NULL. */
PCUB_ORC_API void orc_encode_bin(int log2N, const double* xprior, const uint8_t* frozen, const double* r,
                                 const uint8_t* fval, const uint8_t* info, uint8_t* x) {
    int N = 1 << log2N;
    double* work = (double*)malloc(bin_work_doubles(log2N) * sizeof(double));
    uint8_t* bits = (uint8_t*)malloc(2 * (size_t)N);
    bin_ctx c = {frozen, r, fval, (uint8_t*)info, NULL, 0, 0, bits};
    bin_rec(&c, xprior, NULL, N, x, work, bits);
    free(bits);
    free(work);
}

/* polarTransformOfBits (BinaryPolarEncoderDecoder.py:494-516): x -> u. */
PCUB_ORC_API void orc_polar_transform_bits(int log2N, const uint8_t* x, uint8_t* u) {
    int N = 1 << log2N;
    if (N == 1) { u[0] = x[0]; return; }
    int half = N / 2;
    uint8_t* v = (uint8_t*)malloc((size_t)N);
    for (int i = 0; i < half; ++i) {
        v[i] = (uint8_t)((x[2 * i] + x[2 * i + 1]) % 2);
        v[half + i] = x[2 * i + 1];
    }
    orc_polar_transform_bits(log2N - 1, v, u);
    orc_polar_transform_bits(log2N - 1, v + half, u + half);
    free(v);
}

/* ------------------------------------------------------------------------ */
/* q-ary memoryless: probs[i][x] stored as p[q*i + x]                        */
/* ------------------------------------------------------------------------ */

/* QaryMemorylessVectorDistribution.py:26-43 (linear domain) */
static void q_minus(int q, const double* p, int len, double* out) {
    for (int h = 0; h < len / 2; ++h) {
        const double* a = p + (size_t)q * (2 * h);
        const double* b = a + q;
        double* o = out + (size_t)q * h;
        for (int u = 0; u < q; ++u) o[u] = 0.0;
        for (int x1 = 0; x1 < q; ++x1)
            for (int x2 = 0; x2 < q; ++x2) {
                int u1 = (x1 + x2) % q;
                o[u1] = o[u1] + a[x1] * b[x2];
            }
    }
}

/* QaryMemorylessVectorDistribution.py:45-64 */
static void q_plus(int q, const double* p, int len, const uint8_t* um, double* out) {
    for (int h = 0; h < len / 2; ++h) {
        const double* a = p + (size_t)q * (2 * h);
        const double* b = a + q;
        double* o = out + (size_t)q * h;
        for (int u2 = 0; u2 < q; ++u2) {
            int x1 = (um[h] + u2) % q;
            int x2 = (q - u2) % q;
            o[u2] = 0.0 + a[x1] * b[x2];
        }
    }
}

/* calcNormalizationVector :92-102 (python sum, left to right) + normalize :104-118 */
static void q_normalize(int q, double* p, int len) {
    for (int i = 0; i < len; ++i) {
        double* r = p + (size_t)q * i;
        double t = 0.0;
        for (int x = 0; x < q; ++x) t = t + r[x];
        if (t != 0.0)
            for (int x = 0; x < q; ++x) r[x] /= t;
    }
}

typedef struct {
    int q;
    const uint8_t* frozen;
    uint8_t* info;
    double* leaf_m;
    int u_index;
    int info_index;
} q_ctx;

/* QaryPolarEncoderDecoder.py:318-401.  The x-tree is computed by the reference
 * but never consulted (frozen symbols are fixed to 0, :347-351), so it is
 * omitted here. */
static void q_rec(q_ctx* c, const double* xy, int len, uint8_t* enc, double* work) {
    int q = c->q;
    if (len == 1) {
        int ui = c->u_index;
        if (!c->frozen[ui]) {
            if (xy) {
                /* calcMarginalizedProbabilities :69-90 then np.argmax (first max) */
                double s = 0.0;
                for (int x = 0; x < q; ++x) s = s + xy[x];
                double best = 0.0;
                int arg = 0;
                for (int x = 0; x < q; ++x) {
                    double m = (s > 0.0) ? xy[x] / s : 1.0 / (double)q;
                    if (c->leaf_m) c->leaf_m[(size_t)q * ui + x] = m;
                    if (x == 0 || m > best) { best = m; arg = x; }
                }
                c->info[c->info_index] = (uint8_t)arg;
            }
            enc[0] = c->info[c->info_index];
            c->info_index++;
        } else {
            enc[0] = 0;
        }
        c->u_index++;
        return;
    }
    int half = len / 2;
    double* ch = work;
    double* sub = work + (size_t)q * half;
    uint8_t* um = (uint8_t*)malloc((size_t)half);
    uint8_t* up = (uint8_t*)malloc((size_t)half);
    if (xy) { q_minus(q, xy, len, ch); q_normalize(q, ch, half); }
    q_rec(c, xy ? ch : NULL, half, um, sub);
    if (xy) { q_plus(q, xy, len, um, ch); q_normalize(q, ch, half); }
    q_rec(c, xy ? ch : NULL, half, up, sub);
    for (int h = 0; h < half; ++h) {
        enc[2 * h] = (uint8_t)((um[h] + up[h]) % q);
        enc[2 * h + 1] = (uint8_t)((q - up[h]) % q);
    }
    free(um);
    free(up);
}

PCUB_ORC_API int orc_sc_decode_qary(int q, int log2N, const double* xy, const uint8_t* frozen, uint8_t* info,
                                     uint8_t* xhat, double* leaf_m) {
    int N = 1 << log2N;
    double* work = (double*)malloc((size_t)q * 4 * (size_t)N * sizeof(double));
    q_ctx c = {q, frozen, info, leaf_m, 0, 0};
    q_rec(&c, xy, N, xhat, work);
    free(work);
    return c.info_index;
}

PCUB_ORC_API void orc_sc_decode_qary_batch(int q, int log2N, int64_t B, const double* xy, const uint8_t* frozen,
                                           int K, uint8_t* info, uint8_t* xhat) {
    int N = 1 << log2N;
    double* work = (double*)malloc((size_t)q * 4 * (size_t)N * sizeof(double));
    for (int64_t b = 0; b < B; ++b) {
        q_ctx c = {q, frozen, info + b * K, NULL, 0, 0};
        q_rec(&c, xy + b * (int64_t)q * N, N, xhat + b * N, work);
    }
    free(work);
}

/* q-ary encode (QaryPolarEncoderDecoder.py:65-88): info symbols at the
 * information positions, 0 at frozen ones, combined bottom-up. */
PCUB_ORC_API void orc_encode_qary(int q, int log2N, const uint8_t* frozen, const uint8_t* info, uint8_t* x) {
    int N = 1 << log2N;
    double* work = (double*)malloc((size_t)q * 4 * (size_t)N * sizeof(double));
    q_ctx c = {q, frozen, (uint8_t*)info, NULL, 0, 0};
    q_rec(&c, NULL, N, x, work);
    free(work);
}
