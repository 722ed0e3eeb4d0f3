/* C restatement of the reference's deletion-channel SC decode (TEST INFRASTRUCTURE ONLY).
 *
 * The same algorithm as oracle/trellis_oracle.py, line for line, in C: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg use it, as the checker and as the
 * deletion workload's CPU baseline (so the three GPU/CPU ratios of the bench compare a C
 * restatement with the kernels alike).  The product path never loads it.
 *
 * Restated (file:line in the reference tree, snapshot 2025-02-04):
 *   guard-band removal  Guardbands.py:47-93
 *   trellis build       VectorDistributions/BinaryTrellis.py:309-438 (single state, uniform input)
 *   minus / plus        VectorDistributions/BinaryTrellis.py:206-258
 *   marginal            VectorDistributions/BinaryTrellis.py:260-278
 *   normalisation       VectorDistributions/BinaryTrellis.py:280-306
 *   collection          VectorDistributions/CollectionOfBinaryTrellises.py:55-103, :106-129
 *   memoryless rows     VectorDistributions/BinaryMemorylessVectorDistribution.py:15-87
 *   SC recursion        BinaryPolarEncoderDecoder.py:223-325 (decode branch, uniform prior:
 *                       frozen u_i = fval_i, :258-262)
 * Every sum runs in the reference's dict insertion order: vertices are kept per layer in
 * insertion order, edges per vertex in insertion order (trellis_oracle.py's dicts).  Build with
 * -O2 -ffp-contract=off (no contraction into fma), like sc_oracle.c. */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------------- trellis */

typedef struct {
    int vpos;
    double prob;
    int nin, nout, cin, cout;
    int *ins, *outs; /* edge indices, insertion order */
} Vtx;

typedef struct {
    int u, v; /* vertex indices */
    int label;
    double prob;
} Edge;

typedef struct {
    int length;
    int nv, cv, ne, ce;
    Vtx* V;
    Edge* E;
    int* lcount; /* vertices per layer */
    int* lcap;
    int** layer; /* per layer: vertex indices in insertion order */
} Trellis;

static void* xrealloc(void* p, size_t n) {
    void* q = realloc(p, n ? n : 1);
    if (!q) abort();
    return q;
}

static void tr_init(Trellis* t, int length) {
    memset(t, 0, sizeof *t);
    t->length = length;
    t->lcount = (int*)calloc((size_t)length + 1, sizeof(int));
    t->lcap = (int*)calloc((size_t)length + 1, sizeof(int));
    t->layer = (int**)calloc((size_t)length + 1, sizeof(int*));
}

static void tr_free(Trellis* t) {
    for (int i = 0; i < t->nv; ++i) {
        free(t->V[i].ins);
        free(t->V[i].outs);
    }
    free(t->V);
    free(t->E);
    for (int l = 0; l <= t->length; ++l) free(t->layer[l]);
    free(t->layer);
    free(t->lcount);
    free(t->lcap);
}

/* the vertex (layer, vpos), created at the end of its layer when new (trellis_oracle.py:90-94) */
static int tr_vertex(Trellis* t, int layer, int vpos) {
    for (int i = 0; i < t->lcount[layer]; ++i)
        if (t->V[t->layer[layer][i]].vpos == vpos) return t->layer[layer][i];
    if (t->nv == t->cv) {
        t->cv = t->cv ? 2 * t->cv : 16;
        t->V = (Vtx*)xrealloc(t->V, (size_t)t->cv * sizeof(Vtx));
    }
    const int id = t->nv++;
    Vtx* v = &t->V[id];
    memset(v, 0, sizeof *v);
    v->vpos = vpos;
    v->prob = -1.0;
    if (t->lcount[layer] == t->lcap[layer]) {
        t->lcap[layer] = t->lcap[layer] ? 2 * t->lcap[layer] : 8;
        t->layer[layer] = (int*)xrealloc(t->layer[layer], (size_t)t->lcap[layer] * sizeof(int));
    }
    t->layer[layer][t->lcount[layer]++] = id;
    return id;
}

static void tr_set_prob(Trellis* t, int layer, int vpos, double p) {
    const int id = tr_vertex(t, layer, vpos); /* may move t->V */
    t->V[id].prob = p;
}

static void push(int** a, int* n, int* c, int x) {
    if (*n == *c) {
        *c = *c ? 2 * *c : 8;
        *a = (int*)xrealloc(*a, (size_t)*c * sizeof(int));
    }
    (*a)[(*n)++] = x;
}

/* BinaryTrellis.py:128-136, 164-175: from-vertex first, then to-vertex, then the edge */
static void tr_add(Trellis* t, int layer, int u, int v, int label, double p) {
    const int fu = tr_vertex(t, layer, u);
    const int tv = tr_vertex(t, layer + 1, v);
    Vtx* U = &t->V[fu];
    for (int i = 0; i < U->nout; ++i) {
        Edge* e = &t->E[U->outs[i]];
        if (t->V[e->v].vpos == v && e->label == label) { /* key (u, v, label) */
            e->prob += p;
            return;
        }
    }
    if (t->ne == t->ce) {
        t->ce = t->ce ? 2 * t->ce : 32;
        t->E = (Edge*)xrealloc(t->E, (size_t)t->ce * sizeof(Edge));
    }
    const int id = t->ne++;
    t->E[id].u = fu;
    t->E[id].v = tv;
    t->E[id].label = label;
    t->E[id].prob = 0.0;
    push(&t->V[fu].outs, &t->V[fu].nout, &t->V[fu].cout, id);
    push(&t->V[tv].ins, &t->V[tv].nin, &t->V[tv].cin, id);
    t->E[id].prob += p;
}

/* BinaryTrellis.py:206-258; dec = NULL for the minus transform */
static void tr_transform(const Trellis* t, const int* dec, Trellis* nw) {
    tr_init(nw, t->length / 2);
    for (int i = 0; i < t->lcount[0]; ++i) {
        const Vtx* v = &t->V[t->layer[0][i]];
        tr_set_prob(nw, 0, v->vpos, v->prob);
    }
    for (int i = 0; i < t->lcount[t->length]; ++i) {
        const Vtx* v = &t->V[t->layer[t->length][i]];
        tr_set_prob(nw, t->length / 2, v->vpos, v->prob);
    }
    for (int mid = 1; mid <= t->length; mid += 2) {
        const int j = (mid - 1) / 2;
        for (int wi = 0; wi < t->lcount[mid]; ++wi) {
            const Vtx* w = &t->V[t->layer[mid][wi]];
            for (int a = 0; a < w->nin; ++a) {
                const Edge* ein = &t->E[w->ins[a]];
                for (int b = 0; b < w->nout; ++b) {
                    const Edge* eout = &t->E[w->outs[b]];
                    const double p = ein->prob * eout->prob;
                    const int lbl = ein->label != eout->label ? 1 : 0;
                    if (!dec) {
                        tr_add(nw, j, t->V[ein->u].vpos, t->V[eout->v].vpos, lbl, p);
                    } else {
                        if (lbl != dec[j]) continue;
                        tr_add(nw, j, t->V[ein->u].vpos, t->V[eout->v].vpos, eout->label, p);
                    }
                }
            }
        }
    }
}

/* BinaryTrellis.py:260-278 with normalize=False (the collection collapse) */
static void tr_marginal(const Trellis* t, double m[2]) {
    m[0] = m[1] = 0.0;
    for (int i = 0; i < t->lcount[0]; ++i) {
        const Vtx* v = &t->V[t->layer[0][i]];
        for (int k = 0; k < v->nout; ++k) {
            const Edge* e = &t->E[v->outs[k]];
            m[e->label] += v->prob * e->prob * t->V[e->v].prob / 1.0;
        }
    }
}

/* BinaryTrellis.py:280-306: per layer the larger label sum of the out-edges, then divide */
static void tr_normalize(Trellis* t) {
    for (int l = 0; l < t->length; ++l) {
        double s[2] = {0.0, 0.0};
        for (int i = 0; i < t->lcount[l]; ++i) {
            const Vtx* v = &t->V[t->layer[l][i]];
            for (int k = 0; k < v->nout; ++k) s[t->E[v->outs[k]].label] += t->E[v->outs[k]].prob;
        }
        double n = s[0] >= s[1] ? s[0] : s[1];
        if (n == 0.0) n = 1.0;
        for (int i = 0; i < t->lcount[l]; ++i) {
            const Vtx* v = &t->V[t->layer[l][i]];
            for (int k = 0; k < v->nout; ++k) t->E[v->outs[k]].prob /= n;
        }
    }
}

static double comb(int n, int k) {
    double c = 1.0;
    for (int i = 1; i <= k; ++i) c = c * (double)(n - k + i) / (double)i; /* small exact integers */
    return c;
}

/* BinaryTrellis.py:309-438: single input state, uniform input, a trimmed segment */
static void tr_build(Trellis* t, const uint8_t* w, int m, int L, double pd, int ones) {
    tr_init(t, L);
    const int dcount = L + 2 * ones - m;
    const double pin = 0.5;
    if (ones > 0) {
        const int mo = ones < m ? ones : m;
        for (int i = 0; i <= mo; ++i)
            tr_set_prob(t, 0, i, comb(ones, i) * pow(1.0 - pd, (double)i) * pow(pd, (double)(ones - i)));
        for (int i = m; i >= m - mo; --i) {
            const int j = m - i;
            tr_set_prob(t, L, i, comb(ones, j) * pow(1.0 - pd, (double)j) * pow(pd, (double)(ones - j)));
        }
    } else {
        tr_set_prob(t, 0, 0, 1.0);
        tr_set_prob(t, L, m, 1.0);
    }
    for (int l = 0; l < L; ++l) {
        int lo, hi;
        if (ones > 0) {
            lo = l + ones - dcount > 0 ? l + ones - dcount : 0;
            hi = l + ones < m ? l + ones : m;
        } else {
            lo = l - dcount > 0 ? l - dcount : 0;
            hi = l < m ? l : m;
        }
        for (int vp = lo; vp <= hi; ++vp) {
            if (vp < m) tr_add(t, l, vp, vp + 1, w[vp], pin * (1.0 - pd));
            if (l + 1 + ones - dcount <= vp) {
                for (int lbl = 0; lbl < 2; ++lbl) {
                    const double p = (lbl == 1 || (0 < vp && vp < m)) ? pin * pd : pin;
                    tr_add(t, l, vp, vp, lbl, p);
                }
            }
        }
    }
}

/* --------------------------------------------------------------------- guard bands */

/* Guardbands.py:66-93 then :47-63: trim, halve, recurse.  Appends the 2^(n-n0) segments of
 * w[0, len) in order as (start, length), starts relative to w. */
static void segments(const uint8_t* w, int len, int n, int n0, int* start, int* slen, int* k) {
    int a = 0, b = len - 1;
    while (a <= b && w[a] != 1) ++a;
    while (b >= a && w[b] != 1) --b;
    const int tl = a <= b ? b - a + 1 : 0;
    if (tl == 0) a = 0;
    if (n <= n0) {
        start[*k] = a;
        slen[*k] = tl;
        ++*k;
        return;
    }
    const int h = tl / 2;
    const int k0 = *k;
    segments(w + a, h, n - 1, n0, start, slen, k);
    const int k1 = *k;
    segments(w + a + h, tl - h, n - 1, n0, start, slen, k);
    for (int i = k0; i < k1; ++i) start[i] += a;
    for (int i = k1; i < *k; ++i) start[i] += a + h;
}

/* --------------------------------------------------------------------- SC recursion */

typedef struct {
    int length;
    int ntr;         /* > 0: a collection of ntr trellises */
    Trellis* tr;
    double* rows;    /* ntr == 0: memoryless rows [length][2] */
} VD;

static void vd_free(VD* d) {
    for (int i = 0; i < d->ntr; ++i) tr_free(&d->tr[i]);
    free(d->tr);
    free(d->rows);
}

/* CollectionOfBinaryTrellises.py:55-82 / BinaryMemorylessVectorDistribution.py:15-47 */
static void vd_transform(const VD* d, const int* dec, VD* out) {
    memset(out, 0, sizeof *out);
    out->length = d->length / 2;
    if (d->ntr) {
        const int T = d->ntr, sub = dec ? (d->length / 2) / T : 0;
        Trellis* kids = (Trellis*)malloc(sizeof(Trellis) * (size_t)T);
        for (int i = 0; i < T; ++i) tr_transform(&d->tr[i], dec ? dec + i * sub : NULL, &kids[i]);
        if (d->length / 2 > T) {
            out->ntr = T;
            out->tr = kids;
            return;
        }
        out->rows = (double*)malloc(sizeof(double) * 2 * (size_t)T);
        for (int i = 0; i < T; ++i) {
            tr_marginal(&kids[i], out->rows + 2 * i);
            tr_free(&kids[i]);
        }
        free(kids);
        return;
    }
    const double* r = d->rows;
    out->rows = (double*)malloc(sizeof(double) * 2 * (size_t)(out->length > 0 ? out->length : 1));
    for (int h = 0; h < d->length / 2; ++h) {
        const double* a = r + 4 * h;
        const double* b = r + 4 * h + 2;
        double* o = out->rows + 2 * h;
        if (!dec) {
            o[0] = a[0] * b[0] + a[1] * b[1];
            o[1] = a[0] * b[1] + a[1] * b[0];
        } else if (dec[h] == 0) {
            o[0] = a[0] * b[0];
            o[1] = a[1] * b[1];
        } else {
            o[0] = a[1] * b[0];
            o[1] = a[0] * b[1];
        }
    }
}

static void vd_normalize(VD* d) {
    if (d->ntr) {
        for (int i = 0; i < d->ntr; ++i) tr_normalize(&d->tr[i]);
        return;
    }
    for (int i = 0; i < d->length; ++i) {
        double* row = d->rows + 2 * i;
        double t = row[0] >= row[1] ? row[0] : row[1];
        if (t == 0.0) t = 1.0;
        row[0] /= t;
        row[1] /= t;
    }
}

typedef struct {
    const uint8_t* frozen;
    const uint8_t* fval;
    int u;
    uint8_t* info;
    int ninfo;
} Ctx;

/* BinaryPolarEncoderDecoder.py:223-325; x receives the node's re-encoded bits */
static void rec(const VD* d, Ctx* c, int* x) {
    if (d->length == 1) {
        const int i = c->u++;
        const double p0 = d->rows[0], p1 = d->rows[1];
        double s = 0.0;
        s += p0;
        s += p1;
        int dec = 0;
        if (s > 0.0) dec = (p0 / s >= p1 / s) ? 0 : 1;
        if (c->frozen[i]) {
            x[0] = c->fval[i];
            return;
        }
        c->info[c->ninfo++] = (uint8_t)dec;
        x[0] = dec;
        return;
    }
    const int H = d->length / 2;
    int* xm = (int*)malloc(sizeof(int) * (size_t)H);
    int* xp = (int*)malloc(sizeof(int) * (size_t)H);
    VD m;
    vd_transform(d, NULL, &m);
    vd_normalize(&m);
    rec(&m, c, xm);
    vd_free(&m);
    VD p;
    vd_transform(d, xm, &p);
    vd_normalize(&p);
    rec(&p, c, xp);
    vd_free(&p);
    for (int h = 0; h < H; ++h) {
        x[2 * h] = (xm[h] + xp[h]) % 2;
        x[2 * h + 1] = xp[h];
    }
    free(xm);
    free(xp);
}

/* decode one received word (buildCollectionOfBinaryTrellises_uniformInput_deletion, then SC):
 * xhat [2^n], info [K] out */
int orc_decode_deletion(const uint8_t* word, int len, int n, int n0, double pd, const uint8_t* frozen,
                        const uint8_t* fval, int ones, uint8_t* xhat, uint8_t* info) {
    if (n0 < 0 || n0 > n || n > 24) return -1;
    const int T = 1 << (n - n0), L = 1 << n0;
    int* start = (int*)malloc(sizeof(int) * (size_t)T);
    int* slen = (int*)malloc(sizeof(int) * (size_t)T);
    int k = 0;
    segments(word, len, n, n0, start, slen, &k);
    VD d;
    memset(&d, 0, sizeof d);
    d.length = 1 << n;
    d.ntr = T;
    d.tr = (Trellis*)malloc(sizeof(Trellis) * (size_t)T);
    for (int i = 0; i < T; ++i) tr_build(&d.tr[i], word + start[i], slen[i], L, pd, ones);
    free(start);
    free(slen);
    Ctx c = {frozen, fval, 0, info, 0};
    int* x = (int*)malloc(sizeof(int) * (size_t)d.length);
    if (d.length == T) {
        /* n0 = 0: every trellis collapses at once (the collection's transform does it) -- not a
         * decoder shape; the reference builds L = 1 trellises */
        free(x);
        vd_free(&d);
        return -1;
    }
    rec(&d, &c, x);
    for (int i = 0; i < d.length; ++i) xhat[i] = (uint8_t)x[i];
    free(x);
    vd_free(&d);
    return c.ninfo;
}

/* a batch of padded words rx [B][stride], lengths rx_len [B]: xhat [B][2^n], info [B][K] */
int orc_decode_deletion_batch(const uint8_t* rx, const int32_t* rx_len, long long B, int stride, int n, int n0,
                              double pd, const uint8_t* frozen, const uint8_t* fval, int ones, int K, uint8_t* xhat,
                              uint8_t* info) {
    for (long long b = 0; b < B; ++b) {
        const int r = orc_decode_deletion(rx + b * stride, rx_len[b], n, n0, pd, frozen, fval, ones,
                                          xhat + b * (1LL << n), info + b * (long long)K);
        if (r != K) return -1;
    }
    return 0;
}
