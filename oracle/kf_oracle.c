/*
 * kf_oracle.c — CPU restatement of the reference's CNN-TDNN forward/backward.
 *
 * TEST INFRASTRUCTURE ONLY (see kf_oracle.h). It follows the reference's own
 * materialising formulation — explicit time splices (forward.go:699-790),
 * explicit im2col patches (forward.go:435-456), dense fp32-accumulated GEMMs
 * (ops.cu:381-392) — so it shares no addressing code with the MI355X kernels
 * that compute the same quantities implicitly.
 *
 * Deliberate differences from the reference's *buggy* pieces:
 *   - conv offsets are Kaldi's cross product (time x height), output layout is
 *     height-major [h*F + f] (Kaldi), not the reference's zipped offsets and
 *     filter-major reorder (forward.go:442-444, :499-508);
 *   - backward is the exact gradient of the forward (the reference's
 *     backwardTDNNF / backwardPrefinal are inconsistent with their forward,
 *     network_backward.go:336-463, :549-656).
 */
#include "kf_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------- */
/* fp16 conversions                                                          */
/* ------------------------------------------------------------------------- */
static inline uint32_t f2u(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    return u;
}
static inline float u2f(uint32_t u) {
    float f;
    memcpy(&f, &u, 4);
    return f;
}

/* IEEE round-to-nearest-even, as internal/fp16/fp16.go:12-70 */
uint16_t orc_f32_to_f16_rne(float f) {
    uint32_t b = f2u(f);
    uint32_t sign = (b >> 31) & 1u;
    int exp = (int)((b >> 23) & 0xFF);
    uint32_t frac = b & 0x7FFFFFu;
    if (exp == 255) {
        if (frac == 0) return (uint16_t)(sign << 15 | 0x7C00u);
        return (uint16_t)(sign << 15 | 0x7C00u | (frac >> 13));
    }
    if (exp > 142) return (uint16_t)(sign << 15 | 0x7C00u);
    if (exp > 112) {
        uint32_t e = (uint32_t)(exp - 112);
        uint32_t round = frac & 0x1FFFu;
        frac >>= 13;
        if (round > 0x1000u || (round == 0x1000u && (frac & 1u))) {
            frac++;
            if (frac > 0x3FFu) {
                frac = 0;
                e++;
                if (e > 30) return (uint16_t)(sign << 15 | 0x7C00u);
            }
        }
        return (uint16_t)(sign << 15 | e << 10 | frac);
    }
    if (exp > 101) {
        unsigned shift = (unsigned)(113 - exp);
        frac |= 0x800000u;
        uint32_t round = frac & ((1u << (shift + 13)) - 1u);
        uint32_t half = 1u << (shift + 12);
        frac >>= (shift + 13);
        if (round > half || (round == half && (frac & 1u))) frac++;
        return (uint16_t)(sign << 15 | frac);
    }
    return (uint16_t)(sign << 15);
}

/* truncating conversion used for weights, internal/gpu/tensor.go:158-173 */
uint16_t orc_f32_to_f16_trunc(float f) {
    uint32_t bits = f2u(f);
    uint16_t sign = (uint16_t)((bits >> 16) & 0x8000u);
    int exp = (int)((bits >> 23) & 0xFF) - 127;
    uint32_t frac = bits & 0x7FFFFFu;
    if (exp > 15) return sign | 0x7C00u;
    if (exp < -14) return sign;
    return (uint16_t)(sign | (uint16_t)((exp + 15) << 10) | (uint16_t)(frac >> 13));
}

/* internal/fp16/fp16.go:73-110 */
float orc_f16_to_f32(uint16_t h) {
    uint32_t sign = (uint32_t)(h >> 15) & 1u;
    uint32_t exp = (uint32_t)(h >> 10) & 0x1Fu;
    uint32_t frac = (uint32_t)h & 0x3FFu;
    if (exp == 31) return u2f(sign << 31 | 0x7F800000u | (frac << 13));
    if (exp == 0) {
        if (frac == 0) return u2f(sign << 31);
        while ((frac & 0x400u) == 0) {
            frac <<= 1;
            exp--;
        }
        frac &= 0x3FFu;
        exp++;
        return u2f(sign << 31 | (exp + 112) << 23 | frac << 13);
    }
    return u2f(sign << 31 | (exp + 112) << 23 | frac << 13);
}

static inline float rh(float x) { return orc_f16_to_f32(orc_f32_to_f16_rne(x)); }

void orc_round_f16(float *x, long long n) {
    for (long long i = 0; i < n; ++i) x[i] = rh(x[i]);
}

/* ------------------------------------------------------------------------- */
/* threading: rows split over threads like gotorch's matmulParallel          */
/* ------------------------------------------------------------------------- */
static int g_threads = 1;
void orc_set_threads(int n) { g_threads = n < 1 ? 1 : n; }
int orc_get_threads(void) { return g_threads; }

typedef void (*range_fn)(void *ctx, int lo, int hi);
typedef struct {
    range_fn fn;
    void *ctx;
    int lo, hi;
} job_t;
static void *job_run(void *p) {
    job_t *j = (job_t *)p;
    j->fn(j->ctx, j->lo, j->hi);
    return NULL;
}
static void parallel_for(int n, range_fn fn, void *ctx) {
    int nt = g_threads;
    if (nt > n) nt = n;
    if (nt <= 1) {
        fn(ctx, 0, n);
        return;
    }
    pthread_t th[256];
    job_t jobs[256];
    if (nt > 256) nt = 256;
    int chunk = (n + nt - 1) / nt;
    int used = 0;
    for (int i = 0; i < nt; ++i) {
        int lo = i * chunk, hi = lo + chunk < n ? lo + chunk : n;
        if (lo >= hi) break;
        jobs[i].fn = fn;
        jobs[i].ctx = ctx;
        jobs[i].lo = lo;
        jobs[i].hi = hi;
        pthread_create(&th[i], NULL, job_run, &jobs[i]);
        used++;
    }
    for (int i = 0; i < used; ++i) pthread_join(th[i], NULL);
}

/* C = A . B  (NN), A [MxK], B [KxN] */
typedef struct {
    int M, N, K;
    const float *A, *B;
    float *C;
} mm_t;
static void mm_nn_rows(void *p, int lo, int hi) {
    mm_t *m = (mm_t *)p;
    for (int i = lo; i < hi; ++i) {
        float *c = m->C + (size_t)i * m->N;
        memset(c, 0, sizeof(float) * (size_t)m->N);
        const float *a = m->A + (size_t)i * m->K;
        for (int k = 0; k < m->K; ++k) {
            const float av = a[k];
            if (av == 0.f) continue;
            const float *b = m->B + (size_t)k * m->N;
            for (int j = 0; j < m->N; ++j) c[j] += av * b[j];
        }
    }
}
void orc_matmul(int M, int N, int K, const float *A, const float *B, float *C) {
    mm_t m = {M, N, K, A, B, C};
    parallel_for(M, mm_nn_rows, &m);
}
/* C = A . B^T, A [MxK], B [NxK] */
static void mm_nt_rows(void *p, int lo, int hi) {
    mm_t *m = (mm_t *)p;
    for (int i = lo; i < hi; ++i) {
        const float *a = m->A + (size_t)i * m->K;
        for (int j = 0; j < m->N; ++j) {
            const float *b = m->B + (size_t)j * m->K;
            float s = 0.f;
            for (int k = 0; k < m->K; ++k) s += a[k] * b[k];
            m->C[(size_t)i * m->N + j] = s;
        }
    }
}
static void matmul_nt(int M, int N, int K, const float *A, const float *B, float *C) {
    mm_t m = {M, N, K, A, B, C};
    parallel_for(M, mm_nt_rows, &m);
}
/* C[MxN] = A^T . B, A [K x M], B [K x N]  (weight gradients; K = frames) */
static void mm_tn_rows(void *p, int lo, int hi) {
    mm_t *m = (mm_t *)p;
    for (int i = lo; i < hi; ++i) memset(m->C + (size_t)i * m->N, 0, sizeof(float) * (size_t)m->N);
    for (int k = 0; k < m->K; ++k) {
        const float *a = m->A + (size_t)k * m->M;
        const float *b = m->B + (size_t)k * m->N;
        for (int i = lo; i < hi; ++i) {
            const float av = a[i];
            if (av == 0.f) continue;
            float *c = m->C + (size_t)i * m->N;
            for (int j = 0; j < m->N; ++j) c[j] += av * b[j];
        }
    }
}
static void matmul_tn(int M, int N, int K, const float *A, const float *B, float *C) {
    mm_t m = {M, N, K, A, B, C};
    parallel_for(M, mm_tn_rows, &m);
}

/* ------------------------------------------------------------------------- */
/* layer pieces                                                              */
/* ------------------------------------------------------------------------- */
static void *xalloc(size_t n) {
    void *p = calloc(n ? n : 1, 1);
    return p;
}

/* ops.cu:171-204 */
static inline float bn_apply(const OrcBN *bn, int d, float v) {
    float norm = (v - bn->mean[d]) / sqrtf(bn->var[d] + bn->eps);
    if (bn->target_rms != 1.0f) return norm * bn->target_rms;
    return bn->gamma[d] * norm + bn->beta[d];
}
static inline float bn_scale(const OrcBN *bn, int d) {
    if (bn->target_rms != 1.0f) return bn->target_rms / sqrtf(bn->var[d] + bn->eps);
    return bn->gamma[d] / sqrtf(bn->var[d] + bn->eps);
}

/* spliceBackward forward.go:699-741: [x(max(t-s,0)) | x(t)] */
static float *splice_minus(const float *x, int T, int d, int s) {
    float *o = (float *)xalloc(sizeof(float) * (size_t)T * 2 * d);
    for (int t = 0; t < T; ++t) {
        int tp = t - s < 0 ? 0 : t - s;
        memcpy(o + (size_t)t * 2 * d, x + (size_t)tp * d, sizeof(float) * d);
        memcpy(o + (size_t)t * 2 * d + d, x + (size_t)t * d, sizeof(float) * d);
    }
    return o;
}
/* spliceForward forward.go:745-790: [x(t) | x(min(t+s,T-1))] */
static float *splice_plus(const float *x, int T, int d, int s) {
    float *o = (float *)xalloc(sizeof(float) * (size_t)T * 2 * d);
    for (int t = 0; t < T; ++t) {
        int tp = t + s > T - 1 ? T - 1 : t + s;
        memcpy(o + (size_t)t * 2 * d, x + (size_t)t * d, sizeof(float) * d);
        memcpy(o + (size_t)t * 2 * d + d, x + (size_t)tp * d, sizeof(float) * d);
    }
    return o;
}
/* im2col forward.go:435-456, Kaldi cross product of offsets, zero padding */
static float *im2col(const OrcLayer *L, const float *x, int T) {
    const int pd = L->noff * L->fin;
    float *p = (float *)xalloc(sizeof(float) * (size_t)T * L->hout * pd);
    for (int t = 0; t < T; ++t)
        for (int h = 0; h < L->hout; ++h) {
            float *row = p + ((size_t)t * L->hout + h) * pd;
            for (int o = 0; o < L->noff; ++o) {
                int ts = t + L->toff[o], hs = h * L->sub + L->hoff[o];
                if (ts < 0 || ts >= T || hs < 0 || hs >= L->hin) continue;
                memcpy(row + (size_t)o * L->fin, x + (size_t)ts * L->hin * L->fin + (size_t)hs * L->fin,
                       sizeof(float) * L->fin);
            }
        }
    return p;
}
static void col2im_add(const OrcLayer *L, const float *dp, int T, float *dx) {
    const int pd = L->noff * L->fin;
    for (int t = 0; t < T; ++t)
        for (int h = 0; h < L->hout; ++h) {
            const float *row = dp + ((size_t)t * L->hout + h) * pd;
            for (int o = 0; o < L->noff; ++o) {
                int ts = t + L->toff[o], hs = h * L->sub + L->hoff[o];
                if (ts < 0 || ts >= T || hs < 0 || hs >= L->hin) continue;
                float *d = dx + (size_t)ts * L->hin * L->fin + (size_t)hs * L->fin;
                for (int f = 0; f < L->fin; ++f) d[f] += row[(size_t)o * L->fin + f];
            }
        }
}

/* relu + BN (+ bias) epilogue; R mode rounds after every reference op */
static void bias_relu_bn(float *z, int rows, int D, const float *bias, const OrcBN *bn,
                         uint8_t *mask, int mode, int relu, const uint8_t *force) {
    for (long long i = 0; i < (long long)rows * D; ++i) {
        int d = (int)(i % D);
        float v = z[i];
        if (mode == ORC_ROUND_REF) v = rh(v); /* cuBLAS fp16 output */
        if (bias) {
            v += bias[d];
            if (mode == ORC_ROUND_REF) v = rh(v);
        }
        if (relu) {
            const int on = force ? force[i] != 0 : v > 0.f;
            if (mask) mask[i] = (uint8_t)on;
            if (!on) v = 0.f;
        }
        if (bn && bn->mean) {
            v = bn_apply(bn, d, v);
            if (mode == ORC_ROUND_REF) v = rh(v);
        }
        z[i] = v;
    }
}

/* ---- restricted attention (forward.go:795-909) -------------------------------
 * proj [T x heads*A] per head [key kd | value vd | query key kd | query ctx]; frame t
 * attends to rows t + (o - nleft)*stride, zero outside [0, T) (the reference pads). The
 * per-head loop is the reference's, float32 with the exp in float64. */
static void att_weights(const OrcLayer *L, const float *proj, int T, int t, int h, float *w) {
    const int A = 2 * L->kd + L->vd + L->ctx, ld = L->heads * A;
    const float *q = proj + (size_t)t * ld + (size_t)h * A + L->kd + L->vd;
    float mx = -1e30f, s = 0.f;
    for (int o = 0; o < L->ctx; ++o) {
        const int r = t + (o - L->nleft) * L->astride;
        float dot = 0.f;
        if (r >= 0 && r < T) {
            const float *k = proj + (size_t)r * ld + (size_t)h * A;
            for (int d = 0; d < L->kd; ++d) dot += q[d] * k[d];
        }
        w[o] = q[L->kd + o] + L->key_scale * dot;
        if (w[o] > mx) mx = w[o];
    }
    for (int o = 0; o < L->ctx; ++o) {
        w[o] = (float)exp((double)(w[o] - mx));
        s += w[o];
    }
    for (int o = 0; o < L->ctx; ++o) w[o] /= s;
}

static void att_forward(const OrcLayer *L, const float *proj, int T, float *out) {
    const int A = 2 * L->kd + L->vd + L->ctx, ld = L->heads * A, od = L->vd + L->ctx;
    float w[64];
    for (int t = 0; t < T; ++t)
        for (int h = 0; h < L->heads; ++h) {
            att_weights(L, proj, T, t, h, w);
            float *y = out + (size_t)t * L->heads * od + (size_t)h * od;
            for (int d = 0; d < L->vd; ++d) y[d] = 0.f;
            for (int o = 0; o < L->ctx; ++o) {
                const int r = t + (o - L->nleft) * L->astride;
                if (r >= 0 && r < T) {
                    const float *v = proj + (size_t)r * ld + (size_t)h * A + L->kd;
                    for (int d = 0; d < L->vd; ++d) y[d] += w[o] * v[d];
                }
                y[L->vd + o] = w[o];
            }
        }
}

/* exact gradient of att_forward: dz [T x heads*od] -> dproj [T x heads*A] */
static void att_backward(const OrcLayer *L, const float *proj, int T, const float *dz, float *dproj) {
    const int A = 2 * L->kd + L->vd + L->ctx, ld = L->heads * A, od = L->vd + L->ctx;
    float w[64], dw[64], db[64];
    memset(dproj, 0, sizeof(float) * (size_t)T * ld);
    for (int t = 0; t < T; ++t)
        for (int h = 0; h < L->heads; ++h) {
            att_weights(L, proj, T, t, h, w);
            const float *g = dz + (size_t)t * L->heads * od + (size_t)h * od;
            const float *qk = proj + (size_t)t * ld + (size_t)h * A + L->kd + L->vd;
            float sw = 0.f;
            for (int o = 0; o < L->ctx; ++o) {
                const int r = t + (o - L->nleft) * L->astride;
                dw[o] = g[L->vd + o];
                if (r >= 0 && r < T) {
                    const float *v = proj + (size_t)r * ld + (size_t)h * A + L->kd;
                    for (int d = 0; d < L->vd; ++d) dw[o] += g[d] * v[d];
                }
                sw += w[o] * dw[o];
            }
            float *dq = dproj + (size_t)t * ld + (size_t)h * A + L->kd + L->vd;
            for (int o = 0; o < L->ctx; ++o) {
                db[o] = w[o] * (dw[o] - sw);
                dq[L->kd + o] += db[o];
                const int r = t + (o - L->nleft) * L->astride;
                if (r < 0 || r >= T) continue;
                const float *k = proj + (size_t)r * ld + (size_t)h * A;
                float *dk = dproj + (size_t)r * ld + (size_t)h * A;
                for (int d = 0; d < L->kd; ++d) {
                    dq[d] += L->key_scale * db[o] * k[d];
                    dk[d] += L->key_scale * db[o] * qk[d];
                }
                for (int d = 0; d < L->vd; ++d) dk[L->kd + d] += w[o] * g[d];
            }
        }
}

static int trainable_below(const OrcNet *net, int cur) {
    if (cur < 0) return 0;
    const OrcLayer *L = &net->layers[cur];
    const int ty = L->type;
    if (ty == ORC_CONV || ty == ORC_TDNNF || ty == ORC_LINEAR || ty == ORC_PREFINAL || ty == ORC_OUTPUT ||
        ty == ORC_ATTENTION)
        return 1;
    return trainable_below(net, L->input) || (ty == ORC_COMBINE && trainable_below(net, L->input2));
}

static int layer_needs_dx(const OrcNet *net, int li) {
    /* does any trainable layer lie below li (inputs, and combine's second input)? */
    return trainable_below(net, net->layers[li].input);
}

/* ---- OCP MXFP8 (e4m3 + E8M0, blocks of 32) quantise-dequantise ---------- */
static float e4m3_rne(float a) { /* 0 <= a <= 448 */
    if (a == 0.f) return 0.f;
    int e;
    frexpf(a, &e);           /* a = m 2^e, m in [0.5, 1) */
    int ex = e - 1;          /* floor(log2 a) */
    if (ex < -6) ex = -6;    /* subnormals: quantum 2^-9 */
    const float q = ldexpf(1.f, ex - 3);
    const float r = nearbyintf(a / q) * q; /* round to nearest even */
    return r > 448.f ? 448.f : r;
}
static void mx_block(const float *x, long long xs, float *y, long long ys) {
    float amax = 0.f;
    for (int j = 0; j < 32; ++j) amax = fmaxf(amax, fabsf(x[j * xs]));
    int ex = 0;
    if (amax > 0.f) {
        int e2;
        frexpf(amax, &e2);
        ex = e2 - 1 - 8;
        if (ex < -126) ex = -126;
        if (ex > 126) ex = 126;
    }
    const float sc = ldexpf(1.f, ex), inv = ldexpf(1.f, -ex);
    for (int j = 0; j < 32; ++j) {
        const float v = x[j * xs] * inv;
        const float a = e4m3_rne(fminf(fabsf(v), 448.f));
        y[j * ys] = (v < 0.f ? -a : a) * sc;
    }
}
void orc_mx_qdq_rows(const float *x, float *y, long long rows, int cols) {
    for (long long r = 0; r < rows; ++r)
        for (int b = 0; b < cols / 32; ++b) mx_block(x + r * cols + 32 * b, 1, y + r * cols + 32 * b, 1);
}
static float *mx_rows_new(const float *x, long long rows, int cols) {
    float *y = (float *)xalloc(sizeof(float) * (size_t)rows * cols);
    orc_mx_qdq_rows(x, y, rows, cols);
    return y;
}
/* weights W [K x N]: blocks of 32 along K for every column */
static float *mx_cols_new(const float *W, int K, int N) {
    float *y = (float *)xalloc(sizeof(float) * (size_t)K * N);
    for (int n = 0; n < N; ++n)
        for (int b = 0; b < K / 32; ++b) mx_block(W + (size_t)32 * b * N + n, N, y + (size_t)32 * b * N + n, N);
    return y;
}
/* mirrors f8_producer of host/network.cpp */
static int mx_producer(const OrcLayer *L) {
    switch (L->type) {
        case ORC_CONV: return L->fin != 1 && L->fout % 32 == 0 && L->out_dim % 128 == 0;
        case ORC_TDNNF:
        case ORC_LINEAR: return 1;
        case ORC_PREFINAL: return L->small_dim % 32 == 0;
        default: return 0;
    }
}

static void alloc_net(OrcNet *net) {
    int n = net->nlayers;
    net->act = (float **)xalloc(sizeof(float *) * n);
    net->mask = (uint8_t **)xalloc(sizeof(uint8_t *) * n);
    net->aux = (float **)xalloc(sizeof(float *) * n);
    net->gW = (float **)xalloc(sizeof(float *) * n);
    net->gb = (float **)xalloc(sizeof(float *) * n);
    net->gW2 = (float **)xalloc(sizeof(float *) * n);
    net->gb2 = (float **)xalloc(sizeof(float *) * n);
    net->gact = (float **)xalloc(sizeof(float *) * n);
    net->act8 = (float **)xalloc(sizeof(float *) * n);
}

#define FM(li) (net->force_mask ? net->force_mask[li] : NULL)
int orc_net_forward(OrcNet *net, const float *features) {
    const int T = net->T, mode = net->round_mode, MX = net->mx8;
    if (!net->act) alloc_net(net);
    for (int li = 0; li < net->nlayers; ++li) {
        const OrcLayer *L = &net->layers[li];
        const float *x = L->input == -2 ? net->ivec : L->input < 0 ? features : net->act[L->input];
        const int din = L->in_dim, dout = L->out_dim;
        float *y = (float *)xalloc(sizeof(float) * (size_t)T * dout);
        if (L->per_seq) { /* linear / batchnorm on the B per-sequence rows */
            const int R = net->B;
            if (L->type == ORC_LINEAR) orc_matmul(R, dout, din, x, L->W, y);
            else if (L->type == ORC_BATCHNORM)
                for (long long i = 0; i < (long long)R * dout; ++i) y[i] = bn_apply(&L->bn, (int)(i % dout), x[i]);
            else { free(y); return -1; }
            if (mode) orc_round_f16(y, (long long)R * dout);
            net->act[li] = y;
            continue;
        }
        /* MXFP8 GEMM input of this layer (the producer's copy), or NULL = fp16 GEMM */
        const float *x8 = !MX ? NULL : L->input >= 0 ? net->act8[L->input] : L->input == -1 ? net->feat8 : NULL;
        float *wq = NULL, *wq2 = NULL;
#define MX_OUT(buf, rows, cols) \
    do { if (MX && mx_producer(L)) net->act8[li] = mx_rows_new(buf, rows, cols); } while (0)
        switch (L->type) {
            case ORC_IDCT:
                orc_matmul(T, dout, din, x, L->W, y);
                if (mode) orc_round_f16(y, (long long)T * dout);
                break;
            case ORC_BATCHNORM:
                for (long long i = 0; i < (long long)T * dout; ++i) y[i] = bn_apply(&L->bn, (int)(i % dout), x[i]);
                if (mode) orc_round_f16(y, (long long)T * dout);
                break;
            case ORC_CONV: {
                float *p = im2col(L, x, T);
                orc_matmul(T * L->hout, L->fout, L->noff * L->fin, p, L->W, y);
                free(p);
                net->mask[li] = (uint8_t *)xalloc((size_t)T * dout);
                bias_relu_bn(y, T * L->hout, L->fout, L->b, &L->bn, net->mask[li], mode, 1, FM(li));
                MX_OUT(y, T, dout);
                if (mode) orc_round_f16(y, (long long)T * dout);
                break;
            }
            case ORC_TDNNF: {
                const int s = L->stride, bn = L->bn_dim;
                const int klin = s > 0 ? 2 * din : din, kaff = s > 0 ? 2 * bn : bn;
                const float *lin_src = x8 ? x8 : x, *Wl = L->W;
                if (x8) Wl = wq = mx_cols_new(L->W, klin, bn);
                const float *lin_in = lin_src;
                float *tmp = NULL;
                if (s > 0) lin_in = tmp = splice_minus(lin_src, T, din, s);
                float *bott = (float *)xalloc(sizeof(float) * (size_t)T * bn);
                orc_matmul(T, bn, klin, lin_in, Wl, bott);
                free(tmp);
                if (mode) orc_round_f16(bott, (long long)T * bn);
                /* the product quantises the stored fp16 bottleneck (network.cpp: kf_quant_mxfp8
                   after the linear GEMM), so the copy is taken after the rounding */
                float *bott8 = MX ? mx_rows_new(bott, T, bn) : NULL;
                const float *aff_src = MX ? bott8 : bott, *Wa = L->W2;
                if (MX) Wa = wq2 = mx_cols_new(L->W2, kaff, dout);
                const float *aff_in = aff_src;
                tmp = NULL;
                if (s > 0) aff_in = tmp = splice_plus(aff_src, T, bn, s);
                orc_matmul(T, dout, kaff, aff_in, Wa, y);
                free(tmp);
                free(bott8);
                net->mask[li] = (uint8_t *)xalloc((size_t)T * dout);
                bias_relu_bn(y, T, dout, L->b2, &L->bn, net->mask[li], mode, 1, FM(li));
                if (L->bypass > 0.f && din == dout) {
                    for (long long i = 0; i < (long long)T * dout; ++i) {
                        float v = y[i] + L->bypass * x[i];
                        y[i] = mode == ORC_ROUND_REF ? rh(v) : v;
                    }
                }
                MX_OUT(y, T, dout);
                if (mode) orc_round_f16(y, (long long)T * dout);
                net->aux[li] = bott;
                break;
            }
            case ORC_LINEAR:
                if (x8) wq = mx_cols_new(L->W, din, dout);
                orc_matmul(T, dout, din, x8 ? x8 : x, x8 ? wq : L->W, y);
                MX_OUT(y, T, dout);
                if (mode) orc_round_f16(y, (long long)T * dout);
                break;
            case ORC_PREFINAL: {
                const int big = L->big_dim, small = L->small_dim;
                float *bg = (float *)xalloc(sizeof(float) * (size_t)T * big);
                if (x8) wq = mx_cols_new(L->W, din, big);
                orc_matmul(T, big, din, x8 ? x8 : x, x8 ? wq : L->W, bg);
                net->mask[li] = (uint8_t *)xalloc((size_t)T * big);
                bias_relu_bn(bg, T, big, L->b, &L->bn, net->mask[li], mode, 1, FM(li));
                float *bg8 = MX ? mx_rows_new(bg, T, big) : NULL;
                if (mode) orc_round_f16(bg, (long long)T * big);
                if (MX) wq2 = mx_cols_new(L->W2, big, small);
                orc_matmul(T, small, big, MX ? bg8 : bg, MX ? wq2 : L->W2, y);
                free(bg8);
                bias_relu_bn(y, T, small, NULL, &L->bn2, NULL, mode, 0, NULL);
                MX_OUT(y, T, small);
                if (mode) orc_round_f16(y, (long long)T * small);
                net->aux[li] = bg;
                break;
            }
            case ORC_COMBINE: { /* Kaldi combine-feature-maps; b broadcast per sequence */
                const int n1 = L->nf1, n2 = L->nf2, nf = n1 + n2, H = L->height;
                const float *b = L->input2 == -2 ? net->ivec : L->input2 < 0 ? features : net->act[L->input2];
                const int bseq = L->input2 == -2 || (L->input2 >= 0 && net->layers[L->input2].per_seq);
                for (int t = 0, s = 0; t < T; ++t) {
                    while (bseq && s + 1 < net->B && net->seq_off[s + 1] <= t) ++s;
                    const float *br = b + (size_t)(bseq ? s : t) * H * n2;
                    for (int h = 0; h < H; ++h)
                        for (int f = 0; f < nf; ++f)
                            y[(size_t)t * dout + h * nf + f] =
                                f < n1 ? x[(size_t)t * H * n1 + h * n1 + f] : br[h * n2 + f - n1];
                }
                break;
            }
            case ORC_ATTENTION: {
                const int A = L->heads * (2 * L->kd + L->vd + L->ctx);
                float *proj = (float *)xalloc(sizeof(float) * (size_t)T * A);
                orc_matmul(T, A, din, x, L->W, proj);
                bias_relu_bn(proj, T, A, L->b, NULL, NULL, mode, 0, NULL);
                if (mode) orc_round_f16(proj, (long long)T * A);  /* the stored fp16 affine output */
                att_forward(L, proj, T, y);
                net->mask[li] = (uint8_t *)xalloc((size_t)T * dout);
                bias_relu_bn(y, T, dout, NULL, &L->bn, net->mask[li], mode, 1, FM(li));
                if (mode) orc_round_f16(y, (long long)T * dout);
                net->aux[li] = proj;
                break;
            }
            case ORC_OUTPUT:
                if (x8) wq = mx_cols_new(L->W, din, dout);
                orc_matmul(T, dout, din, x8 ? x8 : x, x8 ? wq : L->W, y);
                bias_relu_bn(y, T, dout, L->b, NULL, NULL, mode, 0, NULL);
                if (mode) orc_round_f16(y, (long long)T * dout);
                if (L->log_softmax) {
                    /* LogSoftmax of the stored fp16 affine output (forward.go:991-997), in
                     * double; the reference's integer-atomicMax row max (ops.cu:120-166)
                     * is wrong for all-negative rows and is not restated */
                    for (int t = 0; t < T; ++t) {
                        float *row = y + (size_t)t * dout;
                        double mx = -INFINITY, s = 0.0;
                        for (int d = 0; d < dout; ++d) mx = row[d] > mx ? row[d] : mx;
                        for (int d = 0; d < dout; ++d) s += exp((double)row[d] - mx);
                        const double lse = mx + log(s);
                        for (int d = 0; d < dout; ++d) row[d] = (float)((double)row[d] - lse);
                    }
                    if (mode) orc_round_f16(y, (long long)T * dout);
                }
                break;
            default:
                free(y);
                return -1;
        }
#undef MX_OUT
        free(wq);
        free(wq2);
        net->act[li] = y;
    }
    return 0;
}

static float *colsum(const float *g, int rows, int D) {
    float *s = (float *)xalloc(sizeof(float) * D);
    for (int r = 0; r < rows; ++r)
        for (int d = 0; d < D; ++d) s[d] += g[(size_t)r * D + d];
    return s;
}

/* the layers whose affine input gradient the MXFP8 train step runs in e4m3: strided
   TDNN-F layers with out_dim % 128 == 0 and as wide as the widest strided TDNN-F layer
   (network.cpp: the dz copies are allocated that wide; no padding columns) */
static int mx_dgrad_layer(const OrcNet *net, int li) {
    const OrcLayer *L = &net->layers[li];
    if (net->mx8 == 2 || L->type != ORC_TDNNF || L->stride <= 0 || L->out_dim % 128) return 0;
    int w = 0;
    for (int j = 0; j < net->nlayers; ++j)
        if (net->layers[j].type == ORC_TDNNF && net->layers[j].stride > 0 && net->layers[j].out_dim > w)
            w = net->layers[j].out_dim;
    return L->out_dim == (w + 127) / 128 * 128;
}

/*
 * Exact backward. v[li] is the fp32 (unrounded) gradient w.r.t. layer li's
 * output; the MI355X build stores g = rne(v) and dz = rne(v * bnscale * mask),
 * and this restatement rounds at exactly those tensors in F mode.
 */
int orc_net_backward(OrcNet *net, const float *features, const float *out_grad) {
    return orc_net_backward_top(net, features, out_grad, net->nlayers - 1);
}

int orc_net_backward_top(OrcNet *net, const float *features, const float *out_grad, int top_li) {
    const int T = net->T, mode = net->round_mode;
    const int n = net->nlayers;
    if (top_li < 0 || top_li >= n) return -1;
    float **v = (float **)xalloc(sizeof(float *) * n);
    {
        const OrcLayer *top = &net->layers[top_li];
        v[top_li] = (float *)xalloc(sizeof(float) * (size_t)T * top->out_dim);
        memcpy(v[top_li], out_grad, sizeof(float) * (size_t)T * top->out_dim);
    }
    for (int li = top_li; li >= 0; --li) {
        const OrcLayer *L = &net->layers[li];
        if (!v[li]) continue;
        const int din = L->in_dim, dout = L->out_dim;
        const float *x = L->input < 0 ? features : net->act[L->input];
        const int need_dx = layer_needs_dx(net, li);
        float *g = v[li];
        /* stored gradient of this layer's output */
        float *gr = (float *)xalloc(sizeof(float) * (size_t)T * dout);
        memcpy(gr, g, sizeof(float) * (size_t)T * dout);
        if (mode) orc_round_f16(gr, (long long)T * dout);
        net->gact[li] = gr;
        float *dx = NULL;
        switch (L->type) {
            case ORC_OUTPUT:
            case ORC_LINEAR: {
                const float *dz = gr;
                net->gW[li] = (float *)xalloc(sizeof(float) * (size_t)din * dout);
                matmul_tn(din, dout, T, x, dz, net->gW[li]);
                if (L->type == ORC_OUTPUT) net->gb[li] = colsum(dz, T, dout);
                if (need_dx) {
                    dx = (float *)xalloc(sizeof(float) * (size_t)T * din);
                    matmul_nt(T, din, dout, dz, L->W, dx); /* W [din x dout] viewed as B^T */
                }
                break;
            }
            case ORC_ATTENTION: {
                const int A = L->heads * (2 * L->kd + L->vd + L->ctx);
                float *dz = (float *)xalloc(sizeof(float) * (size_t)T * dout);
                for (long long i = 0; i < (long long)T * dout; ++i)
                    dz[i] = net->mask[li][i] ? g[i] * bn_scale(&L->bn, (int)(i % dout)) : 0.f;
                if (mode) orc_round_f16(dz, (long long)T * dout);
                float *dp = (float *)xalloc(sizeof(float) * (size_t)T * A);
                att_backward(L, net->aux[li], T, dz, dp);
                free(dz);
                if (mode) orc_round_f16(dp, (long long)T * A);  /* stored fp16 on the GPU */
                net->gW[li] = (float *)xalloc(sizeof(float) * (size_t)din * A);
                matmul_tn(din, A, T, x, dp, net->gW[li]);
                net->gb[li] = colsum(dp, T, A);
                if (need_dx) {
                    dx = (float *)xalloc(sizeof(float) * (size_t)T * din);
                    matmul_nt(T, din, A, dp, L->W, dx);
                }
                free(dp);
                break;
            }
            case ORC_CONV: {
                float *dz = (float *)xalloc(sizeof(float) * (size_t)T * dout);
                for (long long i = 0; i < (long long)T * dout; ++i) {
                    int f = (int)(i % L->fout);
                    dz[i] = net->mask[li][i] ? g[i] * bn_scale(&L->bn, f) : 0.f;
                }
                if (mode) orc_round_f16(dz, (long long)T * dout);
                const int pd = L->noff * L->fin, rows = T * L->hout;
                float *p = im2col(L, x, T);
                net->gW[li] = (float *)xalloc(sizeof(float) * (size_t)pd * L->fout);
                matmul_tn(pd, L->fout, rows, p, dz, net->gW[li]);
                free(p);
                net->gb[li] = colsum(dz, rows, L->fout);
                if (need_dx) {
                    float *dp = (float *)xalloc(sizeof(float) * (size_t)rows * pd);
                    matmul_nt(rows, pd, L->fout, dz, L->W, dp);
                    dx = (float *)xalloc(sizeof(float) * (size_t)T * din);
                    col2im_add(L, dp, T, dx);
                    free(dp);
                }
                free(dz);
                break;
            }
            case ORC_TDNNF: {
                const int s = L->stride, bn = L->bn_dim;
                /* implicit dz (kf_oracle.h): the GPU's dx_epilogue stores no dz for this layer */
                const int imp = net->implicit_dz && mode == ORC_ROUND_FUSED && !net->mx8 && li != top_li &&
                                L->bypass > 0.f && din == dout && dout > 128 && !(dout % 160 == 0 && dout <= 320);
                float *dz = (float *)xalloc(sizeof(float) * (size_t)T * dout);
                for (long long i = 0; i < (long long)T * dout; ++i) {
                    int d = (int)(i % dout);
                    if (imp) dz[i] = net->mask[li][i] ? gr[i] : 0.f;  /* rne(v) masked, unscaled */
                    else dz[i] = net->mask[li][i] ? g[i] * bn_scale(&L->bn, d) : 0.f;
                }
                /* MXFP8 train step (network.cpp backward_impl): the affine input gradient of a
                   strided layer reads the e4m3 copy of the unrounded dz and of W2's rows, except
                   for row T-1 (the clamped-edge row), which stays fp16 */
                float *dz8 = NULL;
                if (net->mx8 && s > 0 && T > 1 && mx_dgrad_layer(net, li)) dz8 = mx_rows_new(dz, T, dout);
                if (mode && !imp) orc_round_f16(dz, (long long)T * dout);
                const float *bott = net->aux[li];
                const int kaff = s > 0 ? 2 * bn : bn, klin = s > 0 ? 2 * din : din;
                float *aff_in = s > 0 ? splice_plus(bott, T, bn, s) : (float *)bott;
                net->gW2[li] = (float *)xalloc(sizeof(float) * (size_t)kaff * dout);
                matmul_tn(kaff, dout, T, aff_in, dz, net->gW2[li]);
                if (s > 0) free(aff_in);
                net->gb2[li] = colsum(dz, T, dout);
                const float *w2 = L->W2;
                float *w2s = NULL;
                if (imp) {
                    /* the BN scale after the reduction (kf_gemm_wgrad_scaled) and folded into
                       rne(W2 * scale) for the input gradient (kf_scale_cols) */
                    for (int r = 0; r < kaff; ++r)
                        for (int d = 0; d < dout; ++d) net->gW2[li][(size_t)r * dout + d] *= bn_scale(&L->bn, d);
                    for (int d = 0; d < dout; ++d) net->gb2[li][d] *= bn_scale(&L->bn, d);
                    w2s = (float *)xalloc(sizeof(float) * (size_t)kaff * dout);
                    for (int r = 0; r < kaff; ++r)
                        for (int d = 0; d < dout; ++d)
                            w2s[(size_t)r * dout + d] = L->W2[(size_t)r * dout + d] * bn_scale(&L->bn, d);
                    orc_round_f16(w2s, (long long)kaff * dout);
                    w2 = w2s;
                }
                float *daff = (float *)xalloc(sizeof(float) * (size_t)T * kaff);
                matmul_nt(T, kaff, dout, dz, w2, daff);
                free(w2s);
                float *daff8 = daff;
                if (dz8) {
                    float *w8 = mx_rows_new(L->W2, kaff, dout);
                    daff8 = (float *)xalloc(sizeof(float) * (size_t)T * kaff);
                    matmul_nt(T, kaff, dout, dz8, w8, daff8);
                    free(w8);
                    free(dz8);
                }
                float *dbott = (float *)xalloc(sizeof(float) * (size_t)T * bn);
                for (int t = 0; t < T; ++t) {
                    const float *da = t == T - 1 ? daff : daff8;
                    for (int c = 0; c < bn; ++c) dbott[(size_t)t * bn + c] += da[(size_t)t * kaff + c];
                }
                if (s > 0)
                    for (int t = 0; t < T; ++t) {
                        int tp = t + s > T - 1 ? T - 1 : t + s;
                        const float *da = tp == T - 1 ? daff : daff8;
                        for (int c = 0; c < bn; ++c)
                            dbott[(size_t)tp * bn + c] += da[(size_t)t * kaff + bn + c];
                    }
                if (daff8 != daff) free(daff8);
                free(daff);
                if (mode) orc_round_f16(dbott, (long long)T * bn);
                float *lin_in = s > 0 ? splice_minus(x, T, din, s) : (float *)x;
                net->gW[li] = (float *)xalloc(sizeof(float) * (size_t)klin * bn);
                matmul_tn(klin, bn, T, lin_in, dbott, net->gW[li]);
                if (s > 0) free(lin_in);
                if (need_dx) {
                    float *dlin = (float *)xalloc(sizeof(float) * (size_t)T * klin);
                    matmul_nt(T, klin, bn, dbott, L->W, dlin);
                    dx = (float *)xalloc(sizeof(float) * (size_t)T * din);
                    if (s > 0) {
                        for (int t = 0; t < T; ++t) {
                            int tp = t - s < 0 ? 0 : t - s;
                            for (int c = 0; c < din; ++c) {
                                dx[(size_t)t * din + c] += dlin[(size_t)t * klin + din + c];
                                dx[(size_t)tp * din + c] += dlin[(size_t)t * klin + c];
                            }
                        }
                    } else {
                        memcpy(dx, dlin, sizeof(float) * (size_t)T * din);
                    }
                    free(dlin);
                    if (L->bypass > 0.f && din == dout)
                        for (long long i = 0; i < (long long)T * din; ++i) dx[i] += L->bypass * gr[i];
                }
                free(dbott);
                free(dz);
                break;
            }
            case ORC_PREFINAL: {
                const int big = L->big_dim, small = L->small_dim;
                float *ds = (float *)xalloc(sizeof(float) * (size_t)T * small);
                for (long long i = 0; i < (long long)T * small; ++i) {
                    int d = (int)(i % small);
                    ds[i] = L->bn2.mean ? g[i] * bn_scale(&L->bn2, d) : g[i];
                }
                if (mode) orc_round_f16(ds, (long long)T * small);
                const float *bg = net->aux[li];
                net->gW2[li] = (float *)xalloc(sizeof(float) * (size_t)big * small);
                matmul_tn(big, small, T, bg, ds, net->gW2[li]);
                float *dbig = (float *)xalloc(sizeof(float) * (size_t)T * big);
                matmul_nt(T, big, small, ds, L->W2, dbig);
                for (long long i = 0; i < (long long)T * big; ++i) {
                    int d = (int)(i % big);
                    dbig[i] = net->mask[li][i] ? dbig[i] * bn_scale(&L->bn, d) : 0.f;
                }
                if (mode) orc_round_f16(dbig, (long long)T * big);
                net->gW[li] = (float *)xalloc(sizeof(float) * (size_t)din * big);
                matmul_tn(din, big, T, x, dbig, net->gW[li]);
                net->gb[li] = colsum(dbig, T, big);
                if (need_dx) {
                    dx = (float *)xalloc(sizeof(float) * (size_t)T * din);
                    matmul_nt(T, din, big, dbig, L->W, dx);
                }
                free(dbig);
                free(ds);
                break;
            }
            case ORC_COMBINE: {
                /* the ivector branch: the broadcast columns summed per sequence (from the
                 * stored fp16 gradient), then back through its batchnorm(s) and linear */
                if (L->input2 < 0 || !net->layers[L->input2].per_seq) break;
                const int n1 = L->nf1, n2 = L->nf2, nf = n1 + n2, H = L->height, R = net->B;
                float *db = (float *)xalloc(sizeof(float) * (size_t)R * H * n2);
                for (int s2 = 0; s2 < R; ++s2)
                    for (int t = net->seq_off[s2]; t < net->seq_off[s2 + 1]; ++t)
                        for (int h = 0; h < H; ++h)
                            for (int q = 0; q < n2; ++q)
                                db[(size_t)s2 * H * n2 + h * n2 + q] += gr[(size_t)t * dout + h * nf + n1 + q];
                if (mode) orc_round_f16(db, (long long)R * H * n2);
                for (int cur = L->input2; cur >= 0; cur = net->layers[cur].input) {
                    const OrcLayer *Q = &net->layers[cur];
                    const int qd = Q->out_dim;
                    if (Q->type == ORC_BATCHNORM) {
                        for (long long i = 0; i < (long long)R * qd; ++i) db[i] *= bn_scale(&Q->bn, (int)(i % qd));
                        if (mode) orc_round_f16(db, (long long)R * qd);
                    } else if (Q->type == ORC_LINEAR) {
                        const float *xq = Q->input == -2 ? net->ivec : net->act[Q->input];
                        net->gW[cur] = (float *)xalloc(sizeof(float) * (size_t)Q->in_dim * qd);
                        matmul_tn(Q->in_dim, qd, R, xq, db, net->gW[cur]);
                        break; /* its input is the ivector input */
                    }
                }
                free(db);
                break;
            }
            case ORC_BATCHNORM:
                if (need_dx) {
                    dx = (float *)xalloc(sizeof(float) * (size_t)T * din);
                    for (long long i = 0; i < (long long)T * din; ++i)
                        dx[i] = g[i] * bn_scale(&L->bn, (int)(i % din));
                }
                break;
            case ORC_IDCT:
                if (need_dx) {
                    dx = (float *)xalloc(sizeof(float) * (size_t)T * din);
                    matmul_nt(T, din, dout, g, L->W, dx);
                }
                break;
            default:
                break;
        }
        if (dx && L->input >= 0) {
            if (v[L->input]) {
                for (long long i = 0; i < (long long)T * din; ++i) v[L->input][i] += dx[i];
                free(dx);
            } else {
                v[L->input] = dx;
            }
        } else {
            free(dx);
        }
    }
    for (int i = 0; i < n; ++i) free(v[i]);
    free(v);
    return 0;
}

void orc_net_free(OrcNet *net) {
    if (!net->act) return;
    for (int i = 0; i < net->nlayers; ++i) {
        free(net->act[i]);
        free(net->mask[i]);
        free(net->aux[i]);
        free(net->gW[i]);
        free(net->gb[i]);
        free(net->gW2[i]);
        free(net->gb2[i]);
        free(net->gact[i]);
        if (net->act8) free(net->act8[i]);
    }
    free(net->act);
    free(net->mask);
    free(net->aux);
    free(net->gW);
    free(net->gb);
    free(net->gW2);
    free(net->gb2);
    free(net->gact);
    free(net->act8);
    net->act8 = NULL;
    net->act = NULL;
}

void orc_sgd(float *w32, const float *g, float *v, float lr, float mom, long long n) {
    for (long long i = 0; i < n; ++i) {
        v[i] = mom * v[i] + g[i];
        w32[i] -= lr * v[i];
    }
}
