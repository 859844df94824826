/*
 * gotorch_net.c — the CNN-TDNN train step in the reference's Go CPU style (SURVEY §8
 * row P2): float64 throughout, each layer computed the way go/gotorch computes its
 * counterpart. A restatement, not Go (no Go toolchain in this image).
 *
 * TEST / BASELINE INFRASTRUCTURE ONLY: loaded by tests/ and bench.py's cpu_baseline.
 *
 * Layer mapping (the network is this build's xconfig, described by OrcLayer):
 *   idct, linear, output, prefinal big / small affines
 *       -> AffineLayer (layers.go:57-110): forward MatMul (ops.go:15-34), rows over
 *          `workers` threads as matmulParallel (ops.go:49-81, gotorch_cpu.c gt_matmul);
 *          backward single-threaded loops: GradB, GradW (b, i, j), gradInput (b, i, j)
 *   TDNN-F linear [x(t-s) | x(t)] and affine [y(t) | y(t+s)]
 *       -> TDNNLayer (layers.go:409-535) with Context {-s, 0} / {0, +s} ({0} at s = 0):
 *          single-threaded (b, t, o, ci, i) loops, edge-clamped context, weights
 *          [(ci * in + i) x out], Bias as the starting sum
 *   conv-relu-batchnorm
 *       -> Conv1DLayer's loop form (cnn_tdnn.go:85-184) over this build's Kaldi
 *          (time, height) offsets: single-threaded (t, h, oc, k, ic) loops, zero padding
 *   ReLU (layers.go:127-157), frozen BatchNorm of the product path (ops.cu:171-204 as
 *   kf_oracle.c bn_apply: gotorch's BatchNormLayer would use batch statistics in train
 *   mode, which costs the same elementwise pass), SGD with momentum 0.9 (model.go:212-279).
 * The arithmetic is the oracle's (kf_oracle.c) in float64; tests/test_gotorch_net.py
 * checks it against the oracle's unrounded mode.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "kf_oracle.h"

void gt_matmul(const double *a, const double *b, double *c, int M, int K, int N, int workers);

typedef struct {
    const OrcLayer *L;
    double *W, *b, *W2, *b2;    /* float64 parameter copies */
    double *gW, *gb, *gW2, *gb2;
    double *vW, *vb, *vW2, *vb2; /* SGD velocities */
    long long nW, nb, nW2, nb2;
    double *bsc, *bsh;   /* frozen BN as y = x * bsc + bsh */
    double *bsc2, *bsh2; /* prefinal's second BN */
    double *y;           /* output activation [T x out] */
    double *aux;         /* TDNN-F bottleneck / prefinal big activation */
    unsigned char *mask; /* ReLU decisions */
} GtLayer;

typedef struct {
    int n, T;
    GtLayer *l;
} GtNet;

static double *dup(const float *p, long long n) {
    if (!p || n <= 0) return NULL;
    double *d = (double *)malloc(sizeof(double) * (size_t)n);
    for (long long i = 0; i < n; ++i) d[i] = p[i];
    return d;
}
static double *zalloc(long long n) { return (double *)calloc((size_t)(n > 0 ? n : 1), sizeof(double)); }

static void bn_prep(const OrcBN *bn, int D, double **sc, double **sh) {
    *sc = *sh = NULL;
    if (!bn->mean) return;
    *sc = zalloc(D);
    *sh = zalloc(D);
    for (int d = 0; d < D; ++d) {
        const double inv = 1.0 / sqrt((double)bn->var[d] + (double)bn->eps);
        if (bn->target_rms != 1.0f) {
            (*sc)[d] = bn->target_rms * inv;
            (*sh)[d] = -bn->mean[d] * bn->target_rms * inv;
        } else {
            (*sc)[d] = bn->gamma[d] * inv;
            (*sh)[d] = bn->beta[d] - bn->gamma[d] * bn->mean[d] * inv;
        }
    }
}

GtNet *gt_net_create(const OrcLayer *layers, int n) {
    GtNet *g = (GtNet *)calloc(1, sizeof(GtNet));
    g->n = n;
    g->l = (GtLayer *)calloc((size_t)n, sizeof(GtLayer));
    for (int i = 0; i < n; ++i) {
        const OrcLayer *L = &layers[i];
        GtLayer *q = &g->l[i];
        q->L = L;
        const int din = L->in_dim, dout = L->out_dim;
        switch (L->type) {
            case ORC_IDCT: q->nW = (long long)din * dout; break;
            case ORC_LINEAR: q->nW = (long long)din * dout; break;
            case ORC_OUTPUT: q->nW = (long long)din * dout, q->nb = dout; break;
            case ORC_CONV: q->nW = (long long)L->noff * L->fin * L->fout, q->nb = L->fout; break;
            case ORC_TDNNF: {
                const int s = L->stride;
                q->nW = (long long)(s > 0 ? 2 * din : din) * L->bn_dim;
                q->nW2 = (long long)(s > 0 ? 2 * L->bn_dim : L->bn_dim) * dout;
                q->nb2 = dout;
                break;
            }
            case ORC_PREFINAL:
                q->nW = (long long)din * L->big_dim, q->nb = L->big_dim;
                q->nW2 = (long long)L->big_dim * L->small_dim;
                break;
            case ORC_BATCHNORM: break;
            default: /* attention / combine / per-sequence branches: not in the gotorch template */
                free(g->l);
                free(g);
                return NULL;
        }
        if (L->per_seq) {
            free(g->l);
            free(g);
            return NULL;
        }
        q->W = dup(L->W, q->nW);
        q->b = dup(L->type == ORC_TDNNF ? NULL : L->b, q->nb);
        q->W2 = dup(L->W2, q->nW2);
        q->b2 = dup(L->b2, q->nb2);
        q->vW = zalloc(q->nW), q->vb = zalloc(q->nb), q->vW2 = zalloc(q->nW2), q->vb2 = zalloc(q->nb2);
        const int bnd = L->type == ORC_CONV ? L->fout : L->type == ORC_PREFINAL ? L->big_dim : dout;
        bn_prep(&L->bn, bnd, &q->bsc, &q->bsh);
        if (L->type == ORC_PREFINAL) bn_prep(&L->bn2, L->small_dim, &q->bsc2, &q->bsh2);
    }
    return g;
}

static void free_step(GtLayer *q) {
    free(q->y), free(q->aux), free(q->mask);
    free(q->gW), free(q->gb), free(q->gW2), free(q->gb2);
    q->y = q->aux = NULL, q->mask = NULL;
    q->gW = q->gb = q->gW2 = q->gb2 = NULL;
}

void gt_net_free(GtNet *g) {
    if (!g) return;
    for (int i = 0; i < g->n; ++i) {
        GtLayer *q = &g->l[i];
        free_step(q);
        free(q->W), free(q->b), free(q->W2), free(q->b2);
        free(q->vW), free(q->vb), free(q->vW2), free(q->vb2);
        free(q->bsc), free(q->bsh), free(q->bsc2), free(q->bsh2);
    }
    free(g->l);
    free(g);
}

/* TDNNLayer.Forward (layers.go:443-475): y[t][o] = bias[o] + sum_ci sum_i
 * x[clamp(t + ctx[ci])][i] * W[(ci * in + i) * out + o] */
static void tdnn_forward(const double *x, int T, int in, const int *ctx, int nctx, const double *W,
                         const double *bias, int out, double *y) {
    for (int t = 0; t < T; ++t)
        for (int o = 0; o < out; ++o) {
            double sum = bias ? bias[o] : 0.0;
            for (int ci = 0; ci < nctx; ++ci) {
                int tc = t + ctx[ci];
                tc = tc < 0 ? 0 : tc >= T ? T - 1 : tc;
                const double *xr = x + (size_t)tc * in;
                for (int i = 0; i < in; ++i) sum += xr[i] * W[((size_t)ci * in + i) * out + o];
            }
            y[(size_t)t * out + o] = sum;
        }
}
/* TDNNLayer.Backward (layers.go:478-522); gx may be NULL (no input gradient needed) */
static void tdnn_backward(const double *x, int T, int in, const int *ctx, int nctx, const double *W, int out,
                          const double *gy, double *gW, double *gb, double *gx) {
    for (int t = 0; t < T; ++t)
        for (int o = 0; o < out; ++o) {
            const double grad = gy[(size_t)t * out + o];
            if (gb) gb[o] += grad;
            for (int ci = 0; ci < nctx; ++ci) {
                int tc = t + ctx[ci];
                tc = tc < 0 ? 0 : tc >= T ? T - 1 : tc;
                const double *xr = x + (size_t)tc * in;
                for (int i = 0; i < in; ++i) {
                    const size_t w = ((size_t)ci * in + i) * out + o;
                    gW[w] += xr[i] * grad;
                    if (gx) gx[(size_t)tc * in + i] += W[w] * grad;
                }
            }
        }
}

/* AffineLayer.Forward (layers.go:57-70) */
static void affine_forward(const double *x, int T, int in, const double *W, const double *bias, int out, double *y,
                           int workers) {
    memset(y, 0, sizeof(double) * (size_t)T * out);
    gt_matmul(x, W, y, T, in, out, workers);
    if (bias)
        for (int t = 0; t < T; ++t)
            for (int j = 0; j < out; ++j) y[(size_t)t * out + j] += bias[j];
}
/* AffineLayer.Backward (layers.go:72-110); gx may be NULL */
static void affine_backward(const double *x, int T, int in, const double *W, int out, const double *gy,
                            double *gW, double *gb, double *gx) {
    if (gb)
        for (int b = 0; b < T; ++b)
            for (int j = 0; j < out; ++j) gb[j] += gy[(size_t)b * out + j];
    for (int b = 0; b < T; ++b)
        for (int i = 0; i < in; ++i) {
            const double xv = x[(size_t)b * in + i];
            for (int j = 0; j < out; ++j) gW[(size_t)i * out + j] += xv * gy[(size_t)b * out + j];
        }
    if (gx)
        for (int b = 0; b < T; ++b)
            for (int i = 0; i < in; ++i) {
                double sum = 0.0;
                for (int j = 0; j < out; ++j) sum += gy[(size_t)b * out + j] * W[(size_t)i * out + j];
                gx[(size_t)b * in + i] = sum;
            }
}

/* ReLU then frozen BN over rows x D (column = i % D), recording the ReLU decisions */
static void relu_bn(double *y, long long n, int D, const double *sc, const double *sh, unsigned char *mask) {
    for (long long i = 0; i < n; ++i) {
        const int d = (int)(i % D);
        double v = y[i];
        if (mask) {
            mask[i] = v > 0.0;
            if (!mask[i]) v = 0.0;
        }
        if (sc) v = v * sc[d] + sh[d];
        y[i] = v;
    }
}

static const double *layer_input(GtNet *g, const OrcLayer *L, const double *features) {
    return L->input < 0 ? features : g->l[L->input].y;
}

int gt_net_forward(GtNet *g, const double *features, int T, int workers) {
    g->T = T;
    for (int li = 0; li < g->n; ++li) {
        GtLayer *q = &g->l[li];
        const OrcLayer *L = q->L;
        free_step(q);
        const double *x = layer_input(g, L, features);
        const int din = L->in_dim, dout = L->out_dim;
        double *y = zalloc((long long)T * dout);
        switch (L->type) {
            case ORC_IDCT:
            case ORC_LINEAR: affine_forward(x, T, din, q->W, NULL, dout, y, workers); break;
            case ORC_OUTPUT:
                affine_forward(x, T, din, q->W, q->b, dout, y, workers);
                if (L->log_softmax)
                    for (int t = 0; t < T; ++t) {
                        double *r = y + (size_t)t * dout, mx = -INFINITY, s = 0.0;
                        for (int d = 0; d < dout; ++d) mx = r[d] > mx ? r[d] : mx;
                        for (int d = 0; d < dout; ++d) s += exp(r[d] - mx);
                        for (int d = 0; d < dout; ++d) r[d] -= mx + log(s);
                    }
                break;
            case ORC_BATCHNORM:
                for (long long i = 0; i < (long long)T * dout; ++i)
                    y[i] = q->bsc ? x[i] * q->bsc[i % dout] + q->bsh[i % dout] : x[i];
                break;
            case ORC_CONV: {
                /* Conv1DLayer.Forward's loop (cnn_tdnn.go:85-124) over (time, height) offsets */
                const int fin = L->fin, fout = L->fout, hin = L->hin;
                for (int t = 0; t < T; ++t)
                    for (int h = 0; h < L->hout; ++h)
                        for (int oc = 0; oc < fout; ++oc) {
                            double sum = 0.0;
                            for (int k = 0; k < L->noff; ++k) {
                                const int ts = t + L->toff[k], hs = h * L->sub + L->hoff[k];
                                if (ts < 0 || ts >= T || hs < 0 || hs >= hin) continue;
                                const double *xr = x + ((size_t)ts * hin + hs) * fin;
                                for (int ic = 0; ic < fin; ++ic) sum += xr[ic] * q->W[((size_t)k * fin + ic) * fout + oc];
                            }
                            y[((size_t)t * L->hout + h) * fout + oc] = sum + q->b[oc];
                        }
                q->mask = (unsigned char *)calloc((size_t)T * dout, 1);
                relu_bn(y, (long long)T * dout, fout, q->bsc, q->bsh, q->mask);
                break;
            }
            case ORC_TDNNF: {
                const int s = L->stride, bn = L->bn_dim;
                const int cl[2] = {-s, 0}, ca[2] = {0, s};
                const int nc = s > 0 ? 2 : 1;
                q->aux = zalloc((long long)T * bn);
                tdnn_forward(x, T, din, s > 0 ? cl : cl + 1, nc, q->W, NULL, bn, q->aux);
                tdnn_forward(q->aux, T, bn, ca, nc, q->W2, q->b2, dout, y);
                q->mask = (unsigned char *)calloc((size_t)T * dout, 1);
                relu_bn(y, (long long)T * dout, dout, q->bsc, q->bsh, q->mask);
                if (L->bypass > 0.f && din == dout)
                    for (long long i = 0; i < (long long)T * dout; ++i) y[i] += (double)L->bypass * x[i];
                break;
            }
            case ORC_PREFINAL: {
                const int big = L->big_dim, small = L->small_dim;
                q->aux = zalloc((long long)T * big);
                affine_forward(x, T, din, q->W, q->b, big, q->aux, workers);
                q->mask = (unsigned char *)calloc((size_t)T * big, 1);
                relu_bn(q->aux, (long long)T * big, big, q->bsc, q->bsh, q->mask);
                affine_forward(q->aux, T, big, q->W2, NULL, small, y, workers);
                relu_bn(y, (long long)T * small, small, q->bsc2, q->bsh2, NULL);
                break;
            }
            default:
                free(y);
                return -1;
        }
        q->y = y;
    }
    return 0;
}

static int trainable_below(const GtNet *g, int cur) {
    if (cur < 0) return 0;
    const int ty = g->l[cur].L->type;
    if (ty == ORC_CONV || ty == ORC_TDNNF || ty == ORC_LINEAR || ty == ORC_PREFINAL || ty == ORC_OUTPUT) return 1;
    return trainable_below(g, g->l[cur].L->input);
}

/* Sequential.Backward (model.go:33-39) from the gradient of the top layer's output */
int gt_net_backward(GtNet *g, const double *features, const double *out_grad, int top) {
    const int T = g->T;
    if (top < 0 || top >= g->n) return -1;
    double **v = (double **)calloc((size_t)g->n, sizeof(double *));
    v[top] = zalloc((long long)T * g->l[top].L->out_dim);
    memcpy(v[top], out_grad, sizeof(double) * (size_t)T * g->l[top].L->out_dim);
    for (int li = top; li >= 0; --li) {
        GtLayer *q = &g->l[li];
        const OrcLayer *L = q->L;
        double *gy = v[li];
        if (!gy) continue;
        const int din = L->in_dim, dout = L->out_dim;
        const double *x = layer_input(g, L, features);
        const int need_dx = trainable_below(g, L->input);
        double *dx = need_dx ? zalloc((long long)T * din) : NULL;
        q->gW = zalloc(q->nW), q->gb = zalloc(q->nb), q->gW2 = zalloc(q->nW2), q->gb2 = zalloc(q->nb2);
        switch (L->type) {
            case ORC_OUTPUT:
            case ORC_LINEAR:
            case ORC_IDCT:
                affine_backward(x, T, din, q->W, dout, gy, q->gW, L->type == ORC_OUTPUT ? q->gb : NULL, dx);
                break;
            case ORC_BATCHNORM:
                if (dx)
                    for (long long i = 0; i < (long long)T * din; ++i) dx[i] = gy[i] * (q->bsc ? q->bsc[i % din] : 1.0);
                break;
            case ORC_CONV: {
                const int fin = L->fin, fout = L->fout, hin = L->hin;
                double *dz = zalloc((long long)T * dout);
                for (long long i = 0; i < (long long)T * dout; ++i)
                    dz[i] = q->mask[i] ? gy[i] * (q->bsc ? q->bsc[i % fout] : 1.0) : 0.0;
                /* Conv1DLayer.Backward's loop (cnn_tdnn.go:128-172) */
                for (int t = 0; t < T; ++t)
                    for (int h = 0; h < L->hout; ++h)
                        for (int oc = 0; oc < fout; ++oc) {
                            const double grad = dz[((size_t)t * L->hout + h) * fout + oc];
                            q->gb[oc] += grad;
                            for (int k = 0; k < L->noff; ++k) {
                                const int ts = t + L->toff[k], hs = h * L->sub + L->hoff[k];
                                if (ts < 0 || ts >= T || hs < 0 || hs >= hin) continue;
                                const size_t xo = ((size_t)ts * hin + hs) * fin;
                                for (int ic = 0; ic < fin; ++ic) {
                                    const size_t w = ((size_t)k * fin + ic) * fout + oc;
                                    q->gW[w] += x[xo + ic] * grad;
                                    if (dx) dx[xo + ic] += q->W[w] * grad;
                                }
                            }
                        }
                free(dz);
                break;
            }
            case ORC_TDNNF: {
                const int s = L->stride, bn = L->bn_dim;
                const int cl[2] = {-s, 0}, ca[2] = {0, s};
                const int nc = s > 0 ? 2 : 1;
                double *dz = zalloc((long long)T * dout);
                for (long long i = 0; i < (long long)T * dout; ++i)
                    dz[i] = q->mask[i] ? gy[i] * (q->bsc ? q->bsc[i % dout] : 1.0) : 0.0;
                double *dbott = zalloc((long long)T * bn);
                tdnn_backward(q->aux, T, bn, ca, nc, q->W2, dout, dz, q->gW2, q->gb2, dbott);
                tdnn_backward(x, T, din, s > 0 ? cl : cl + 1, nc, q->W, bn, dbott, q->gW, NULL, dx);
                if (dx && L->bypass > 0.f && din == dout)
                    for (long long i = 0; i < (long long)T * din; ++i) dx[i] += (double)L->bypass * gy[i];
                free(dz);
                free(dbott);
                break;
            }
            case ORC_PREFINAL: {
                const int big = L->big_dim, small = L->small_dim;
                double *ds = zalloc((long long)T * small);
                for (long long i = 0; i < (long long)T * small; ++i)
                    ds[i] = gy[i] * (q->bsc2 ? q->bsc2[i % small] : 1.0);
                double *dbig = zalloc((long long)T * big);
                affine_backward(q->aux, T, big, q->W2, small, ds, q->gW2, NULL, dbig);
                for (long long i = 0; i < (long long)T * big; ++i)
                    dbig[i] = q->mask[i] ? dbig[i] * (q->bsc ? q->bsc[i % big] : 1.0) : 0.0;
                affine_backward(x, T, din, q->W, big, dbig, q->gW, q->gb, dx);
                free(ds);
                free(dbig);
                break;
            }
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
    for (int i = 0; i < g->n; ++i) free(v[i]);
    free(v);
    return 0;
}

/* SGD.Step (model.go:236-268): momentum 0.9, no weight decay */
static void sgd1(double *p, const double *gr, double *v, long long n, double lr, double mom) {
    if (!p || !gr) return;
    for (long long j = 0; j < n; ++j) v[j] = mom * v[j] + gr[j];
    for (long long j = 0; j < n; ++j) p[j] -= lr * v[j];
}
void gt_net_sgd(GtNet *g, double lr, double mom) {
    for (int i = 0; i < g->n; ++i) {
        GtLayer *q = &g->l[i];
        if (q->L->type == ORC_IDCT) continue; /* fixed matrix, not a parameter */
        sgd1(q->W, q->gW, q->vW, q->nW, lr, mom);
        sgd1(q->b, q->gb, q->vb, q->nb, lr, mom);
        sgd1(q->W2, q->gW2, q->vW2, q->nW2, lr, mom);
        sgd1(q->b2, q->gb2, q->vb2, q->nb2, lr, mom);
    }
}

/* accessors: which = 0 output activation, 1 gW, 2 gb, 3 gW2, 4 gb2, 5 W, 6 W2 */
const double *gt_net_tensor(const GtNet *g, int li, int which, long long *n) {
    if (li < 0 || li >= g->n) return NULL;
    const GtLayer *q = &g->l[li];
    switch (which) {
        case 0: *n = (long long)g->T * q->L->out_dim; return q->y;
        case 1: *n = q->nW; return q->gW;
        case 2: *n = q->nb; return q->gb;
        case 3: *n = q->nW2; return q->gW2;
        case 4: *n = q->nb2; return q->gb2;
        case 5: *n = q->nW; return q->W;
        case 6: *n = q->nW2; return q->W2;
        default: return NULL;
    }
}
