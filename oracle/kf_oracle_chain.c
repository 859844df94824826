/*
 * kf_oracle_chain.c — CPU restatement of the reference's chain LF-MMI objective.
 *
 * TEST INFRASTRUCTURE ONLY (see kf_oracle.h): the checker for the HIP chain
 * kernels and the CPU baseline's objective leg. Plain sequential C, in the
 * reference's data types (float32 state vectors, float64 log-correction and
 * initial probabilities):
 *   - denominator: cpp/cuda/chain_den.cu:122-706 with the initial-prob rule of
 *     internal/nnet/denominator.go:131-171;
 *   - numerator:   the deterministic log-domain forward-backward of
 *     cpp/cuda/chain_det.cu:26-237 (fixed arc order, LogAdd of :26-35,
 *     posterior clamp of chain.cu:309-311);
 *   - objective:   ComputeChainObjfAndDeriv, internal/nnet/backward.go:224-371,
 *     with the pieces of cpp/cuda/chain_backward.cu:27-180.
 */
#include "kf_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

static const float kLogZero = -1.0e+30f;

static void *zalloc(size_t n) {
    void *p = calloc(n ? n : 1, 1);
    if (!p) abort();
    return p;
}

/* denominator.go:131-171 */
void orc_den_initial_probs(int S, int A, const int *src, const int *dst, const float *tp,
                           int start, float *init_out) {
    double *cur = zalloc(sizeof(double) * S), *next = zalloc(sizeof(double) * S);
    double *avg = zalloc(sizeof(double) * S);
    cur[start] = 1.0;
    for (int it = 0; it < 100; ++it) {
        for (int s = 0; s < S; ++s) avg[s] += cur[s] / 100.0;
        memset(next, 0, sizeof(double) * S);
        for (int a = 0; a < A; ++a) next[dst[a]] += cur[src[a]] * (double)tp[a];
        double tot = 0.0;
        for (int s = 0; s < S; ++s) tot += next[s];
        if (tot > 0) {
            double inv = 1.0 / tot;
            for (int s = 0; s < S; ++s) next[s] *= inv;
        }
        double *t = cur;
        cur = next;
        next = t;
    }
    for (int s = 0; s < S; ++s) init_out[s] = (float)avg[s];
    free(cur);
    free(next);
    free(avg);
}

static float fsum(const float *x, int n) {
    float s = 0.f;
    for (int i = 0; i < n; ++i) s += x[i];
    return s;
}

/* chain_den.cu:496-706 (den_forward :371-472 is its first half) */
float orc_den_forward_backward(const OrcDen *d, const float *nnet, int T, float leaky, float *post) {
    const int S = d->S, P = d->P, A = d->A;
    float *ex = zalloc(sizeof(float) * (size_t)T * P);
    for (long long i = 0; i < (long long)T * P; ++i) { /* kernel_apply_exp :122-131 */
        float v = nnet[i];
        v = fmaxf(-30.0f, fminf(30.0f, v));
        ex[i] = expf(v);
    }
    float *adash = zalloc(sizeof(float) * (size_t)(T + 1) * S);
    float *alpha = zalloc(sizeof(float) * S);
    float *asum = zalloc(sizeof(float) * (T + 1));
    /* AlphaFirstFrame + AlphaDash(0) */
    memcpy(alpha, d->init, sizeof(float) * S);
    asum[0] = fsum(alpha, S);
    for (int s = 0; s < S; ++s) adash[s] = alpha[s] + asum[0] * leaky * d->init[s];
    double logc = 0.0;
    for (int t = 1; t <= T; ++t) {
        const float *xa = ex + (size_t)(t - 1) * P;
        const float *ap = adash + (size_t)(t - 1) * S;
        memset(alpha, 0, sizeof(float) * S);
        for (int a = 0; a < A; ++a) { /* kernel_den_forward_transitions :158-183 */
            float sv = ap[d->src[a]];
            if (sv <= 0.0f) continue;
            int p = d->pdf0[a];
            float xv = (p >= 0 && p < P) ? xa[p] : 0.0f;
            float c = sv * d->tp[a] * xv;
            if (c > 0.0f) alpha[d->dst[a]] += c;
        }
        if (asum[t - 1] > 0.0f) {
            float inv = 1.0f / asum[t - 1];
            for (int s = 0; s < S; ++s) alpha[s] *= inv;
            logc += log((double)asum[t - 1]);
        }
        asum[t] = fsum(alpha, S);
        float *an = adash + (size_t)t * S;
        for (int s = 0; s < S; ++s) an[s] = alpha[s] + asum[t] * leaky * d->init[s];
    }
    float total = fsum(adash + (size_t)T * S, S);
    float logprob = (float)(log((double)total) + logc);
    if (post) {
        float *bd = zalloc(sizeof(float) * S), *b = zalloc(sizeof(float) * S);
        memset(post, 0, sizeof(float) * (size_t)T * P);
        float inv_tot = total > 0.0f ? 1.0f / total : 0.0f;
        for (int s = 0; s < S; ++s) bd[s] = inv_tot;
        float dot = 0.f;
        for (int s = 0; s < S; ++s) dot += d->init[s] * bd[s];
        float tb = leaky * dot;
        for (int s = 0; s < S; ++s) b[s] = bd[s] + tb;
        for (int t = T - 1; t >= 0; --t) {
            const float *xt = ex + (size_t)t * P;
            const float *ap = adash + (size_t)t * S;
            float *gt = post + (size_t)t * P;
            memset(bd, 0, sizeof(float) * S);
            for (int a = 0; a < A; ++a) {
                int p = d->pdf0[a];
                float bv = b[d->dst[a]];
                if (bv > 0.0f) { /* kernel_den_backward_transitions :222-247 */
                    float xv = (p >= 0 && p < P) ? xt[p] : 0.0f;
                    float c = bv * d->tp[a] * xv;
                    if (c > 0.0f) bd[d->src[a]] += c;
                }
                if (p < 0 || p >= P) continue; /* kernel_den_posteriors :253-280 */
                float av = ap[d->src[a]];
                if (av <= 0.0f || bv <= 0.0f) continue;
                float g = av * d->tp[a] * xt[p] * bv;
                if (g > 0.0f) gt[p] += g;
            }
            if (asum[t] > 0.0f) {
                float inv = 1.0f / asum[t];
                for (int s = 0; s < S; ++s) bd[s] *= inv;
                for (int p = 0; p < P; ++p) gt[p] *= inv;
            }
            dot = 0.f;
            for (int s = 0; s < S; ++s) dot += d->init[s] * bd[s];
            tb = leaky * dot;
            for (int s = 0; s < S; ++s) b[s] = bd[s] + tb;
        }
        free(bd);
        free(b);
    }
    free(ex);
    free(adash);
    free(alpha);
    free(asum);
    return logprob;
}

/* chain_det.cu:26-35 */
static float logadd(float a, float b) {
    if (a <= kLogZero) return b;
    if (b <= kLogZero) return a;
    float mx = fmaxf(a, b), mn = fminf(a, b);
    return mx + log1pf(expf(mn - mx));
}

/* chain_det.cu:55-237 (forward by destination over incoming arcs in arc order,
 * backward by source, posteriors in (source, arc) order). */
float orc_num_forward_backward(const OrcNum *n, const float *nnet, int T, int P, float *post) {
    const int S = n->S, A = n->A;
    float *alpha = zalloc(sizeof(float) * (size_t)(T + 1) * S);
    float *beta = zalloc(sizeof(float) * (size_t)(T + 1) * S);
    int *src = zalloc(sizeof(int) * (A > 0 ? A : 1));
    for (int s = 0; s < S; ++s)
        for (int a = n->row_ptr[s]; a < n->row_ptr[s + 1]; ++a) src[a] = s;
    for (long long i = 0; i < (long long)(T + 1) * S; ++i) alpha[i] = beta[i] = kLogZero;
    alpha[n->start] = 0.0f;
    for (int t = 0; t < T; ++t) {
        float *an = alpha + (size_t)(t + 1) * S;
        const float *ac = alpha + (size_t)t * S;
        /* incoming arcs of every dst in arc-index order == sequential arc sweep */
        for (int a = 0; a < A; ++a) {
            int p = n->pdf1[a];
            if (p <= 0 || p > P) continue;
            float sa = ac[src[a]];
            if (sa <= kLogZero) continue;
            float v = sa + nnet[(size_t)t * P + (p - 1)] + n->logw[a];
            an[n->dst[a]] = logadd(an[n->dst[a]], v);
        }
    }
    float total = kLogZero;
    for (int i = 0; i < n->nfinal; ++i)
        total = logadd(total, alpha[(size_t)T * S + n->final_state[i]] + n->final_w[i]);
    for (int i = 0; i < n->nfinal; ++i) beta[(size_t)T * S + n->final_state[i]] = n->final_w[i];
    for (int t = T - 1; t >= 0; --t) {
        float *bc = beta + (size_t)t * S;
        const float *bn = beta + (size_t)(t + 1) * S;
        for (int s = 0; s < S; ++s) {
            float v = kLogZero;
            for (int a = n->row_ptr[s]; a < n->row_ptr[s + 1]; ++a) {
                int p = n->pdf1[a];
                if (p <= 0 || p > P) continue;
                float b = bn[n->dst[a]];
                if (b <= kLogZero) continue;
                v = logadd(v, b + nnet[(size_t)t * P + (p - 1)] + n->logw[a]);
            }
            bc[s] = v;
        }
    }
    if (post) {
        memset(post, 0, sizeof(float) * (size_t)T * P);
        for (int t = 0; t < T; ++t)
            for (int s = 0; s < S; ++s) {
                float a0 = alpha[(size_t)t * S + s];
                if (a0 <= kLogZero) continue;
                for (int a = n->row_ptr[s]; a < n->row_ptr[s + 1]; ++a) {
                    int p = n->pdf1[a];
                    if (p <= 0 || p > P) continue;
                    float b = beta[(size_t)(t + 1) * S + n->dst[a]];
                    if (b <= kLogZero) continue;
                    float lp = a0 + nnet[(size_t)t * P + (p - 1)] + n->logw[a] + b - total;
                    if (lp > 0.0f) lp = 0.0f;
                    post[(size_t)t * P + (p - 1)] += expf(lp);
                }
            }
    }
    free(alpha);
    free(beta);
    free(src);
    return total;
}

/* backward.go:224-371 for one sequence */
int orc_chain_objf(const OrcChainOpts *o, const OrcDen *den, const OrcNum *num, const float *nnet,
                   int T, float *deriv, OrcChainResult *r) {
    const int P = den->P;
    const long long n = (long long)T * P;
    float w = o->supervision_weight;
    memset(r, 0, sizeof(*r));
    r->frames = T;
    r->ok = 1;
    memset(deriv, 0, sizeof(float) * n);
    float *dpost = zalloc(sizeof(float) * n), *npost = zalloc(sizeof(float) * n);
    float *x16 = zalloc(sizeof(float) * n);
    r->den_logprob = orc_den_forward_backward(den, nnet, T, o->leaky_hmm_coefficient, dpost);
    if (o->out_of_range_regularize > 0.0f) { /* chain_backward.cu:27-67 */
        const float limit = 30.0f, scale = 2.0f * o->out_of_range_regularize;
        for (long long i = 0; i < n; ++i) {
            if ((i / P) % 2 != 0) continue;
            float v = nnet[i];
            if (v < -limit) {
                deriv[i] += (-limit - v) * scale;
                r->out_of_range++;
            } else if (v > limit) {
                deriv[i] += (limit - v) * scale;
                r->out_of_range++;
            }
        }
    }
    for (long long i = 0; i < n; ++i) x16[i] = orc_f16_to_f32(orc_f32_to_f16_rne(nnet[i]));
    r->num_logprob = orc_num_forward_backward(num, x16, T, P, npost);
    for (long long i = 0; i < n; ++i) { /* addGradientFromPosteriors: += w*num; -= w*den */
        deriv[i] += w * npost[i];
        deriv[i] -= w * dpost[i];
    }
    if (o->l2_regularize > 0.0f) { /* chain_backward.cu:111-148, :242-274 */
        float l2s = w * o->l2_regularize;
        double sq = 0.0;
        for (long long i = 0; i < n; ++i) {
            deriv[i] -= l2s * nnet[i];
            sq += (double)nnet[i] * nnet[i];
        }
        r->l2_term = (float)(-0.5 * l2s * sq);
    }
    double objf = (double)w * (r->num_logprob - r->den_logprob);
    if (isnan(objf) || isinf(objf)) {
        memset(deriv, 0, sizeof(float) * n);
        objf = -10.0 * w * T;
        r->l2_term = 0.0;
        r->ok = 0;
    }
    r->objf = objf;
    r->total_weight = (double)w * T;
    free(dpost);
    free(npost);
    free(x16);
    return 0;
}
