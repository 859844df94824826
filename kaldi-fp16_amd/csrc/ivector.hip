// ivector.hip — the Kaldi ivector input path of a CNN-TDNN:
//   ivector-linear input=ReplaceIndex(ivector, t, 0)  -> per-sequence rows (B, not T)
//   combine-feature-maps input=Append(idct-batchnorm, ivector-batchnorm)
//   cnn1 with num-filters-in = nf1 + nf2 (6 in Kaldi's recipes: not a multiple of 32)
// ReplaceIndex(x, t, 0) means "the row of x at t = 0 of this sequence" for every frame, so
// the per-sequence rows are broadcast to their frames inside the combine kernel instead of
// being materialised. The reference aliases the ivector rows and appends tensors of
// different row counts (forward.go:263-296), which is undefined; this path follows Kaldi.
//
// Kernels (all HBM-bound, one output element or one 8-wide group per thread):
//   k_combine_fm      out[t][h*(n1+n2) + f] = f < n1 ? a[t][h*n1 + f] : b[seq(t)][h*n2 + f-n1]
//                     (Kaldi combine-feature-maps; ops.cu:258-287's interleave)
//   k_combine_fm_bwd  db[s][h*n2 + g] = sum over t in s of dy[t][h*(n1+n2) + n1 + g]
//                     (fixed frame order: deterministic)
//   k_im2col_small    P[(t, ho)][tap*fin + c] = x[t + dt][ho*sub + dh][c], zero outside,
//                     columns [ntaps*fin, kp) zero: a small-fin conv becomes one GEMM
//   k_col2im_small    dx[t][h][c] = sum over taps of dP[(t - dt, ho)][tap*fin + c],
//                     ho*sub + dh = h (gather form: deterministic)
//   k_scale_cols      y[r][c] = x[r][c] * scale[c] (frozen BatchNorm backward)
#include "kf_common.h"
#include "../../include/kf_ops.h"

namespace {

// sequence of frame t: the last s with seq_off[s] <= t (seq_off[B] = T)
__device__ __forceinline__ int seq_of(const int *seq_off, int B, int t) {
    int lo = 0, hi = B - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (seq_off[mid] <= t) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

__global__ void k_combine_fm(const h16 *a, long long lda, const h16 *b, long long ldb, const int *seq_off, int B,
                             h16 *out, long long ldo, int T, int height, int n1, int n2) {
    const int nf = n1 + n2, width = height * nf;
    const long long total = (long long)T * width;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const int t = (int)(i / width), d = (int)(i - (long long)t * width);
        const int h = d / nf, f = d - h * nf;
        h16 v;
        if (f < n1) {
            v = a[(long long)t * lda + h * n1 + f];
        } else {
            const int r = seq_off ? seq_of(seq_off, B, t) : t;
            v = b[(long long)r * ldb + h * n2 + (f - n1)];
        }
        out[(long long)t * ldo + d] = v;
    }
}

// one block per (sequence, 64 columns of b): 16 frame groups x 64 columns; group q sums
// frames q, q+16, ... of the sequence in order, then the 16 partials are added in
// group order (deterministic)
constexpr int kFmGroups = 16;
__global__ __launch_bounds__(64 * kFmGroups) void k_combine_fm_bwd(const h16 *dy, long long ldy, const int *seq_off,
                                                                 int B, h16 *db, long long ldb, int height, int n1,
                                                                 int n2) {
    __shared__ float part[kFmGroups][64];
    const int nb = height * n2, nchunk = (nb + 63) / 64;
    const int s = blockIdx.x / nchunk, c = (blockIdx.x % nchunk) * 64 + (threadIdx.x & 63);
    const int q = threadIdx.x >> 6, nf = n1 + n2;
    float acc = 0.f;
    if (s < B && c < nb) {
        const int h = c / n2, g = c - h * n2;
        const h16 *col = dy + h * nf + n1 + g;
        for (int t = seq_off[s] + q; t < seq_off[s + 1]; t += kFmGroups) acc += (float)col[(long long)t * ldy];
    }
    part[q][threadIdx.x & 63] = acc;
    __syncthreads();
    if (q == 0 && s < B && c < nb) {
        float sum = 0.f;
#pragma unroll
        for (int k = 0; k < kFmGroups; ++k) sum += part[k][threadIdx.x];
        db[(long long)s * ldb + c] = (h16)sum;
    }
}

struct SmallConv {
    int T, hin, hout, sub, fin, ntaps, kp;
    int dt[KF_MAX_PARTS], dh[KF_MAX_PARTS];
};

// one thread per 8 consecutive columns of a row (kp % 8 == 0): one 16-byte store
__global__ void k_im2col_small(const h16 *x, long long ldx, SmallConv c, h16 *P) {
    const long long rows = (long long)c.T * c.hout;
    const int kg = c.kp / 8;
    const long long total = rows * kg;
    const int kr = c.ntaps * c.fin;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const long long m = i / kg;
        const int k0 = (int)(i - m * kg) * 8;
        const int t = (int)(m / c.hout), ho = (int)(m - (long long)t * c.hout);
        half8 o;
        int tap = k0 / c.fin, ch = k0 - tap * c.fin;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            h16 v = (h16)0.f;
            if (k0 + e < kr) {
                const int ts = t + c.dt[tap], hs = ho * c.sub + c.dh[tap];
                if (ts >= 0 && ts < c.T && hs >= 0 && hs < c.hin) v = x[(long long)ts * ldx + hs * c.fin + ch];
            }
            o[e] = v;
            if (++ch == c.fin) {
                ch = 0;
                ++tap;
            }
        }
        *reinterpret_cast<half8 *>(P + m * c.kp + k0) = o;
    }
}

__global__ void k_col2im_small(const h16 *dP, SmallConv c, h16 *dx, long long ldx) {
    const int width = c.hin * c.fin;
    const long long total = (long long)c.T * width;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const int t = (int)(i / width), d = (int)(i - (long long)t * width);
        const int h = d / c.fin, ch = d - h * c.fin;
        float acc = 0.f;
        for (int tap = 0; tap < c.ntaps; ++tap) {
            const int to = t - c.dt[tap], num = h - c.dh[tap];
            if (to < 0 || to >= c.T || num < 0 || num % c.sub) continue;
            const int ho = num / c.sub;
            if (ho >= c.hout) continue;
            acc += (float)dP[((long long)to * c.hout + ho) * c.kp + tap * c.fin + ch];
        }
        dx[(long long)t * ldx + d] = (h16)acc;
    }
}

__global__ void k_scale_cols(const h16 *x, long long ldx, const float *scale, h16 *y, long long ldy, int rows,
                             int cols) {
    const long long total = (long long)rows * cols;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const int r = (int)(i / cols), c = (int)(i - (long long)r * cols);
        // the fp32 product, then one RNE to fp16 (the oracle's rounding points); without the
        // barrier hipcc fuses both into v_fma_mixlo_f16, which rounds the exact product once
        // and differs from rne(fp32 product) at near-ties
        float p = (float)x[(long long)r * ldx + c] * scale[c];
        asm volatile("" : "+v"(p));
        y[(long long)r * ldy + c] = (h16)p;
    }
}

// per-sequence linear-component (R = B rows, any dims): y = x . W, fp32 accumulation
__global__ void k_rows_gemm(const h16 *x, long long ldx, const h16 *W, long long ldw, h16 *y, long long ldy, int R,
                            int K, int N) {
    const long long total = (long long)R * N;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const int r = (int)(i / N), n = (int)(i - (long long)r * N);
        float acc = 0.f;
        for (int k = 0; k < K; ++k) acc += (float)x[(long long)r * ldx + k] * (float)W[(long long)k * ldw + n];
        y[(long long)r * ldy + n] = (h16)acc;
    }
}

// its weight gradient: dW[m][n] = sum_r x[r][m] g[r][n] (fp32, overwritten, rows in order)
__global__ void k_rows_wgrad(const h16 *x, long long ldx, const h16 *g, long long ldg, float *dW, long long ldd,
                             int R, int M, int N) {
    const long long total = (long long)M * N;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const int m = (int)(i / N), n = (int)(i - (long long)m * N);
        float acc = 0.f;
        for (int r = 0; r < R; ++r) acc += (float)x[(long long)r * ldx + m] * (float)g[(long long)r * ldg + n];
        dW[(long long)m * ldd + n] = acc;
    }
}

int launch_check(const char *what) {
    if (hipGetLastError() != hipSuccess) {
        kf_report_error("%s: launch failed", what);
        return -1;
    }
    return 0;
}

bool small_conv(SmallConv &c, int T, int hin, int hout, int sub, int fin, int ntaps, const int *dt,
                const int *dh, int kp, const char *what) {
    if (T <= 0 || hin <= 0 || hout <= 0 || sub <= 0 || fin <= 0 || ntaps <= 0 || ntaps > KF_MAX_PARTS ||
        kp < ntaps * fin || !dt || !dh) {
        kf_report_error("%s: bad shape (T %d hin %d hout %d sub %d fin %d taps %d kp %d)", what, T, hin, hout, sub,
                        fin, ntaps, kp);
        return false;
    }
    c.T = T;
    c.hin = hin;
    c.hout = hout;
    c.sub = sub;
    c.fin = fin;
    c.ntaps = ntaps;
    c.kp = kp;
    for (int i = 0; i < ntaps; ++i) {
        c.dt[i] = dt[i];
        c.dh[i] = dh[i];
    }
    return true;
}

}  // namespace

extern "C" int kf_combine_feature_maps(const void *a, long long lda, const void *b, long long ldb,
                                       const int *dev_seq_off, int B, void *out, long long ldo, int T, int height,
                                       int nf1, int nf2) {
    if (T <= 0) return 0;
    if (!a || !b || !out || height <= 0 || nf1 <= 0 || nf2 <= 0 || lda < (long long)height * nf1 ||
        ldb < (long long)height * nf2 || ldo < (long long)height * (nf1 + nf2) || (dev_seq_off && B <= 0)) {
        kf_report_error("kf_combine_feature_maps: bad arguments");
        return -1;
    }
    const long long total = (long long)T * height * (nf1 + nf2);
    k_combine_fm<<<kf_blocks(total, 256, 16384), 256, 0, kf_stream()>>>((const h16 *)a, lda, (const h16 *)b, ldb,
                                                                        dev_seq_off, B, (h16 *)out, ldo, T,
                                                                        height, nf1, nf2);
    return launch_check("kf_combine_feature_maps");
}

extern "C" int kf_combine_feature_maps_backward(const void *dy, long long ldy, const int *dev_seq_off, int B,
                                                void *db, long long ldb, int height, int nf1, int nf2) {
    if (B <= 0) return 0;
    if (!dy || !dev_seq_off || !db || height <= 0 || nf1 < 0 || nf2 <= 0 ||
        ldy < (long long)height * (nf1 + nf2) || ldb < (long long)height * nf2) {
        kf_report_error("kf_combine_feature_maps_backward: bad arguments");
        return -1;
    }
    const int nchunk = (height * nf2 + 63) / 64;
    k_combine_fm_bwd<<<B * nchunk, 64 * kFmGroups, 0, kf_stream()>>>((const h16 *)dy, ldy, dev_seq_off, B,
                                                                     (h16 *)db, ldb, height, nf1, nf2);
    return launch_check("kf_combine_feature_maps_backward");
}

extern "C" int kf_im2col_small(const void *x, long long ldx, int T, int hin, int hout, int sub, int fin,
                               int ntaps, const int *dt, const int *dh, void *P, int kp) {
    SmallConv c;
    if (!x || !P || !small_conv(c, T, hin, hout, sub, fin, ntaps, dt, dh, kp, "kf_im2col_small")) return -1;
    if (kp % 8 || ((uintptr_t)P & 15)) {
        kf_report_error("kf_im2col_small: kp must be a multiple of 8 and P 16-byte aligned");
        return -1;
    }
    const long long total = (long long)T * hout * (kp / 8);
    k_im2col_small<<<kf_blocks(total, 256, 16384), 256, 0, kf_stream()>>>((const h16 *)x, ldx, c, (h16 *)P);
    return launch_check("kf_im2col_small");
}

extern "C" int kf_col2im_small(const void *dP, int T, int hin, int hout, int sub, int fin, int ntaps,
                               const int *dt, const int *dh, int kp, void *dx, long long ldx) {
    SmallConv c;
    if (!dP || !dx || !small_conv(c, T, hin, hout, sub, fin, ntaps, dt, dh, kp, "kf_col2im_small")) return -1;
    const long long total = (long long)T * hin * fin;
    k_col2im_small<<<kf_blocks(total, 256, 16384), 256, 0, kf_stream()>>>((const h16 *)dP, c, (h16 *)dx, ldx);
    return launch_check("kf_col2im_small");
}

extern "C" int kf_scale_cols(const void *x, long long ldx, const float *scale, void *y, long long ldy, int rows,
                             int cols) {
    if (rows <= 0 || cols <= 0) return 0;
    if (!x || !scale || !y) {
        kf_report_error("kf_scale_cols: null argument");
        return -1;
    }
    k_scale_cols<<<kf_blocks((long long)rows * cols, 256, 16384), 256, 0, kf_stream()>>>(
        (const h16 *)x, ldx, scale, (h16 *)y, ldy, rows, cols);
    return launch_check("kf_scale_cols");
}

extern "C" int kf_rows_gemm(const void *x, long long ldx, const void *W, long long ldw, void *y, long long ldy, int R,
                            int K, int N) {
    if (R <= 0 || N <= 0) return 0;
    if (!x || !W || !y || K <= 0) {
        kf_report_error("kf_rows_gemm: bad arguments");
        return -1;
    }
    k_rows_gemm<<<kf_blocks((long long)R * N, 256, 8192), 256, 0, kf_stream()>>>(
        (const h16 *)x, ldx, (const h16 *)W, ldw, (h16 *)y, ldy, R, K, N);
    return launch_check("kf_rows_gemm");
}

extern "C" int kf_rows_wgrad(const void *x, long long ldx, const void *g, long long ldg, float *dW, long long ldd,
                             int R, int M, int N) {
    if (M <= 0 || N <= 0) return 0;
    if (!x || !g || !dW || R <= 0) {
        kf_report_error("kf_rows_wgrad: bad arguments");
        return -1;
    }
    k_rows_wgrad<<<kf_blocks((long long)M * N, 256, 8192), 256, 0, kf_stream()>>>(
        (const h16 *)x, ldx, (const h16 *)g, ldg, dW, ldd, R, M, N);
    return launch_check("kf_rows_wgrad");
}
