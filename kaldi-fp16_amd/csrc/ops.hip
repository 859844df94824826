// ops.hip — reference ABI compute ops (include/ops.h) on gfx950.
// Semantics follow cpp/cuda/ops.cu:26-643 and cpp/cuda/backward_wrappers.cu:41-291:
// fp16 in, fp32 math, one round-to-nearest-even fp16 store. Kernels are
// grid-stride loops over 8-element (16-byte) vectors with a scalar tail, so
// they run at HBM rate for any count (the reference uses one thread per
// element and 2-byte accesses).
#include "kf_common.h"
#include "../../include/ops.h"
#include "../../include/kf_ops.h"

KF_DECLARE_ERR(ops)

int kf_ops_gemm_impl(int M, int N, int K, float alpha, const void *A, int lda, const void *B,
                     int ldb, float beta, void *C, int ldc, char *err, size_t errlen);

static int ops_check(const char *what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        ops_set_error("%s: %s", what, hipGetErrorString(e));
        return -1;
    }
    return 0;
}

static inline bool aligned16(const void *p) { return ((uintptr_t)p & 15) == 0; }

// Generic element-wise driver: f(i, ...) applied per element; vector path when
// all pointers are 16-byte aligned.
#define GRID_STRIDE(i, n)                                                          \
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < (n); \
         i += (long long)gridDim.x * blockDim.x)

// ------------------------------- activations -------------------------------
enum { ACT_RELU, ACT_SIGMOID, ACT_TANH, ACT_CLIPPED };

__device__ __forceinline__ float act_apply(int kind, float x, float ceil_) {
    switch (kind) {
        case ACT_RELU: return x < 0.f ? 0.f : x;
        case ACT_SIGMOID: return 1.f / (1.f + expf(-x));
        case ACT_TANH: return tanhf(x);
        default: return fmaxf(0.f, fminf(x, ceil_));
    }
}

__global__ void k_act(h16 *d, long long n, int kind, float ceil_, int vec) {
    if (vec) {
        GRID_STRIDE(i, n / 8) {
            half8 v = load_h8(d + 8 * i);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = f2h(act_apply(kind, (float)v[e], ceil_));
            store_h8(d + 8 * i, v);
        }
        GRID_STRIDE(i, n % 8) {
            long long j = n / 8 * 8 + i;
            d[j] = f2h(act_apply(kind, h2f(d[j]), ceil_));
        }
    } else {
        GRID_STRIDE(i, n) d[i] = f2h(act_apply(kind, h2f(d[i]), ceil_));
    }
}

static int run_act(void *data, int count, int kind, float c, const char *name) {
    kf_take_pending(__func__);
    if (count < 0) {
        ops_set_error("%s: negative count", name);
        return -1;
    }
    if (count == 0) return 0;
    k_act<<<kf_blocks(count / 8 + 1, 256, 8192), 256, 0, kf_stream()>>>(
        (h16 *)data, count, kind, c, aligned16(data));
    return ops_check(name);
}

// ------------------------------- softmax -----------------------------------
// one 256-thread block per row; true max via wave/block reduction
__device__ __forceinline__ float block_reduce(float v, bool is_max, float *sh) {
    for (int o = 32; o > 0; o >>= 1) {
        float w = __shfl_xor(v, o);
        v = is_max ? fmaxf(v, w) : v + w;
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) sh[wid] = v;
    __syncthreads();
    const int nw = blockDim.x >> 6;
    float r = sh[0];
    for (int i = 1; i < nw; ++i) r = is_max ? fmaxf(r, sh[i]) : r + sh[i];
    return r;
}

__global__ void k_softmax(h16 *data, int cols, int logmode) {
    __shared__ float sh[16];
    h16 *row = data + (long long)blockIdx.x * cols;
    float mx = -INFINITY;
    for (int j = threadIdx.x; j < cols; j += blockDim.x) mx = fmaxf(mx, h2f(row[j]));
    mx = block_reduce(mx, true, sh);
    if (logmode) {
        float s = 0.f;
        for (int j = threadIdx.x; j < cols; j += blockDim.x) s += expf(h2f(row[j]) - mx);
        s = block_reduce(s, false, sh);
        const float lse = mx + logf(s);
        for (int j = threadIdx.x; j < cols; j += blockDim.x) row[j] = f2h(h2f(row[j]) - lse);
    } else {
        // the reference's two rounding points (ops.cu:70-118): exp is stored as fp16,
        // the sum is taken over the unrounded fp32 values, then fp16(fp16(e) * (1/sum))
        float s2 = 0.f;
        for (int j = threadIdx.x; j < cols; j += blockDim.x) {
            const float e = expf(h2f(row[j]) - mx);
            row[j] = f2h(e);
            s2 += e;
        }
        s2 = block_reduce(s2, false, sh);
        const float inv = 1.f / s2;
        for (int j = threadIdx.x; j < cols; j += blockDim.x) row[j] = f2h(h2f(row[j]) * inv);
    }
}

// ------------------------------- row-vector layout ------------------------
// [rows x cols] element-wise ops on 8-column (16-byte) vectors: a thread owns ONE column
// vector cv for all its rows (its per-column parameters are loaded once, no per-element
// index division) and walks rows r0, r0 + R, ... Consecutive threads take consecutive
// column vectors of a row, then the next row, so a wave reads contiguous row bytes.
struct RowVec {
    int ncv;      // column vectors per row
    long long R;  // row stride of the walk (threads = ncv * R)
};
static inline RowVec rowvec_plan(long long rows, int ncv, int &blocks) {
    long long R = 262144 / ncv;  // ~256K threads in flight, four 16-byte loads each
    if (R < 1) R = 1;
    if (R > rows) R = rows;
    blocks = (int)((ncv * R + 255) / 256);
    return RowVec{ncv, R};
}
#define ROWVEC_THREAD(P, cv, r0)                                          \
    const long long g_ = (long long)blockIdx.x * blockDim.x + threadIdx.x; \
    if (g_ >= (long long)(P).ncv * (P).R) return;                         \
    const int cv = (int)(g_ % (P).ncv);                                   \
    const long long r0 = g_ / (P).ncv

// ------------------------------- batchnorm ---------------------------------
// norm = (x - mean) / sqrtf(var + eps); gamma * norm + beta (or norm * target_rms), the
// reference's expression per element (ops.cu:171-204). The vector form evaluates the
// same expression with the per-column sqrtf taken once per thread.
__global__ void k_bn(h16 *x, long long total, int D, const float *mean, const float *var,
                     const float *gamma, const float *beta, float target_rms, float eps,
                     int rms) {
    GRID_STRIDE(i, total) {
        const int d = (int)(i % D);
        const float norm = (h2f(x[i]) - mean[d]) / sqrtf(var[d] + eps);
        x[i] = f2h(rms ? norm * target_rms : gamma[d] * norm + beta[d]);
    }
}
__global__ __launch_bounds__(256) void k_bn_v8(h16 *x, long long rows, RowVec P, const float *mean,
                                               const float *var, const float *gamma, const float *beta,
                                               float target_rms, float eps, int rms) {
    ROWVEC_THREAD(P, cv, r0);
    float mu[8], sd[8], g[8], b[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const int c = 8 * cv + e;
        mu[e] = mean[c];
        sd[e] = sqrtf(var[c] + eps);
        g[e] = rms ? target_rms : gamma[c];
        b[e] = rms ? 0.f : beta[c];
    }
    const long long ld = 8LL * P.ncv;
    h16 *p = x + 8LL * cv;
    long long r = r0;
    for (; r + 3 * P.R < rows; r += 4 * P.R) {  // four rows in flight per thread
        half8 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = load_h8(p + (r + u * P.R) * ld);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const float norm = ((float)v[u][e] - mu[e]) / sd[e];
                v[u][e] = f2h(rms ? norm * g[e] : g[e] * norm + b[e]);
            }
            store_h8(p + (r + u * P.R) * ld, v[u]);
        }
    }
    for (; r < rows; r += P.R) {
        half8 v = load_h8(p + r * ld);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const float norm = ((float)v[e] - mu[e]) / sd[e];
            v[e] = f2h(rms ? norm * g[e] : g[e] * norm + b[e]);
        }
        store_h8(p + r * ld, v);
    }
}

__global__ void k_bn_bwd(const h16 *go, h16 *gi, const float *gamma, const float *var,
                         float eps, long long total, int cols) {
    GRID_STRIDE(i, total) {
        const int d = (int)(i % cols);
        gi[i] = f2h(h2f(go[i]) * (gamma[d] / sqrtf(var[d] + eps)));
    }
}
__global__ __launch_bounds__(256) void k_bn_bwd_v8(const h16 *go, h16 *gi, const float *gamma,
                                                   const float *var, float eps, long long rows, RowVec P) {
    ROWVEC_THREAD(P, cv, r0);
    float sc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) sc[e] = gamma[8 * cv + e] / sqrtf(var[8 * cv + e] + eps);
    const long long ld = 8LL * P.ncv, c0 = 8LL * cv;
    long long r = r0;
    for (; r + 3 * P.R < rows; r += 4 * P.R) {
        half8 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = load_h8(go + (r + u * P.R) * ld + c0);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[u][e] = f2h((float)v[u][e] * sc[e]);
            store_h8(gi + (r + u * P.R) * ld + c0, v[u]);
        }
    }
    for (; r < rows; r += P.R) {
        half8 v = load_h8(go + r * ld + c0);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = f2h((float)v[e] * sc[e]);
        store_h8(gi + r * ld + c0, v);
    }
}

// column placement (concat) / extraction (slice) of 8-column vectors: dst row r, column
// dcol0 + 8 cv  <-  src row r, column scol0 + 8 cv
__global__ __launch_bounds__(256) void k_cols_copy_v8(h16 *dst, long long ldd, int dcol0, const h16 *src,
                                                      long long lds, int scol0, long long rows, RowVec P) {
    ROWVEC_THREAD(P, cv, r0);
    h16 *d = dst + dcol0 + 8LL * cv;
    const h16 *s = src + scol0 + 8LL * cv;
    long long r = r0;
    for (; r + 3 * P.R < rows; r += 4 * P.R) {
        half8 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = load_h8(s + (r + u * P.R) * lds);
#pragma unroll
        for (int u = 0; u < 4; ++u) store_h8(d + (r + u * P.R) * ldd, v[u]);
    }
    for (; r < rows; r += P.R) store_h8(d + r * ldd, load_h8(s + r * lds));
}

// ------------------------------- element-wise ------------------------------
__global__ void k_add_scaled(h16 *dst, const h16 *src, long long n, float a, float b, int vec) {
    if (vec) {
        GRID_STRIDE(i, n / 8) {
            half8 d = load_h8(dst + 8 * i), s = load_h8(src + 8 * i);
#pragma unroll
            for (int e = 0; e < 8; ++e) d[e] = f2h(a * (float)s[e] + b * (float)d[e]);
            store_h8(dst + 8 * i, d);
        }
        GRID_STRIDE(i, n % 8) {
            long long j = n / 8 * 8 + i;
            dst[j] = f2h(a * h2f(src[j]) + b * h2f(dst[j]));
        }
    } else {
        GRID_STRIDE(i, n) dst[i] = f2h(a * h2f(src[i]) + b * h2f(dst[i]));
    }
}

// ops_copy on 16-byte vectors, four in flight per thread (hipMemcpyAsync's blit kernel
// reached ~3.4 TB/s on the splice row-view copies)
__global__ __launch_bounds__(256) void k_copy_v8(h16 *dst, const h16 *src, long long n8) {
    const long long S = (long long)gridDim.x * blockDim.x;
    long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 3 * S < n8; i += 4 * S) {
        half8 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = load_h8(src + 8 * (i + u * S));
#pragma unroll
        for (int u = 0; u < 4; ++u) store_h8(dst + 8 * (i + u * S), v[u]);
    }
    for (; i < n8; i += S) store_h8(dst + 8 * i, load_h8(src + 8 * i));
}

__global__ void k_fill(h16 *dst, long long n, float v, int vec) {
    const h16 hv = f2h(v);
    if (vec) {
        half8 w;
#pragma unroll
        for (int e = 0; e < 8; ++e) w[e] = hv;
        GRID_STRIDE(i, n / 8) store_h8(dst + 8 * i, w);
        GRID_STRIDE(i, n % 8) dst[n / 8 * 8 + i] = hv;
    } else {
        GRID_STRIDE(i, n) dst[i] = hv;
    }
}

__global__ void k_concat_cols(h16 *dst, int T, int dst_cols, const h16 *src, int src_cols,
                              int off) {
    GRID_STRIDE(i, (long long)T * src_cols) {
        const long long t = i / src_cols, c = i - t * src_cols;
        dst[t * dst_cols + off + c] = src[i];
    }
}

__global__ void k_slice_cols(h16 *dst, int T, int dst_cols, const h16 *src, int src_cols,
                             int off) {
    GRID_STRIDE(i, (long long)T * dst_cols) {
        const long long t = i / dst_cols, c = i - t * dst_cols;
        dst[i] = src[t * src_cols + off + c];
    }
}

__global__ void k_combine_fm(h16 *out, const h16 *in, int T, int total, int H, int nf1,
                             int nf2) {
    GRID_STRIDE(i, (long long)T * total) {
        const long long t = i / total;
        const int d = (int)(i - t * total);
        const int nf = nf1 + nf2, h = d / nf, f = d - h * nf;
        const long long src = f < nf1 ? t * total + (long long)h * nf1 + f
                                      : t * total + (long long)H * nf1 + (long long)h * nf2 + (f - nf1);
        out[i] = in[src];
    }
}

__global__ void k_subsample_rows(h16 *dst, const h16 *src, int out_rows, int cols, int stride,
                                 int off) {
    GRID_STRIDE(i, (long long)out_rows * cols) {
        const long long r = i / cols, c = i - r * cols;
        dst[i] = src[(off + r * stride) * cols + c];
    }
}

__device__ __forceinline__ float act_bwd_elem(int kind, float xv, float gv) {
    // no fma contraction: LLVM would fold fpext(fp16 product) into an fp32 fma and
    // drop the intermediate fp16 rounding the reference's __hmul chain performs
#pragma clang fp contract(off)
    // fp16 arithmetic as the reference's __hmul / __hsub chain
    // (backward_wrappers.cu:41-74): every product / difference rounds to fp16
    // (a product of two fp16 values is exact in fp32, so one RNE matches __hmul)
    if (kind == ACT_RELU) return xv > 0.f ? gv : 0.f;
    if (kind == ACT_SIGMOID) return h2f(f2h(gv * xv)) * h2f(f2h(1.f - xv));
    return gv * h2f(f2h(1.f - h2f(f2h(xv * xv))));
}
__global__ void k_act_bwd(const h16 *x, h16 *g, long long n, int kind, int vec) {
#pragma clang fp contract(off)
    if (vec) {
        GRID_STRIDE(i, n / 8) {
            const half8 xv = load_h8(x + 8 * i);
            half8 gv = load_h8(g + 8 * i);
#pragma unroll
            for (int e = 0; e < 8; ++e) gv[e] = f2h(act_bwd_elem(kind, (float)xv[e], (float)gv[e]));
            store_h8(g + 8 * i, gv);
        }
        GRID_STRIDE(i, n % 8) {
            const long long j = n / 8 * 8 + i;
            g[j] = f2h(act_bwd_elem(kind, h2f(x[j]), h2f(g[j])));
        }
    } else {
        GRID_STRIDE(i, n) g[i] = f2h(act_bwd_elem(kind, h2f(x[i]), h2f(g[i])));
    }
}

// tiled transpose through LDS (dst[N x M] = src[M x N]^T), coalesced both ways
__global__ void k_transpose(const h16 *src, h16 *dst, int M, int N) {
    __shared__ h16 tile[64][65];
    const int bx = blockIdx.x * 64, by = blockIdx.y * 64;
    for (int r = threadIdx.y; r < 64; r += blockDim.y) {
        const int m = by + r, n = bx + threadIdx.x;
        if (m < M && n < N) tile[r][threadIdx.x] = src[(long long)m * N + n];
    }
    __syncthreads();
    for (int r = threadIdx.y; r < 64; r += blockDim.y) {
        const int n = bx + r, m = by + threadIdx.x;
        if (m < M && n < N) dst[(long long)n * M + m] = tile[threadIdx.x][r];
    }
}

__global__ void k_h2f(const h16 *s, float *d, long long n, int vec) {
    if (vec) {
        GRID_STRIDE(i, n / 8) {
            const half8 v = load_h8(s + 8 * i);
            float4v a, b;
#pragma unroll
            for (int e = 0; e < 4; ++e) a[e] = (float)v[e], b[e] = (float)v[4 + e];
            *reinterpret_cast<float4v *>(d + 8 * i) = a;
            *reinterpret_cast<float4v *>(d + 8 * i + 4) = b;
        }
        GRID_STRIDE(i, n % 8) d[n / 8 * 8 + i] = h2f(s[n / 8 * 8 + i]);
    } else {
        GRID_STRIDE(i, n) d[i] = h2f(s[i]);
    }
}

// kf_dp_debug KF_DP_DEBUG_PEER_MEAN (csrc/dp.cpp): a two-rank average whose other rank's
// bucket is `peer`, on the communication stream
__global__ void k_dp_peer_mean(float *buf, const float *peer, long long n) {
    GRID_STRIDE(i, n) buf[i] = (buf[i] + peer[i]) * 0.5f;
}
int kf_dp_debug_mean_launch(float *buf, const float *peer, size_t n, hipStream_t s) {
    kf_take_pending(__func__);
    if (!n) return 0;
    const long long blocks = ((long long)n + 255) / 256;
    hipLaunchKernelGGL(k_dp_peer_mean, dim3((unsigned)(blocks < 4096 ? blocks : 4096)), dim3(256), 0, s, buf, peer,
                       (long long)n);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

__device__ __forceinline__ void sgd_elem(float *w32, h16 *w16, const h16 *g, float *v, float lr, float mom,
                                         long long i) {
    const float vv = mom * v[i] + h2f(g[i]);
    v[i] = vv;
    const float w = w32[i] - lr * vv;
    w32[i] = w;
    w16[i] = f2h(w);
}
// vec: every pointer 16-byte aligned; 8 parameters per thread (two float4 of w32 / v)
__global__ void k_sgd(float *w32, h16 *w16, const h16 *g, float *v, float lr, float mom,
                      long long n, int vec) {
    if (!vec) {
        GRID_STRIDE(i, n) sgd_elem(w32, w16, g, v, lr, mom, i);
        return;
    }
    GRID_STRIDE(i, n / 8) {
        const half8 gv = load_h8(g + 8 * i);
        half8 wh;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            float4v vv = *reinterpret_cast<const float4v *>(v + 8 * i + 4 * q);
            float4v ww = *reinterpret_cast<const float4v *>(w32 + 8 * i + 4 * q);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                vv[e] = mom * vv[e] + (float)gv[4 * q + e];
                ww[e] = ww[e] - lr * vv[e];
                wh[4 * q + e] = f2h(ww[e]);
            }
            *reinterpret_cast<float4v *>(v + 8 * i + 4 * q) = vv;
            *reinterpret_cast<float4v *>(w32 + 8 * i + 4 * q) = ww;
        }
        store_h8(w16 + 8 * i, wh);
    }
    GRID_STRIDE(i, n % 8) sgd_elem(w32, w16, g, v, lr, mom, n / 8 * 8 + i);
}

// ---------------------------------------------------------------------------
extern "C" {

const char *ops_last_error(void) { return ops_err_.get(); }
void ops_clear_error(void) { ops_err_.clear(); }

int ops_gemm(void *handle, int M, int N, int K, float alpha, const void *A, int lda,
             const void *B, int ldb, float beta, void *C, int ldc) {
    (void)handle;
    char err[512];
    if (kf_ops_gemm_impl(M, N, K, alpha, A, lda, B, ldb, beta, C, ldc, err, sizeof err)) {
        ops_set_error("%s", err);
        return -1;
    }
    return 0;
}

int ops_gemm_strided(void *handle, int M, int N, int K, float alpha, const void *A, int lda,
                     int64_t strideA, const void *B, int ldb, int64_t strideB, float beta,
                     void *C, int ldc, int64_t strideC, int batch_count) {
    (void)handle;
    char err[512];
    for (int b = 0; b < batch_count; ++b) {
        if (kf_ops_gemm_impl(M, N, K, alpha, (const h16 *)A + b * strideA, lda,
                             (const h16 *)B + b * strideB, ldb, beta, (h16 *)C + b * strideC,
                             ldc, err, sizeof err)) {
            ops_set_error("strided batch %d: %s", b, err);
            return -1;
        }
    }
    return 0;
}

int ops_relu(void *data, int count) { return run_act(data, count, ACT_RELU, 0.f, "relu kernel"); }
int ops_sigmoid(void *data, int count) { return run_act(data, count, ACT_SIGMOID, 0.f, "sigmoid"); }
int ops_tanh_act(void *data, int count) { return run_act(data, count, ACT_TANH, 0.f, "tanh"); }
int ops_clipped_relu(void *data, int count, float ceiling) {
    return run_act(data, count, ACT_CLIPPED, ceiling, "clipped_relu");
}

int ops_softmax(void *data, int rows, int cols) {
    kf_take_pending(__func__);
    if (rows <= 0 || cols <= 0) return 0;
    k_softmax<<<rows, 256, 0, kf_stream()>>>((h16 *)data, cols, 0);
    return ops_check("softmax kernel");
}
// Row-wise log-softmax with the row held in registers: one wave per row, 16-byte loads,
// max / sum by wave shuffles, one read and one write of the row (k_softmax re-reads it
// three times). The reference's LogSoftmax (ops.cu:120-166) takes the row max with an
// integer atomicMax on float bits, which is wrong for all-negative rows; this one is not.
constexpr int kLsmMaxChunks = 8;  // cols <= 64 lanes * 8 chunks * 8 = 4096
__global__ __launch_bounds__(256) void k_log_softmax_rows(h16 *data, int rows, int cols) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows) return;  // whole wave
    half8 *r = reinterpret_cast<half8 *>(data + (long long)row * cols);
    const int nch = cols >> 3;
    half8 v[kLsmMaxChunks];
    float mx = -INFINITY;
#pragma unroll
    for (int k = 0; k < kLsmMaxChunks; ++k) {
        const int c = lane + 64 * k;
        v[k] = c < nch ? r[c] : half8{};
        if (c < nch)
#pragma unroll
            for (int e = 0; e < 8; ++e) mx = fmaxf(mx, (float)v[k][e]);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < kLsmMaxChunks; ++k)
        if (lane + 64 * k < nch)
#pragma unroll
            for (int e = 0; e < 8; ++e) s += expf((float)v[k][e] - mx);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    const float lse = mx + logf(s);
#pragma unroll
    for (int k = 0; k < kLsmMaxChunks; ++k) {
        const int c = lane + 64 * k;
        if (c < nch) {
            half8 w;
#pragma unroll
            for (int e = 0; e < 8; ++e) w[e] = (h16)((float)v[k][e] - lse);
            r[c] = w;
        }
    }
}

int ops_log_softmax(void *data, int rows, int cols) {
    kf_take_pending(__func__);
    if (rows <= 0 || cols <= 0) return 0;
    if (cols % 8 == 0 && cols <= 64 * 8 * kLsmMaxChunks && aligned16(data)) {
        k_log_softmax_rows<<<(rows + 3) / 4, 256, 0, kf_stream()>>>((h16 *)data, rows, cols);
        return ops_check("log_softmax kernel");
    }
    k_softmax<<<rows, 256, 0, kf_stream()>>>((h16 *)data, cols, 1);
    return ops_check("log_softmax kernel");
}

static int run_bn(void *x, int T, int D, const float *mean, const float *var, const float *gamma,
                  const float *beta, float target_rms, float eps, int rms, const char *name) {
    kf_take_pending(__func__);
    const long long total = (long long)T * D;
    if (D % 8 == 0 && aligned16(x)) {
        int blocks;
        const RowVec P = rowvec_plan(T, D / 8, blocks);
        k_bn_v8<<<blocks, 256, 0, kf_stream()>>>((h16 *)x, T, P, mean, var, gamma, beta, target_rms, eps, rms);
    } else {
        k_bn<<<kf_blocks(total, 256, 8192), 256, 0, kf_stream()>>>((h16 *)x, total, D, mean, var, gamma, beta,
                                                                  target_rms, eps, rms);
    }
    return ops_check(name);
}

int ops_batchnorm_forward(void *x, int T, int D, const float *mean, const float *var,
                          const float *gamma, const float *beta, float epsilon) {
    long long total = (long long)T * D;
    if (total <= 0) return 0;
    return run_bn(x, T, D, mean, var, gamma, beta, 1.f, epsilon, 0, "batchnorm kernel");
}
int ops_batchnorm_forward_rms(void *x, int T, int D, const float *mean, const float *var,
                              float target_rms, float epsilon) {
    long long total = (long long)T * D;
    if (total <= 0) return 0;
    return run_bn(x, T, D, mean, var, nullptr, nullptr, target_rms, epsilon, 1, "batchnorm rms kernel");
}

int ops_add_scaled(void *dst, const void *src, int count, float alpha, float beta) {
    kf_take_pending(__func__);
    if (count <= 0) return 0;
    k_add_scaled<<<kf_blocks(count / 8 + 1, 256, 8192), 256, 0, kf_stream()>>>(
        (h16 *)dst, (const h16 *)src, count, alpha, beta, aligned16(dst) && aligned16(src));
    return ops_check("add_scaled");
}
int ops_add(void *dst, const void *src, int count) {
    return ops_add_scaled(dst, src, count, 1.f, 1.f);
}
int ops_copy(void *dst, const void *src, int count) {
    kf_take_pending(__func__);
    if (count <= 0) return 0;
    if (count % 8 == 0 && aligned16(dst) && aligned16(src)) {
        const long long n8 = count / 8;
        k_copy_v8<<<kf_blocks(n8, 256, 8192), 256, 0, kf_stream()>>>((h16 *)dst, (const h16 *)src, n8);
        return ops_check("copy");
    }
    hipError_t e = hipMemcpyAsync(dst, src, (size_t)count * 2, hipMemcpyDeviceToDevice, kf_stream());
    if (e != hipSuccess) {
        ops_set_error("copy: %s", hipGetErrorString(e));
        return -1;
    }
    return 0;
}
int ops_fill(void *dst, int count, float val) {
    kf_take_pending(__func__);
    if (count <= 0) return 0;
    k_fill<<<kf_blocks(count / 8 + 1, 256, 8192), 256, 0, kf_stream()>>>((h16 *)dst, count, val, aligned16(dst));
    return ops_check("fill");
}

int ops_concat_cols(void *dst, int T, int dst_cols, const void *src, int src_cols,
                    int dst_col_offset) {
    kf_take_pending(__func__);
    if ((long long)T * src_cols <= 0) return 0;
    if (dst_col_offset < 0 || dst_col_offset + src_cols > dst_cols) {
        ops_set_error("concat_cols: offset %d + %d > %d", dst_col_offset, src_cols, dst_cols);
        return -1;
    }
    if (src_cols % 8 == 0 && dst_cols % 8 == 0 && dst_col_offset % 8 == 0 && aligned16(dst) && aligned16(src)) {
        int blocks;
        const RowVec P = rowvec_plan(T, src_cols / 8, blocks);
        k_cols_copy_v8<<<blocks, 256, 0, kf_stream()>>>((h16 *)dst, dst_cols, dst_col_offset, (const h16 *)src,
                                                        src_cols, 0, T, P);
    } else {
        k_concat_cols<<<kf_blocks((long long)T * src_cols, 256, 8192), 256, 0, kf_stream()>>>(
            (h16 *)dst, T, dst_cols, (const h16 *)src, src_cols, dst_col_offset);
    }
    return ops_check("concat_cols");
}
int ops_slice_cols(const void *src, int T, int src_cols, void *dst, int dst_cols,
                   int src_col_offset) {
    kf_take_pending(__func__);
    if ((long long)T * dst_cols <= 0) return 0;
    if (src_col_offset < 0 || src_col_offset + dst_cols > src_cols) {
        ops_set_error("slice_cols: offset %d + %d > %d", src_col_offset, dst_cols, src_cols);
        return -1;
    }
    if (src_cols % 8 == 0 && dst_cols % 8 == 0 && src_col_offset % 8 == 0 && aligned16(dst) && aligned16(src)) {
        int blocks;
        const RowVec P = rowvec_plan(T, dst_cols / 8, blocks);
        k_cols_copy_v8<<<blocks, 256, 0, kf_stream()>>>((h16 *)dst, dst_cols, 0, (const h16 *)src, src_cols,
                                                        src_col_offset, T, P);
    } else {
        k_slice_cols<<<kf_blocks((long long)T * dst_cols, 256, 8192), 256, 0, kf_stream()>>>(
            (h16 *)dst, T, dst_cols, (const h16 *)src, src_cols, src_col_offset);
    }
    return ops_check("slice_cols");
}

int ops_combine_feature_maps(void *data, int T, int total_dim, int height, int nf1, int nf2) {
    kf_take_pending(__func__);
    const long long total = (long long)T * total_dim;
    if (total <= 0) return 0;
    if ((long long)height * (nf1 + nf2) != total_dim) {
        ops_set_error("combine_feature_maps: height*(nf1+nf2)=%d != %d", height * (nf1 + nf2),
                      total_dim);
        return -1;
    }
    void *tmp = kf_workspace(total * 2, 1);
    if (!tmp) {
        ops_set_error("combine alloc: out of memory");
        return -1;
    }
    hipMemcpyAsync(tmp, data, total * 2, hipMemcpyDeviceToDevice, kf_stream());
    k_combine_fm<<<kf_blocks(total, 256, 8192), 256, 0, kf_stream()>>>(
        (h16 *)data, (const h16 *)tmp, T, total_dim, height, nf1, nf2);
    return ops_check("combine_feature_maps");
}

void ops_subsample_rows(void *dst, const void *src, int in_rows, int cols, int stride,
                        int row_offset) {
    if (stride <= 0) return;
    const int out_rows = (in_rows - row_offset + stride - 1) / stride;
    if (out_rows <= 0 || cols <= 0) return;
    k_subsample_rows<<<kf_blocks((long long)out_rows * cols, 256, 8192), 256, 0, kf_stream()>>>(
        (h16 *)dst, (const h16 *)src, out_rows, cols, stride, row_offset);
}

int ops_relu_backward(const void *x, void *grad, int count) {
    kf_take_pending(__func__);
    if (count <= 0) return 0;
    k_act_bwd<<<kf_blocks(count / 8 + 1, 256, 8192), 256, 0, kf_stream()>>>(
        (const h16 *)x, (h16 *)grad, count, ACT_RELU, aligned16(x) && aligned16(grad));
    return ops_check("relu_backward");
}
int ops_sigmoid_backward(const void *out, void *grad, int count) {
    kf_take_pending(__func__);
    if (count <= 0) return 0;
    k_act_bwd<<<kf_blocks(count / 8 + 1, 256, 8192), 256, 0, kf_stream()>>>(
        (const h16 *)out, (h16 *)grad, count, ACT_SIGMOID, aligned16(out) && aligned16(grad));
    return ops_check("sigmoid_backward");
}
int ops_tanh_backward(const void *out, void *grad, int count) {
    kf_take_pending(__func__);
    if (count <= 0) return 0;
    k_act_bwd<<<kf_blocks(count / 8 + 1, 256, 8192), 256, 0, kf_stream()>>>(
        (const h16 *)out, (h16 *)grad, count, ACT_TANH, aligned16(out) && aligned16(grad));
    return ops_check("tanh_backward");
}
// several transposes in one launch (the network's transposed weight copies after an
// update): block b belongs to the job whose tile range [blk0[j], blk0[j + 1]) holds it
struct TransposeJobs {
    const h16 *src[KF_TRANSPOSE_MAX];
    h16 *dst[KF_TRANSPOSE_MAX];
    int M[KF_TRANSPOSE_MAX], N[KF_TRANSPOSE_MAX], gx[KF_TRANSPOSE_MAX];
    int blk0[KF_TRANSPOSE_MAX + 1];
    int n;
};
__global__ void k_transpose_batch(TransposeJobs J) {
    __shared__ h16 tile[64][65];
    int j = 0;
    while (j + 1 < J.n && (int)blockIdx.x >= J.blk0[j + 1]) ++j;
    const int b = blockIdx.x - J.blk0[j];
    const int bx = (b % J.gx[j]) * 64, by = (b / J.gx[j]) * 64, M = J.M[j], N = J.N[j];
    const h16 *src = J.src[j];
    h16 *dst = J.dst[j];
    for (int r = threadIdx.y; r < 64; r += blockDim.y) {
        const int m = by + r, n = bx + threadIdx.x;
        if (m < M && n < N) tile[r][threadIdx.x] = src[(long long)m * N + n];
    }
    __syncthreads();
    for (int r = threadIdx.y; r < 64; r += blockDim.y) {
        const int n = bx + r, m = by + threadIdx.x;
        if (m < M && n < N) dst[(long long)n * M + m] = tile[threadIdx.x][r];
    }
}
extern "C" int kf_transpose_batch(int n, const void *const *src, void *const *dst, const int *M, const int *N) {
    kf_take_pending(__func__);
    if (n < 0 || n > KF_TRANSPOSE_MAX) {
        kf_report_error("kf_transpose_batch: %d jobs (at most %d)", n, KF_TRANSPOSE_MAX);
        return -1;
    }
    TransposeJobs J{};
    int tot = 0;
    for (int i = 0; i < n; ++i) {
        if (M[i] <= 0 || N[i] <= 0) {
            kf_report_error("kf_transpose_batch: job %d is %d x %d", i, M[i], N[i]);
            return -1;
        }
        J.src[i] = (const h16 *)src[i];
        J.dst[i] = (h16 *)dst[i];
        J.M[i] = M[i];
        J.N[i] = N[i];
        J.gx[i] = (N[i] + 63) / 64;
        J.blk0[i] = tot;
        tot += J.gx[i] * ((M[i] + 63) / 64);
    }
    J.blk0[n] = tot;
    J.n = n;
    if (!tot) return 0;
    k_transpose_batch<<<tot, dim3(64, 4), 0, kf_stream()>>>(J);
    return ops_check("transpose_batch");
}

int ops_transpose(const void *src, void *dst, int M, int N) {
    kf_take_pending(__func__);
    if (M <= 0 || N <= 0) return 0;
    dim3 grid((N + 63) / 64, (M + 63) / 64);
    k_transpose<<<grid, dim3(64, 4), 0, kf_stream()>>>((const h16 *)src, (h16 *)dst, M, N);
    return ops_check("transpose");
}
int ops_batchnorm_backward(const void *grad_out, void *grad_in, const float *gamma,
                           const float *variance, float eps, int rows, int cols) {
    kf_take_pending(__func__);
    const long long total = (long long)rows * cols;
    if (total <= 0) return 0;
    if (cols % 8 == 0 && aligned16(grad_out) && aligned16(grad_in)) {
        int blocks;
        const RowVec P = rowvec_plan(rows, cols / 8, blocks);
        k_bn_bwd_v8<<<blocks, 256, 0, kf_stream()>>>((const h16 *)grad_out, (h16 *)grad_in, gamma, variance, eps,
                                                     rows, P);
    } else {
        k_bn_bwd<<<kf_blocks(total, 256, 8192), 256, 0, kf_stream()>>>(
            (const h16 *)grad_out, (h16 *)grad_in, gamma, variance, eps, total, cols);
    }
    return ops_check("batchnorm_backward");
}
int ops_fp16_to_fp32(const void *src, float *dst, int count) {
    kf_take_pending(__func__);
    if (count <= 0) return 0;
    k_h2f<<<kf_blocks(count / 8 + 1, 256, 8192), 256, 0, kf_stream()>>>((const h16 *)src, dst, count,
                                                                       aligned16(src) && aligned16(dst));
    return ops_check("fp16_to_fp32");
}
int ops_sgd_update(float *w_fp32, void *w_fp16, const void *grad_fp16, float *velocity,
                   float lr, float momentum, int count) {
    kf_take_pending(__func__);
    if (count <= 0) return 0;
    const int vec = aligned16(w_fp32) && aligned16(w_fp16) && aligned16(grad_fp16) && aligned16(velocity);
    k_sgd<<<kf_blocks(count / 8 + 1, 256, 8192), 256, 0, kf_stream()>>>(
        w_fp32, (h16 *)w_fp16, (const h16 *)grad_fp16, velocity, lr, momentum, count, vec);
    return ops_check("sgd_update");
}

}  // extern "C"
