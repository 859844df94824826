// layers.hip — the few CNN-TDNN pieces that are not MFMA-shaped:
//   * IDCT (K = 40 dense, forward.go:317-330) — a register dot per output group;
//   * the first conv layer, whose input has one filter so im2col K = 9
//     (forward.go:418-524 with num-filters-in = 1): direct 9-tap kernel with the
//     bias / ReLU / mask / BatchNorm epilogue fused, and its weight gradient as a
//     deterministic two-pass reduction;
//   * the flat multi-tensor SGD with fp32 master weights
//     (backward_wrappers.cu:129-142 applied to every parameter in one launch).
// All are HBM-bound; every lane moves 16-byte vectors.
#include "kf_common.h"
#include "../../include/kf_ops.h"

KF_DECLARE_ERR(lay)

static int lay_check(const char *what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        lay_set_error("%s: %s", what, hipGetErrorString(e));
        return -1;
    }
    return 0;
}
extern "C" const char *kf_layers_last_error(void) { return lay_err_.get(); }

// y[t][j..j+7] = sum_k x[t][k] * M[k][j..j+7]; K <= 64, N % 8 == 0, M fp16 [K x N]
__global__ void k_small_gemm(const h16 *x, int ldx, const h16 *Mw, h16 *y, int ldy, int T, int K,
                             int N) {
    __shared__ float sm[64 * 64];
    for (int i = threadIdx.x; i < K * N; i += blockDim.x) sm[i] = h2f(Mw[i]);
    __syncthreads();
    const int groups = N / 8;
    const long long total = (long long)T * groups;
    for (long long it = (long long)blockIdx.x * blockDim.x + threadIdx.x; it < total;
         it += (long long)gridDim.x * blockDim.x) {
        const int t = (int)(it / groups), g = (int)(it - (long long)t * groups);
        float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        const h16 *xr = x + (long long)t * ldx;
        for (int k = 0; k < K; ++k) {
            const float xv = h2f(xr[k]);
#pragma unroll
            for (int e = 0; e < 8; ++e) acc[e] += xv * sm[k * N + 8 * g + e];
        }
        half8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = f2h(acc[e]);
        store_h8(y + (long long)t * ldy + 8 * g, o);
    }
}

// first conv layer, one input filter: x [T x hin], out [(t*hout+h) x fout]
struct ConvC1 {
    int T, hin, hout, sub, fout, noff;
    int dt[9], dh[9];
};

// First conv layer (one input filter, K <= 9, too thin for MFMA), forward with ReLU,
// mask and frozen BatchNorm. The input frames a workgroup touches are staged in LDS
// once: a workgroup owns C1_TB frames (all output heights), its input tile is
// [C1_TB + dtmax - dtmin frames][heights dhmin .. (hout-1)*sub + dhmax] as fp32 with the
// time / height padding as zeros, and every (row, 8-filter group) item reads its <= 9
// taps from LDS (the 8 groups of a row broadcast one address, consecutive heights are
// consecutive words) instead of as 2-byte global loads (361 -> 187 us per launch for
// cnn1 at T = 96,000 against the global-load form). Each thread keeps one 8-filter
// group's 9 x 8 weights in registers.
#define C1_TB 16
__global__ __launch_bounds__(256) void k_conv_c1_fwd_tile(ConvC1 c, int dtmin, int dtmax, int dhmin, int dhmax,
                                                          const h16 *x, const h16 *W, const h16 *bias,
                                                          const float *scale, const float *shift, h16 *y,
                                                          uint8_t *mask) {
    extern __shared__ float xs[];
    const int groups = c.fout / 8, tid = threadIdx.x;
    const int t0 = blockIdx.x * C1_TB, nt = min(C1_TB, c.T - t0);
    const int wd = (c.hout - 1) * c.sub + dhmax - dhmin + 1, nf = nt + dtmax - dtmin;
    for (int i = tid; i < nf * wd; i += 256) {
        const int tt = i / wd, hh = i - tt * wd;
        const int ts = t0 + dtmin + tt, hs = dhmin + hh;
        xs[i] = (ts >= 0 && ts < c.T && hs >= 0 && hs < c.hin) ? h2f(x[(long long)ts * c.hin + hs]) : 0.f;
    }
    const int g = tid % groups;
    float w[9][8], b[8], sc[8], sf[8];
#pragma unroll
    for (int o = 0; o < 9; ++o)
#pragma unroll
        for (int e = 0; e < 8; ++e) w[o][e] = o < c.noff ? h2f(W[o * c.fout + 8 * g + e]) : 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        b[e] = bias ? h2f(bias[8 * g + e]) : 0.f;
        sc[e] = scale ? scale[8 * g + e] : 1.f;
        sf[e] = scale ? shift[8 * g + e] : 0.f;
    }
    int tap[9];  // LDS word offset of each tap relative to (row's frame, h * sub)
#pragma unroll
    for (int o = 0; o < 9; ++o) tap[o] = o < c.noff ? (c.dt[o] - dtmin) * wd + c.dh[o] - dhmin : 0;
    __syncthreads();
    const int rows = nt * c.hout, step = 256 / groups;
    for (int row = tid / groups; row < rows; row += step) {
        const int tl = row / c.hout, h = row - tl * c.hout;
        const float *xr = xs + tl * wd + h * c.sub;
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = b[e];
#pragma unroll
        for (int o = 0; o < 9; ++o) {
            const float xv = o < c.noff ? xr[tap[o]] : 0.f;
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = fmaf(xv, w[o][e], v[e]);
        }
        unsigned bits = 0;
        half8 out;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            float a = v[e];
            if (a > 0.f) bits |= 1u << e;
            else a = 0.f;
            if (scale) a = fmaf(a, sc[e], sf[e]);
            out[e] = f2h(a);
        }
        const long long idx = ((long long)(t0 + tl) * c.hout + h) * c.fout + 8 * g;
        store_h8(y + idx, out);
        if (mask) mask[idx >> 3] = (uint8_t)bits;
    }
}

// partial dW / db of the 1-filter conv. Thread = (row group, 8 consecutive
// filters): 16-byte dz loads, the <= 9 input taps per row read through L1.
// Each block reduces a contiguous range of rows in a fixed order into
// slab[block][noff+1][fout] (row noff = bias): deterministic, HBM-rate. The input frames
// of the block's rows sit in LDS as fp32 with zero padding (as k_conv_c1_fwd_tile), so
// the taps are LDS reads, not 2-byte global loads.
constexpr int C1_UNROLL = 4;
constexpr int C1_RED = 4 * 32 * 80;  // cross-wave image: 4 waves x (fout / 8 <= 32) lanes x 80 floats
__global__ __launch_bounds__(256) void k_conv_c1_wgrad(ConvC1 c, int dtmin, int dtmax, int dhmin, int dhmax,
                                                       const h16 *x, const h16 *dz, float *slab,
                                                       int rows_per_block) {
    extern __shared__ __attribute__((aligned(16))) float red[];  // [4 waves x fg][10*8], then the input tile
    const int fg = c.fout / 8;                 // threads per row
    const int lane_f = threadIdx.x % fg, rg = threadIdx.x / fg, nrg = blockDim.x / fg;
    const int rows = c.T * c.hout;             // < 2^31, checked on the host
    const int r0 = blockIdx.x * rows_per_block;
    const int r1 = min(rows, r0 + rows_per_block);
    float *xs = red + C1_RED;
    const int tb = r0 / c.hout, wd = (c.hout - 1) * c.sub + dhmax - dhmin + 1;
    const int nf = (max(r1 - 1, r0) / c.hout - tb + 1) + dtmax - dtmin;
    for (int i = threadIdx.x; i < nf * wd; i += 256) {
        const int tt = i / wd, hh = i - tt * wd;
        const int ts = tb + dtmin + tt, hs = dhmin + hh;
        xs[i] = (ts >= 0 && ts < c.T && hs >= 0 && hs < c.hin) ? h2f(x[(long long)ts * c.hin + hs]) : 0.f;
    }
    int tap[9];
#pragma unroll
    for (int o = 0; o < 9; ++o) tap[o] = o < c.noff ? (c.dt[o] - dtmin) * wd + c.dh[o] - dhmin : 0;
    __syncthreads();
    float acc[10][8];
#pragma unroll
    for (int o = 0; o < 10; ++o)
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[o][e] = 0.f;
    for (int rb = r0 + rg; rb < r1; rb += nrg * C1_UNROLL) {
        half8 g[C1_UNROLL];
        float xv[C1_UNROLL][9];
#pragma unroll
        for (int u = 0; u < C1_UNROLL; ++u) {
            const int r = rb + u * nrg;
            const bool live = r < r1;
            const int rr = live ? r : r0;  // clamped: every load is issued, dead rows add zero
            g[u] = load_h8(dz + (long long)rr * c.fout + 8 * lane_f);
            if (!live) g[u] = half8{};
            const int t = rr / c.hout, h = rr - t * c.hout;
            const float *xr = xs + (t - tb) * wd + h * c.sub;
#pragma unroll
            for (int o = 0; o < 9; ++o) xv[u][o] = o < c.noff ? xr[tap[o]] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < C1_UNROLL; ++u)
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const float gv = (float)g[u][e];
#pragma unroll
                for (int o = 0; o < 9; ++o) acc[o][e] = fmaf(gv, xv[u][o], acc[o][e]);
                acc[9][e] += gv;
            }
    }
    // sum over the row groups in a fixed order: first the wave's row groups (lanes
    // fg apart) by a butterfly over the lane bits above lane_f, then the waves through LDS
    // (an 80-float image per thread needed 80 KB of LDS and held the kernel to one workgroup
    // per CU)
#pragma unroll
    for (int o = 0; o < 10; ++o)
#pragma unroll
        for (int e = 0; e < 8; ++e)
            for (int m = fg; m < 64; m <<= 1) acc[o][e] += __shfl_xor(acc[o][e], m);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane < fg) {
        float *mine = red + (wave * fg + lane) * 80;
#pragma unroll
        for (int o = 0; o < 10; ++o)
#pragma unroll
            for (int e = 0; e < 8; ++e) mine[o * 8 + e] = acc[o][e];
    }
    __syncthreads();
    float *out = slab + (long long)blockIdx.x * (c.noff + 1) * c.fout;
    const int nw = blockDim.x / 64;
    for (int i = threadIdx.x; i < (c.noff + 1) * c.fout; i += blockDim.x) {
        const int o = i / c.fout, f = i - o * c.fout;
        const int src = o == c.noff ? 9 : o;
        const int tf = f / 8, e = f - tf * 8;
        float s = 0.f;
        for (int k = 0; k < nw; ++k) s += red[(k * fg + tf) * 80 + src * 8 + e];
        out[i] = s;
    }
}

// one 256-thread block per output: thread j sums slabs j, j+256, ... then a
// fixed-order tree over the block (deterministic)
__global__ void k_conv_c1_reduce(const float *slab, int nblk, int n, float *dW, float *db,
                                 int wcount) {
    __shared__ float sh[256];
    const int i = blockIdx.x;
    float s = 0.f;
    for (int b = threadIdx.x; b < nblk; b += blockDim.x) s += slab[(long long)b * n + i];
    sh[threadIdx.x] = s;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w) sh[threadIdx.x] += sh[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        if (i < wcount) dW[i] = sh[0];
        else if (db) db[i - wcount] = sh[0];
    }
}

// flat SGD with momentum and fp32 master weights; fp32 gradient
__global__ void k_sgd_flat(float *w32, h16 *w16, const float *g, float *v, float lr, float mom,
                           long long n) {
    const long long n4 = n / 4;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
         i += (long long)gridDim.x * blockDim.x) {
        float4v gv = reinterpret_cast<const float4v *>(g)[i];
        float4v vv = reinterpret_cast<float4v *>(v)[i];
        float4v wv = reinterpret_cast<float4v *>(w32)[i];
        half4 hv;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            vv[e] = mom * vv[e] + gv[e];
            wv[e] = wv[e] - lr * vv[e];
            hv[e] = f2h(wv[e]);
        }
        reinterpret_cast<float4v *>(v)[i] = vv;
        reinterpret_cast<float4v *>(w32)[i] = wv;
        reinterpret_cast<half4 *>(w16)[i] = hv;
    }
    for (long long i = n4 * 4 + (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x) {
        const float vv = mom * v[i] + g[i];
        v[i] = vv;
        w32[i] -= lr * vv;
        w16[i] = f2h(w32[i]);
    }
}

// fp16 <- fp32 for a flat parameter set (master -> working copy)
__global__ void k_f32_to_f16_flat(const float *s, h16 *d, long long n) {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x)
        d[i] = f2h(s[i]);
}

// fused frozen BatchNorm on a [rows x D] fp16 tensor (y = x*scale + shift)
__global__ void k_bn_apply(const h16 *x, h16 *y, long long rows, int D, const float *scale,
                           const float *shift) {
    const long long total = rows * D;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const int d = (int)(i % D);
        y[i] = f2h(fmaf(h2f(x[i]), scale[d], shift[d]));
    }
}

extern "C" {

int kf_small_gemm(const void *x, int ldx, const void *Mw, void *y, int ldy, int T, int K, int N) {
    kf_take_pending(__func__);
    if (K > 64 || N > 64 || N % 8) {
        lay_set_error("small_gemm: K=%d N=%d unsupported", K, N);
        return -1;
    }
    if (T <= 0) return 0;
    k_small_gemm<<<kf_blocks((long long)T * (N / 8), 256, 4096), 256, 0, kf_stream()>>>(
        (const h16 *)x, ldx, (const h16 *)Mw, (h16 *)y, ldy, T, K, N);
    return lay_check("small_gemm");
}

int kf_bn_apply(const void *x, void *y, long long rows, int D, const float *scale,
                const float *shift) {
    kf_take_pending(__func__);
    if (rows <= 0) return 0;
    k_bn_apply<<<kf_blocks(rows * D, 256, 8192), 256, 0, kf_stream()>>>(
        (const h16 *)x, (h16 *)y, rows, D, scale, shift);
    return lay_check("bn_apply");
}

int kf_conv_c1_forward(int T, int hin, int hout, int sub, int fout, int noff, const int *dt,
                       const int *dh, const void *x, const void *W, const void *bias,
                       const float *scale, const float *shift, void *y, uint8_t *mask) {
    kf_take_pending(__func__);
    if (noff > 9 || fout % 8 || fout > 256 || 256 % (fout / 8) ||
        (long long)T * hout * fout >= (1LL << 31)) {
        lay_set_error("conv_c1_forward: noff=%d fout=%d T*hout=%lld unsupported", noff, fout,
                      (long long)T * hout);
        return -1;
    }
    ConvC1 c{T, hin, hout, sub, fout, noff, {0}, {0}};
    for (int i = 0; i < noff; ++i) {
        c.dt[i] = dt[i];
        c.dh[i] = dh[i];
    }
    // (a row-per-thread form with all 64 filters measured slower)
    int dtmin = 0, dtmax = 0, dhmin = 0, dhmax = 0;
    for (int i = 0; i < noff; ++i) {
        dtmin = std::min(dtmin, dt[i]);
        dtmax = std::max(dtmax, dt[i]);
        dhmin = std::min(dhmin, dh[i]);
        dhmax = std::max(dhmax, dh[i]);
    }
    const size_t lds = (size_t)4 * (C1_TB + dtmax - dtmin) * ((hout - 1) * sub + dhmax - dhmin + 1);
    if (lds > 64 * 1024) {
        lay_set_error("conv_c1_forward: input tile of %zu bytes exceeds the LDS budget", lds);
        return -1;
    }
    if (T <= 0) return 0;
    k_conv_c1_fwd_tile<<<(T + C1_TB - 1) / C1_TB, 256, lds, kf_stream()>>>(
        c, dtmin, dtmax, dhmin, dhmax, (const h16 *)x, (const h16 *)W, (const h16 *)bias, scale, shift, (h16 *)y,
        mask);
    return lay_check("conv_c1_forward");
}

int kf_conv_c1_wgrad(int T, int hin, int hout, int sub, int fout, int noff, const int *dt,
                     const int *dh, const void *x, const void *dz, float *dW, float *db) {
    kf_take_pending(__func__);
    if (noff > 9 || fout % 8 || fout > 256 || 256 % (fout / 8) ||
        (long long)T * hout * fout >= (1LL << 31)) {
        lay_set_error("conv_c1_wgrad: noff=%d fout=%d T*hout=%lld unsupported", noff, fout,
                      (long long)T * hout);
        return -1;
    }
    ConvC1 c{T, hin, hout, sub, fout, noff, {0}, {0}};
    for (int i = 0; i < noff; ++i) {
        c.dt[i] = dt[i];
        c.dh[i] = dh[i];
    }
    const long long rows = (long long)T * hout;
    // one round of workgroups, three per CU (rocprof, T = 96,000: 181 us at 768 against
    // 191 / 204 / 273 us at 1536 / 2048 / 4096); KF_C1_NBLK: another count (A/B)
    static const int env_nblk = getenv("KF_C1_NBLK") ? atoi(getenv("KF_C1_NBLK")) : 0;
    int cus = 0, dev = 0;
    hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    int nblk = env_nblk > 0 ? env_nblk : 3 * cus;
    int rpb = (int)((rows + nblk - 1) / nblk);
    if (rpb < 256) rpb = 256;
    nblk = (int)((rows + rpb - 1) / rpb);
    const int n = (noff + 1) * fout;
    float *slab = (float *)kf_workspace((size_t)nblk * n * 4, 2);
    if (!slab) {
        lay_set_error("conv_c1_wgrad: workspace");
        return -1;
    }
    int dtmin = 0, dtmax = 0, dhmin = 0, dhmax = 0;
    for (int i = 0; i < noff; ++i) {
        dtmin = std::min(dtmin, dt[i]);
        dtmax = std::max(dtmax, dt[i]);
        dhmin = std::min(dhmin, dh[i]);
        dhmax = std::max(dhmax, dh[i]);
    }
    // input tile: the frames of rpb rows (+1 for a range straddling frames) plus the time
    // offsets, heights dhmin .. (hout-1)*sub + dhmax
    const size_t tile = (size_t)4 * ((rpb + hout - 1) / hout + 1 + dtmax - dtmin) *
                        ((hout - 1) * sub + dhmax - dhmin + 1);
    // (before it: the cross-wave image, C1_RED floats)
    if (C1_RED * 4 + tile > 160 * 1024) {
        lay_set_error("conv_c1_wgrad: input tile of %zu bytes exceeds the LDS", tile);
        return -1;
    }
    k_conv_c1_wgrad<<<nblk, 256, C1_RED * 4 + tile, kf_stream()>>>(c, dtmin, dtmax, dhmin, dhmax, (const h16 *)x,
                                                                   (const h16 *)dz, slab, rpb);
    k_conv_c1_reduce<<<n, 256, 0, kf_stream()>>>(slab, nblk, n, dW, db, noff * fout);
    return lay_check("conv_c1_wgrad");
}

// ---------------------------------------------------------------------------
// Supervised-row sets of the row-subsampled train step (kf_nnet.h
// nnet_set_row_subsampling): compact row c of a layer above the conv stack is source row
// crow(c) = 3c for c < tc0, else (T - 1) - 3 (tc - 1 - c) (the clamped-edge tail). One
// thread moves 16 bytes; row_bytes % 16 == 0.
// ---------------------------------------------------------------------------
__device__ __forceinline__ long long crow_of(long long c, int T, int tc0, int tc) {
    return c < tc0 ? 3 * c : (long long)(T - 1) - 3 * ((long long)tc - 1 - c);
}
__global__ __launch_bounds__(256) void k_gather_rows(uint4 *dst, const uint4 *src, long long vpr, int T, int tc0,
                                                     int tc) {
    const long long n = (long long)tc * vpr;
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
        const long long c = i / vpr, v = i - c * vpr;
        dst[i] = src[crow_of(c, T, tc0, tc) * vpr + v];
    }
}
// full rows t < T: the compact row whose source row t is, else zero
// (rows r0 .. T - 1 only, dst row 0 = full row r0)
__global__ __launch_bounds__(256) void k_scatter_rows(uint4 *dst, const uint4 *src, long long vpr, int T, int tc0,
                                                      int tc, int r0) {
    const long long n = (long long)(T - r0) * vpr;
    const int nt = tc - tc0, rt = (T - 1) % 3;
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
        const long long t = r0 + i / vpr, v = i % vpr;
        long long c = -1;
        if (t % 3 == 0 && t / 3 < tc0) c = t / 3;
        else if (nt > 0 && t % 3 == rt && t >= (long long)(T - 1) - 3LL * (nt - 1)) c = tc - 1 - ((T - 1) - t) / 3;
        dst[i] = c >= 0 ? src[c * vpr + v] : uint4{0u, 0u, 0u, 0u};
    }
}
struct BlockMap {
    int n;
    int src[32];
};
// dst block b = src block M.src[b], or zeros where M.src[b] < 0 (blocks of vpb uint4)
__global__ __launch_bounds__(256) void k_copy_blocks(uint4 *dst, const uint4 *src, long long vpb, BlockMap M) {
    const long long n = (long long)M.n * vpb;
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
        const int b = (int)(i / vpb);
        const int sb = M.src[b];
        dst[i] = sb >= 0 ? src[sb * vpb + (i - b * vpb)] : uint4{0u, 0u, 0u, 0u};
    }
}
struct RowList {
    int n;
    int row[4];
};
// edge[c] = rne(sum over the listed rows, in list order, of src[row][c]) (fp32 sum)
__global__ __launch_bounds__(256) void k_rows_sum_list(h16 *edge, const h16 *src, long long ld, RowList L, int cols) {
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c >= cols) return;
    float s = 0.f;
    for (int i = 0; i < L.n; ++i) s += h2f(src[(long long)L.row[i] * ld + c]);
    edge[c] = f2h(s);
}

int kf_gather_rows(void *dst, const void *src, long long row_bytes, int T, int tc0, int tc) {
    kf_take_pending(__func__);
    if (row_bytes <= 0 || row_bytes % 16 || tc0 < 0 || tc < tc0 || T <= 0 || 3LL * (tc0 - 1) > T - 1) {
        lay_set_error("gather_rows: bad geometry (row_bytes %lld T %d tc0 %d tc %d)", row_bytes, T, tc0, tc);
        return -1;
    }
    if (tc == 0) return 0;
    const long long vpr = row_bytes / 16;
    k_gather_rows<<<kf_blocks((long long)tc * vpr, 256, 16384), 256, 0, kf_stream()>>>((uint4 *)dst, (const uint4 *)src,
                                                                                    vpr, T, tc0, tc);
    return lay_check("gather_rows");
}
int kf_scatter_rows_from(void *dst, const void *src, long long row_bytes, int T, int tc0, int tc, int r0) {
    kf_take_pending(__func__);
    if (row_bytes <= 0 || row_bytes % 16 || tc0 < 0 || tc < tc0 || T <= 0 || 3LL * (tc0 - 1) > T - 1 || r0 < 0 ||
        r0 >= T) {
        lay_set_error("scatter_rows: bad geometry (row_bytes %lld T %d tc0 %d tc %d r0 %d)", row_bytes, T, tc0, tc, r0);
        return -1;
    }
    const long long vpr = row_bytes / 16;
    k_scatter_rows<<<kf_blocks((long long)(T - r0) * vpr, 256, 16384), 256, 0, kf_stream()>>>(
        (uint4 *)dst, (const uint4 *)src, vpr, T, tc0, tc, r0);
    return lay_check("scatter_rows");
}
int kf_scatter_rows(void *dst, const void *src, long long row_bytes, int T, int tc0, int tc) {
    return kf_scatter_rows_from(dst, src, row_bytes, T, tc0, tc, 0);
}
int kf_copy_blocks(void *dst, const void *src, long long block_bytes, const int *map, int nblocks) {
    kf_take_pending(__func__);
    if (block_bytes <= 0 || block_bytes % 16 || nblocks < 0 || nblocks > 32 || (nblocks && !map)) {
        lay_set_error("copy_blocks: bad geometry (block_bytes %lld nblocks %d)", block_bytes, nblocks);
        return -1;
    }
    if (!nblocks) return 0;
    BlockMap M;
    M.n = nblocks;
    for (int b = 0; b < 32; ++b) M.src[b] = b < nblocks ? map[b] : -1;
    const long long vpb = block_bytes / 16;
    k_copy_blocks<<<kf_blocks((long long)nblocks * vpb, 256, 4096), 256, 0, kf_stream()>>>((uint4 *)dst,
                                                                                       (const uint4 *)src, vpb, M);
    return lay_check("copy_blocks");
}
int kf_rows_sum_list(void *edge, const void *src, long long ld, const int *rows, int n, int cols) {
    kf_take_pending(__func__);
    if (n < 0 || n > 4 || cols <= 0 || (n && !rows)) {
        lay_set_error("rows_sum_list: %d rows (at most 4), %d columns", n, cols);
        return -1;
    }
    RowList L{n, {0, 0, 0, 0}};
    for (int i = 0; i < n; ++i) L.row[i] = rows[i];
    k_rows_sum_list<<<(cols + 255) / 256, 256, 0, kf_stream()>>>((h16 *)edge, (const h16 *)src, ld, L, cols);
    return lay_check("rows_sum_list");
}

int kf_sgd_flat(float *w32, void *w16, const float *g, float *v, float lr, float mom,
                long long n) {
    kf_take_pending(__func__);
    if (n <= 0) return 0;
    k_sgd_flat<<<kf_blocks(n / 4 + 1, 256, 8192), 256, 0, kf_stream()>>>(w32, (h16 *)w16, g, v, lr,
                                                                        mom, n);
    return lay_check("sgd_flat");
}

int kf_f32_to_f16_flat(const float *src, void *dst, long long n) {
    kf_take_pending(__func__);
    if (n <= 0) return 0;
    k_f32_to_f16_flat<<<kf_blocks(n, 256, 8192), 256, 0, kf_stream()>>>(src, (h16 *)dst, n);
    return lay_check("f32_to_f16_flat");
}

}  // extern "C"
