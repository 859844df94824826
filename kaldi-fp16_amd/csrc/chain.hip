// chain.hip — chain LF-MMI objective on MI355X (gfx950).
//
// Two workgroup-resident kernels replace the reference's per-frame launch
// storms (chain.cu launches T kernels per pass with CAS atomics;
// chain_den.cu ~10 launches + 3 blocking D2H copies per frame):
//
//   k_logfb   log-domain forward-backward of one FST per workgroup, all frames
//             in one launch, fixed arc order (the deterministic algorithm of
//             chain_det.cu:55-237; posteriors summed per pdf in arc order, i.e.
//             exactly the order of chain_det.cu:147-190's single thread).
//   k_den_fb  probability-space denominator of chain_den.cu:496-706 with the
//             leaky HMM, one sequence per workgroup: alpha'/beta state vectors
//             and the frame's exp(x) row live in LDS; arcs are streamed from a
//             sliced, degree-sorted table (SELL-64: lane = state, one coalesced
//             8-byte record per arc and step); den posteriors accumulate in LDS
//             as 2^-44 fixed point (ds_add_u64 — order-independent, hence
//             deterministic); the product mode fuses the whole objective
//             assembly of backward.go:224-371 (penalty, +w*num, -w*den, L2, NaN
//             rule) into the per-frame epilogue and writes the fp16 gradient
//             row straight into the network's output-gradient matrix.
//
// The C-ABI of chain.h / chain_den.h / chain_backward_api.h is served by the same
// kernels; kf_chain.h is the batched, device-resident product interface.
#include "kf_common.h"
#include "../../include/chain.h"
#include "../../include/chain_backward_api.h"
#include "../../include/chain_den.h"
#include "../../include/kf_chain.h"
#include "../../include/kf_ops.h"

#include <cmath>
#include <map>
#include <mutex>
#include <vector>

KF_DECLARE_ERR(chain)
KF_DECLARE_ERR(den)
KF_DECLARE_ERR(kfc)

extern "C" const char *chain_last_error(void) { return chain_err_.get(); }
extern "C" void chain_clear_error(void) { chain_err_.clear(); }
extern "C" const char *den_last_error(void) { return den_err_.get(); }
extern "C" void den_clear_error(void) { den_err_.clear(); }
extern "C" const char *kf_chain_last_error(void) { return kfc_err_.get(); }
extern "C" void kf_chain_clear_error(void) { kfc_err_.clear(); }

static const float kLogZero = -1.0e+30f;
static const float kFix = 17592186044416.0f;          // 2^44
static const double kInvFix = 1.0 / 17592186044416.0;  // 2^-44

// ===========================================================================
// Device helpers
// ===========================================================================
__device__ __forceinline__ float logadd_dev(float a, float b) {  // chain_det.cu:26-35
    if (a <= kLogZero) return b;
    if (b <= kLogZero) return a;
    float mx = fmaxf(a, b), mn = fminf(a, b);
    return mx + log1pf(expf(mn - mx));
}

template <typename XT>
__device__ __forceinline__ float ld_x(const XT *p) { return (float)*p; }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
// Deterministic block sum: wave butterflies, then the per-wave sums in wave order.
// Every thread returns the same value. Contains one barrier; `red` must not be
// reused before the next barrier.
template <int NW>
__device__ __forceinline__ float block_sum(float v, float *red) {
    v = wave_sum(v);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) s += red[w];
    return s;
}
template <int NW>
__device__ __forceinline__ double block_sum_d(double v, double *red) {
    v = wave_sum_d(v);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < NW; ++w) s += red[w];
    return s;
}

// ===========================================================================
// Log-domain forward-backward (numerator; chain.h ABI)
// ===========================================================================
struct LogFstDev {
    const int *row_ptr, *in_ptr, *in_arc, *arc_src, *arc_dst, *arc_pdf;
    const float *arc_w;
    const int *grp_ptr, *grp_pdf, *grp_arc;
    // pre-gathered copies for the LDS-resident kernel (k_num_fb)
    const int *in_src, *in_g, *arc_g, *gsrc, *gdst;
    const float *in_w, *gw;
    const int *fin_state;
    const float *fin_w;
    int S, A, G, nfinal, start, T;
    int mode;        // bit0: forward+backward, bit1: posteriors
    int stride;
    long long row0;  // frame t -> nnet row row0 + t*stride
    float *alpha, *beta;  // [(T+1) x S]
    float *post_sparse;   // [T x G] or null
    float *post_dense;    // [T x P] or null
    float *total;         // [1] (in: when mode has no forward)
};

enum { LF_FB = 1, LF_POST = 2 };

__global__ __launch_bounds__(256) void k_logfb(const LogFstDev *fsts, const h16 *nnet, long long ld,
                                               int P) {
    const LogFstDev f = fsts[blockIdx.x];
    const int S = f.S, T = f.T, tid = threadIdx.x;
    if (S <= 0 || T < 0) return;
    float total;
    if (f.mode & LF_FB) {
        for (int s = tid; s < S; s += 256) f.alpha[s] = (s == f.start) ? 0.0f : kLogZero;
        __syncthreads();
        for (int t = 0; t < T; ++t) {
            const h16 *xr = nnet + (f.row0 + (long long)t * f.stride) * ld;
            const float *ac = f.alpha + (size_t)t * S;
            float *an = f.alpha + (size_t)(t + 1) * S;
            for (int d = tid; d < S; d += 256) {
                float v = kLogZero;
                for (int k = f.in_ptr[d]; k < f.in_ptr[d + 1]; ++k) {
                    int a = f.in_arc[k];
                    int p = f.arc_pdf[a];
                    if (p <= 0 || p > P) continue;
                    float sa = ac[f.arc_src[a]];
                    if (sa <= kLogZero) continue;
                    v = logadd_dev(v, sa + (float)xr[p - 1] + f.arc_w[a]);
                }
                an[d] = v;
            }
            __syncthreads();
        }
        total = kLogZero;
        for (int i = 0; i < f.nfinal; ++i)
            total = logadd_dev(total, f.alpha[(size_t)T * S + f.fin_state[i]] + f.fin_w[i]);
        if (tid == 0) *f.total = total;
        float *bT = f.beta + (size_t)T * S;
        for (int s = tid; s < S; s += 256) bT[s] = kLogZero;
        __syncthreads();
        if (tid == 0)
            for (int i = 0; i < f.nfinal; ++i) bT[f.fin_state[i]] = f.fin_w[i];
        __syncthreads();
    } else {
        total = *f.total;
    }
    for (int t = T - 1; t >= 0; --t) {
        const h16 *xr = nnet + (f.row0 + (long long)t * f.stride) * ld;
        const float *bn = f.beta + (size_t)(t + 1) * S;
        if (f.mode & LF_FB) {
            float *bc = f.beta + (size_t)t * S;
            for (int s = tid; s < S; s += 256) {
                float v = kLogZero;
                for (int a = f.row_ptr[s]; a < f.row_ptr[s + 1]; ++a) {
                    int p = f.arc_pdf[a];
                    if (p <= 0 || p > P) continue;
                    float b = bn[f.arc_dst[a]];
                    if (b <= kLogZero) continue;
                    v = logadd_dev(v, b + (float)xr[p - 1] + f.arc_w[a]);
                }
                bc[s] = v;
            }
        }
        if (f.mode & LF_POST) {
            float *pd = f.post_dense ? f.post_dense + (size_t)t * P : nullptr;
            if (pd) {
                for (int p = tid; p < P; p += 256) pd[p] = 0.0f;
                __syncthreads();
            }
            const float *ac = f.alpha + (size_t)t * S;
            for (int g = tid; g < f.G; g += 256) {
                int p = f.grp_pdf[g];
                float acc = 0.0f;
                if (p > 0 && p <= P) {
                    float xv = (float)xr[p - 1];
                    for (int k = f.grp_ptr[g]; k < f.grp_ptr[g + 1]; ++k) {
                        int a = f.grp_arc[k];
                        float av = ac[f.arc_src[a]];
                        if (av <= kLogZero) continue;
                        float b = bn[f.arc_dst[a]];
                        if (b <= kLogZero) continue;
                        float lp = av + xv + f.arc_w[a] + b - total;
                        if (lp > 0.0f) lp = 0.0f;  // chain.cu:309-311
                        acc += expf(lp);
                    }
                    if (pd) pd[p - 1] = acc;
                }
                if (f.post_sparse) f.post_sparse[(size_t)t * f.G + g] = acc;
            }
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// Product numerator: the whole FST (arcs pre-gathered per incoming / outgoing /
// pdf-group order) lives in LDS; per frame only the G distinct pdf values of the
// output row are fetched, one frame ahead. Same arithmetic and order as k_logfb.
// ---------------------------------------------------------------------------
#define NUM_THREADS 256
#define NUM_PRE 4  // S, G <= 1024 (larger FSTs use k_logfb)

struct NumLds {  // word offsets into dynamic LDS
    int a0, a1, xg0, xg1, in_ptr, in_src, in_g, in_w, row_ptr, arc_dst, arc_g, arc_w, gpdf, misc, words;
};
__host__ __device__ inline NumLds num_lds_layout(int S, int A, int G, int Ag) {
    (void)Ag;  // the pdf-group arcs are read by k_num_post from global memory
    NumLds L;
    int o = 0;
    L.a0 = o; o += S;
    L.a1 = o; o += S;
    L.xg0 = o; o += G;
    L.xg1 = o; o += G;
    L.in_ptr = o; o += S + 1;
    L.in_src = o; o += A;
    L.in_g = o; o += A;
    L.in_w = o; o += A;
    L.row_ptr = o; o += S + 1;
    L.arc_dst = o; o += A;
    L.arc_g = o; o += A;
    L.arc_w = o; o += A;
    L.gpdf = o; o += G;
    L.misc = o; o += 4;
    L.words = o;
    return L;
}

// Workgroups [0, nseq) run the forwards (alpha rows and the total), [nseq, 2 nseq) the
// backwards at the same time (the backward needs neither alpha nor the total: it stores
// its beta rows); k_num_post then forms the posteriors from the stored rows. (One
// workgroup per sequence running both passes took 2.7 ms alone, 4.6 ms beside the den
// recursion; the split takes 1.8 + 0.7 ms and costs the recursion ~0.25 ms less.)
__global__ __launch_bounds__(NUM_THREADS) void k_num_fb(const LogFstDev *fsts, const h16 *nnet,
                                                        long long ld, int P, int nseq) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const bool do_fwd = (int)blockIdx.x < nseq;
    const LogFstDev f = fsts[(int)blockIdx.x % nseq];
    const int S = f.S, A = f.A, G = f.G, T = f.T, tid = threadIdx.x;
    const int Ag = f.G > 0 ? f.grp_ptr[f.G] : 0;
    const NumLds L = num_lds_layout(S, A, G, Ag);
    float *W = reinterpret_cast<float *>(smem);
    int *I = reinterpret_cast<int *>(smem);
    // stage the FST; arcs whose pdf is outside [1, P] get group -1 (skipped)
    for (int i = tid; i <= S; i += NUM_THREADS) {
        I[L.in_ptr + i] = f.in_ptr[i];
        I[L.row_ptr + i] = f.row_ptr[i];
    }
    for (int q = tid; q < G; q += NUM_THREADS) I[L.gpdf + q] = f.grp_pdf[q];
    for (int k = tid; k < A; k += NUM_THREADS) {
        int g0 = f.in_g[k], g1 = f.arc_g[k];
        int p0 = g0 >= 0 ? f.grp_pdf[g0] : 0, p1 = g1 >= 0 ? f.grp_pdf[g1] : 0;
        I[L.in_src + k] = f.in_src[k];
        I[L.in_g + k] = (p0 > 0 && p0 <= P) ? g0 : -1;
        W[L.in_w + k] = f.in_w[k];
        I[L.arc_dst + k] = f.arc_dst[k];
        I[L.arc_g + k] = (p1 > 0 && p1 <= P) ? g1 : -1;
        W[L.arc_w + k] = f.arc_w[k];
    }
    float *cur = W + L.a0, *nxt = W + L.a1;
    if (do_fwd)
        for (int s = tid; s < S; s += NUM_THREADS) {
            float v = (s == f.start) ? 0.0f : kLogZero;
            cur[s] = v;
            f.alpha[s] = v;
        }
    __syncthreads();
    auto row_of = [&](int t) { return nnet + (f.row0 + (long long)t * f.stride) * ld; };
    float pre[NUM_PRE];
    auto fetch_x = [&](int t) {
        const h16 *xr = row_of(t);
#pragma unroll
        for (int i = 0; i < NUM_PRE; ++i) {  // unconditional (clamped) loads, then select
            int q = tid + i * NUM_THREADS;
            int p = q < G ? I[L.gpdf + q] : 0;
            float v = (float)xr[min(max(p, 1), P) - 1];
            pre[i] = (p > 0 && p <= P) ? v : 0.0f;
        }
    };
    auto store_x = [&](float *xg) {
#pragma unroll
        for (int i = 0; i < NUM_PRE; ++i) {
            int q = tid + i * NUM_THREADS;
            if (q < G) xg[q] = pre[i];
        }
    };
    // ---- forward
    if (do_fwd) {
    if (T > 0) {
        fetch_x(0);
        store_x(W + L.xg0);
        if (T > 1) fetch_x(1);
    }
    __syncthreads();
    for (int t = 0; t < T; ++t) {
        const float *xg = W + ((t & 1) ? L.xg1 : L.xg0);
        float *an = f.alpha + (size_t)(t + 1) * S;
        for (int d = tid; d < S; d += NUM_THREADS) {
            float v = kLogZero;
            for (int k = I[L.in_ptr + d]; k < I[L.in_ptr + d + 1]; ++k) {
                int g = I[L.in_g + k];
                if (g < 0) continue;
                float sa = cur[I[L.in_src + k]];
                if (sa <= kLogZero) continue;
                v = logadd_dev(v, sa + xg[g] + W[L.in_w + k]);
            }
            nxt[d] = v;
            an[d] = v;
        }
        if (t + 1 < T) {
            store_x(W + ((t & 1) ? L.xg0 : L.xg1));
            if (t + 2 < T) fetch_x(t + 2);
        }
        __syncthreads();
        float *tmp = cur;
        cur = nxt;
        nxt = tmp;
    }
    // total over the finals, in order (chain.cu:213-240)
    if (tid == 0) {
        float tot = kLogZero;
        for (int i = 0; i < f.nfinal; ++i) tot = logadd_dev(tot, cur[f.fin_state[i]] + f.fin_w[i]);
        W[L.misc] = tot;
        *f.total = tot;
    }
        return;
    }  // forward
    // ---- backward: beta rows into f.beta (rows 0 .. T)
    float *bn = W + L.a0, *bc = W + L.a1;  // beta[t+1], beta[t]
    __syncthreads();
    for (int s = tid; s < S; s += NUM_THREADS) bn[s] = kLogZero;
    if (T > 0) {
        fetch_x(T - 1);
        store_x(W + L.xg0);
        if (T > 1) fetch_x(T - 2);
    }
    __syncthreads();
    if (tid == 0)
        for (int i = 0; i < f.nfinal; ++i) bn[f.fin_state[i]] = f.fin_w[i];
    __syncthreads();
    for (int s = tid; s < S; s += NUM_THREADS) f.beta[(size_t)T * S + s] = bn[s];
    for (int t = T - 1, it = 0; t >= 0; --t, ++it) {
        const float *xg = W + ((it & 1) ? L.xg1 : L.xg0);
        for (int s = tid; s < S; s += NUM_THREADS) {
            float v = kLogZero;
            for (int k = I[L.row_ptr + s]; k < I[L.row_ptr + s + 1]; ++k) {
                int g = I[L.arc_g + k];
                if (g < 0) continue;
                float b = bn[I[L.arc_dst + k]];
                if (b <= kLogZero) continue;
                v = logadd_dev(v, b + xg[g] + W[L.arc_w + k]);
            }
            bc[s] = v;
            f.beta[(size_t)t * S + s] = v;
        }
        if (t > 0) {
            store_x(W + ((it & 1) ? L.xg0 : L.xg1));
            if (t > 1) fetch_x(t - 2);
        }
        __syncthreads();
        float *tmp = bn;
        bn = bc;
        bc = tmp;
    }
}

// posteriors of the numerator (after k_num_fb): one workgroup per (sequence,
// NUM_POST_FR frames) from the stored alpha[t], beta[t+1] and the total — the arithmetic
// and order of k_num_fb's fused posterior loop
#define NUM_POST_FR 8
__global__ __launch_bounds__(NUM_THREADS) void k_num_post(const LogFstDev *fsts, const h16 *nnet, long long ld,
                                                          int P, int nfb) {
    const LogFstDev f = fsts[blockIdx.x / nfb];
    const int t0 = (blockIdx.x % nfb) * NUM_POST_FR;
    const float total = *f.total;
    for (int t = t0; t < min(f.T, t0 + NUM_POST_FR); ++t) {
    const float *ar = f.alpha + (size_t)t * f.S, *bn = f.beta + (size_t)(t + 1) * f.S;
    const h16 *xr = nnet + (f.row0 + (long long)t * f.stride) * ld;
    float *ps = f.post_sparse + (size_t)t * f.G;
    for (int q = threadIdx.x; q < f.G; q += NUM_THREADS) {
        const int p = f.grp_pdf[q];
        float acc = 0.0f;
        if (p > 0 && p <= P) {
            const float xv = (float)xr[p - 1];
            for (int k = f.grp_ptr[q]; k < f.grp_ptr[q + 1]; ++k) {
                float av = ar[f.gsrc[k]];
                if (av <= kLogZero) continue;
                float b = bn[f.gdst[k]];
                if (b <= kLogZero) continue;
                float lp = av + xv + f.gw[k] + b - total;
                if (lp > 0.0f) lp = 0.0f;  // chain.cu:309-311
                acc += expf(lp);
            }
        }
        ps[q] = acc;
    }
    }
}

// ===========================================================================
// Denominator (prob space, leaky HMM) — SELL-64 arc tables
// ===========================================================================
struct SellDev {  // sliced ELL, 64 rows per slice, rows sorted by degree
    int nsl;
    const int *perm, *len, *off;
    // records {f1 | f2 << 16, tp} with f1, f2 as the LDS byte offsets of their operands
    // in rows interleaving NS sequences (f, b) or frames (q): 4 * NS * f1, 4 * NS * f2,
    // index NS - 1 — one address add per gather
    const uint2 *arc_p[2];
    const float *initp;   // init[perm[c]] in slice order (0 for padding rows), f and b only
    // Slice ownership for G = 1, 2, 4, 8 blocks per sequence (index log2 G): the slices
    // are spread over the G x DEN_WAVES (block, wave) pairs by length, longest first onto
    // the least loaded pair, so the slowest wave of a frame carries about the mean share
    // (round-robin ownership left it 1.3-1.4x the mean on the den graph's degree-sorted
    // slices). slot[lgG][gi * spg + k]: the slice in slot k of block gi, processed by
    // wave k % DEN_WAVES (-1: empty). The q table keeps only its G = 1 lists (the
    // posterior kernel's waves).
    const int *slot[4];
    int spg[4];
};
struct DenDev {
    int S, P;
    SellDev f;  // rows = destination states: {src, pdf0}
    SellDev b;  // rows = source states:      {dst, pdf0}
    SellDev q;  // rows = pdfs:               {src, dst}
    const float *init;
    int pair_ok;  // the NS = 2 recursion fits the LDS
};

struct DenRun {
    const void *nnet;
    long long ld;
    const long long *row0;  // [nseq]
    const int *frames;      // [nseq]
    int stride, max_frames;
    float leaky;
    int backward;           // 0: forward only
    float *den_out;         // [nseq][2] {total_prob, log-prob} from k_den_fwd
    unsigned long long *trace;  // optional phase timestamps (kf_chain_trace), null = off
    float *alpha_store;     // [nseq][max_frames+1][nsl_f*64], forward-table slice order
    float *beta_store;      // [nseq][max_frames+1][nsl_b*64], backward-table slice order
    float *asum_store;      // [nseq][max_frames+1] alpha sums (alpha'[t] = row + asum[t]*leaky*init)
    float *bsum_store;      // [nseq][max_frames+1] <init, beta'[t]> (beta[t] = row + leaky*bsum[t])
    float *stats;           // [nseq][8]
    // ABI mode
    float *post_dense;      // [T x P] (single sequence)
    // product mode
    const LogFstDev *nums;  // [nseq] numerator descriptors (total, G, grp_pdf, post_sparse)
    h16 *out_grad;
    long long ldg;
    KfChainOpts opts;
};

enum { DEN_ABI = 0, DEN_PRODUCT = 1 };
#define DEN_THREADS 1024
#define DEN_WAVES 16
#define DEN_MAXPT 4  // P <= 4096
#define DEN_MAXS 8  // S <= 8192

// Row prefetch held in registers between frames: fp16 rows stay packed (2 per VGPR).
// Loads are unconditional (index clamped); the out-of-range select at issue makes the
// fetch wait for its row, which measured faster than a select at use (5.87 vs 6.13 ms
// for k_den_fb: the consume loads then no longer queue behind the HBM row in vmcnt).
template <typename XT> struct RowPre {
    float v[DEN_MAXPT];
    __device__ __forceinline__ void fetch(const XT *row, int P) {
#pragma unroll
        for (int i = 0; i < DEN_MAXPT; ++i) {
            int p = threadIdx.x + i * DEN_THREADS;
            float x = (float)row[min(p, P - 1)];
            v[i] = p < P ? x : 0.0f;
        }
    }
    __device__ __forceinline__ float get(int i, int) const { return v[i]; }
};
template <> struct RowPre<h16> {
    uint32_t v[DEN_MAXPT / 2];
    __device__ __forceinline__ void fetch(const h16 *row, int P) {
        const unsigned short *u = reinterpret_cast<const unsigned short *>(row);
#pragma unroll
        for (int i = 0; i < DEN_MAXPT / 2; ++i) {
            int p0 = threadIdx.x + (2 * i) * DEN_THREADS, p1 = p0 + DEN_THREADS;
            uint32_t lo = __builtin_nontemporal_load(u + min(p0, P - 1));
            uint32_t hi = __builtin_nontemporal_load(u + min(p1, P - 1));
            v[i] = (p0 < P ? lo : 0u) | ((p1 < P ? hi : 0u) << 16);
        }
    }
    __device__ __forceinline__ float get(int i, int) const {
        unsigned short b = (unsigned short)((i & 1) ? (v[i >> 1] >> 16) : (v[i >> 1] & 0xFFFF));
        return (float)__builtin_bit_cast(h16, b);
    }
};
struct StatePre {  // alpha' row prefetch (S <= DEN_MAXS * DEN_THREADS)
    float v[DEN_MAXS];
    __device__ __forceinline__ void fetch(const float *row, int S) {
#pragma unroll
        for (int i = 0; i < DEN_MAXS; ++i) {
            int s = threadIdx.x + i * DEN_THREADS;
            float x = __builtin_nontemporal_load(row + min(s, S - 1));
            v[i] = s < S ? x : 0.0f;
        }
    }
};

// fwd / bwd LDS: reduction scratch, the NS-interleaved state row (va or vb, nsl * 64
// entries in the table's slice order) and exp row (xe), and the table's slice metadata
// (len / off / this block's slots)
#define DEN_LDS_TOTAL (160 * 1024)
static size_t den_rec_fixed_bytes(int P, int nsl, int spg, int ns) {
    return (size_t)4 * (64 + (size_t)ns * ((size_t)nsl * 64 + P + (P & 1)) + 2 * (size_t)nsl + spg) + 64;
}
// posteriors: the alpha' and beta rows of `pair` frames in the f / b tables' slice orders
// (rs = nsl * 64 entries each), the gamma rows and the q table's perm / len / off
static size_t den_post_lds_bytes(int rs, int P, int nslq, int pair = 1) {
    return (size_t)4 * (64 + 2 * (size_t)pair * rs + (size_t)pair * P + (size_t)nslq * 66);
}

// ---------------------------------------------------------------------------
// Cross-workgroup exchange (G workgroups per sequence). Hand-off recipe of
// cdna_hip_programming.md §6 Guideline 16 (R1, counter form, all-sc1): every
// payload word is stored write-through (sc1) by its wave, every storing wave
// drains vmcnt, the workgroup barriers, one lane adds to the sequence's counter
// (agent scope); consumers poll that counter relaxed (bounded, s_sleep), barrier,
// and read every payload word with sc1 loads. Counters and the per-launch timeout
// word are zeroed by hipMemsetAsync before every launch; a block that gives up also
// adds to a sticky word that only kf_chain_result / the den ABI read and clear, so a
// timed-out launch is reported even when later launches succeed.
// ---------------------------------------------------------------------------
typedef __attribute__((address_space(1))) unsigned int gu32_t;
#define RLX_AGENT __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT

__device__ __forceinline__ void st_sc1(float *p, float v) {
    __hip_atomic_store((gu32_t *)p, __float_as_uint(v), RLX_AGENT);
}
__device__ __forceinline__ float ld_sc1(const float *p) {
    return __uint_as_float(__hip_atomic_load((gu32_t *)p, RLX_AGENT));
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t den_rsrc(const void *base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), (short)0, (int)0xFFFFFFFF, 0x00020000);
}
// Exchange word access. LOC: every block of the sequence runs on one XCD, so they share
// one L2 — plain stores (written through the CU's L1 into that L2, acknowledged there)
// and sc0 loads (which miss the L1) hand the data over without the write-through to
// memory that agent scope (sc1) needs across XCDs. `base` is uniform, `i` a word index.
template <bool LOC>
__device__ __forceinline__ void x_st(float *base, int i, float v) {
    if constexpr (LOC)
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), den_rsrc(base), i * 4, 0, 0);
    else
        st_sc1(base + i, v);
}
template <bool LOC>
__device__ __forceinline__ float x_ld(const float *base, int i) {
    if constexpr (LOC)
        return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(den_rsrc(base), i * 4, 0, 1 /* sc0 */));
    else
        return ld_sc1(base + i);
}

// NS = 2: the blocks of a unit run two sequences at once. The LDS state is
// interleaved (float2 per state), so one SELL record, one pair of address adds and
// two 8-byte gathers serve both sequences (the record stream and the gather issue of
// the arc phase halve per sequence); G doubles so the grid keeps every CU busy.
struct DenX {
    float *buf;     // [nseq][2][G][blk]; blk = 64: [q * DEN_WAVES + wave] = that wave's partial
                    // sum of sequence q of the unit (the state slices themselves are exchanged
                    // through the alpha / beta stores)
    unsigned *cnt;  // [nseq] arrivals (zeroed before each launch)
    unsigned *xm;   // [nseq] XCD census: 4-bit arrival count per XCD (zeroed before each launch)
    int force_sys;  // 1: agent-scope exchange even when a unit's blocks share an XCD (tests)
    unsigned *tmo;  // per-launch timeout word (zeroed before each launch)
    unsigned *sticky;  // timed-out blocks since the last read (never zeroed by a launch)
    unsigned spin_limit;  // polls before a wait gives up (kf_chain_debug_spin_limit)
    int G, lgG, spg, blk;  // spg: exchange slots per block (the table's at this G)
    int nseq;              // exchange units (NS sequences each: 2u, 2u+1 for NS = 2)
    int nseqs, ns;         // sequences, sequences per unit
    unsigned lds_f, lds_b; // dynamic LDS of the fwd / bwd kernels
};

// unit / slice-owner of this block; the G blocks of a unit share an XCD when the grid
// allows it (blocks b and b+8 share one, MI355X_MICROARCH.md)
__device__ __forceinline__ void den_map(const DenX &X, int &unit, int &gi) {
    const int nb = X.nseq * X.G, b = blockIdx.x;
    int w = b;
    if (nb % 8 == 0 && (nb / 8) % X.G == 0) w = (b % 8) * (nb / 8) + b / 8;
    unit = w >> X.lgG;
    gi = w & (X.G - 1);
}

// publish: every wave stores its NS partial sums (lane 0, tail slots q * DEN_WAVES +
// wave); every wave drains vmcnt, the workgroup barriers, one lane adds the arrival
// (one store drain per frame)
template <bool LOC, int NS>
__device__ __forceinline__ void den_publish(const DenX &X, float *tail, const float (&wsum)[NS], int unit) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (lane == 0) {
#pragma unroll
        for (int q = 0; q < NS; ++q) x_st<LOC>(tail, q * DEN_WAVES + wave, wsum[q]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) __hip_atomic_fetch_add((gu32_t *)&X.cnt[unit], 1u, RLX_AGENT);
}
// one lane polls `word` until done(value); false on timeout, uniform. *val: the last value
template <class Done>
__device__ __forceinline__ bool den_poll(const DenX &X, const unsigned *word, Done done, int *lds_flag,
                                         unsigned *val = nullptr) {
    if (threadIdx.x == 0) {
        int ok = 1;
        for (unsigned it = 0;; ++it) {
            const unsigned v = __hip_atomic_load((gu32_t *)word, RLX_AGENT);
            if (val) *val = v;
            if (done(v)) break;
            if ((it & 255) == 255 && __hip_atomic_load((gu32_t *)X.tmo, RLX_AGENT)) {
                ok = 0;
                break;
            }
            if (it >= X.spin_limit) {  // ~seconds by default: a partner block is not resident
                __hip_atomic_store((gu32_t *)X.tmo, 1u, RLX_AGENT);
                __hip_atomic_fetch_add((gu32_t *)X.sticky, 1u, RLX_AGENT);
                ok = 0;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        *lds_flag = ok;
    }
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    return *lds_flag != 0;
}
// wait for `target` arrivals; false on timeout, uniform
__device__ __forceinline__ bool den_wait(const DenX &X, int unit, unsigned target, int *lds_flag) {
    return den_poll(X, &X.cnt[unit], [&](unsigned v) { return v >= target; }, lds_flag);
}
// XCD census before the first exchange: 1 if all G blocks of the unit run on one XCD
// (the placement den_map asks the dispatcher for, not a guarantee), 0 if not or
// forced, -1 on timeout; uniform. Each block adds 1 to its XCD's 4-bit field.
__device__ __forceinline__ int den_xcd_local(const DenX &X, int unit, int *lds_flag) {
    if (unit >= X.nseq) return 0;  // grid padding: no exchange
    unsigned *word = X.xm + unit;
    if (threadIdx.x == 0) {
        const unsigned xcc = __builtin_amdgcn_s_getreg((20) | (3 << 11)) & 7;  // HW_REG_XCC_ID
        __hip_atomic_fetch_add((gu32_t *)word, 1u << (4 * xcc), RLX_AGENT);
    }
    auto total = [](unsigned v) {
        unsigned n = 0;
        for (int k = 0; k < 8; ++k) n += (v >> (4 * k)) & 15;
        return n;
    };
    unsigned *vl = reinterpret_cast<unsigned *>(lds_flag) + 1;
    if (!den_poll(X, word, [&](unsigned v) { return total(v) >= (unsigned)X.G; }, lds_flag, vl)) return -1;
    const unsigned v = *vl;
    bool one = false;
    for (int k = 0; k < 8; ++k)
        if (((v >> (4 * k)) & 15) == (unsigned)X.G) one = true;
    return one && !X.force_sys ? 1 : 0;
}
// NS values per state: the LDS state row is NS-interleaved (one 4 * NS-byte word per state)
template <int NS> struct DenV {
    float x[NS];
};
template <int NS>
__device__ __forceinline__ DenV<NS> lds_v(const unsigned char *base, unsigned off) {
    DenV<NS> r;
    if constexpr (NS == 2) {
        const float2 t = *reinterpret_cast<const float2 *>(base + off);
        r.x[0] = t.x;
        r.x[1] = t.y;
    } else {
        r.x[0] = *reinterpret_cast<const float *>(base + off);
    }
    return r;
}

// Exchanged state rows of the NS sequences of a unit (rows[q], slice order: every slice
// stored by the block that owns it) and the G x DEN_WAVES partial sums of buffer `buf`:
// first sum(q, total) for every live q (fixed order, equal in every lane), then
// f(slice position, values, initp) per position. Only live sequences are loaded (rows[q] of a sequence
// past its last frame is never read); their values are 0 in f. The partial sums load
// with the rows, so one round trip serves both.
template <bool LOC, int NS, class FS, class F>
__device__ __forceinline__ void den_consume(const DenX &X, int unit, int buf, float *const (&rows)[NS],
                                            const bool (&live)[NS], int nsl, const float *initp, FS sum, F f) {
    int tid = threadIdx.x;
    // opaque to the optimiser: the row addresses below are rebuilt every frame instead of
    // being hoisted out of the frame loop as 64-bit values
    asm volatile("" : "+v"(tid));
    const int n = nsl * 64, lane = tid & 63;
    const float *xb = X.buf + ((size_t)unit * 2 + buf) * X.G * X.blk;
    float pv[NS];
#pragma unroll
    for (int q = 0; q < NS; ++q) pv[q] = 0.0f;
    for (int i = lane; i < X.G * DEN_WAVES; i += 64) {
#pragma unroll
        for (int q = 0; q < NS; ++q)
            if (live[q]) pv[q] += x_ld<LOC>(xb, (i / DEN_WAVES) * X.blk + q * DEN_WAVES + i % DEN_WAVES);
    }
    float v[NS][DEN_MAXS], ip[DEN_MAXS];
#pragma unroll
    for (int m = 0; m < DEN_MAXS; ++m) ip[m] = initp ? initp[min(tid + m * DEN_THREADS, n - 1)] : 0.0f;
#pragma unroll
    for (int q = 0; q < NS; ++q) {
        if (live[q]) {
#pragma unroll
            for (int m = 0; m < DEN_MAXS; ++m) v[q][m] = x_ld<LOC>(rows[q], min(tid + m * DEN_THREADS, n - 1));
        } else {
#pragma unroll
            for (int m = 0; m < DEN_MAXS; ++m) v[q][m] = 0.0f;
        }
    }
#pragma unroll
    for (int q = 0; q < NS; ++q)
        if (live[q]) sum(q, wave_sum(pv[q]));
#pragma unroll
    for (int m = 0; m < DEN_MAXS; ++m) {
        const int c = tid + m * DEN_THREADS;
        if (c < n) {
            DenV<NS> val;
#pragma unroll
            for (int q = 0; q < NS; ++q) val.x[q] = v[q][m];
            f(c, val, ip[m]);
        }
    }
}

// new state values of the live sequences into the NS-interleaved LDS row (a sequence
// past its last frame keeps its final state for the end-of-launch totals)
template <int NS>
__device__ __forceinline__ void den_put(float *row, int st, const DenV<NS> &v, const bool (&live)[NS]) {
    if constexpr (NS == 2) {
        float2 *p = reinterpret_cast<float2 *>(row) + st;
        if (live[0] && live[1]) *p = make_float2(v.x[0], v.x[1]);
        else if (live[0]) row[2 * st] = v.x[0];
        else if (live[1]) row[2 * st + 1] = v.x[1];
    } else {
        if (live[0]) row[st] = v.x[0];
    }
}

// gather-sum over one slice of a SELL table for the NS sequences (fixed arc order per
// sequence). Records carry LDS byte offsets pre-scaled for the NS layout: state row at
// `sv`, exp row at `sx`.
template <int NS>
__device__ __forceinline__ void sell_slice(const uint2 *arcs, int len, int off, int lane, const unsigned char *sv,
                                           const unsigned char *sx, float (&acc)[NS]) {
#pragma clang fp contract(off)  // (a * tp) * x + acc rounded as the oracle does, any NS
    const uint2 *e = arcs + (size_t)off * 64 + lane;
#pragma unroll
    for (int q = 0; q < NS; ++q) acc[q] = 0.f;
    for (int k = 0; k < len; k += 8) {  // 8 records in flight per lane (len is a multiple of 8)
        uint2 rr[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) rr[i] = e[(k + i) * 64];
        DenV<NS> a[8], x[8];  // all 16 gathers in flight before the first product
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            a[i] = lds_v<NS>(sv, rr[i].x & 0xFFFF);
            x[i] = lds_v<NS>(sx, rr[i].x >> 16);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const float tp = __uint_as_float(rr[i].y);
#pragma unroll
            for (int q = 0; q < NS; ++q) acc[q] += a[i].x[q] * tp * x[i].x[q];
        }
    }
}

// Per-block SELL state: len / off of every slice and this block's slot list (slot k is
// processed by wave k % DEN_WAVES; -1 = empty) in LDS; initp stays in global memory
// (L2-resident, read once per position per frame), which keeps the NS = 2 recursion small
// enough to share a CU with the numerator kernel on the side stream. States are named by
// slice position (make_den_tables), so no permutation is needed: positions >= S are
// padding.
struct SellLds {
    const int *len, *off;  // [nsl] each
    const int *slot;       // [spg]
    const float *initp;    // [nsl*64], global
};
__device__ __forceinline__ SellLds stage_sell(const SellDev &T, int lgG, int gi, int spg, unsigned char *base) {
    int *lenl = reinterpret_cast<int *>(base), *offl = lenl + T.nsl;
    int *slotl = offl + T.nsl;
    for (int i = threadIdx.x; i < T.nsl; i += DEN_THREADS) {
        lenl[i] = T.len[i];
        offl[i] = T.off[i];
    }
    for (int i = threadIdx.x; i < spg; i += DEN_THREADS) slotl[i] = T.slot[lgG][gi * spg + i];
    SellLds L{lenl, offl, slotl, T.initp};
    return L;
}

// The NS sequences of unit `unit` (sequence NS*unit + q; absent past nseqs) and their frame
// counts, row offsets and liveness at iteration `it` of a recursion.
template <int NS> struct DenUnit {
    int seq[NS], T[NS];
    long long r0[NS];
    bool has[NS];
    __device__ __forceinline__ DenUnit(const DenRun &r, const DenX &X, int unit) {
#pragma unroll
        for (int q = 0; q < NS; ++q) {
            seq[q] = unit * NS + q;
            has[q] = unit < X.nseq && seq[q] < X.nseqs;
            T[q] = has[q] ? r.frames[seq[q]] : 0;
            r0[q] = has[q] ? r.row0[seq[q]] : 0;
        }
    }
    __device__ __forceinline__ int tmax() const {
        int m = 0;
#pragma unroll
        for (int q = 0; q < NS; ++q) m = max(m, T[q]);
        return m;
    }
};

// exp(clamp(x)) of the NS prefetched rows into the interleaved exp row; 0 for a sequence
// with no row (`on` false)
template <typename XT, int NS>
__device__ __forceinline__ void den_put_exp(float *xe, int P, const RowPre<XT> (&pre)[NS], const bool (&on)[NS]) {
#pragma unroll
    for (int i = 0; i < DEN_MAXPT; ++i) {
        const int p = threadIdx.x + i * DEN_THREADS;
        if (p < P) {
#pragma unroll
            for (int q = 0; q < NS; ++q)  // kernel_apply_exp
                xe[NS * p + q] = on[q] ? expf(fmaxf(-30.0f, fminf(30.0f, pre[q].get(i, P)))) : 0.0f;
        }
    }
}

// Forward pass (chain_den.cu:583-620), G blocks per unit: block gi computes alpha[t+1]
// for the destination rows of its slices (a load-balanced share, SellDev::slot) for the
// NS sequences and stores them into row t+1 of each sequence's alpha store, which is also
// the exchange: all blocks rebuild the full alpha'[t+1] in LDS from those rows. The store
// keeps the slices before the leaky term: alpha'[t] = row[t] + asum[t] * leaky * init,
// which k_den_post applies when it loads the row (one write per frame, not two).
template <typename XT, bool LOC, int NS>
__device__ __forceinline__ void den_fwd_body(const DenDev &g, const DenRun &r, const DenX &X,
                                             unsigned char *smem, int unit, int gi) {
    const int S = g.S, P = g.P, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int G = X.G, nsl = g.f.nsl, spg = X.spg;
    const int PP = P + (P & 1);
    float *red = reinterpret_cast<float *>(smem);          // [32]
    int *flag = reinterpret_cast<int *>(smem) + 32;        // [32]
    const int rs = nsl * 64;  // rows (LDS and stored) are in slice order: contiguous, whole lines
    float *va = reinterpret_cast<float *>(smem) + 64;      // [rs][NS] alpha'[t]
    float *xe = va + NS * rs;                              // [PP][NS] exp(clamp(x))
    unsigned char *sbase = reinterpret_cast<unsigned char *>(xe + NS * PP);
    const unsigned char *sv = reinterpret_cast<const unsigned char *>(va);
    const unsigned char *sx = reinterpret_cast<const unsigned char *>(xe);

    const DenUnit<NS> U(r, X, unit);
    const int Tm = U.tmax();
    const XT *nnet = reinterpret_cast<const XT *>(r.nnet);
    const float leaky = r.leaky;
    float *astore[NS], *asum[NS];
#pragma unroll
    for (int q = 0; q < NS; ++q) {
        const int sq = U.has[q] ? U.seq[q] : 0;
        astore[q] = r.alpha_store + (size_t)sq * (r.max_frames + 1) * rs;
        asum[q] = r.asum_store + (size_t)sq * (r.max_frames + 1);
    }
    const uint2 *arcs = g.f.arc_p[NS - 1];
    const SellLds F = stage_sell(g.f, X.lgG, gi, spg, sbase);
    float part = 0.f;
    for (int s = tid; s < S; s += DEN_THREADS) part += g.init[s];
    const float as0 = block_sum<DEN_WAVES>(part, red);  // AlphaFirstFrame + AlphaDash(0)
    float as[NS];
#pragma unroll
    for (int q = 0; q < NS; ++q) as[q] = as0;
    for (int c = tid; c < rs; c += DEN_THREADS) {
        const float ip = F.initp[c];  // init of the state at position c (0 for padding)
        const float v = ip + as0 * leaky * ip;
#pragma unroll
        for (int q = 0; q < NS; ++q) va[NS * c + q] = v;
    }
    if (gi == 0) {
#pragma unroll
        for (int q = 0; q < NS; ++q) {
            if (!U.has[q]) continue;
            for (int c = tid; c < rs; c += DEN_THREADS) __builtin_nontemporal_store(F.initp[c], astore[q] + c);
            if (tid == 0) {
                asum[q][0] = as0;
                r.stats[(size_t)U.seq[q] * 8 + 3] = 0.0f;  // accumulated by k_den_post
                r.stats[(size_t)U.seq[q] * 8 + 6] = 0.0f;
            }
        }
    }
    RowPre<XT> pre[NS];
    bool on[NS];
#pragma unroll
    for (int q = 0; q < NS; ++q) {
        on[q] = U.T[q] > 0;
        if (on[q]) pre[q].fetch(nnet + U.r0[q] * r.ld, P);
    }
    den_put_exp<XT, NS>(xe, P, pre, on);
    __syncthreads();
    const bool tr = r.trace && unit == 0 && gi == 0 && tid == 0;
#define DEN_TP(i) \
    if (tr && t >= 16 && t < 48) r.trace[(t - 16) * 8 + (i)] = wall_clock64();
    for (int t = 0; t < Tm; ++t) {
        DEN_TP(0);
        bool live[NS];
        float *arow[NS], inv[NS], pq[NS];
#pragma unroll
        for (int q = 0; q < NS; ++q) {
            live[q] = t < U.T[q];
            arow[q] = astore[q] + (size_t)(t + 1) * rs;
            inv[q] = as[q] > 0.0f ? 1.0f / as[q] : 1.0f;
            pq[q] = 0.f;
        }
        const int buf = (t + 1) & 1;
        float *tail = X.buf + (((size_t)unit * 2 + buf) * G + gi) * X.blk;
        for (int k = wave; k < spg; k += DEN_WAVES) {
            const int j = F.slot[k];
            if (j < 0) continue;
            const bool real = j * 64 + lane < S;  // padding positions stay 0
            float acc[NS];
            sell_slice<NS>(arcs, F.len[j], F.off[j], lane, sv, sx, acc);
#pragma unroll
            for (int q = 0; q < NS; ++q) {
                const float v = real ? acc[q] * inv[q] : 0.0f;
                if (live[q]) x_st<LOC>(arow[q], j * 64 + lane, v);
                pq[q] += v;
            }
        }
        if (r.trace && unit == 0 && gi < 2 && lane == 0 && t >= 16 && t < 48)  // per-wave arc end, blocks 0, 1
            r.trace[256 + ((t - 16) * 2 + gi) * DEN_WAVES + wave] = wall_clock64();
        DEN_TP(1);
        float ws[NS];
#pragma unroll
        for (int q = 0; q < NS; ++q) ws[q] = wave_sum(pq[q]);
        den_publish<LOC, NS>(X, tail, ws, unit);
        DEN_TP(2);
        // the next frame's output rows: fetched after the publish, so their latency hides
        // under the exchange wait (fetched at the frame start, the record loads' in-order
        // vmcnt waits queue behind them)
#pragma unroll
        for (int q = 0; q < NS; ++q) {
            on[q] = t + 1 < U.T[q];
            if (on[q]) pre[q].fetch(nnet + (U.r0[q] + (long long)(t + 1) * r.stride) * r.ld, P);
        }
        DEN_TP(3);
        if (!den_wait(X, unit, (unsigned)(G * (t + 1)), flag)) return;
        DEN_TP(4);
        float as1[NS];
#pragma unroll
        for (int q = 0; q < NS; ++q) as1[q] = as[q];
        DEN_TP(5);
        den_consume<LOC, NS>(X, unit, buf, arow, live, nsl, F.initp,
                             [&](int q, float v) { as1[q] = v; },
                             [&](int st, DenV<NS> v, float ip) {
#pragma unroll
                                 for (int q = 0; q < NS; ++q) v.x[q] += as1[q] * leaky * ip;
                                 den_put<NS>(va, st, v, live);
                             });
        DEN_TP(6);
        // past the publish barrier nothing reads this frame's xe
        den_put_exp<XT, NS>(xe, P, pre, on);
        if (gi == 0 && tid == 0) {
#pragma unroll
            for (int q = 0; q < NS; ++q)
                if (live[q]) asum[q][t + 1] = as1[q];
        }
#pragma unroll
        for (int q = 0; q < NS; ++q) as[q] = as1[q];
        __syncthreads();
        DEN_TP(7);
    }
#undef DEN_TP
    if (gi != 0) return;
    // total_prob = sum(alpha'[T]); log_correction = sum_{t<T} log(alpha_sum[t])
#pragma unroll
    for (int q = 0; q < NS; ++q) {
        if (!U.has[q]) continue;  // uniform
        part = 0.f;
        for (int c = tid; c < rs; c += DEN_THREADS) part += va[NS * c + q];
        const float total = block_sum<DEN_WAVES>(part, red);
        double lc = 0.0;
        for (int t = tid; t < U.T[q]; t += DEN_THREADS) {
            float a = asum[q][t];
            if (a > 0.0f) lc += log((double)a);
        }
        double *redd = reinterpret_cast<double *>(smem) + 8;  // red[16..31]
        __syncthreads();
        lc = block_sum_d<DEN_WAVES>(lc, redd);
        if (tid == 0) {
            const int sq = U.seq[q];
            r.den_out[sq * 2 + 0] = total;
            r.den_out[sq * 2 + 1] = (float)(log((double)total) + lc);
            r.stats[(size_t)sq * 8 + 1] = r.den_out[sq * 2 + 1];
        }
        __syncthreads();
    }
}
template <typename XT, int NS>
__global__ __launch_bounds__(DEN_THREADS) void k_den_fwd(const DenDev g, const DenRun r, const DenX X) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    int unit, gi;
    den_map(X, unit, gi);
    const int loc = den_xcd_local(X, unit, reinterpret_cast<int *>(smem) + 32);
    if (loc > 0) den_fwd_body<XT, true, NS>(g, r, X, smem, unit, gi);
    else if (loc == 0) den_fwd_body<XT, false, NS>(g, r, X, smem, unit, gi);
}

// Backward recursion (chain_den.cu:632-684 without the posteriors), G blocks per unit:
// beta'[t] over the source rows of this block's slices for the NS sequences, stored into
// row t of each sequence's beta store, which is also the exchange; beta[t] = beta'[t] +
// leaky*<init, beta'[t]>, the second term kept per frame in bsum (k_den_post adds it).
// The reference scales beta'[t] by 1/sum(alpha[t]) and starts from 1/total_prob; any
// positive per-frame factor gives the same posteriors once k_den_post normalises each
// frame (the den posteriors of a frame sum to one: they are d log p / d x_t), so this
// pass scales by 1/<init, beta'[t+1]> and starts from ones — it needs nothing from the
// forward pass and runs beside it. Iteration `it` is frame T_q - 1 - it of sequence q.
template <typename XT, bool LOC, int NS>
__device__ __forceinline__ void den_bwd_body(const DenDev &g, const DenRun &r, const DenX &X,
                                             unsigned char *smem, int unit, int gi) {
    const int S = g.S, P = g.P, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int G = X.G, nsl = g.b.nsl, spg = X.spg;
    const int PP = P + (P & 1);
    float *red = reinterpret_cast<float *>(smem);      // [32]
    int *flag = reinterpret_cast<int *>(smem) + 32;    // [32]
    const int rs = nsl * 64;
    float *vb = reinterpret_cast<float *>(smem) + 64;  // [rs][NS] beta[t+1], slice order
    float *xe = vb + NS * rs;                          // [PP][NS] exp(clamp(x))
    unsigned char *sbase = reinterpret_cast<unsigned char *>(xe + NS * PP);
    const unsigned char *sv = reinterpret_cast<const unsigned char *>(vb);
    const unsigned char *sx = reinterpret_cast<const unsigned char *>(xe);

    const DenUnit<NS> U(r, X, unit);
    const int Tm = U.tmax();
    const XT *nnet = reinterpret_cast<const XT *>(r.nnet);
    const float leaky = r.leaky;
    float *bstore[NS], *bsum[NS];
#pragma unroll
    for (int q = 0; q < NS; ++q) {
        const int sq = U.has[q] ? U.seq[q] : 0;
        bstore[q] = r.beta_store + (size_t)sq * (r.max_frames + 1) * rs;
        bsum[q] = r.bsum_store + (size_t)sq * (r.max_frames + 1);
    }
    const uint2 *arcs = g.b.arc_p[NS - 1];
    const SellLds B = stage_sell(g.b, X.lgG, gi, spg, sbase);
    // BetaDashLastFrame up to the per-frame factor: beta'[T] = 1, <init, 1> = sum(init)
    float part = 0.f;
    for (int s = tid; s < S; s += DEN_THREADS) part += g.init[s];
    const float n0 = block_sum<DEN_WAVES>(part, red);
    float nrm[NS];
#pragma unroll
    for (int q = 0; q < NS; ++q) nrm[q] = n0;
    for (int c = tid; c < rs; c += DEN_THREADS) {
#pragma unroll
        for (int q = 0; q < NS; ++q) vb[NS * c + q] = 1.0f + leaky * n0;
    }
    if (gi == 0) {
#pragma unroll
        for (int q = 0; q < NS; ++q) {
            if (!U.has[q]) continue;
            float *bT = bstore[q] + (size_t)U.T[q] * rs;
            for (int c = tid; c < rs; c += DEN_THREADS) __builtin_nontemporal_store(1.0f, bT + c);
            if (tid == 0) bsum[q][U.T[q]] = n0;
        }
    }
    RowPre<XT> pre[NS];
    bool on[NS];
#pragma unroll
    for (int q = 0; q < NS; ++q) {
        on[q] = U.T[q] > 0;
        if (on[q]) pre[q].fetch(nnet + (U.r0[q] + (long long)(U.T[q] - 1) * r.stride) * r.ld, P);
    }
    den_put_exp<XT, NS>(xe, P, pre, on);
    __syncthreads();
    for (int it = 0; it < Tm; ++it) {
        bool live[NS];
        int tq[NS];
        float *brow[NS], inv[NS], pq[NS];
#pragma unroll
        for (int q = 0; q < NS; ++q) {
            tq[q] = U.T[q] - 1 - it;
            live[q] = tq[q] >= 0;
            brow[q] = bstore[q] + (size_t)max(tq[q], 0) * rs;
            inv[q] = nrm[q] > 0.0f ? 1.0f / nrm[q] : 1.0f;
            pq[q] = 0.f;
        }
        const int buf = it & 1;
        float *tail = X.buf + (((size_t)unit * 2 + buf) * G + gi) * X.blk;
        for (int k = wave; k < spg; k += DEN_WAVES) {  // kernel_den_backward_transitions
            const int j = B.slot[k];
            if (j < 0) continue;
            const bool real = j * 64 + lane < S;  // padding positions stay 0
            const float ip = B.initp[j * 64 + lane];
            float acc[NS];
            sell_slice<NS>(arcs, B.len[j], B.off[j], lane, sv, sx, acc);
#pragma unroll
            for (int q = 0; q < NS; ++q) {
                const float bd = real ? acc[q] * inv[q] : 0.0f;
                if (live[q]) x_st<LOC>(brow[q], j * 64 + lane, bd);
                pq[q] += ip * bd;
            }
        }
        float ws[NS];
#pragma unroll
        for (int q = 0; q < NS; ++q) ws[q] = wave_sum(pq[q]);
        den_publish<LOC, NS>(X, tail, ws, unit);
#pragma unroll
        for (int q = 0; q < NS; ++q) {  // as den_fwd_body
            on[q] = tq[q] > 0;
            if (on[q]) pre[q].fetch(nnet + (U.r0[q] + (long long)(tq[q] - 1) * r.stride) * r.ld, P);
        }
        if (!den_wait(X, unit, (unsigned)(G * (it + 1)), flag)) return;
        float tb[NS];
#pragma unroll
        for (int q = 0; q < NS; ++q) tb[q] = 0.f;
        den_consume<LOC, NS>(X, unit, buf, brow, live, nsl, nullptr,
                             [&](int q, float v) {
                                 nrm[q] = v;  // <init, beta'[t]>: the next factor
                                 tb[q] = leaky * v;
                             },
                             [&](int st, DenV<NS> v, float) {
#pragma unroll
                                 for (int q = 0; q < NS; ++q) v.x[q] += tb[q];
                                 den_put<NS>(vb, st, v, live);
                             });
        if (gi == 0 && tid == 0) {
#pragma unroll
            for (int q = 0; q < NS; ++q)
                if (live[q]) bsum[q][tq[q]] = nrm[q];
        }
        den_put_exp<XT, NS>(xe, P, pre, on);
        __syncthreads();
    }
}

// Forward and backward recursions of every unit in one launch: blocks of the first half
// run alpha with exchange XF, the second half beta with XB (the two passes are
// independent, see den_bwd_body). One launch keeps all 2*units*G blocks co-resident,
// which the bounded exchange polls rely on; the XCD grouping of den_map is kept (G
// consecutive ids share an XCD).
template <typename XT, int NS>
__global__ __launch_bounds__(DEN_THREADS) void k_den_fb(const DenDev g, const DenRun r, const DenX XF,
                                                        const DenX XB) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    // the numerator kernel's waves share some of these CUs (side stream, it has ~2 ms of
    // slack under this launch): the recursion's waves win the issue arbitration
    __builtin_amdgcn_s_setprio(3);
    const int half = XF.nseq * XF.G, nb = 2 * half, b = blockIdx.x;
    int w = b;
    if (nb % 8 == 0 && (nb / 8) % XF.G == 0) w = (b % 8) * (nb / 8) + b / 8;
    const bool bwd = w >= half;
    const int inner = bwd ? w - half : w;
    const int unit = inner >> XF.lgG, gi = inner & (XF.G - 1);
    const int loc = den_xcd_local(bwd ? XB : XF, unit, reinterpret_cast<int *>(smem) + 32);
    if (loc < 0) return;  // timed out (reported through the timeout words)
    if (bwd) {
        if (loc) den_bwd_body<XT, true, NS>(g, r, XB, smem, unit, gi);
        else den_bwd_body<XT, false, NS>(g, r, XB, smem, unit, gi);
    } else {
        if (loc) den_fwd_body<XT, true, NS>(g, r, XF, smem, unit, gi);
        else den_fwd_body<XT, false, NS>(g, r, XF, smem, unit, gi);
    }
}

// Posteriors (kernel_den_posteriors, chain_den.cu:253-280) for every (sequence,
// frame) in parallel — gamma[t] needs only the stored alpha'[t] and beta[t+1] — by
// pdf rows in arc order (no atomics), and in the product mode the objective
// assembly of backward.go:224-371 into the fp16 gradient row. The whole pass always
// runs; a non-finite objective only zeroes what is written. PAIR frames share one
// stream of the pdf-ordered arc records (the pass is bound by that L2 stream).
#define POST_FRAMES 2  // frames per block (one two-frame pass: 1.82 -> 1.76 ms against 4)
// records carry LDS byte offsets into the PAIR-interleaved alpha' / beta rows (one
// 8-byte gather per operand serves both frames)
template <int PAIR>
__device__ __forceinline__ void post_slice(const uint2 *arcs, int len, int off, int lane,
                                           const unsigned char *sva, const unsigned char *svb, float acc[PAIR]) {
#pragma clang fp contract(off)  // (alpha * tp) * beta + acc, as the oracle rounds
    const uint2 *e = arcs + (size_t)off * 64 + lane;
#pragma unroll
    for (int f = 0; f < PAIR; ++f) acc[f] = 0.f;
    // (16 records in flight instead of 8: 1738 -> 1812 us per launch, r5)
    for (int k = 0; k < len; k += 8) {
        uint2 rr[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) rr[i] = e[(k + i) * 64];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const DenV<PAIR> a = lds_v<PAIR>(sva, rr[i].x & 0xFFFF), b = lds_v<PAIR>(svb, rr[i].x >> 16);
            const float tp = __uint_as_float(rr[i].y);
#pragma unroll
            for (int f = 0; f < PAIR; ++f) acc[f] += a.x[f] * tp * b.x[f];
        }
    }
}
template <typename XT, int MODE, int PAIR>
__global__ __launch_bounds__(DEN_THREADS) void k_den_post(const DenDev g, const DenRun r, int nfb) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int S = g.S, P = g.P, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int seq = blockIdx.x / nfb, fb = blockIdx.x % nfb;
    const int nslq = g.q.nsl;
    const int rsf = g.f.nsl * 64, rsb = g.b.nsl * 64;  // slice-ordered rows (k_den_fb)
    float *red = reinterpret_cast<float *>(smem);      // [32]
    float *va = reinterpret_cast<float *>(smem) + 64;  // [rsf][PAIR] alpha'[t+f], f-table slice order
    float *vb = va + PAIR * rsf;                       // [rsb][PAIR] beta[t+f+1], b-table slice order
    float *gam = vb + PAIR * rsb;                      // [PAIR][P] den, then the gradient
    int *metaq = reinterpret_cast<int *>(gam + PAIR * P);
    const int *permq = metaq, *lenq = metaq + nslq * 64, *offq = metaq + nslq * 65;
    for (int i = tid; i < nslq * 64; i += DEN_THREADS) metaq[i] = g.q.perm[i];
    for (int i = tid; i < nslq; i += DEN_THREADS) {
        metaq[nslq * 64 + i] = g.q.len[i];
        metaq[nslq * 65 + i] = g.q.off[i];
    }

    const int T = r.frames[seq];
    const int t0 = fb * POST_FRAMES, t1 = min(T, t0 + POST_FRAMES);
    if (t0 >= t1) return;
    const long long row0 = r.row0[seq];
    const XT *nnet = reinterpret_cast<const XT *>(r.nnet);
    const float *astore = r.alpha_store + (size_t)seq * (r.max_frames + 1) * rsf;
    const float *bstore = r.beta_store + (size_t)seq * (r.max_frames + 1) * rsb;
    const float *asum = r.asum_store + (size_t)seq * (r.max_frames + 1);
    const float *bsum = r.bsum_store + (size_t)seq * (r.max_frames + 1);
    const float leaky = r.leaky;

    int ok = 1;
    float w = 1.0f;
    const LogFstDev *nf = nullptr;
    int NG = 0;
    if (MODE == DEN_PRODUCT) {
        nf = &r.nums[seq];
        NG = nf->G;
        w = r.opts.supervision_weight;
        const float num_lp = *nf->total;
        const float den_lp = r.den_out[seq * 2 + 1];
        double objf = (double)w * ((double)num_lp - (double)den_lp);
        ok = !(isnan(objf) || isinf(objf));
        if (fb == 0 && tid == 0) {
            float *st8 = r.stats + (size_t)seq * 8;
            st8[0] = num_lp;
            st8[1] = den_lp;
            st8[2] = ok ? (float)objf : (float)(-10.0 * w * T);  // backward.go:356-363
            st8[4] = w * (float)T;
            st8[5] = (float)T;
            st8[7] = ok ? 1.0f : 0.0f;
        }
    }
    const float l2s = r.opts.supervision_weight * r.opts.l2_regularize;
    const float oscale = 2.0f * r.opts.out_of_range_regularize;
    const bool do_oor = MODE == DEN_PRODUCT && r.opts.out_of_range_regularize > 0.0f;
    const bool do_l2 = MODE == DEN_PRODUCT && r.opts.l2_regularize > 0.0f;
    float oor = 0.f, sq = 0.f;
    // this thread's positions c = tid + m * DEN_THREADS of the alpha' rows: the initial
    // probability, once for the block's frames (rs <= DEN_MAXS * DEN_THREADS); the rows
    // are copied to LDS position for position (the records name slice positions)
    float ipf[DEN_MAXS];
#pragma unroll
    for (int m = 0; m < DEN_MAXS; ++m) {
        const int c = tid + m * DEN_THREADS;
        ipf[m] = c < rsf ? g.f.initp[c] : 0.f;
    }
    for (int t = t0; t < t1; t += PAIR) {
        const int nf2 = min(PAIR, t1 - t);
        // stage alpha'[t+f], beta[t+f+1] (a missing second frame computes zeros); the
        // stored rows lack the leaky terms (den_fwd_body, den_bwd_body), added here as the
        // recursions add them
        // both frames' rows are loaded before the first LDS store, which then writes each
        // position's PAIR values as one vector (a PAIR-strided scalar store is 2-way conflicted)
        float va_[PAIR][DEN_MAXS], vb_[PAIR][DEN_MAXS], as1[PAIR], tb[PAIR];
#pragma unroll
        for (int f = 0; f < PAIR; ++f) {
            const bool live = f < nf2;
            // (a missing frame reads frame t's rows, which exist, and stores zeros)
            const int tf = live ? t + f : t;
            const float *ar = astore + (size_t)tf * rsf, *br = bstore + (size_t)(tf + 1) * rsb;
            as1[f] = live ? asum[t + f] : 0.f;
            tb[f] = live ? leaky * bsum[t + f + 1] : 0.f;
#pragma unroll
            for (int m = 0; m < DEN_MAXS; ++m) {  // unconditional loads (index clamped)
                const int c = tid + m * DEN_THREADS;
                va_[f][m] = __builtin_nontemporal_load(ar + min(c, rsf - 1));
                vb_[f][m] = __builtin_nontemporal_load(br + min(c, rsb - 1));
            }
        }
#pragma unroll
        for (int m = 0; m < DEN_MAXS; ++m) {
            const int c = tid + m * DEN_THREADS;
            DenV<PAIR> a, b;
#pragma unroll
            for (int f = 0; f < PAIR; ++f) {
                const bool live = f < nf2;
                a.x[f] = live ? va_[f][m] + as1[f] * leaky * ipf[m] : 0.f;
                b.x[f] = live ? vb_[f][m] + tb[f] : 0.f;
            }
            if constexpr (PAIR == 2) {
                if (c < rsf) reinterpret_cast<float2 *>(va)[c] = make_float2(a.x[0], a.x[1]);
                if (c < rsb) reinterpret_cast<float2 *>(vb)[c] = make_float2(b.x[0], b.x[1]);
            } else {
                if (c < rsf) va[c] = a.x[0];
                if (c < rsb) vb[c] = b.x[0];
            }
        }
        __syncthreads();
        float gpart[PAIR];
#pragma unroll
        for (int f = 0; f < PAIR; ++f) gpart[f] = 0.f;
        for (int k = wave; k < g.q.spg[0]; k += DEN_WAVES) {
            const int j = g.q.slot[0][k];
            if (j < 0) continue;
            const int pdf = permq[j * 64 + lane];
            float acc[PAIR];
            post_slice<PAIR>(g.q.arc_p[PAIR - 1], lenq[j], offq[j], lane, reinterpret_cast<const unsigned char *>(va),
                             reinterpret_cast<const unsigned char *>(vb), acc);
            if (pdf < 0) continue;
#pragma unroll
            for (int f = 0; f < PAIR; ++f) {
                if (f >= nf2) break;
                const float x = (float)nnet[(row0 + (long long)(t + f) * r.stride) * r.ld + pdf];
                const float gv = acc[f] * expf(fmaxf(-30.0f, fminf(30.0f, x)));  // kernel_apply_exp
                gam[f * P + pdf] = gv;
                gpart[f] += gv;
            }
        }
#pragma unroll
        for (int f = 0; f < PAIR; ++f) {
            if (f >= nf2) break;
            const int tf = t + f;
            // the frame's occupation sums to one (alpha and beta carry arbitrary
            // per-frame factors, see den_bwd_body): normalise in a fixed order
            const float gsum = block_sum<DEN_WAVES>(gpart[f], red);
            const float ginv = gsum > 0.0f ? 1.0f / gsum : 0.0f;
            float *gm = gam + f * P;
            if (MODE == DEN_ABI) {
                for (int pdf = tid; pdf < P; pdf += DEN_THREADS)
                    r.post_dense[(size_t)tf * P + pdf] = gm[pdf] * ginv;
            } else {
                // d = (oor) + w*num - w*den - l2: -w*den first, the numerator's sparse
                // posteriors (its pdf set) added in place, then the dense pass
                for (int pdf = tid; pdf < P; pdf += DEN_THREADS) gm[pdf] = -(w * (gm[pdf] * ginv));
                __syncthreads();
                const float *nps = nf->post_sparse + (size_t)tf * NG;
                for (int q = tid; q < NG; q += DEN_THREADS) {
                    const int p = nf->grp_pdf[q];
                    if (p > 0 && p <= P) gm[p - 1] = w * nps[q] + gm[p - 1];
                }
                __syncthreads();
                const XT *xrow = nnet + (row0 + (long long)tf * r.stride) * r.ld;
                h16 *orow = r.out_grad + (row0 + (long long)tf * r.stride) * r.ldg;
                const bool even = (tf & 1) == 0;
                for (int pdf = tid; pdf < P; pdf += DEN_THREADS) {
                    const float x = (float)xrow[pdf];
                    float d = 0.0f;
                    if (do_oor && even) {  // chain_backward.cu:27-67
                        if (x < -30.0f) {
                            d += (-30.0f - x) * oscale;
                            oor += 1.0f;
                        } else if (x > 30.0f) {
                            d += (30.0f - x) * oscale;
                            oor += 1.0f;
                        }
                    }
                    d += gm[pdf];
                    if (do_l2) {
                        d -= l2s * x;
                        sq += x * x;
                    }
                    orow[pdf] = ok ? (h16)(-d) : (h16)0.0f;  // loss gradient = -deriv
                }
            }
            __syncthreads();
        }
    }
    if (MODE == DEN_PRODUCT) {
        float o = block_sum<DEN_WAVES>(oor, red);
        __syncthreads();
        float q = block_sum<DEN_WAVES>(sq, red);
        if (tid == 0) {
            float *st8 = r.stats + (size_t)seq * 8;
            if (o > 0.0f) atomicAdd(&st8[6], o);
            if (do_l2 && ok) atomicAdd(&st8[3], -0.5f * l2s * q);
        }
    }
}

// initp[c] = init[perm[c]] (0 for padding rows): the initial probabilities in a
// SELL table's slice order, so the exchange consumers load them with the payload
__global__ void k_perm_gather(const int *perm, const float *init, float *out, int n) {
    int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c < n) out[c] = perm[c] >= 0 ? init[perm[c]] : 0.0f;
}

// ===========================================================================
// Host: SELL-64 tables and graph objects
// ===========================================================================
namespace {

struct Sell {
    std::vector<int> perm, len, off;
    std::vector<uint2> arcs;
};

// rows = key states; each row lists (other | pdf<<16, tp) in arc order
// rows = values of key[] in [0, nrows); each row lists {f1 | f2<<16, tp} in arc order
// slice position of every row of a SELL table keyed by `key` (rows sorted by degree,
// stable: the order build_sell uses)
std::vector<int> sell_positions(int nrows, int A, const int32_t *key) {
    std::vector<int> deg(nrows, 0), order(nrows), pos(nrows);
    for (int a = 0; a < A; ++a) deg[key[a]]++;
    for (int i = 0; i < nrows; ++i) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return deg[a] > deg[b]; });
    for (int i = 0; i < nrows; ++i) pos[order[i]] = i;
    return pos;
}

Sell build_sell(int nrows, int A, const int32_t *key, const int32_t *f1, const int32_t *f2,
                const float *tp, int n1, int n2) {
    Sell s;
    std::vector<int> deg(nrows, 0);
    for (int a = 0; a < A; ++a) deg[key[a]]++;
    std::vector<int> order(nrows);
    for (int i = 0; i < nrows; ++i) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return deg[a] > deg[b]; });
    const int nsl = (nrows + 63) / 64;
    s.perm.assign((size_t)nsl * 64, -1);
    s.len.resize(nsl);
    s.off.resize(nsl);
    std::vector<int> rowpos(nrows);
    int tot = 0;
    for (int j = 0; j < nsl; ++j) {
        int mx = 0;
        for (int l = 0; l < 64; ++l) {
            int r = j * 64 + l;
            if (r < nrows) {
                s.perm[r] = order[r];
                rowpos[order[r]] = r;
                mx = std::max(mx, deg[order[r]]);
            }
        }
        mx = (mx + 7) & ~7;  // whole 8-record steps; the padding records have tp = 0
        s.len[j] = mx;
        s.off[j] = tot;
        tot += mx;
    }
    s.arcs.assign((size_t)tot * 64, make_uint2(0u, 0u));  // tp = 0 padding
    // arcs of every row, in arc order
    std::vector<std::vector<int>> rows(nrows);
    for (int a = 0; a < A; ++a) rows[key[a]].push_back(a);
    // Place each row's arcs into the slice's steps so that, per step and per
    // 32-lane half-wave, the two LDS gathers (f1 and f2 indices) fall in distinct
    // banks ((index) mod 32 for ds_read_b32) as far as possible; padding records
    // (tp = 0) take indices of free banks. Summation order per row changes, but
    // stays fixed.
    for (int j = 0; j < nsl; ++j) {
        for (int half = 0; half < 2; ++half) {
            std::vector<std::vector<int>> rem(32);
            for (int l = 0; l < 32; ++l) {
                int r = j * 64 + half * 32 + l;
                if (r < nrows) rem[l] = rows[s.perm[r]];
            }
            for (int k = 0; k < s.len[j]; ++k) {
                bool used1[32] = {false}, used2[32] = {false};
                // rows with the most remaining arcs choose first
                int order[32];
                for (int l = 0; l < 32; ++l) order[l] = l;
                std::stable_sort(order, order + 32,
                                 [&](int x, int y) { return rem[x].size() > rem[y].size(); });
                for (int oi = 0; oi < 32; ++oi) {
                    const int l = order[oi];
                    uint2 rec = make_uint2(0u, 0u);
                    if (!rem[l].empty()) {
                        size_t best = 0;
                        int bestc = 3;
                        for (size_t q = 0; q < rem[l].size() && bestc > 0; ++q) {
                                const int a = rem[l][q];
                                int c = (used1[f1[a] & 31] ? 1 : 0) + (used2[f2[a] & 31] ? 1 : 0);
                                if (c < bestc) {
                                    bestc = c;
                                    best = q;
                                }
                            }
                        const int a = rem[l][best];
                        rem[l].erase(rem[l].begin() + best);
                        used1[f1[a] & 31] = used2[f2[a] & 31] = true;
                        uint32_t tpu;
                        memcpy(&tpu, &tp[a], 4);
                        rec = make_uint2((uint32_t)f1[a] | ((uint32_t)f2[a] << 16), tpu);
                    } else {  // padding: valid indices on free banks
                        const int m1 = std::min(32, n1) - 1, m2 = std::min(32, n2) - 1;
                        int b1 = 0, b2 = 0;
                        while (b1 < m1 && used1[b1]) ++b1;
                        while (b2 < m2 && used2[b2]) ++b2;
                        used1[b1] = used2[b2] = true;
                        rec = make_uint2((uint32_t)b1 | ((uint32_t)b2 << 16), 0u);
                    }
                    s.arcs[((size_t)s.off[j] + k) * 64 + half * 32 + l] = rec;
                }
            }
        }
    }
    return s;
}

template <typename T>
T *dev_upload(const std::vector<T> &v, std::vector<void *> &owned) {
    void *p = nullptr;
    size_t bytes = std::max<size_t>(v.size() * sizeof(T), 16);
    if (hipMalloc(&p, bytes) != hipSuccess) return nullptr;
    owned.push_back(p);
    if (!v.empty()) hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice);
    return (T *)p;
}

// Slice ownership of SellDev::slot for G blocks of DEN_WAVES waves: longest
// slice first onto the least loaded (block, wave) pair (a slice costs its rows plus a
// fixed 4 for its per-slice work); bin b is block b % G, wave b / G, so the largest
// slices also spread over the blocks.
void den_balance(const std::vector<int> &len, int G, std::vector<int> &slot, int &spg) {
    const int nsl = (int)len.size(), bins = G * DEN_WAVES;
    std::vector<int> order(nsl);
    for (int j = 0; j < nsl; ++j) order[j] = j;
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return len[a] > len[b]; });
    std::vector<long long> load(bins, 0);
    std::vector<std::vector<int>> lists(bins);
    for (int j : order) {
        int b = 0;
        for (int i = 1; i < bins; ++i)
            if (load[i] < load[b]) b = i;
        lists[b].push_back(j);
        load[b] += len[j] + 4;
    }
    size_t maxc = 1;
    for (auto &l : lists) maxc = std::max(maxc, l.size());
    spg = (int)maxc * DEN_WAVES;
    slot.assign((size_t)G * spg, -1);
    for (int b = 0; b < bins; ++b) {
        const int gi = b % G, w = b / G;
        for (size_t i = 0; i < lists[b].size(); ++i) slot[(size_t)gi * spg + w + DEN_WAVES * (int)i] = lists[b][i];
    }
}

struct DenTables {
    DenDev dev{};
    std::vector<void *> owned;
    ~DenTables() {
        for (void *p : owned) hipFree(p);
    }
};

DenTables *make_den_tables(int S, int P, int A, const int32_t *src, const int32_t *dst,
                           const int32_t *pdf0, const float *tp, const char **why) {
    if (S <= 0 || P <= 0 || A <= 0) {
        *why = "empty denominator graph";
        return nullptr;
    }
    if (S > 65535 || P > 65535) {
        *why = "den graph needs num_states, num_pdfs <= 65535 (16-bit arc fields)";
        return nullptr;
    }
    if (P > DEN_MAXPT * DEN_THREADS) {
        *why = "num_pdfs > 4096 not supported";
        return nullptr;
    }
    // S < 8192: the pair records hold 8 * (slice position) as a 16-bit LDS byte offset
    const int rsS = (S + 63) / 64 * 64;
    if (den_post_lds_bytes(rsS, P, (P + 63) / 64) > DEN_LDS_TOTAL ||
        den_rec_fixed_bytes(P, (S + 63) / 64, (S + 63) / 64, 1) > DEN_LDS_TOTAL || S >= DEN_MAXS * DEN_THREADS) {
        *why = "den graph too large for the LDS-resident kernels (S < 8192, ~12*S + 14*P B)";
        return nullptr;
    }
    for (int a = 0; a < A; ++a)
        if (src[a] < 0 || src[a] >= S || dst[a] < 0 || dst[a] >= S || pdf0[a] < 0 ||
            pdf0[a] >= P || !(tp[a] >= 0.0f)) {
            *why = "den transition out of range (state, pdf or negative probability)";
            return nullptr;
        }
    // The recursions and the posteriors keep their state rows in LDS in the f (alpha') and
    // b (beta) tables' slice orders, the layout the stores use: the records name states
    // by slice position, so the per-frame row copies into LDS are linear (no permutation,
    // no bank conflicts) and the padding positions hold zeros (or, in beta rows, values
    // only tp = 0 padding records read).
    const std::vector<int> posf = sell_positions(S, A, dst), posb = sell_positions(S, A, src);
    std::vector<int32_t> src_f(A), dst_b(A);
    for (int a = 0; a < A; ++a) {
        src_f[a] = posf[src[a]];
        dst_b[a] = posb[dst[a]];
    }
    Sell sf = build_sell(S, A, dst, src_f.data(), pdf0, tp, rsS, P);
    Sell sb = build_sell(S, A, src, dst_b.data(), pdf0, tp, rsS, P);
    Sell sq = build_sell(P, A, pdf0, src_f.data(), dst_b.data(), tp, rsS, rsS);
    auto *t = new DenTables();
    DenDev &d = t->dev;
    d.S = S;
    d.P = P;
    bool ok = true;
    auto put = [&](SellDev &o, const Sell &h, int ngs) {
        o.nsl = (int)h.len.size();
        o.perm = dev_upload(h.perm, t->owned);
        o.len = dev_upload(h.len, t->owned);
        o.off = dev_upload(h.off, t->owned);
        ok = ok && o.perm && o.len && o.off;
        for (int lg = 0; lg < 4; ++lg) {
            o.slot[lg] = nullptr;
            o.spg[lg] = 0;
            if (lg >= ngs) continue;
            std::vector<int> slot;
            den_balance(h.len, 1 << lg, slot, o.spg[lg]);
            o.slot[lg] = dev_upload(slot, t->owned);
            ok = ok && o.slot[lg];
        }
    };
    put(d.f, sf, 4);
    put(d.b, sb, 4);
    put(d.q, sq, 1);
    d.pair_ok = 1;
    for (int lg = 0; lg < 4 && ok; ++lg) {
        const int spg = std::max(d.f.spg[lg], d.b.spg[lg]);
        if (den_rec_fixed_bytes(P, d.f.nsl, spg, 1) > DEN_LDS_TOTAL) {
            delete t;
            *why = "den graph too large for the LDS-resident kernels (slice lists)";
            return nullptr;
        }
        if (den_rec_fixed_bytes(P, d.f.nsl, spg, 2) > DEN_LDS_TOTAL) d.pair_ok = 0;
    }
    // records with LDS byte offsets for the interleaved rows (den_fwd_body / den_bwd_body,
    // k_den_post)
    auto scaled = [&](const Sell &h, uint32_t ns) {
        std::vector<uint2> a(h.arcs);
        for (auto &r : a) {
            const uint32_t f1 = r.x & 0xFFFF, f2 = r.x >> 16;
            r.x = (4 * ns * f1) | ((4 * ns * f2) << 16);
        }
        return a;
    };
    for (int ns = 1; ns <= 2; ++ns) {
        d.f.arc_p[ns - 1] = dev_upload(scaled(sf, ns), t->owned);
        d.b.arc_p[ns - 1] = dev_upload(scaled(sb, ns), t->owned);
        d.q.arc_p[ns - 1] = dev_upload(scaled(sq, ns), t->owned);
        ok = ok && d.f.arc_p[ns - 1] && d.b.arc_p[ns - 1] && d.q.arc_p[ns - 1];
    }
    std::vector<float> zf(sf.perm.size(), 0.0f), zb(sb.perm.size(), 0.0f);
    d.f.initp = dev_upload(zf, t->owned);  // filled by den_tables_set_init
    d.b.initp = dev_upload(zb, t->owned);
    ok = ok && d.f.initp && d.b.initp;
    if (!ok) {
        delete t;
        *why = "hipMalloc failed for den tables";
        return nullptr;
    }
    return t;
}

// (re)derive the slice-ordered initial probabilities from a device init vector
void den_tables_set_init(const DenDev &d, const float *d_init, hipStream_t st) {
    const int nf = d.f.nsl * 64, nb = d.b.nsl * 64;
    hipLaunchKernelGGL(k_perm_gather, dim3((nf + 255) / 256), dim3(256), 0, st, d.f.perm, d_init,
                       (float *)d.f.initp, nf);
    hipLaunchKernelGGL(k_perm_gather, dim3((nb + 255) / 256), dim3(256), 0, st, d.b.perm, d_init,
                       (float *)d.b.initp, nb);
}

// denominator.go:131-171
void compute_initial_probs(int S, int A, const int32_t *src, const int32_t *dst, const float *tp,
                   int start, float *out) {
    std::vector<double> cur(S, 0.0), next(S, 0.0), avg(S, 0.0);
    cur[start] = 1.0;
    for (int it = 0; it < 100; ++it) {
        for (int s = 0; s < S; ++s) avg[s] += cur[s] / 100.0;
        std::fill(next.begin(), next.end(), 0.0);
        for (int a = 0; a < A; ++a) next[dst[a]] += cur[src[a]] * (double)tp[a];
        double tot = 0.0;
        for (int s = 0; s < S; ++s) tot += next[s];
        if (tot > 0) {
            double inv = 1.0 / tot;
            for (int s = 0; s < S; ++s) next[s] *= inv;
        }
        cur.swap(next);
    }
    for (int s = 0; s < S; ++s) out[s] = (float)avg[s];
}

// G blocks per sequence: as many as the CUs allow (every block must be resident:
// the exchange polls are bounded, so a shortfall ends in the timeout word, not a hang)
int den_pick_G(int nseq) {
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 1;
    }
    for (int G = 4; G > 1; G /= 2)
        if (nseq * G <= cus) return G;
    return 1;
}

// exchange buffers + counters for up to nseq sequences at G blocks each
struct DenXBuf {
    float *buf = nullptr;
    unsigned *cnt = nullptr;
    size_t buf_cap = 0, cnt_cap = 0;
    ~DenXBuf() {
        if (buf) hipFree(buf);
        if (cnt) hipFree(cnt);
        if (h_word) hipHostFree(h_word);
    }
    // nseqs sequences in units of ns, G blocks per unit, over table `tb` (the f table for
    // the forward recursion, b for the backward)
    bool make(const DenDev &g, const SellDev &tb, int nseqs, int ns, int G, DenX &X) {
        X.G = G;
        X.ns = ns;
        X.nseqs = nseqs;
        X.nseq = (nseqs + ns - 1) / ns;
        X.lgG = G == 8 ? 3 : G == 4 ? 2 : G == 2 ? 1 : 0;
        X.spg = tb.spg[X.lgG];
        X.blk = 64;  // partial sums only: the slices go through the alpha / beta stores
        X.lds_f = (unsigned)den_rec_fixed_bytes(g.P, g.f.nsl, g.f.spg[X.lgG], ns);
        X.lds_b = (unsigned)den_rec_fixed_bytes(g.P, g.b.nsl, g.b.spg[X.lgG], ns);
        size_t nb = (size_t)X.nseq * 2 * G * X.blk * 4;
        size_t nc = (((size_t)X.nseq * 2 + 2) * 4 + 15) / 16 * 16;  // sticky, timeout, counters, census
        if (nb > buf_cap) {
            if (buf) hipFree(buf);
            buf = nullptr;
            buf_cap = 0;
            if (hipMalloc(&buf, nb) != hipSuccess) return false;
            buf_cap = nb;
        }
        if (nc > cnt_cap) {
            unsigned *grown = nullptr;
            if (hipMalloc(&grown, nc) != hipSuccess) return false;
            hipMemsetAsync(grown, 0, nc, kf_stream());
            if (cnt) {  // the sticky count survives the reallocation
                hipMemcpyAsync(grown, cnt, 4, hipMemcpyDeviceToDevice, kf_stream());
                hipStreamSynchronize(kf_stream());
                hipFree(cnt);
            }
            cnt = grown;
            cnt_cap = nc;
        }
        X.buf = buf;
        X.sticky = cnt;
        X.tmo = cnt + 1;
        X.cnt = cnt + 2;
        X.xm = cnt + 2 + X.nseq;
        X.spin_limit = spin_limit;
        X.force_sys = force_sys;
        last_units = X.nseq;
        last_G = G;
        return true;
    }
    int last_units = 0, last_G = 0;
    // units of the last launch whose G workgroups all ran on one XCD (the census words
    // stay in memory after the launch); -1 on a read error
    int census_local(hipStream_t st) {
        if (!cnt || !last_units) return 0;
        std::vector<unsigned> w(last_units);
        hipMemcpyAsync(w.data(), cnt + 2 + last_units, (size_t)last_units * 4, hipMemcpyDeviceToHost, st);
        if (hipStreamSynchronize(st) != hipSuccess) return -1;
        int n = 0;
        for (unsigned v : w)
            for (int k = 0; k < 8; ++k)
                if (((v >> (4 * k)) & 15) == (unsigned)last_G) {
                    ++n;
                    break;
                }
        return n;
    }
    // counters and the per-launch timeout word; never the sticky word
    void zero(hipStream_t st) { hipMemsetAsync(cnt + 1, 0, cnt_cap - 4, st); }
    unsigned spin_limit = 1u << 21;
    int force_sys = 0;
    // blocks that timed out since the last call (stream-ordered read, then cleared)
    // (read through a pinned word: a stream-ordered copy into pageable memory left
    // hipErrorStreamCaptureUnsupported pending on the calling thread in the r6 bench)
    unsigned *h_word = nullptr;
    unsigned take_timeouts(hipStream_t st) {
        if (!cnt) return 0;
        if (!h_word && hipHostMalloc((void **)&h_word, 64, hipHostMallocDefault) != hipSuccess) {
            h_word = nullptr;
            kf_take_pending("DenXBuf::take_timeouts hipHostMalloc");
            return 0;
        }
        *h_word = 0;
        hipMemcpyAsync(h_word, cnt, 4, hipMemcpyDeviceToHost, st);
        kf_take_pending("DenXBuf::take_timeouts hipMemcpyAsync");
        hipStreamSynchronize(st);
        kf_take_pending("DenXBuf::take_timeouts hipStreamSynchronize");
        const unsigned v = *h_word;
        if (v) {
            hipMemsetAsync(cnt, 0, 4, st);
            hipStreamSynchronize(st);
        }
        return v;
    }
};

void launch_den_fwd(const DenDev &g, const DenRun &r, const DenX &X, DenXBuf &xb, bool fp32_in) {
    size_t lds = X.lds_f;
    hipStream_t st = kf_stream();
    xb.zero(st);
    dim3 grid(X.nseq * X.G);
    if (fp32_in)  // the den ABI: one sequence (X.ns == 1)
        hipLaunchKernelGGL((k_den_fwd<float, 1>), grid, dim3(DEN_THREADS), lds, st, g, r, X);
    else if (X.ns == 2)
        hipLaunchKernelGGL((k_den_fwd<h16, 2>), grid, dim3(DEN_THREADS), lds, st, g, r, X);
    else
        hipLaunchKernelGGL((k_den_fwd<h16, 1>), grid, dim3(DEN_THREADS), lds, st, g, r, X);
}
// both recursions in one launch (k_den_fb); XF / XB from two exchange buffers
void launch_den_fb(const DenDev &g, const DenRun &r, const DenX &XF, DenXBuf &xf, const DenX &XB,
                   DenXBuf &xbb, bool fp32_in) {
    hipStream_t st = kf_stream();
    xf.zero(st);
    xbb.zero(st);
    dim3 grid(2 * XF.nseq * XF.G);
    const size_t lds = std::max(XF.lds_f, XB.lds_b);
    if (fp32_in) hipLaunchKernelGGL((k_den_fb<float, 1>), grid, dim3(DEN_THREADS), lds, st, g, r, XF, XB);
    else if (XF.ns == 2) hipLaunchKernelGGL((k_den_fb<h16, 2>), grid, dim3(DEN_THREADS), lds, st, g, r, XF, XB);
    else hipLaunchKernelGGL((k_den_fb<h16, 1>), grid, dim3(DEN_THREADS), lds, st, g, r, XF, XB);
}
void launch_den_post(const DenDev &g, const DenRun &r, const DenX &X, bool fp32_in, int mode) {
    hipStream_t st = kf_stream();
    const int nfb = (r.max_frames + POST_FRAMES - 1) / POST_FRAMES;
    dim3 pgrid(X.nseqs * nfb);  // per sequence
    // frame pairs share the arc stream when both frames' alpha/beta fit in LDS
    const int rs = g.f.nsl * 64;  // = g.b.nsl * 64
    const bool pair = den_post_lds_bytes(rs, g.P, g.q.nsl, 2) <= DEN_LDS_TOTAL;
    size_t plds = den_post_lds_bytes(rs, g.P, g.q.nsl, pair ? 2 : 1);
#define KF_POST(XT_, MODE_, PAIR_) \
    hipLaunchKernelGGL((k_den_post<XT_, MODE_, PAIR_>), pgrid, dim3(DEN_THREADS), plds, st, g, r, nfb)
    if (mode == DEN_PRODUCT) {
        if (pair) KF_POST(h16, DEN_PRODUCT, 2);
        else KF_POST(h16, DEN_PRODUCT, 1);
    } else if (fp32_in) {
        if (pair) KF_POST(float, DEN_ABI, 2);
        else KF_POST(float, DEN_ABI, 1);
    } else {
        if (pair) KF_POST(h16, DEN_ABI, 2);
        else KF_POST(h16, DEN_ABI, 1);
    }
#undef KF_POST
}

// ---- numerator FST host preparation (reverse CSR + pdf groups) -------------
struct NumHost {  // one FST, local indices
    int S, A, nfinal, start;
    std::vector<int> row_ptr, in_ptr, in_arc, arc_src, arc_dst, arc_pdf, grp_ptr, grp_pdf, grp_arc,
        fin_state, in_src, in_g, arc_g, gsrc, gdst;
    std::vector<float> arc_w, fin_w, in_w, gw;
};

bool prepare_num(NumHost &h, const char **why) {
    const int S = h.S, A = h.A;
    if (S <= 0) {
        *why = "FST has no states";
        return false;
    }
    if ((int)h.row_ptr.size() != S + 1 || h.row_ptr[0] != 0 || h.row_ptr[S] != A) {
        *why = "row_ptr does not describe num_arcs arcs";
        return false;
    }
    h.arc_src.assign(A, 0);
    for (int s = 0; s < S; ++s) {
        if (h.row_ptr[s + 1] < h.row_ptr[s]) {
            *why = "row_ptr not monotone";
            return false;
        }
        for (int a = h.row_ptr[s]; a < h.row_ptr[s + 1]; ++a) h.arc_src[a] = s;
    }
    for (int a = 0; a < A; ++a)
        if (h.arc_dst[a] < 0 || h.arc_dst[a] >= S) {
            *why = "arc destination out of range";
            return false;
        }
    for (int i = 0; i < h.nfinal; ++i)
        if (h.fin_state[i] < 0 || h.fin_state[i] >= S) {
            *why = "final state out of range";
            return false;
        }
    if (h.start < 0 || h.start >= S) {
        *why = "start state out of range";
        return false;
    }
    // reverse CSR, incoming arcs in arc-index order (chain_det.cu:243-290)
    h.in_ptr.assign(S + 1, 0);
    for (int a = 0; a < A; ++a) h.in_ptr[h.arc_dst[a] + 1]++;
    for (int s = 0; s < S; ++s) h.in_ptr[s + 1] += h.in_ptr[s];
    h.in_arc.assign(A, 0);
    std::vector<int> pos(h.in_ptr.begin(), h.in_ptr.end() - 1);
    for (int a = 0; a < A; ++a) h.in_arc[pos[h.arc_dst[a]]++] = a;
    // pdf groups, arcs in arc-index order inside each group
    std::vector<int> idx;
    for (int a = 0; a < A; ++a)
        if (h.arc_pdf[a] > 0) idx.push_back(a);
    std::stable_sort(idx.begin(), idx.end(),
                     [&](int x, int y) { return h.arc_pdf[x] < h.arc_pdf[y]; });
    h.grp_ptr.assign(1, 0);
    h.grp_pdf.clear();
    h.grp_arc = idx;
    for (size_t i = 0; i < idx.size(); ++i) {
        if (i == 0 || h.arc_pdf[idx[i]] != h.arc_pdf[idx[i - 1]]) {
            if (i) h.grp_ptr.push_back((int)i);
            h.grp_pdf.push_back(h.arc_pdf[idx[i]]);
        }
    }
    if (!idx.empty()) h.grp_ptr.push_back((int)idx.size());
    // pre-gathered arc fields for k_num_fb
    h.arc_g.assign(A, -1);
    for (size_t q = 0; q + 1 < h.grp_ptr.size(); ++q)
        for (int k = h.grp_ptr[q]; k < h.grp_ptr[q + 1]; ++k) h.arc_g[h.grp_arc[k]] = (int)q;
    h.in_src.resize(A);
    h.in_g.resize(A);
    h.in_w.resize(A);
    for (int k = 0; k < A; ++k) {
        int a = h.in_arc[k];
        h.in_src[k] = h.arc_src[a];
        h.in_g[k] = h.arc_g[a];
        h.in_w[k] = h.arc_w[a];
    }
    h.gsrc.resize(idx.size());
    h.gdst.resize(idx.size());
    h.gw.resize(idx.size());
    for (size_t k = 0; k < idx.size(); ++k) {
        h.gsrc[k] = h.arc_src[idx[k]];
        h.gdst[k] = h.arc_dst[idx[k]];
        h.gw[k] = h.arc_w[idx[k]];
    }
    return true;
}

// Packs many NumHost into one device blob; fills LogFstDev pointer fields.
struct NumDevice {
    std::vector<LogFstDev> desc;  // per FST, pointers set, run fields unset
    std::vector<int> G, Ag;
    std::vector<void *> owned;
    ~NumDevice() {
        for (void *p : owned) hipFree(p);
    }
};

template <typename T>
void append(std::vector<int32_t> &blob, const std::vector<T> &v, std::vector<size_t> &offs) {
    offs.push_back(blob.size());
    size_t n = blob.size();
    blob.resize(n + v.size());
    if (!v.empty()) memcpy(blob.data() + n, v.data(), v.size() * 4);
}

// the numerator tables of a minibatch as one int32 blob; offs[i] = the 19 table offsets of
// FST i inside it
static void pack_nums(std::vector<NumHost> &hs, std::vector<int32_t> &blob,
                      std::vector<std::vector<size_t>> &offs) {
    blob.clear();
    offs.assign(hs.size(), {});
    for (size_t i = 0; i < hs.size(); ++i) {
        NumHost &h = hs[i];
        auto &o = offs[i];
        append(blob, h.row_ptr, o);
        append(blob, h.in_ptr, o);
        append(blob, h.in_arc, o);
        append(blob, h.arc_src, o);
        append(blob, h.arc_dst, o);
        append(blob, h.arc_pdf, o);
        append(blob, h.arc_w, o);
        append(blob, h.grp_ptr, o);
        append(blob, h.grp_pdf, o);
        append(blob, h.grp_arc, o);
        append(blob, h.fin_state, o);
        append(blob, h.fin_w, o);
        append(blob, h.in_src, o);
        append(blob, h.in_g, o);
        append(blob, h.arc_g, o);
        append(blob, h.gsrc, o);
        append(blob, h.gdst, o);
        append(blob, h.in_w, o);
        append(blob, h.gw, o);
    }
}

// descriptors of the FSTs packed at device address d
static void num_descs(const std::vector<NumHost> &hs, const std::vector<std::vector<size_t>> &offs,
                      const int32_t *d, NumDevice *nd) {
    nd->desc.clear();
    nd->G.clear();
    nd->Ag.clear();
    for (size_t i = 0; i < hs.size(); ++i) {
        const auto &o = offs[i];
        LogFstDev f{};
        f.row_ptr = d + o[0];
        f.in_ptr = d + o[1];
        f.in_arc = d + o[2];
        f.arc_src = d + o[3];
        f.arc_dst = d + o[4];
        f.arc_pdf = d + o[5];
        f.arc_w = reinterpret_cast<const float *>(d + o[6]);
        f.grp_ptr = d + o[7];
        f.grp_pdf = d + o[8];
        f.grp_arc = d + o[9];
        f.fin_state = d + o[10];
        f.fin_w = reinterpret_cast<const float *>(d + o[11]);
        f.in_src = d + o[12];
        f.in_g = d + o[13];
        f.arc_g = d + o[14];
        f.gsrc = d + o[15];
        f.gdst = d + o[16];
        f.in_w = reinterpret_cast<const float *>(d + o[17]);
        f.gw = reinterpret_cast<const float *>(d + o[18]);
        f.S = hs[i].S;
        f.A = hs[i].A;
        f.G = (int)hs[i].grp_pdf.size();
        f.nfinal = hs[i].nfinal;
        f.start = hs[i].start;
        nd->desc.push_back(f);
        nd->G.push_back(f.G);
        nd->Ag.push_back((int)hs[i].grp_arc.size());
    }
}

NumDevice *upload_nums(std::vector<NumHost> &hs, const char **why) {
    std::vector<int32_t> blob;
    std::vector<std::vector<size_t>> offs;
    pack_nums(hs, blob, offs);
    auto *nd = new NumDevice();
    int32_t *d = dev_upload(blob, nd->owned);
    if (!d) {
        delete nd;
        *why = "hipMalloc failed for numerator FSTs";
        return nullptr;
    }
    num_descs(hs, offs, d, nd);
    return nd;
}

// ABI helper: device ChainFstGPU -> host NumHost
bool fetch_fst(const ChainFstGPU *fst, NumHost &h, const char **why) {
    if (!fst || fst->num_states <= 0 || fst->num_arcs < 0 || fst->num_final < 0) {
        *why = "invalid ChainFstGPU";
        return false;
    }
    h.S = fst->num_states;
    h.A = fst->num_arcs;
    h.nfinal = fst->num_final;
    h.start = fst->start_state;
    h.row_ptr.resize(h.S + 1);
    h.arc_dst.resize(h.A);
    h.arc_pdf.resize(h.A);
    h.arc_w.resize(h.A);
    h.fin_state.resize(h.nfinal);
    h.fin_w.resize(h.nfinal);
    hipStreamSynchronize(kf_stream());
    bool ok = hipMemcpy(h.row_ptr.data(), fst->row_ptr, (h.S + 1) * 4, hipMemcpyDeviceToHost) == hipSuccess;
    if (h.A) {
        ok = ok && hipMemcpy(h.arc_dst.data(), fst->col_idx, h.A * 4, hipMemcpyDeviceToHost) == hipSuccess;
        ok = ok && hipMemcpy(h.arc_pdf.data(), fst->labels, h.A * 4, hipMemcpyDeviceToHost) == hipSuccess;
        ok = ok && hipMemcpy(h.arc_w.data(), fst->weights, h.A * 4, hipMemcpyDeviceToHost) == hipSuccess;
    }
    if (h.nfinal) {
        ok = ok && hipMemcpy(h.fin_state.data(), fst->final_states, h.nfinal * 4, hipMemcpyDeviceToHost) == hipSuccess;
        ok = ok && hipMemcpy(h.fin_w.data(), fst->final_weights, h.nfinal * 4, hipMemcpyDeviceToHost) == hipSuccess;
    }
    if (!ok) {
        *why = "device->host copy of the FST failed";
        return false;
    }
    return prepare_num(h, why);
}

struct DevBuf {
    void *p = nullptr;
    ~DevBuf() {
        if (p) hipFree(p);
    }
    bool alloc(size_t n) {
        return hipMalloc(&p, std::max<size_t>(n, 16)) == hipSuccess;
    }
};

// Runs k_logfb over `fsts` (already filled) and returns the totals.
bool run_logfb(std::vector<LogFstDev> &fsts, const void *nnet16, long long ld, int P,
               std::vector<float> &totals, const char **why) {
    kf_take_pending(__func__);
    DevBuf d, tot;
    size_t n = fsts.size();
    if (!tot.alloc(n * sizeof(float)) || !d.alloc(n * sizeof(LogFstDev))) {
        *why = "hipMalloc failed";
        return false;
    }
    hipStream_t st = kf_stream();
    for (size_t i = 0; i < n; ++i)
        if (!(fsts[i].mode & LF_FB)) {
            hipMemcpyAsync((float *)tot.p + i, &totals[i], 4, hipMemcpyHostToDevice, st);
        }
    for (size_t i = 0; i < n; ++i) fsts[i].total = (float *)tot.p + i;
    hipMemcpyAsync(d.p, fsts.data(), n * sizeof(LogFstDev), hipMemcpyHostToDevice, st);
    hipLaunchKernelGGL(k_logfb, dim3(n), dim3(256), 0, st, (const LogFstDev *)d.p,
                       (const h16 *)nnet16, ld, P);
    totals.resize(n);
    hipMemcpyAsync(totals.data(), tot.p, n * 4, hipMemcpyDeviceToHost, st);
    hipError_t e = hipStreamSynchronize(st);
    if (e != hipSuccess || hipGetLastError() != hipSuccess) {
        *why = hipGetErrorString(e);
        return false;
    }
    return true;
}

}  // namespace

// ===========================================================================
// chain.h ABI
// ===========================================================================
extern "C" size_t chain_workspace_bytes(int T, int num_states) {
    return 2 * (size_t)(T + 1) * num_states * sizeof(float);
}

static int fb_common(const void *nnet, const ChainFstGPU *fst, int T, int P, float *alpha,
                     float *beta, float *total, int mode, const float *post_in_total,
                     float *post) {
    const char *why = nullptr;
    if (!nnet || !alpha || !beta || T < 0 || P <= 0) {
        chain_set_error("chain_forward_backward: invalid arguments");
        return -1;
    }
    NumHost h;
    if (!fetch_fst(fst, h, &why)) {
        chain_set_error("chain_forward_backward: %s", why);
        return -1;
    }
    std::vector<NumHost> hs{h};
    NumDevice *nd = upload_nums(hs, &why);
    if (!nd) {
        chain_set_error("chain_forward_backward: %s", why);
        return -1;
    }
    std::vector<LogFstDev> fs{nd->desc[0]};
    LogFstDev &f = fs[0];
    // the caller's own arrays are authoritative for arcs and finals
    f.arc_dst = fst->col_idx;
    f.arc_pdf = fst->labels;
    f.arc_w = fst->weights;
    f.fin_state = fst->final_states;
    f.fin_w = fst->final_weights;
    f.T = T;
    f.mode = mode;
    f.stride = 1;
    f.row0 = 0;
    f.alpha = alpha;
    f.beta = beta;
    f.post_dense = post;
    std::vector<float> tot{post_in_total ? *post_in_total : 0.0f};
    bool ok = run_logfb(fs, nnet, P, P, tot, &why);
    delete nd;
    if (!ok) {
        chain_set_error("chain_forward_backward: %s", why);
        return -1;
    }
    if (total) *total = tot[0];
    return 0;
}

extern "C" int chain_forward_backward(const void *nnet_output, const ChainFstGPU *fst, int T,
                                      int num_pdfs, float *alpha, float *beta,
                                      float *total_logprob) {
    return fb_common(nnet_output, fst, T, num_pdfs, alpha, beta, total_logprob, LF_FB, nullptr,
                     nullptr);
}
extern "C" int chain_forward_backward_det(const void *nnet_output, const ChainFstGPU *fst, int T,
                                          int num_pdfs, float *alpha, float *beta,
                                          float *total_logprob) {
    return chain_forward_backward(nnet_output, fst, T, num_pdfs, alpha, beta, total_logprob);
}
extern "C" int chain_compute_posteriors(const void *nnet_output, const ChainFstGPU *fst, int T,
                                        int num_pdfs, const float *alpha, const float *beta,
                                        float total_logprob, float *posteriors) {
    if (!posteriors) {
        chain_set_error("chain_compute_posteriors: posteriors is NULL");
        return -1;
    }
    return fb_common(nnet_output, fst, T, num_pdfs, const_cast<float *>(alpha),
                     const_cast<float *>(beta), nullptr, LF_POST, &total_logprob, posteriors);
}
extern "C" int chain_compute_posteriors_det(const void *nnet_output, const ChainFstGPU *fst,
                                            int T, int num_pdfs, const float *alpha,
                                            const float *beta, float total_logprob,
                                            float *posteriors) {
    return chain_compute_posteriors(nnet_output, fst, T, num_pdfs, alpha, beta, total_logprob,
                                    posteriors);
}

__global__ void k_chain_gradient(h16 *g, const float *num, const float *den, long long n, float w) {
    long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float v = (den[i] - num[i]) * w;  // chain.cu:330-352
    g[i] = (h16)fmaxf(-30.0f, fminf(30.0f, v));
}

extern "C" int chain_compute_loss(const void *nnet_output, const ChainFstGPU *num_fst,
                                  const ChainFstGPU *den_fst, int T, int num_pdfs,
                                  void *grad_output, ChainLossResult *result) {
    const char *why = nullptr;
    if (!nnet_output || !result || T < 0 || num_pdfs <= 0) {
        chain_set_error("chain_compute_loss: invalid arguments");
        return -1;
    }
    std::vector<NumHost> hs(2);
    if (!fetch_fst(num_fst, hs[0], &why) || !fetch_fst(den_fst, hs[1], &why)) {
        chain_set_error("chain_compute_loss: %s", why);
        return -1;
    }
    NumDevice *nd = upload_nums(hs, &why);
    if (!nd) {
        chain_set_error("chain_compute_loss: %s", why);
        return -1;
    }
    const size_t TP = (size_t)T * num_pdfs;
    DevBuf ws, post;
    size_t wsn = 2 * (size_t)(T + 1) * (hs[0].S + hs[1].S);
    if (!ws.alloc(wsn * 4) || !post.alloc(2 * TP * 4)) {
        delete nd;
        chain_set_error("chain_compute_loss: hipMalloc failed");
        return -1;
    }
    std::vector<LogFstDev> fs = nd->desc;
    float *w = (float *)ws.p;
    for (int i = 0; i < 2; ++i) {
        fs[i].T = T;
        fs[i].mode = LF_FB | (grad_output ? LF_POST : 0);
        fs[i].stride = 1;
        fs[i].row0 = 0;
        fs[i].alpha = w;
        w += (size_t)(T + 1) * hs[i].S;
        fs[i].beta = w;
        w += (size_t)(T + 1) * hs[i].S;
        fs[i].post_dense = grad_output ? (float *)post.p + i * TP : nullptr;
    }
    std::vector<float> tot(2, 0.0f);
    bool ok = run_logfb(fs, nnet_output, num_pdfs, num_pdfs, tot, &why);
    delete nd;
    if (!ok) {
        chain_set_error("chain_compute_loss: %s", why);
        return -1;
    }
    result->num_logprob = tot[0];
    result->den_logprob = tot[1];
    result->loss = -(tot[0] - tot[1]);
    if (grad_output && TP) {
        hipLaunchKernelGGL(k_chain_gradient, dim3(kf_blocks(TP, 256)), dim3(256), 0, kf_stream(),
                           (h16 *)grad_output, (const float *)post.p, (const float *)post.p + TP,
                           (long long)TP, 1.0f);
        if (hipStreamSynchronize(kf_stream()) != hipSuccess) {
            chain_set_error("chain_compute_loss: gradient kernel failed");
            return -1;
        }
    }
    return 0;
}

__global__ void k_f32_to_f16(const float *in, h16 *out, long long n) {
    long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = (h16)in[i];
}

static float num_fb_fp32(const int *row_ptr, const int *col_idx, const float *weights,
                         const int *pdf_ids, const int *final_states, const float *final_weights,
                         int S, int A, int F, const float *nnet, float *num_post, int T, int P,
                         void *stream) {
    if (!nnet || !num_post || T < 0 || P <= 0) {
        chain_set_error("chain_num_forward_backward: invalid arguments");
        return -1e30f;
    }
    hipStream_t saved = kf_stream();
    if (stream) kf_set_stream(stream);
    ChainFstGPU fst{(int32_t *)row_ptr, (int32_t *)col_idx, (int32_t *)pdf_ids, (float *)weights,
                    (int32_t *)final_states, (float *)final_weights, S, A, F, 0};
    const size_t TP = (size_t)T * P;
    DevBuf x16, ws;
    float result = -1e30f;
    if (x16.alloc(TP * 2) && ws.alloc(chain_workspace_bytes(T, S))) {
        hipLaunchKernelGGL(k_f32_to_f16, dim3(kf_blocks(TP, 256)), dim3(256), 0, kf_stream(),
                           nnet, (h16 *)x16.p, (long long)TP);
        float *a = (float *)ws.p, *b = a + (size_t)(T + 1) * S;
        float tot = 0.f;
        if (fb_common(x16.p, &fst, T, P, a, b, &tot, LF_FB | LF_POST, nullptr, num_post) == 0)
            result = tot;
    } else {
        chain_set_error("chain_num_forward_backward: hipMalloc failed");
    }
    if (stream) kf_set_stream((void *)saved);
    return result;
}

extern "C" float chain_num_forward_backward(const int *fst_row_ptr, const int *fst_col_idx,
                                            const float *fst_weights, const int *fst_pdf_ids,
                                            const int *fst_final_states,
                                            const float *fst_final_weights, int num_states,
                                            int num_arcs, int num_final, const float *nnet_output,
                                            float *num_post, int T, int num_pdfs, void *stream) {
    return num_fb_fp32(fst_row_ptr, fst_col_idx, fst_weights, fst_pdf_ids, fst_final_states,
                       fst_final_weights, num_states, num_arcs, num_final, nnet_output, num_post,
                       T, num_pdfs, stream);
}
extern "C" float chain_num_forward_backward_det(
    const int *fst_row_ptr, const int *fst_col_idx, const float *fst_weights,
    const int *fst_pdf_ids, const int *fst_final_states, const float *fst_final_weights,
    int num_states, int num_arcs, int num_final, const float *nnet_output, float *num_post, int T,
    int num_pdfs, void *stream) {
    return num_fb_fp32(fst_row_ptr, fst_col_idx, fst_weights, fst_pdf_ids, fst_final_states,
                       fst_final_weights, num_states, num_arcs, num_final, nnet_output, num_post,
                       T, num_pdfs, stream);
}

// ===========================================================================
// chain_backward_api.h ABI (element-wise objective pieces)
// ===========================================================================
__global__ void k_combine16(const float *num, const float *den, float w, h16 *g, long long n) {
    long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) g[i] = (h16)(w * (num[i] - den[i]));
}
__global__ void k_add_post(const float *num, const float *den, float *g, float w, long long n) {
    long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) g[i] += w * (num[i] - den[i]);
}
__global__ void k_penalize(const float *x, float *g, float limit, float scale, int T, int P,
                           int *count) {
    long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    int c = 0;
    if (i < (long long)T * P && ((i / P) % 2) == 0) {
        float v = x[i];
        if (v < -limit) {
            g[i] += (-limit - v) * scale;
            c = 1;
        } else if (v > limit) {
            g[i] += (limit - v) * scale;
            c = 1;
        }
    }
    float cf = wave_sum((float)c);
    if ((threadIdx.x & 63) == 0 && cf > 0.0f) atomicAdd(count, (int)cf);
}
__global__ void k_l2(const float *x, float *g, float s, long long n, double *acc) {
    long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    double q = 0.0;
    if (i < n) {
        float v = x[i];
        g[i] -= s * v;
        q = (double)v * v;
    }
    q = wave_sum_d(q);
    if ((threadIdx.x & 63) == 0) atomicAdd(acc, q);
}

extern "C" int chain_combine_gradient(const float *num_post, const float *den_post, float weight,
                                      int T, int num_pdfs, void *grad_output) {
    kf_take_pending(__func__);
    long long n = (long long)T * num_pdfs;
    if (n <= 0) return 0;
    hipLaunchKernelGGL(k_combine16, dim3(kf_blocks(n, 256)), dim3(256), 0, kf_stream(), num_post,
                       den_post, weight, (h16 *)grad_output, n);
    if (hipGetLastError() != hipSuccess) {
        chain_set_error("chain_combine_gradient: launch failed");
        return -1;
    }
    return 0;
}
extern "C" int chain_add_posterior_gradient(const float *num_post, const float *den_post,
                                            float *grad, float weight, int total_elements) {
    kf_take_pending(__func__);
    if (total_elements <= 0) return 0;
    hipLaunchKernelGGL(k_add_post, dim3(kf_blocks(total_elements, 256)), dim3(256), 0, kf_stream(),
                       num_post, den_post, grad, weight, (long long)total_elements);
    if (hipGetLastError() != hipSuccess) {
        chain_set_error("chain_add_posterior_gradient: launch failed");
        return -1;
    }
    return 0;
}
extern "C" int chain_penalize_out_of_range(const float *nnet_output, float *grad_output,
                                           float limit, float scale, int T, int num_pdfs) {
    long long n = (long long)T * num_pdfs;
    if (n <= 0) return 0;
    DevBuf cnt;
    if (!cnt.alloc(4)) return 0;
    hipStream_t st = kf_stream();
    hipMemsetAsync(cnt.p, 0, 4, st);
    hipLaunchKernelGGL(k_penalize, dim3(kf_blocks(n, 256)), dim3(256), 0, st, nnet_output,
                       grad_output, limit, scale, T, num_pdfs, (int *)cnt.p);
    int h = 0;
    hipMemcpyAsync(&h, cnt.p, 4, hipMemcpyDeviceToHost, st);
    hipStreamSynchronize(st);
    return h;
}
extern "C" float chain_l2_regularize(const float *nnet_output, float *grad_output, float l2_scale,
                                     int total_elements) {
    if (total_elements <= 0) return 0.0f;
    DevBuf acc;
    if (!acc.alloc(8)) return 0.0f;
    hipStream_t st = kf_stream();
    hipMemsetAsync(acc.p, 0, 8, st);
    hipLaunchKernelGGL(k_l2, dim3(kf_blocks(total_elements, 256)), dim3(256), 0, st, nnet_output,
                       grad_output, l2_scale, (long long)total_elements, (double *)acc.p);
    double h = 0.0;
    hipMemcpyAsync(&h, acc.p, 8, hipMemcpyDeviceToHost, st);
    hipStreamSynchronize(st);
    return (float)(-0.5 * l2_scale * h);
}
extern "C" int chain_grad_fp32_to_fp16(const float *grad_fp32, void *grad_fp16,
                                       int total_elements) {
    if (total_elements <= 0) return 0;
    hipLaunchKernelGGL(k_f32_to_f16, dim3(kf_blocks(total_elements, 256)), dim3(256), 0,
                       kf_stream(), grad_fp32, (h16 *)grad_fp16, (long long)total_elements);
    return 0;
}

// ===========================================================================
// chain_den.h ABI
// ===========================================================================
static std::mutex g_den_mu;
static std::map<const void *, DenTables *> g_den_tables;  // keyed by DenFstGPU::src_states

extern "C" int den_fst_upload(DenFstGPU *fst, const int32_t *src, const int32_t *dst,
                              const int32_t *pdf, const float *trans_probs, int num_trans,
                              int num_states, int num_pdfs) {
    const char *why = nullptr;
    if (!fst || !src || !dst || !pdf || !trans_probs) {
        den_set_error("den_fst_upload: NULL argument");
        return -1;
    }
    DenTables *t = make_den_tables(num_states, num_pdfs, num_trans, src, dst, pdf, trans_probs, &why);
    if (!t) {
        den_set_error("den_fst_upload: %s", why);
        return -1;
    }
    std::vector<int32_t> vs(src, src + num_trans), vd(dst, dst + num_trans), vp(pdf, pdf + num_trans);
    std::vector<float> vt(trans_probs, trans_probs + num_trans);
    std::vector<void *> owned;
    fst->src_states = dev_upload(vs, owned);
    fst->dst_states = dev_upload(vd, owned);
    fst->pdf_ids = dev_upload(vp, owned);
    fst->transition_probs = dev_upload(vt, owned);
    if (!fst->src_states || !fst->dst_states || !fst->pdf_ids || !fst->transition_probs) {
        for (void *p : owned) hipFree(p);
        delete t;
        den_set_error("den_fst_upload: hipMalloc failed");
        return -1;
    }
    fst->num_transitions = num_trans;
    fst->num_states = num_states;
    fst->num_pdfs = num_pdfs;
    std::lock_guard<std::mutex> lk(g_den_mu);
    g_den_tables[fst->src_states] = t;
    return 0;
}

extern "C" void den_fst_free(DenFstGPU *fst) {
    if (!fst) return;
    {
        std::lock_guard<std::mutex> lk(g_den_mu);
        auto it = g_den_tables.find(fst->src_states);
        if (it != g_den_tables.end()) {
            delete it->second;
            g_den_tables.erase(it);
        }
    }
    hipFree(fst->src_states);
    hipFree(fst->dst_states);
    hipFree(fst->pdf_ids);
    hipFree(fst->transition_probs);
    fst->src_states = fst->dst_states = fst->pdf_ids = nullptr;
    fst->transition_probs = nullptr;
}

static float den_abi(const DenFstGPU *fst, const float *h_nnet, const float *h_init, int T,
                     float leaky, float *h_post) {
    kf_take_pending(__func__);
    DenTables *t = nullptr;
    {
        std::lock_guard<std::mutex> lk(g_den_mu);
        auto it = fst ? g_den_tables.find(fst->src_states) : g_den_tables.end();
        if (it != g_den_tables.end()) t = it->second;
    }
    if (!t) {
        den_set_error("den_forward: FST was not uploaded with den_fst_upload");
        return -1e30f;
    }
    if (!h_nnet || !h_init || T < 0) {
        den_set_error("den_forward: invalid arguments");
        return -1e30f;
    }
    const int S = t->dev.S, P = t->dev.P;
    const size_t TP = (size_t)T * P;
    DevBuf x, init, as, bs, ast, bst, stats, post, row0, frames, dout;
    const size_t rs = (size_t)t->dev.f.nsl * 64;  // slice-ordered rows
    if (!x.alloc(TP * 4) || !init.alloc(S * 4) || !as.alloc((size_t)(T + 1) * rs * 4) ||
        (h_post && !bs.alloc((size_t)(T + 1) * rs * 4)) ||
        !ast.alloc((T + 1) * 4) || !bst.alloc((T + 1) * 4) || !stats.alloc(32) || !row0.alloc(8) || !frames.alloc(4) ||
        !dout.alloc(8) ||
        (h_post && !post.alloc(TP * 4))) {
        den_set_error("den_forward: hipMalloc failed");
        return -1e30f;
    }
    hipStream_t st = kf_stream();
    long long r0 = 0;
    hipMemcpyAsync(x.p, h_nnet, TP * 4, hipMemcpyHostToDevice, st);
    hipMemcpyAsync(init.p, h_init, S * 4, hipMemcpyHostToDevice, st);
    hipMemcpyAsync(row0.p, &r0, 8, hipMemcpyHostToDevice, st);
    hipMemcpyAsync(frames.p, &T, 4, hipMemcpyHostToDevice, st);
    DenDev g = t->dev;
    g.init = (const float *)init.p;
    den_tables_set_init(g, g.init, st);
    DenRun r{};
    r.nnet = x.p;
    r.ld = P;
    r.row0 = (const long long *)row0.p;
    r.frames = (const int *)frames.p;
    r.stride = 1;
    r.max_frames = T;
    r.leaky = leaky;
    r.backward = h_post != nullptr;
    r.alpha_store = (float *)as.p;
    r.beta_store = (float *)bs.p;
    r.asum_store = (float *)ast.p;
    r.bsum_store = (float *)bst.p;
    r.stats = (float *)stats.p;
    r.post_dense = (float *)post.p;
    r.den_out = (float *)dout.p;
    DenX X{}, XB{};
    DenXBuf xbuf, xbuf2;
    const int G = h_post ? den_pick_G(2) : den_pick_G(1);
    if (!xbuf.make(g, g.f, 1, 1, G, X) || (h_post && !xbuf2.make(g, g.b, 1, 1, G, XB))) {
        den_set_error("den_forward: hipMalloc failed");
        return -1e30f;
    }
    if (h_post) {
        launch_den_fb(g, r, X, xbuf, XB, xbuf2, true);
        launch_den_post(g, r, X, true, DEN_ABI);
    } else {
        launch_den_fwd(g, r, X, xbuf, true);
    }
    float st8[8] = {0};
    hipMemcpyAsync(st8, stats.p, 32, hipMemcpyDeviceToHost, st);
    if (h_post) hipMemcpyAsync(h_post, post.p, TP * 4, hipMemcpyDeviceToHost, st);
    hipError_t e = hipStreamSynchronize(st);
    if (e != hipSuccess || hipGetLastError() != hipSuccess) {
        den_set_error("den_forward_backward: %s", hipGetErrorString(e));
        return -1e30f;
    }
    if (xbuf.take_timeouts(st) + (h_post ? xbuf2.take_timeouts(st) : 0u)) {
        den_set_error("den_forward_backward: cross-workgroup exchange timed out");
        return -1e30f;
    }
    return st8[1];
}

extern "C" float den_forward(const DenFstGPU *fst, const float *nnet_output,
                             const float *initial_probs, int T, float leaky_hmm_coeff) {
    return den_abi(fst, nnet_output, initial_probs, T, leaky_hmm_coeff, nullptr);
}
extern "C" float den_forward_backward(const DenFstGPU *fst, const float *nnet_output,
                                      const float *initial_probs, int T, float leaky_hmm_coeff,
                                      float *grad_output) {
    if (!grad_output) {
        den_set_error("den_forward_backward: grad_output is NULL");
        return -1e30f;
    }
    return den_abi(fst, nnet_output, initial_probs, T, leaky_hmm_coeff, grad_output);
}

// ===========================================================================
// kf_chain.h — batched product interface
// ===========================================================================
struct KfDenGraph {
    DenTables *t = nullptr;
    int num_arcs = 0;
    std::vector<float> init;
    float *d_init = nullptr;
    ~KfDenGraph() {
        delete t;
        if (d_init) hipFree(d_init);
    }
};

struct KfNumBatch {
    NumDevice *nd = nullptr;
    std::vector<int> S;
    unsigned gen = 0;                  // bumped by every refill (kf_chain_compute's layout cache)
    // kf_num_batch_refill: device blob and its pinned host staging (grow only)
    int32_t *d_blob = nullptr;
    size_t d_cap = 0;                  // int32 entries
    int32_t *h_blob = nullptr;
    size_t h_cap = 0;
    hipEvent_t ev_copy = nullptr;      // the last refill's copy (h_blob is reused after it)
    ~KfNumBatch() {
        delete nd;
        if (ev_copy) {
            hipEventSynchronize(ev_copy);
            hipEventDestroy(ev_copy);
        }
        if (d_blob) hipFree(d_blob);
        if (h_blob) hipHostFree(h_blob);
    }
};

struct KfChain {
    const KfDenGraph *den = nullptr;
    DenXBuf xbuf2;  // the backward recursion's exchange (k_den_fb)
    int max_seqs = 0, max_frames = 0;
    float *alpha_store = nullptr, *beta_store = nullptr, *asum_store = nullptr, *bsum_store = nullptr;
    float *stats = nullptr;
    float *h_stats = nullptr;     // pinned [max_seqs][8] (kf_chain_result)
    float *num_ab = nullptr;      // numerator alpha/beta
    size_t num_ab_cap = 0;
    float *num_post = nullptr;    // sparse numerator posteriors
    size_t num_post_cap = 0;
    LogFstDev *d_desc = nullptr;  // [max_seqs]
    long long *d_row0 = nullptr;
    int *d_frames = nullptr;
    float *d_num_total = nullptr;
    // cache of the last run's layout (re-uploaded only when it changes)
    const KfNumBatch *last_num = nullptr;
    unsigned last_gen = 0;
    // pinned staging of the layout upload: two slots, each reused after its copy's event
    char *h_stage[2] = {nullptr, nullptr};
    hipEvent_t ev_stage[2] = {nullptr, nullptr};
    int stage_slot = 0;
    std::vector<int> last_row0, last_frames;
    int last_stride = -1, last_nseq = 0;
    const void *last_nnet = nullptr;
    long long last_ld = -1, last_rows = -1;
    std::vector<LogFstDev> host_desc;
    size_t num_lds = 0;           // dynamic LDS of k_num_fb, 0 = use k_logfb
    float *den_out = nullptr;     // [max_seqs][2]
    hipStream_t side = nullptr;   // numerator stream (overlaps the den forward)
    hipEvent_t ev_in = nullptr, ev_num = nullptr;
    DenXBuf xbuf;
    unsigned long long *trace = nullptr;  // kf_chain_trace (diagnostics)
    int den_pairs = 1;                     // kf_chain_debug_den_pairs (tests)
    ~KfChain() {
        for (int i = 0; i < 2; ++i) {
            if (ev_stage[i]) {
                hipEventSynchronize(ev_stage[i]);
                hipEventDestroy(ev_stage[i]);
            }
            if (h_stage[i]) hipHostFree(h_stage[i]);
        }
        if (h_stats) hipHostFree(h_stats);
        if (side) hipStreamDestroy(side);
        if (ev_in) hipEventDestroy(ev_in);
        if (ev_num) hipEventDestroy(ev_num);
        if (den_out) hipFree(den_out);
        for (void *p : {(void *)alpha_store, (void *)beta_store, (void *)asum_store, (void *)bsum_store,
                        (void *)stats, (void *)num_ab,
                        (void *)num_post, (void *)d_desc, (void *)d_num_total})
            if (p) hipFree(p);
    }
};

extern "C" KfDenGraph *kf_den_graph_create(int S, int P, int A, const int32_t *src,
                                           const int32_t *dst, const int32_t *pdf0,
                                           const float *tp, int start_state,
                                           const float *initial_probs) {
    const char *why = nullptr;
    if (!src || !dst || !pdf0 || !tp || start_state < 0 || start_state >= S) {
        kfc_set_error("kf_den_graph_create: invalid arguments");
        return nullptr;
    }
    DenTables *t = make_den_tables(S, P, A, src, dst, pdf0, tp, &why);
    if (!t) {
        kfc_set_error("kf_den_graph_create: %s", why);
        return nullptr;
    }
    auto *g = new KfDenGraph();
    g->t = t;
    g->num_arcs = A;
    g->init.resize(S);
    if (initial_probs)
        memcpy(g->init.data(), initial_probs, S * 4);
    else
        compute_initial_probs(S, A, src, dst, tp, start_state, g->init.data());
    std::vector<void *> owned;
    g->d_init = dev_upload(g->init, owned);
    if (!g->d_init) {
        delete g;
        kfc_set_error("kf_den_graph_create: hipMalloc failed");
        return nullptr;
    }
    g->t->dev.init = g->d_init;
    den_tables_set_init(g->t->dev, g->d_init, kf_stream());
    if (hipStreamSynchronize(kf_stream()) != hipSuccess) {
        delete g;
        kfc_set_error("kf_den_graph_create: initial-probability gather failed");
        return nullptr;
    }
    return g;
}

extern "C" int kf_den_graph_initial_probs(const KfDenGraph *g, float *out) {
    if (!g || !out) return -1;
    memcpy(out, g->init.data(), g->init.size() * 4);
    return 0;
}
extern "C" void kf_den_graph_free(KfDenGraph *g) {
    kf_take_pending(__func__);
    delete g;
    kf_take_pending("the return of kf_den_graph_free");
}

// host CSR arrays (kf_chain.h layout) -> prepared numerator FSTs
static bool num_hosts(const char *fn, int nseq, const int32_t *state_off, const int32_t *arc_off,
                      const int32_t *row_ptr, const int32_t *dst, const int32_t *pdf1, const float *logw,
                      const int32_t *final_off, const int32_t *final_state, const float *final_logw,
                      std::vector<NumHost> &hs) {
    const char *why = nullptr;
    if (nseq <= 0 || !state_off || !arc_off || !row_ptr || !final_off) {
        kfc_set_error("%s: invalid arguments", fn);
        return false;
    }
    hs.assign(nseq, NumHost());
    for (int i = 0; i < nseq; ++i) {
        NumHost &h = hs[i];
        h.S = state_off[i + 1] - state_off[i];
        h.A = arc_off[i + 1] - arc_off[i];
        h.nfinal = final_off[i + 1] - final_off[i];
        h.start = 0;
        if (h.S <= 0 || h.A < 0 || h.nfinal < 0) {
            kfc_set_error("%s: sequence %d has an empty FST", fn, i);
            return false;
        }
        const int32_t *rp = row_ptr + state_off[i] + i;
        h.row_ptr.assign(rp, rp + h.S + 1);
        h.arc_dst.assign(dst + arc_off[i], dst + arc_off[i + 1]);
        h.arc_pdf.assign(pdf1 + arc_off[i], pdf1 + arc_off[i + 1]);
        h.arc_w.assign(logw + arc_off[i], logw + arc_off[i + 1]);
        h.fin_state.assign(final_state + final_off[i], final_state + final_off[i + 1]);
        h.fin_w.assign(final_logw + final_off[i], final_logw + final_off[i + 1]);
        if (!prepare_num(h, &why)) {
            kfc_set_error("%s: sequence %d: %s", fn, i, why);
            return false;
        }
    }
    return true;
}

extern "C" KfNumBatch *kf_num_batch_create(int nseq, const int32_t *state_off,
                                           const int32_t *arc_off, const int32_t *row_ptr,
                                           const int32_t *dst, const int32_t *pdf1,
                                           const float *logw, const int32_t *final_off,
                                           const int32_t *final_state, const float *final_logw) {
    const char *why = nullptr;
    std::vector<NumHost> hs;
    if (!num_hosts("kf_num_batch_create", nseq, state_off, arc_off, row_ptr, dst, pdf1, logw, final_off,
                   final_state, final_logw, hs))
        return nullptr;
    NumDevice *nd = upload_nums(hs, &why);
    if (!nd) {
        kfc_set_error("kf_num_batch_create: %s", why);
        return nullptr;
    }
    auto *b = new KfNumBatch();
    b->nd = nd;
    for (auto &h : hs) b->S.push_back(h.S);
    return b;
}

// TrainStep's per-minibatch numerator upload (chain_loss.go:44-97) without a device-wide
// stall: host preparation into pinned staging, one asynchronous copy on `stream` into
// buffers that only grow. The caller orders the copy after every kernel that still reads
// the batch's previous contents (e.g. `stream` waits for an event recorded after the
// kf_chain_compute that used it).
extern "C" int kf_num_batch_refill(KfNumBatch *b, int nseq, const int32_t *state_off,
                                   const int32_t *arc_off, const int32_t *row_ptr, const int32_t *dst,
                                   const int32_t *pdf1, const float *logw, const int32_t *final_off,
                                   const int32_t *final_state, const float *final_logw, void *stream) {
    if (!b) {
        kfc_set_error("kf_num_batch_refill: NULL batch");
        return -1;
    }
    std::vector<NumHost> hs;
    if (!num_hosts("kf_num_batch_refill", nseq, state_off, arc_off, row_ptr, dst, pdf1, logw, final_off,
                   final_state, final_logw, hs))
        return -1;
    std::vector<int32_t> blob;
    std::vector<std::vector<size_t>> offs;
    pack_nums(hs, blob, offs);
    const size_t n = std::max<size_t>(blob.size(), 4);
    hipStream_t st = stream ? (hipStream_t)stream : kf_stream();
    if (b->ev_copy) hipEventSynchronize(b->ev_copy);  // h_blob may still feed the last copy
    else if (hipEventCreateWithFlags(&b->ev_copy, hipEventDisableTiming) != hipSuccess) {
        kfc_set_error("kf_num_batch_refill: hipEventCreate failed");
        return -1;
    }
    if (n > b->h_cap) {
        if (b->h_blob) hipHostFree(b->h_blob);
        b->h_blob = nullptr;
        b->h_cap = 0;
        if (hipHostMalloc((void **)&b->h_blob, n * 4, 0) != hipSuccess) {
            kfc_set_error("kf_num_batch_refill: hipHostMalloc failed");
            return -1;
        }
        b->h_cap = n;
    }
    if (n > b->d_cap) {
        // growing: the old blob (this batch's own, or the create-time one) may still be
        // read by queued kernels; hipFree waits for the device
        if (b->d_blob) hipFree(b->d_blob);
        b->d_blob = nullptr;
        b->d_cap = 0;
        if (hipMalloc((void **)&b->d_blob, n * 4) != hipSuccess) {
            kfc_set_error("kf_num_batch_refill: hipMalloc failed");
            return -1;
        }
        b->d_cap = n;
    }
    if (b->nd && !b->nd->owned.empty()) {  // the create-time upload is no longer referenced
        hipDeviceSynchronize();
        for (void *p : b->nd->owned) hipFree(p);
        b->nd->owned.clear();
    }
    if (!b->nd) b->nd = new NumDevice();
    memcpy(b->h_blob, blob.data(), blob.size() * 4);
    if (hipMemcpyAsync(b->d_blob, b->h_blob, blob.size() * 4, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipEventRecord(b->ev_copy, st) != hipSuccess) {
        kfc_set_error("kf_num_batch_refill: copy failed");
        return -1;
    }
    num_descs(hs, offs, b->d_blob, b->nd);
    b->S.clear();
    for (auto &h : hs) b->S.push_back(h.S);
    ++b->gen;
    return 0;
}
extern "C" void kf_num_batch_free(KfNumBatch *b) {
    kf_take_pending(__func__);
    delete b;
    kf_take_pending("the return of kf_num_batch_free");
}

extern "C" KfChain *kf_chain_create(const KfDenGraph *den, int max_seqs, int max_frames) {
    if (!den || max_seqs <= 0 || max_frames <= 0) {
        kfc_set_error("kf_chain_create: invalid arguments");
        return nullptr;
    }
    auto *c = new KfChain();
    c->den = den;
    c->max_seqs = max_seqs;
    c->max_frames = max_frames;
    const int S = den->t->dev.S;
    const size_t rs = (size_t)den->t->dev.f.nsl * 64;  // slice-ordered state rows
    bool ok = hipMalloc(&c->alpha_store, (size_t)max_seqs * (max_frames + 1) * rs * 4) == hipSuccess;
    ok = ok && hipMalloc(&c->beta_store, (size_t)max_seqs * (max_frames + 1) * rs * 4) == hipSuccess;
    ok = ok && hipMalloc(&c->asum_store, (size_t)max_seqs * (max_frames + 1) * 4) == hipSuccess;
    ok = ok && hipMalloc(&c->bsum_store, (size_t)max_seqs * (max_frames + 1) * 4) == hipSuccess;
    ok = ok && hipMalloc(&c->stats, (size_t)max_seqs * 8 * 4) == hipSuccess;
    // descriptors, row offsets and frame counts in one allocation, laid out as the pinned
    // staging slot, so a layout change is one copy
    ok = ok && hipMalloc(&c->d_desc, (size_t)max_seqs * (sizeof(LogFstDev) + 12)) == hipSuccess;
    if (ok) {
        c->d_row0 = reinterpret_cast<long long *>(reinterpret_cast<char *>(c->d_desc) + (size_t)max_seqs * sizeof(LogFstDev));
        c->d_frames = reinterpret_cast<int *>(reinterpret_cast<char *>(c->d_row0) + (size_t)max_seqs * 8);
    }
    ok = ok && hipMalloc(&c->d_num_total, (size_t)max_seqs * 4) == hipSuccess;
    ok = ok && hipMalloc(&c->den_out, (size_t)max_seqs * 8) == hipSuccess;
    ok = ok && hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking) == hipSuccess;
    ok = ok && hipEventCreateWithFlags(&c->ev_in, hipEventDisableTiming) == hipSuccess;
    ok = ok && hipEventCreateWithFlags(&c->ev_num, hipEventDisableTiming) == hipSuccess;
    for (int i = 0; i < 2; ++i) {
        ok = ok && hipEventCreateWithFlags(&c->ev_stage[i], hipEventDisableTiming) == hipSuccess;
        ok = ok && hipHostMalloc((void **)&c->h_stage[i], (size_t)max_seqs * (sizeof(LogFstDev) + 12), 0) ==
                       hipSuccess;
    }
    if (!ok) {
        delete c;
        kfc_set_error("kf_chain_create: hipMalloc failed");
        return nullptr;
    }
    hipMemset(c->stats, 0, (size_t)max_seqs * 32);
    return c;
}
extern "C" void kf_chain_free(KfChain *c) {
    kf_take_pending(__func__);
    delete c;
    kf_take_pending("the return of kf_chain_free");
}

extern "C" int kf_chain_compute(KfChain *c, const KfNumBatch *num, const KfChainOpts *opts,
                                const void *nnet_output, long long ld, long long num_rows, int nseq,
                                const int32_t *seq_row0, const int32_t *seq_frames, int stride,
                                void *out_grad, long long ldg) {
    kf_take_pending(__func__);
    if (!c || !num || !opts || !nnet_output || !out_grad || !seq_row0 || !seq_frames) {
        kfc_set_error("kf_chain_compute: NULL argument");
        return -1;
    }
    const int P = c->den->t->dev.P;
    if (nseq <= 0 || nseq > c->max_seqs || nseq != (int)num->nd->desc.size() || stride <= 0 ||
        ld < P || ldg < P) {
        kfc_set_error("kf_chain_compute: nseq %d (max %d, batch %zu), stride %d, ld %lld/%lld vs P %d",
                      nseq, c->max_seqs, num->nd->desc.size(), stride, ld, ldg, P);
        return -1;
    }
    hipStream_t st = kf_stream();
    // a refilled numerator batch (kf_num_batch_refill): its copy lands before anything reads it
    if (num->ev_copy) hipStreamWaitEvent(st, num->ev_copy, 0);
    bool same = c->last_num == num && c->last_gen == num->gen && c->last_nseq == nseq && c->last_stride == stride &&
                c->last_nnet == nnet_output && c->last_ld == ld && c->last_rows == num_rows &&
                std::equal(seq_row0, seq_row0 + nseq, c->last_row0.begin(), c->last_row0.end()) &&
                std::equal(seq_frames, seq_frames + nseq, c->last_frames.begin(),
                           c->last_frames.end());
    if (!same) {
        for (int i = 0; i < nseq; ++i)
            if (seq_frames[i] < 0 || seq_frames[i] > c->max_frames || seq_row0[i] < 0 ||
                (seq_frames[i] > 0 &&
                 seq_row0[i] + (long long)(seq_frames[i] - 1) * stride >= num_rows)) {
                kfc_set_error("kf_chain_compute: sequence %d: %d frames (max %d), row0 %d, "
                              "stride %d outside %lld rows", i, seq_frames[i], c->max_frames,
                              seq_row0[i], stride, num_rows);
                return -1;
            }
        size_t ab = 0, ps = 0;
        for (int i = 0; i < nseq; ++i) {
            ab += 2 * (size_t)(seq_frames[i] + 1) * num->S[i];
            ps += (size_t)seq_frames[i] * num->nd->G[i];
        }
        if ((ab > c->num_ab_cap && c->num_ab) || (ps > c->num_post_cap && c->num_post))
            hipDeviceSynchronize();  // growing: queued numerator kernels may still use the old buffers
        if (ab > c->num_ab_cap) {
            if (c->num_ab) hipFree(c->num_ab);
            c->num_ab = nullptr;
            if (hipMalloc(&c->num_ab, ab * 4) != hipSuccess) {
                c->num_ab_cap = 0;
                kfc_set_error("kf_chain_compute: hipMalloc failed");
                return -1;
            }
            c->num_ab_cap = ab;
        }
        if (ps > c->num_post_cap) {
            if (c->num_post) hipFree(c->num_post);
            c->num_post = nullptr;
            if (hipMalloc(&c->num_post, std::max<size_t>(ps, 1) * 4) != hipSuccess) {
                c->num_post_cap = 0;
                kfc_set_error("kf_chain_compute: hipMalloc failed");
                return -1;
            }
            c->num_post_cap = ps;
        }
        c->host_desc = num->nd->desc;
        float *ab_p = c->num_ab, *ps_p = c->num_post;
        std::vector<long long> r0(nseq);
        for (int i = 0; i < nseq; ++i) {
            LogFstDev &f = c->host_desc[i];
            f.T = seq_frames[i];
            f.mode = LF_FB | LF_POST;
            f.stride = stride;
            f.row0 = seq_row0[i];
            f.alpha = ab_p;
            ab_p += (size_t)(f.T + 1) * f.S;
            f.beta = ab_p;
            ab_p += (size_t)(f.T + 1) * f.S;
            f.post_sparse = ps_p;
            ps_p += (size_t)f.T * f.G;
            f.post_dense = nullptr;
            f.total = c->d_num_total + i;
            r0[i] = seq_row0[i];
        }
        size_t lds = 0;
        bool fits = true;
        for (int i = 0; i < nseq; ++i) {
            const LogFstDev &f = c->host_desc[i];
            int Ag = (int)num->nd->Ag[i];
            lds = std::max(lds, (size_t)num_lds_layout(f.S, f.A, f.G, Ag).words * 4);
            fits = fits && f.S <= NUM_PRE * NUM_THREADS && f.G <= NUM_PRE * NUM_THREADS;
        }
        c->num_lds = (fits && lds <= 64 * 1024) ? lds : 0;
        // asynchronous on st (every earlier reader of d_desc / d_row0 / d_frames is ahead of it
        // on st: the den kernels, and the numerator kernels through ev_num), from a pinned slot
        // whose previous copy has retired: no host stall when the batch changes every step
        const int slot = c->stage_slot;
        c->stage_slot ^= 1;
        hipEventSynchronize(c->ev_stage[slot]);
        char *hs_ = c->h_stage[slot];
        memcpy(hs_, c->host_desc.data(), nseq * sizeof(LogFstDev));
        memcpy(hs_ + (size_t)c->max_seqs * sizeof(LogFstDev), r0.data(), nseq * 8);
        memcpy(hs_ + (size_t)c->max_seqs * (sizeof(LogFstDev) + 8), seq_frames, nseq * 4);
        bool cp = hipMemcpyAsync(c->d_desc, hs_, (size_t)c->max_seqs * (sizeof(LogFstDev) + 12),
                                 hipMemcpyHostToDevice, st) == hipSuccess;
        cp = cp && hipEventRecord(c->ev_stage[slot], st) == hipSuccess;
        if (!cp) {
            c->last_num = nullptr;
            kfc_set_error("kf_chain_compute: layout upload failed");
            return -1;
        }
        c->last_num = num;
        c->last_gen = num->gen;
        c->last_nseq = nseq;
        c->last_stride = stride;
        c->last_nnet = nnet_output;
        c->last_ld = ld;
        c->last_rows = num_rows;
        c->last_row0.assign(seq_row0, seq_row0 + nseq);
        c->last_frames.assign(seq_frames, seq_frames + nseq);
    }
    double num_arcs = 0, frames = 0;
    for (int i = 0; i < nseq; ++i) {
        num_arcs += (double)c->host_desc[i].A * seq_frames[i];
        frames += seq_frames[i];
    }
    // numerator on the side stream, overlapping the denominator forward
    hipEventRecord(c->ev_in, st);
    hipStreamWaitEvent(c->side, c->ev_in, 0);
    {
        hipStream_t saved = kf_stream();
        kf_set_stream((void *)c->side);
        int pn = kf_prof_start(KF_PROF_CHAIN_NUM, num_arcs);
        if (c->num_lds) {
            // forwards and backwards at the same time, then the posteriors (the numerator
            // shares CUs with the den recursion: the shorter, the less it costs it)
            hipLaunchKernelGGL(k_num_fb, dim3(2 * nseq), dim3(NUM_THREADS), c->num_lds, c->side,
                               (const LogFstDev *)c->d_desc, (const h16 *)nnet_output, ld, P, nseq);
            int maxT = 0;
            for (int i = 0; i < nseq; ++i) maxT = std::max(maxT, seq_frames[i]);
            const int nfb = (maxT + NUM_POST_FR - 1) / NUM_POST_FR;
            if (maxT > 0)
                hipLaunchKernelGGL(k_num_post, dim3(nseq * nfb), dim3(NUM_THREADS), 0, c->side,
                                   (const LogFstDev *)c->d_desc, (const h16 *)nnet_output, ld, P, nfb);
        }
        else
            hipLaunchKernelGGL(k_logfb, dim3(nseq), dim3(256), 0, c->side,
                               (const LogFstDev *)c->d_desc, (const h16 *)nnet_output, ld, P);
        kf_prof_stop(pn);
        kf_set_stream((void *)saved);
    }
    hipEventRecord(c->ev_num, c->side);
    DenRun r{};
    r.nnet = nnet_output;
    r.ld = ld;
    r.row0 = c->d_row0;
    r.frames = c->d_frames;
    r.stride = stride;
    r.max_frames = c->max_frames;
    r.leaky = opts->leaky_hmm_coefficient;
    r.backward = 1;
    r.alpha_store = c->alpha_store;
    r.beta_store = c->beta_store;
    r.asum_store = c->asum_store;
    r.bsum_store = c->bsum_store;
    r.stats = c->stats;
    r.den_out = c->den_out;
    r.trace = c->trace;
    r.nums = c->d_desc;
    r.out_grad = (h16 *)out_grad;
    r.ldg = ldg;
    r.opts = *opts;
    // algorithmic bytes: per frame three streamed passes over the
    // packed arc records, alpha' stored and re-read, the output row read twice
    // and the gradient row written once
    const DenDev &dd = c->den->t->dev;
    double bytes = frames * (3.0 * 8.0 * c->den->num_arcs + 8.0 * dd.S + 6.0 * dd.P);
    int pd = kf_prof_start(KF_PROF_CHAIN_DEN, bytes);
    DenX X{}, XB{};
    // forward and backward blocks share the CUs; sequence pairs (NS = 2) share each
    // record and gather when their interleaved rows fit the LDS
    const int ns = nseq >= 2 && dd.pair_ok && c->den_pairs ? 2 : 1;
    const int G = den_pick_G(2 * ((nseq + ns - 1) / ns));
    if (!c->xbuf.make(dd, dd.f, nseq, ns, G, X) || !c->xbuf2.make(dd, dd.b, nseq, ns, G, XB)) {
        kfc_set_error("kf_chain_compute: hipMalloc failed");
        return -1;
    }
    launch_den_fb(dd, r, X, c->xbuf, XB, c->xbuf2, false);
    hipStreamWaitEvent(st, c->ev_num, 0);  // the numerator is needed from here on
    launch_den_post(dd, r, X, false, DEN_PRODUCT);
    kf_prof_stop(pd);
    if (hipGetLastError() != hipSuccess) {
        kfc_set_error("kf_chain_compute: launch failed");
        return -1;
    }
    return 0;
}

// Diagnostics: when `buf` (device, 32*8 + 32*2*16 u64) is non-null, the den forward
// kernel of sequence 0 / block 0 records 8 phase timestamps (wall_clock64, 100 MHz) for
// frames 16..47 of every later compute, then the arc-phase end of every wave of blocks
// 0 and 1 of sequence 0. Not part of the product contract.
extern "C" void kf_chain_trace(KfChain *c, unsigned long long *buf) {
    if (c) c->trace = buf;
}

// diagnostics (tests): polls an exchange wait makes before it gives up; 0 forces the
// timeout path on the first wait that is not already satisfied. 0xFFFFFFFF = default.
extern "C" void kf_chain_debug_spin_limit(KfChain *c, unsigned polls) {
    if (!c) return;
    const unsigned v = polls == 0xFFFFFFFFu ? (1u << 21) : polls;
    c->xbuf.spin_limit = c->xbuf2.spin_limit = v;
}

// diagnostics (tests): 0 runs the den recursions one sequence per unit (NS = 1) even
// where sequence pairs fit; 1 = default
extern "C" void kf_chain_debug_den_pairs(KfChain *c, int pairs) {
    if (c) c->den_pairs = pairs ? 1 : 0;
}

// diagnostics (tests): 1 makes the den exchange use agent scope (sc1 through to memory)
// even where the blocks of a sequence share an XCD; 0 = default (L2-local when they do)
extern "C" void kf_chain_debug_exchange_sys(KfChain *c, int force) {
    if (c) c->xbuf.force_sys = c->xbuf2.force_sys = force ? 1 : 0;
}

// diagnostics (tests): the XCD census of the last compute's den launch. *units = exchange
// units per direction, *G = workgroups per unit; *local_fwd / *local_bwd = units whose G
// workgroups all ran on one XCD, i.e. took the L2-local exchange unless
// kf_chain_debug_exchange_sys forced agent scope (*forced = 1). 0, or -1 on error.
extern "C" int kf_chain_debug_census(KfChain *c, int *units, int *local_fwd, int *local_bwd, int *forced, int *G) {
    if (!c) return -1;
    hipStream_t st = kf_stream();
    const int f = c->xbuf.census_local(st), b = c->xbuf2.census_local(st);
    if (f < 0 || b < 0) {
        kfc_set_error("kf_chain_debug_census: read failed");
        return -1;
    }
    if (units) *units = c->xbuf.last_units;
    if (local_fwd) *local_fwd = f;
    if (local_bwd) *local_bwd = b;
    if (forced) *forced = c->xbuf.force_sys;
    if (G) *G = c->xbuf.last_G;
    return 0;
}

extern "C" const float *kf_chain_seq_stats(const KfChain *c) { return c ? c->stats : nullptr; }

extern "C" int kf_chain_result(KfChain *c, KfChainResult *out) {
    if (!c || !out) return -1;
    kf_take_pending("kf_chain_result");
    const int n = c->last_nseq;
    hipStream_t st = kf_stream();
    // pinned staging (a stream-ordered copy into pageable memory left a spurious
    // hipErrorStreamCaptureUnsupported pending on the calling thread)
    if (n && !c->h_stats &&
        hipHostMalloc((void **)&c->h_stats, (size_t)c->max_seqs * 8 * 4, hipHostMallocDefault) != hipSuccess) {
        c->h_stats = nullptr;
        kf_take_pending("kf_chain_result hipHostMalloc");
        kfc_set_error("kf_chain_result: pinned staging allocation failed");
        return -1;
    }
    if (n && hipMemcpyAsync(c->h_stats, c->stats, (size_t)n * 8 * 4, hipMemcpyDeviceToHost, st) != hipSuccess) {
        kf_take_pending("kf_chain_result hipMemcpyAsync");
        kfc_set_error("kf_chain_result: statistics copy failed");
        return -1;
    }
    if (hipStreamSynchronize(st) != hipSuccess) {
        kf_take_pending("kf_chain_result hipStreamSynchronize");
        kfc_set_error("kf_chain_result: stream error");
        return -1;
    }
    kf_take_pending("kf_chain_result after the statistics copy");
    const float *s = c->h_stats;
    // every compute since the last result: the sticky count is never reset by a launch
    if (const unsigned nt = c->xbuf.take_timeouts(st) + c->xbuf2.take_timeouts(st)) {
        kfc_set_error("kf_chain_result: den cross-workgroup exchange timed out in %u block(s) since the last "
                      "result (blocks not resident); the objective and gradients of those computes are invalid",
                      nt);
        return -1;
    }
    memset(out, 0, sizeof(*out));
    for (int i = 0; i < n; ++i) {
        const float *v = &s[(size_t)i * 8];
        out->num_logprob += v[0];
        out->den_logprob += v[1];
        out->objf += v[2];
        out->l2_term += v[3];
        out->total_weight += v[4];
        out->frames += (int)v[5];
        out->out_of_range += (int)v[6];
        out->num_ok += v[7] > 0.5f;
    }
    out->num_seqs = n;
    return 0;
}
