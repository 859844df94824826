// gemm.hip — FP16 MFMA GEMMs for gfx950 (MI355X).
//
// One kernel template covers every dense contraction of the CNN-TDNN step:
//   forward   Y = epi(X . W)           A k-contiguous (activations), B = W[K][N]
//   input grad dX = epi(dZ . W^T)      A k-contiguous (dZ),  B = W rows (k-contiguous)
//   weight grad dW = X^T . dZ          A and B both reduction-major (split-K, fp32)
//   ABI ops_gemm C = a.A.B + b.C       A k-contiguous, B = [K][N]
// replacing the reference's cublasGemmEx (cpp/cuda/ops.cu:381-392) plus the
// separate splice / transpose / bias / relu / BN / bypass kernels around it
// (internal/nnet/forward.go:589-790, internal/gpu/backward_ops.go:162-253).
//
// Structure (256 threads = 4 waves; each wave owns a (BM/WM) x (BN/WN) sub-tile):
//   * operands are fetched in 16-byte chunks through the KfOperand addressing
//     rule (kf_ops.h), so TDNN splices and conv im2col are never materialised;
//     invalid chunks (padding, edges) are zero-filled in registers;
//   * register-staged double-buffered LDS, one barrier per K-step;
//   * k-contiguous tiles live as [rows][BK] with a 16-byte XOR swizzle and are read
//     with ds_read_b128; reduction-major tiles live as [BK][W] with an 8-byte XOR
//     swizzle and are read with ds_read_b64_tr_b16 (hardware transpose) — both
//     images are bank-conflict free for the v_mfma_f32_16x16x32_f16 fragment maps
//     (checked offline for the ds_read lane groups of MI355X_MICROARCH §LDS);
//   * fused epilogue: accumulators are staged through LDS as fp32 and every lane
//     then owns 8 consecutive columns of one row, so bias/BN/bypass operands are
//     read and fp16 results written as 16-byte vectors (coalesced).
#include "kf_common.h"
#include "../../include/kf_ops.h"
#include "../../include/ops.h"

KF_DECLARE_ERR(kf)

extern "C" const char *kf_last_error(void) { return kf_err_.get(); }
extern "C" void kf_clear_error(void) { kf_err_.clear(); }

// ---------------------------------------------------------------------------
// operand addressing
// ---------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ T sel9(const T (&a)[KF_MAX_PARTS], int p) {
    T v = a[0];
#pragma unroll
    for (int i = 1; i < KF_MAX_PARTS; ++i)
        if (p == i) v = a[i];
    return v;
}

__device__ __forceinline__ bool op_plain(const KfOperand &d) {
    return d.nparts == 1 && d.hout == 1 && d.dt[0] == 0 && d.edge_t[0] < 0;
}

// pointer to the 8-element chunk Op[r][c..c+7], or nullptr when it reads as zero
__device__ __forceinline__ const h16 *op_chunk(const KfOperand &d, bool plain, int r, int c) {
    if (r >= d.nrows || c >= d.ncols) return nullptr;
    const h16 *base = (const h16 *)d.base;
    if (plain) return base + (long long)r * d.ld + c;
    int p = 0, kk = c;
    if (d.nparts > 1) {
        p = c / d.part_width;
        kk = c - p * d.part_width;
    }
    int t = r, h = 0;
    if (d.hout > 1) {
        t = r / d.hout;
        h = r - t * d.hout;
    }
    const int et = sel9(d.edge_t, p);
    if (et >= 0 && t == et) return (const h16 *)sel9(d.edge_ptr, p) + kk;
    int st = t + sel9(d.dt, p);
    if (st < 0 || st >= d.T) {
        if (d.tpolicy != KF_CLAMP) return nullptr;
        st = st < 0 ? 0 : d.T - 1;
    }
    int sh = h * d.hmul + sel9(d.dh, p);
    if (d.hdiv > 1) {
        if (sh < 0 || (sh % d.hdiv) != 0) return nullptr;
        sh /= d.hdiv;
    }
    if (sh < 0 || sh >= d.hsrc) return nullptr;
    return base + (long long)st * d.ld + (long long)sh * d.part_width + kk;
}

// ---------------------------------------------------------------------------
// LDS images
// ---------------------------------------------------------------------------
// k-contiguous [rows][BK] halves, 16-byte chunk c of row r stored at c ^ ((r>>1)&(CPR-1))
template <int BK>
__device__ __forceinline__ int kc_off(int r, int c) {
    constexpr int CPR = BK / 8;
    return r * (BK * 2) + 16 * (c ^ ((r >> 1) & (CPR - 1)));
}
// reduction-major [BK][W] halves, 8-byte unit u of row r stored at u ^ swz(r)
template <int W>
__device__ __forceinline__ int mn_swz(int r) {
    if constexpr (W == 64) return ((r & 2) << 1) ^ (((r >> 3) & 1) << 3);
    else if constexpr (W == 128 || W == 256) return ((r & 3) << 2) ^ (((r >> 3) & 1) << 4);
    else if constexpr (W % 32 == 0) return ((r >> 3) & 1) << 2;
    else return 0;
}
template <int W>
__device__ __forceinline__ int mn_off(int r, int u) {
    return r * (W * 2) + 8 * (u ^ mn_swz<W>(r));
}

typedef __attribute__((address_space(3))) short4v lds_s4;

// fragment for v_mfma_f32_16x16x32_f16: lane l holds Op[idx0 + (l&15)][k = 32s + 8(l>>4) + j]
template <bool KC, int W, int BK>
__device__ __forceinline__ half8 load_frag(const char *tile, int idx0, int s, int lane) {
    if constexpr (KC) {
        const int r = idx0 + (lane & 15);
        const int c = s * 4 + (lane >> 4);
        return *reinterpret_cast<const half8 *>(tile + kc_off<BK>(r, c));
    } else {
        const int q = (lane & 15) >> 2, p = lane & 3, g = lane >> 4;
        const int r0 = s * 32 + 8 * g + q;
        const int u = (idx0 >> 2) + p;
        short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4 *)(tile + mn_off<W>(r0, u)));
        short4v hi =
            __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4 *)(tile + mn_off<W>(r0 + 4, u)));
        typedef short short8v __attribute__((ext_vector_type(8)));
        short8v v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
        return __builtin_bit_cast(half8, v);
    }
}

// ---------------------------------------------------------------------------
// epilogue on 8 consecutive columns of one row
// ---------------------------------------------------------------------------
__device__ __forceinline__ void epilogue8(const KfEpilogue &E, int m, int n, float v[8]) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] *= E.alpha;
    if (E.beta != 0.f) {
        half8 o = load_h8((const h16 *)E.out + (long long)m * E.ldo + n);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += E.beta * (float)o[e];
    }
    if (E.bias) {
        half8 b = load_h8((const h16 *)E.bias + n);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += (float)b[e];
    }
    if (E.relu) {
        unsigned bits = 0;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            if (v[e] > 0.f) bits |= 1u << e;
            else v[e] = 0.f;
        }
        if (E.mask_out) E.mask_out[((long long)m * E.ldo + n) >> 3] = (uint8_t)bits;
    }
    if (E.scale) {
        float4v s0 = *reinterpret_cast<const float4v *>(E.scale + n);
        float4v s1 = *reinterpret_cast<const float4v *>(E.scale + n + 4);
        float4v b0 = *reinterpret_cast<const float4v *>(E.shift + n);
        float4v b1 = *reinterpret_cast<const float4v *>(E.shift + n + 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            v[e] = fmaf(v[e], s0[e], b0[e]);
            v[e + 4] = fmaf(v[e + 4], s1[e], b1[e]);
        }
    }
    if (E.resid) {
        half8 r = load_h8((const h16 *)E.resid + (long long)m * E.ldr + n);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = fmaf(E.resid_alpha, (float)r[e], v[e]);
    }
    if (E.out) {
        half8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = f2h(v[e]);
        store_h8((h16 *)E.out + (long long)m * E.ldo + n, o);
    }
    if (E.out2) {
        float w[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) w[e] = v[e];
        if (E.scale2) {
            float4v s0 = *reinterpret_cast<const float4v *>(E.scale2 + n);
            float4v s1 = *reinterpret_cast<const float4v *>(E.scale2 + n + 4);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                w[e] *= s0[e];
                w[e + 4] *= s1[e];
            }
        }
        if (E.mask_in) {
            unsigned bits = E.mask_in[((long long)m * E.ldo2 + n) >> 3];
#pragma unroll
            for (int e = 0; e < 8; ++e)
                if (!((bits >> e) & 1u)) w[e] = 0.f;
        }
        half8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = f2h(w[e]);
        store_h8((h16 *)E.out2 + (long long)m * E.ldo2 + n, o);
    }
}

// ---------------------------------------------------------------------------
// the kernel
// ---------------------------------------------------------------------------
struct WgradArgs {
    float *slab;        // [splits][M][N] fp32 partials
    float *bias_slab;   // [splits][N] fp32 column sums of B, or nullptr
    int k_per_split;    // multiple of BK
};

template <int BM, int BN, int BK>
struct SmemSize {
    static constexpr int pipe = 2 * (BM + BN) * BK * 2;
    static constexpr int epi = BM * (BN + 4) * 4;
    static constexpr int bytes = pipe > epi ? pipe : epi;
};

template <int BM, int BN, int BK, int WM, int WN, bool AKC, bool BKC, bool WGRAD>
__global__ __launch_bounds__(256, 2) void gemm_kernel(int M, int N, int K, KfOperand A,
                                                      KfOperand B, KfEpilogue E, WgradArgs G,
                                                      int n_ntiles) {
    static_assert(WM * WN == 4, "4 waves");
    constexpr int WTM = BM / WM, WTN = BN / WN;
    constexpr int TM = WTM / 16, TN = WTN / 16;
    static_assert(TM * 16 == WTM && TN * 16 == WTN, "wave tile multiple of 16");
    constexpr int KS = BK / 32;
    constexpr int CA = BM * BK / 8 / 256, CB = BN * BK / 8 / 256;
    static_assert(CA * 256 * 8 == BM * BK && CB * 256 * 8 == BN * BK, "chunk split");
    constexpr int A_STAGE = BM * BK * 2, B_STAGE = BN * BK * 2;

    __shared__ __attribute__((aligned(16))) char smem[SmemSize<BM, BN, BK>::bytes];
    auto sA = [&](int buf) { return smem + buf * A_STAGE; };
    auto sB = [&](int buf) { return smem + 2 * A_STAGE + buf * B_STAGE; };

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WN, wn = wave % WN;
    const int tile = blockIdx.x;
    const int mt = tile / n_ntiles, nt = tile - mt * n_ntiles;
    const int m0 = mt * BM, n0 = nt * BN;
    int kbeg = 0, kend = K;
    if constexpr (WGRAD) {
        kbeg = blockIdx.y * G.k_per_split;
        kend = min(K, kbeg + G.k_per_split);
    }
    const int nk = (kend - kbeg + BK - 1) / BK;
    const bool aplain = op_plain(A), bplain = op_plain(B);

    uint4 ra[CA], rb[CB];
    auto ldg = [&](int k0) {
#pragma unroll
        for (int i = 0; i < CA; ++i) {
            const int id = tid + 256 * i;
            int r, c;
            if constexpr (AKC) {
                r = m0 + id / (BK / 8);
                c = k0 + 8 * (id % (BK / 8));
            } else {
                r = k0 + id / (BM / 8);
                c = m0 + 8 * (id % (BM / 8));
            }
            const bool inb = AKC ? (c < kend) : (r < kend);
            const h16 *p = inb ? op_chunk(A, aplain, r, c) : nullptr;
            ra[i] = p ? *reinterpret_cast<const uint4 *>(p) : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < CB; ++i) {
            const int id = tid + 256 * i;
            int r, c;
            if constexpr (BKC) {
                r = n0 + id / (BK / 8);
                c = k0 + 8 * (id % (BK / 8));
            } else {
                r = k0 + id / (BN / 8);
                c = n0 + 8 * (id % (BN / 8));
            }
            const bool inb = BKC ? (c < kend) : (r < kend);
            const h16 *p = inb ? op_chunk(B, bplain, r, c) : nullptr;
            rb[i] = p ? *reinterpret_cast<const uint4 *>(p) : make_uint4(0, 0, 0, 0);
        }
    };
    auto sts = [&](int buf) {
#pragma unroll
        for (int i = 0; i < CA; ++i) {
            const int id = tid + 256 * i;
            int off;
            if constexpr (AKC) off = kc_off<BK>(id / (BK / 8), id % (BK / 8));
            else off = mn_off<BM>(id / (BM / 8), 2 * (id % (BM / 8)));
            *reinterpret_cast<uint4 *>(sA(buf) + off) = ra[i];
        }
#pragma unroll
        for (int i = 0; i < CB; ++i) {
            const int id = tid + 256 * i;
            int off;
            if constexpr (BKC) off = kc_off<BK>(id / (BK / 8), id % (BK / 8));
            else off = mn_off<BN>(id / (BN / 8), 2 * (id % (BN / 8)));
            *reinterpret_cast<uint4 *>(sB(buf) + off) = rb[i];
        }
    };

    float4v acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = float4v{0.f, 0.f, 0.f, 0.f};

    // column sums of B (bias gradient) by the blocks of the first M tile
    const bool do_bsum = WGRAD && G.bias_slab != nullptr && mt == 0 && !BKC;
    float bsum = 0.f;

    if (nk > 0) {
        ldg(kbeg);
        sts(0);
        __syncthreads();
    }
    for (int kt = 0; kt < nk; ++kt) {
        const int cur = kt & 1;
        if (kt + 1 < nk) ldg(kbeg + (kt + 1) * BK);
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            half8 fa[TM], fb[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i)
                fa[i] = load_frag<AKC, BM, BK>(sA(cur), wm * WTM + i * 16, s, lane);
#pragma unroll
            for (int j = 0; j < TN; ++j)
                fb[j] = load_frag<BKC, BN, BK>(sB(cur), wn * WTN + j * 16, s, lane);
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[i], fb[j], acc[i][j],
                                                                       0, 0, 0);
        }
        if constexpr (WGRAD && !BKC) {
            if (do_bsum && tid < BN) {
                for (int r = 0; r < BK; ++r) {
                    const int u = tid >> 2;
                    const char *p = sB(cur) + mn_off<BN>(r, u) + 2 * (tid & 3);
                    bsum += (float)*reinterpret_cast<const h16 *>(p);
                }
            }
        }
        if (kt + 1 < nk) sts(cur ^ 1);
        __syncthreads();
    }

    if constexpr (WGRAD) {
        float *slab = G.slab + (long long)blockIdx.y * M * N;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int n = n0 + wn * WTN + j * 16 + (lane & 15);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int m = m0 + wm * WTM + i * 16 + 4 * (lane >> 4) + e;
                    if (m < M && n < N) slab[(long long)m * N + n] = acc[i][j][e];
                }
            }
        if (do_bsum && tid < BN && n0 + tid < N)
            G.bias_slab[(long long)blockIdx.y * N + n0 + tid] = bsum;
    } else {
        // stage fp32 accumulators through LDS: [BM][BN+4]
        float *st = reinterpret_cast<float *>(smem);
        constexpr int LDT = BN + 4;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int c = wn * WTN + j * 16 + (lane & 15);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int r = wm * WTM + i * 16 + 4 * (lane >> 4) + e;
                    st[r * LDT + c] = acc[i][j][e];
                }
            }
        __syncthreads();
        constexpr int GROUPS = BM * BN / 8;
        for (int it = tid; it < GROUPS; it += 256) {
            const int r = it / (BN / 8), cg = it - r * (BN / 8);
            const int m = m0 + r, n = n0 + 8 * cg;
            if (m >= M || n >= N) continue;
            float v[8];
            float4v x0 = *reinterpret_cast<const float4v *>(st + r * LDT + 8 * cg);
            float4v x1 = *reinterpret_cast<const float4v *>(st + r * LDT + 8 * cg + 4);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                v[e] = x0[e];
                v[e + 4] = x1[e];
            }
            epilogue8(E, m, n, v);
        }
    }
}

// split-K reduction: dst[m][n] (+)= sum_s slab[s][m][n]
__global__ void k_slab_reduce(const float *slab, int splits, int M, int N, float *dst,
                              long long ldw, int accumulate) {
    const long long total = (long long)M * N;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        float s = 0.f;
        for (int k = 0; k < splits; ++k) s += slab[k * total + i];
        const long long m = i / N, n = i - m * N;
        float *d = dst + m * ldw + n;
        *d = accumulate ? *d + s : s;
    }
}

__global__ void k_rows_sum(h16 *edge, const h16 *src, long long ld, int r0, int r1, int cols) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= cols) return;
    float s = 0.f;
    for (int r = r0; r < r1; ++r) s += h2f(src[(long long)r * ld + c]);
    edge[c] = f2h(s);
}

// ---------------------------------------------------------------------------
// optional per-launch HIP-event timing (kf_prof_*), used by bench.py to price
// the dominant kernel class over the timed region on the stream it runs on
// ---------------------------------------------------------------------------
#include <vector>
namespace {
struct ProfRec {
    hipEvent_t a, b;
    int cls;
    double flops;
};
bool g_prof = false;
std::vector<ProfRec> g_prof_recs;
std::vector<hipEvent_t> g_prof_pool;
hipEvent_t prof_event() {
    if (!g_prof_pool.empty()) {
        hipEvent_t e = g_prof_pool.back();
        g_prof_pool.pop_back();
        return e;
    }
    hipEvent_t e;
    hipEventCreate(&e);
    return e;
}
}  // namespace
enum { KF_PROF_FUSED = 0, KF_PROF_WGRAD = 1, KF_PROF_NCLS = 2 };

extern "C" void kf_prof_enable(int on) { g_prof = on != 0; }
// sums per class since the last collect: count, milliseconds, flops
extern "C" int kf_prof_collect(int cls, long long *count, double *ms, double *flops) {
    long long c = 0;
    double t = 0, f = 0;
    for (auto &r : g_prof_recs) {
        if (r.cls != cls) continue;
        hipEventSynchronize(r.b);
        float e = 0.f;
        hipEventElapsedTime(&e, r.a, r.b);
        c++;
        t += e;
        f += r.flops;
    }
    if (count) *count = c;
    if (ms) *ms = t;
    if (flops) *flops = f;
    return 0;
}
extern "C" void kf_prof_reset(void) {
    for (auto &r : g_prof_recs) {
        hipEventSynchronize(r.b);
        g_prof_pool.push_back(r.a);
        g_prof_pool.push_back(r.b);
    }
    g_prof_recs.clear();
}

// ---------------------------------------------------------------------------
// host side: tile selection and launch
// ---------------------------------------------------------------------------
template <int BM, int BN, int BK, int WM, int WN, bool AKC, bool BKC, bool WGRAD>
static int launch(int M, int N, int K, const KfOperand &A, const KfOperand &B,
                  const KfEpilogue &E, const WgradArgs &G, int splits) {
    const int mt = (M + BM - 1) / BM, nt = (N + BN - 1) / BN;
    dim3 grid(mt * nt, WGRAD ? splits : 1);
    ProfRec rec{};
    if (g_prof) {
        rec.a = prof_event();
        rec.b = prof_event();
        rec.cls = WGRAD ? KF_PROF_WGRAD : KF_PROF_FUSED;
        rec.flops = 2.0 * M * N * (double)K;
        hipEventRecord(rec.a, kf_stream());
    }
    gemm_kernel<BM, BN, BK, WM, WN, AKC, BKC, WGRAD>
        <<<grid, 256, 0, kf_stream()>>>(M, N, K, A, B, E, G, nt);
    if (g_prof) {
        hipEventRecord(rec.b, kf_stream());
        g_prof_recs.push_back(rec);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        kf_set_error("gemm launch (M=%d N=%d K=%d): %s", M, N, K, hipGetErrorString(e));
        return -1;
    }
    return 0;
}

static bool check_operand(const KfOperand &d, const char *name) {
    if (!d.base) {
        kf_set_error("operand %s: null base", name);
        return false;
    }
    if (d.nparts < 1 || d.nparts > KF_MAX_PARTS || d.part_width <= 0 || d.hout < 1 ||
        d.hdiv < 1) {
        kf_set_error("operand %s: bad addressing (nparts=%d width=%d hout=%d hdiv=%d)", name,
                     d.nparts, d.part_width, d.hout, d.hdiv);
        return false;
    }
    if (d.part_width % 8 != 0 || d.ncols % 8 != 0 || d.ld % 8 != 0 ||
        ((uintptr_t)d.base & 15) != 0) {
        kf_set_error("operand %s: columns / ld / base must be 16-byte granular", name);
        return false;
    }
    for (int p = 0; p < d.nparts; ++p)
        if (d.edge_t[p] >= 0 && (((uintptr_t)d.edge_ptr[p]) & 15)) {
            kf_set_error("operand %s: edge row %d misaligned", name, p);
            return false;
        }
    return true;
}

extern "C" int kf_gemm_fused(int M, int N, int K, const KfOperand *A, const KfOperand *B,
                             const KfEpilogue *epi) {
    if (M <= 0 || N <= 0) return 0;
    if (!check_operand(*A, "A") || !check_operand(*B, "B")) return -1;
    if (N % 8 != 0) {
        kf_set_error("kf_gemm_fused: N=%d must be a multiple of 8", N);
        return -1;
    }
    if (!A->kcontig) {
        kf_set_error("kf_gemm_fused: A must be k-contiguous");
        return -1;
    }
    const KfEpilogue &E = *epi;
    if ((E.out && E.ldo % 8) || (E.out2 && E.ldo2 % 8) || (E.resid && E.ldr % 8) ||
        (E.mask_out && E.ldo % 8)) {
        kf_set_error("kf_gemm_fused: leading dimensions must be multiples of 8");
        return -1;
    }
    WgradArgs G{nullptr, nullptr, 0};
    // tile choice by output width
    if (B->kcontig) {
        if (N % 160 == 0 && N <= 320)
            return launch<128, 160, 64, 2, 2, true, true, false>(M, N, K, *A, *B, E, G, 1);
        if (N <= 64) return launch<256, 64, 32, 4, 1, true, true, false>(M, N, K, *A, *B, E, G, 1);
        return launch<128, 128, 64, 2, 2, true, true, false>(M, N, K, *A, *B, E, G, 1);
    } else {
        if (N % 160 == 0 && N <= 320)
            return launch<128, 160, 64, 2, 2, true, false, false>(M, N, K, *A, *B, E, G, 1);
        if (N <= 64)
            return launch<256, 64, 32, 4, 1, true, false, false>(M, N, K, *A, *B, E, G, 1);
        return launch<128, 128, 64, 2, 2, true, false, false>(M, N, K, *A, *B, E, G, 1);
    }
}

extern "C" int kf_gemm_wgrad(int M, int N, int K, const KfOperand *A, const KfOperand *B,
                             float *dW, long long ldw, float *bias_grad, int accumulate) {
    if (M <= 0 || N <= 0) return 0;
    if (!check_operand(*A, "A") || !check_operand(*B, "B")) return -1;
    if (A->kcontig || B->kcontig) {
        kf_set_error("kf_gemm_wgrad: A and B must be reduction-major");
        return -1;
    }
    // tile + split choice: aim for >= ~2 workgroups per CU
    int BMc = 128, BNc = (N % 160 == 0 && N <= 320) ? 160 : (N <= 64 ? 64 : 128);
    if (BNc == 64) BMc = 256;
    const int tiles = ((M + BMc - 1) / BMc) * ((N + BNc - 1) / BNc);
    const int BK = (BNc == 64) ? 32 : 64;
    int splits = (512 + tiles - 1) / tiles;
    const int maxsplit = (K + 4 * BK - 1) / (4 * BK);  // at least 4 K-steps per split
    if (splits > maxsplit) splits = maxsplit;
    if (splits < 1) splits = 1;
    int kps = (K + splits - 1) / splits;
    kps = (kps + BK - 1) / BK * BK;
    splits = (K + kps - 1) / kps;
    size_t slab_bytes = (size_t)splits * M * N * 4;
    size_t bias_bytes = bias_grad ? (size_t)splits * N * 4 : 0;
    char *ws = (char *)kf_workspace(slab_bytes + bias_bytes + 256, 0);
    if (!ws) {
        kf_set_error("kf_gemm_wgrad: workspace allocation of %zu bytes failed",
                     slab_bytes + bias_bytes);
        return -1;
    }
    WgradArgs G{(float *)ws, bias_grad ? (float *)(ws + ((slab_bytes + 255) & ~(size_t)255))
                                       : nullptr,
                kps};
    KfEpilogue E{};
    int rc;
    if (BNc == 160) rc = launch<128, 160, 64, 2, 2, false, false, true>(M, N, K, *A, *B, E, G, splits);
    else if (BNc == 64) rc = launch<256, 64, 32, 4, 1, false, false, true>(M, N, K, *A, *B, E, G, splits);
    else rc = launch<128, 128, 64, 2, 2, false, false, true>(M, N, K, *A, *B, E, G, splits);
    if (rc) return rc;
    k_slab_reduce<<<kf_blocks((long long)M * N, 256, 4096), 256, 0, kf_stream()>>>(
        G.slab, splits, M, N, dW, ldw, accumulate);
    if (bias_grad)
        k_slab_reduce<<<kf_blocks(N, 256, 64), 256, 0, kf_stream()>>>(G.bias_slab, splits, 1, N,
                                                                      bias_grad, N, accumulate);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        kf_set_error("wgrad reduce: %s", hipGetErrorString(e));
        return -1;
    }
    return 0;
}

extern "C" int kf_rows_sum(void *edge, const void *src, long long ld, int r0, int r1, int cols) {
    if (cols <= 0) return 0;
    k_rows_sum<<<(cols + 255) / 256, 256, 0, kf_stream()>>>((h16 *)edge, (const h16 *)src, ld,
                                                            r0, r1, cols);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        kf_set_error("rows_sum: %s", hipGetErrorString(e));
        return -1;
    }
    return 0;
}

// helpers for plain operands (used by the ABI GEMM below and by the host layer)
static KfOperand plain_operand(const void *p, long long ld, int rows, int cols, int kcontig) {
    KfOperand d;
    memset(&d, 0, sizeof(d));
    d.base = p;
    d.ld = ld;
    d.nrows = rows;
    d.ncols = cols;
    d.kcontig = kcontig;
    d.nparts = 1;
    d.part_width = cols;
    d.T = rows;
    d.hout = 1;
    d.hsrc = 1;
    d.hmul = 0;
    d.hdiv = 1;
    d.tpolicy = KF_ZERO;
    for (int i = 0; i < KF_MAX_PARTS; ++i) d.edge_t[i] = -1;
    return d;
}

// ---------------------------------------------------------------------------
// reference ABI GEMM (ops.h) on the same kernels
// ---------------------------------------------------------------------------
struct KfGemmCtx {
    int magic;
};

extern "C" void *ops_cublas_create(void) {
    KfGemmCtx *c = new KfGemmCtx;
    c->magic = 0x6b663136;
    return c;
}
extern "C" void ops_cublas_destroy(void *h) { delete (KfGemmCtx *)h; }

// scalar fallback for shapes the MFMA path cannot address (unaligned / odd N)
__global__ void k_gemm_small(int M, int N, int K, float alpha, const h16 *A, int lda,
                             const h16 *B, int ldb, float beta, h16 *C, int ldc) {
    const long long total = (long long)M * N;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const int m = (int)(i / N), n = (int)(i - (long long)m * N);
        float s = 0.f;
        for (int k = 0; k < K; ++k) s += h2f(A[(long long)m * lda + k]) * h2f(B[(long long)k * ldb + n]);
        float v = alpha * s;
        if (beta != 0.f) v += beta * h2f(C[(long long)m * ldc + n]);
        C[(long long)m * ldc + n] = f2h(v);
    }
}

int kf_ops_gemm_impl(int M, int N, int K, float alpha, const void *A, int lda, const void *B,
                     int ldb, float beta, void *C, int ldc, char *err, size_t errlen) {
    if (M < 0 || N < 0 || K < 0) {
        snprintf(err, errlen, "ops_gemm: negative dims (M=%d N=%d K=%d)", M, N, K);
        return -1;
    }
    if (M == 0 || N == 0) return 0;
    if (lda <= 0) lda = K;
    if (ldb <= 0) ldb = N;
    if (ldc <= 0) ldc = N;
    const bool fast = (K % 8 == 0) && (N % 8 == 0) && (lda % 8 == 0) && (ldb % 8 == 0) &&
                      (ldc % 8 == 0) && !(((uintptr_t)A | (uintptr_t)B | (uintptr_t)C) & 15);
    if (!fast || K == 0) {
        k_gemm_small<<<kf_blocks((long long)M * N, 256, 8192), 256, 0, kf_stream()>>>(
            M, N, K, alpha, (const h16 *)A, lda, (const h16 *)B, ldb, beta, (h16 *)C, ldc);
    } else {
        KfOperand a = plain_operand(A, lda, M, K, 1);
        KfOperand b = plain_operand(B, ldb, K, N, 0);
        KfEpilogue E;
        memset(&E, 0, sizeof(E));
        E.out = C;
        E.ldo = ldc;
        E.alpha = alpha;
        E.beta = beta;
        if (kf_gemm_fused(M, N, K, &a, &b, &E) != 0) {
            snprintf(err, errlen, "%s", kf_last_error() ? kf_last_error() : "gemm failed");
            return -1;
        }
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        snprintf(err, errlen, "ops_gemm (M=%d N=%d K=%d): %s", M, N, K, hipGetErrorString(e));
        return -1;
    }
    return 0;
}
