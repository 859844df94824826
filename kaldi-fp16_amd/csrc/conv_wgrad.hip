// conv_wgrad.hip — weight gradient of the 3x3 convolutions with the source halo in LDS.
//
// dW[(p, c)][n] = sum over output rows m = (t, h) of X[t + dt_p][h * hmul + dh_p][c] . dZ[m][n]
// (the reference's backward: im2col of the cached input, transposed, times the output
// gradient — internal/gpu/backward_ops.go:162-253 over forward.go:435-456's im2col).
//
// The im2col GEMM (gemm_kernel with the reduction-major im2col operand) stages every
// tap's 64-channel slab of every output row separately: for the 64-filter layers its
// 192 x 64 tiles move ~20 KB through L2 per MFLOP and run at ~270 TF/s. Here one
// workgroup owns ALL nine taps of one 64-channel chunk (a 576-row tile) and, per
// K-step of 64 output rows, loads the source frames those rows touch ONCE (the same
// halo image as the forward's conv_halo_kernel: padded heights, de-interleaved by
// parity for height-subsampled layers); every tap's A fragment is then a transposed
// LDS read (ds_read_b64_tr_b16) at a per-tap row offset, each lane addressing the
// halo row of its own output rows. B (dZ rows) streams through the usual
// reduction-major stager. Split over the reduction into fp32 slabs like kf_gemm_wgrad;
// the slab reduce is gemm.hip's.
#include <algorithm>
#include <cstdlib>

#include "gemm_common.h"

namespace {

constexpr int WTAPS = 9;         // taps per tile (3 x 3 kernels)
constexpr int WWM = 4;           // wave rows: 576 / 4 = 144 tile rows (9 MFMA blocks) per wave
constexpr int WROWS = WTAPS * 64;

// LDS image swizzle of halo row R: 16-byte chunk c lives at slot c ^ hsw(R). Bits 1
// and 3 of R make the eight rows a ds_read_b64_tr_b16 lane group reads (k, k + 1, ..,
// k + 3, k + 8, .., k + 11) land on disjoint banks (checked exhaustively offline; a
// frame boundary inside the group can still cost one 2-way conflict).
__device__ __forceinline__ int hsw(int R) { return (((R >> 1) & 1) | (((R >> 3) & 1) << 1)) << 1; }

constexpr int HPW_MAX = 8;       // halo pieces per wave per K-step (host-checked)

// s_waitcnt vmcnt(n) for a wave-uniform runtime n (the immediate is compile-time)
__device__ __forceinline__ void wait_vmcnt_rt(int n) {
    switch (n) {
        case 0: wait_vmcnt<0>(); break;
        case 1: wait_vmcnt<1>(); break;
        case 2: wait_vmcnt<2>(); break;
        case 3: wait_vmcnt<3>(); break;
        case 4: wait_vmcnt<4>(); break;
        case 5: wait_vmcnt<5>(); break;
        case 6: wait_vmcnt<6>(); break;
        case 7: wait_vmcnt<7>(); break;
        case 8: wait_vmcnt<8>(); break;
        case 9: wait_vmcnt<9>(); break;
        case 10: wait_vmcnt<10>(); break;
        case 11: wait_vmcnt<11>(); break;
        case 12: wait_vmcnt<12>(); break;
        case 13: wait_vmcnt<13>(); break;
        case 14: wait_vmcnt<14>(); break;
        case 15: wait_vmcnt<15>(); break;
        default: wait_vmcnt<0>(); break;
    }
}

struct WHalo {
    const h16 *x;        // source [T x hsrc x fin] (row = frame, ld elements)
    long long ld;
    int T, hout, hmul, hsrc, fin, pad, hpe, hpos, nf, dtmin;
    int ts, toff;        // output frame t reads source frames ts * t + toff + dt (KfOperand.tmul / t0)
    int rows, npieces, halo_bytes;
    int hpw;             // halo pieces issued per wave per K-step (ceil(npieces / waves))
    unsigned inv_hout;   // ceil(2^16 / hout): exact x / hout for x * hout < 2^16
    int ctap[WTAPS];
    int mout;            // T * hout (the reduction)
    int kps;             // K-steps (64 rows) per split
    int splits, ctiles, ntiles;
    float *slab, *bias_slab;
    int Mtot, N;         // dW rows (9 * fin), columns (fout)
};

// NW waves (4: two workgroups per CU, 8: one); NS-stage LDS ring of {halo, dZ rows}
template <int BN, int NW, int NS>
__global__ __launch_bounds__(64 * NW, 8 / NW) void conv_wgrad_halo_kernel(OpD B, WHalo H) {
    constexpr int WNW = NW;
    constexpr int WN = WNW / WWM;
    constexpr int WTM = WROWS / WWM, WTN = BN / WN;
    constexpr int TM = WTM / 16, TN = WTN / 16;
    constexpr int B_STAGE = BN * BK * 2;
    static_assert(TM * 16 == WTM && TN * 16 == WTN, "wave tile");
    using SB = Stager<false, BN, OP_SIMPLE, WNW>;
    extern __shared__ __attribute__((aligned(16))) char dsm[];
    char *bring = dsm + NS * H.halo_bytes;
    char *dummy = bring + NS * B_STAGE;  // 1 KiB sink for the padding loads (never read)

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / WN, wn = wave % WN;

    // work item: the tiles of one split are consecutive, and consecutive items share an
    // XCD (block b runs on XCD b % 8), so a split's halo and dZ rows are L2-shared
    const int tiles = H.ctiles * H.ntiles, total = tiles * H.splits;
    int w = blockIdx.x;
    {
        const int q = total / 8, rmd = total % 8, xcd = w % 8, loc = w / 8;
        w = (xcd < rmd ? xcd * (q + 1) : rmd * (q + 1) + (xcd - rmd) * q) + loc;
    }
    const int split = w / tiles, tile = w - split * tiles;
    const int cc = tile / H.ntiles, nt = tile - cc * H.ntiles;
    const int n0 = nt * BN;
    const int nks = (H.mout + BK - 1) / BK;
    const int ks0 = split * H.kps, ks1 = min(nks, ks0 + H.kps);

    SB sb;
    sb.init(B, n0, wave, lane);
    const Rsrc rx = make_rsrc(H.x), rb = make_rsrc(B.base);

    // halo of K-step ks into image `img`: source frames tb + dtmin .. + nf - 1. Every
    // wave issues exactly hpw pieces (the surplus ones load zeros into `dummy`), so the
    // ring's counted waits see the same number of loads per step on every wave.
    // The row -> (frame, height) map does not depend on the K-step: each lane keeps
    // its pieces' frame index and in-frame byte offset (-1: a padding height).
    // packed (frame << 20) | in-frame byte offset, -1 for a padding height (host-checked:
    // offsets < 2^20, frames < 2^11)
    int pfo[HPW_MAX];
    static_for<HPW_MAX>([&](auto I) {
        constexpr int i = decltype(I)::value;
        const int R = 8 * (wave + i * WNW) + (lane >> 3);
        pfo[i] = -1;
        if (i < H.hpw && R < H.rows) {
            const int f = R / H.hpos, pos = R - f * H.hpos;
            const int par = pos / H.hpe, idx = pos - par * H.hpe;
            const int sh = idx * H.hmul + par - H.pad;
            const int kc = (lane & 7) ^ hsw(R);  // logical chunk of this slot
            if ((unsigned)sh < (unsigned)H.hsrc) pfo[i] = (f << 20) | ((sh * H.fin + cc * BK + kc * 8) * 2);
        }
    });
    const unsigned ldb = (unsigned)(H.ld * 2);
    auto halo_issue = [&](int ks, int img) {
        char *dst = dsm + img * H.halo_bytes;
        const int tb = H.ts * ((ks * BK) / H.hout) + H.toff + H.dtmin;
        static_for<HPW_MAX>([&](auto I) {
            constexpr int i = decltype(I)::value;
            if (i < H.hpw) {
                const int q = wave + i * WNW;
                const int t = tb + (pfo[i] >> 20);
                const unsigned voff = pfo[i] >= 0 && (unsigned)t < (unsigned)H.T
                                          ? (unsigned)t * ldb + (unsigned)(pfo[i] & 0xFFFFF) : BAD;
                char *d = q < H.npieces ? dst + q * 1024 : dummy;
                lds_dma<16>(rx, d, voff);
            }
        });
    };
    const int lps = H.hpw + SB::NC;  // LDS-DMA loads per thread per K-step

    // per fragment I of this wave: tap and channel base (wave-uniform)
    int ct[TM], cpart[TM];
    const int lp = lane & 3;
    static_for<TM>([&](auto I) {
        const int r = wm * WTM + I * 16;
        const int tap = r >> 6, c0 = r & 63;
        ct[I] = H.ctap[tap];
        cpart[I] = (c0 >> 3) + (lp >> 1);
    });
    const int lo8 = 8 * (lp & 1);
    const int g = lane >> 4, q4 = (lane & 15) >> 2;

    float4v acc[TM][TN];
    static_for<TM>([&](auto I) {
        static_for<TN>([&](auto J) { acc[I][J] = float4v{0.f, 0.f, 0.f, 0.f}; });
    });
    // bias gradient (column sums of dZ): one extra MFMA per column block with an A
    // fragment of ones, on the first wave row of the channel-chunk-0 tiles
    const bool do_bsum = H.bias_slab != nullptr && cc == 0 && wm == 0;
    float4v accb[TN];
    static_for<TN>([&](auto J) { accb[J] = float4v{0.f, 0.f, 0.f, 0.f}; });
    half8 ones;
#pragma unroll
    for (int e = 0; e < 8; ++e) ones[e] = (h16)1.0f;

    static_for<NS - 1>([&](auto I) {
        constexpr int i = decltype(I)::value;
        if (ks0 + i < ks1) {
            halo_issue(ks0 + i, i);
            sb.issue(B, rb, (ks0 + i) * BK, H.mout, bring + i * B_STAGE, wave, lane);
        }
    });
    int st = 0;
    for (int ks = ks0; ks < ks1; ++ks) {
        // stages ks + 1 .. ks + NS - 2 stay in flight; only stage ks is retired
        if (ks + NS - 2 < ks1) wait_vmcnt_rt((NS - 2) * lps);
        else wait_vmcnt<0>();
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        if (ks + NS - 1 < ks1) {
            const int sn = st == 0 ? NS - 1 : st - 1;  // (st + NS - 1) % NS
            halo_issue(ks + NS - 1, sn);
            sb.issue(B, rb, (ks + NS - 1) * BK, H.mout, bring + sn * B_STAGE, wave, lane);
        }
        const char *ta = dsm + st * H.halo_bytes;
        const char *tb = bring + st * B_STAGE;
        // halo row of this lane's output rows (k = 32 s + 8 g + q4, + 4), tap offset 0
        const int r0 = ks * BK - ((ks * BK) / H.hout) * H.hout;  // first row's height
        int base[2][2];
        static_for<2>([&](auto S) {
            static_for<2>([&](auto HI) {
                const int x = r0 + 32 * S + 8 * g + q4 + 4 * HI;
                const int df = (int)(((unsigned)x * H.inv_hout) >> 16);
                base[S][HI] = H.ts * df * H.hpos + (x - df * H.hout);
            });
        });
        static_for<BK / 32>([&](auto S) {
            constexpr int s = decltype(S)::value;
            half8 fa[TM], fb[TN];
            static_for<TM>([&](auto I) {
                short4v v[2];
                static_for<2>([&](auto HI) {
                    const int R = base[s][HI] + ct[I];
                    const int off = (R << 7) + (((cpart[I] ^ hsw(R)) << 4) | lo8);
                    v[HI] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4 *)(ta + off));
                });
                typedef short short8v __attribute__((ext_vector_type(8)));
                short8v x8 = __builtin_shufflevector(v[0], v[1], 0, 1, 2, 3, 4, 5, 6, 7);
                fa[I] = __builtin_bit_cast(half8, x8);
            });
            static_for<TN>([&](auto J) { fb[J] = load_frag<false, BN>(tb, wn * WTN + J * 16, s, lane); });
            static_for<TM>([&](auto I) {
                static_for<TN>([&](auto J) {
                    acc[I][J] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[I], fb[J], acc[I][J], 0, 0, 0);
                });
            });
            if (do_bsum)
                static_for<TN>([&](auto J) {
                    accb[J] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ones, fb[J], accb[J], 0, 0, 0);
                });
        });
        __builtin_amdgcn_sched_barrier(0);
        st = st + 1 == NS ? 0 : st + 1;
    }

    // fp32 partials: tile row (tap, c) is dW row tap * fin + cc * 64 + c
    float *slab = H.slab + (long long)split * H.Mtot * H.N;
    static_for<TM>([&](auto I) {
        const int r = wm * WTM + I * 16;
        const int row0 = (r >> 6) * H.fin + cc * 64 + (r & 63) + 4 * (lane >> 4);
        static_for<TN>([&](auto J) {
            const int n = n0 + wn * WTN + J * 16 + (lane & 15);
            static_for<4>([&](auto EI) {
                if (n < H.N) slab[(long long)(row0 + EI) * H.N + n] = acc[I][J][decltype(EI)::value];
            });
        });
    });
    if (do_bsum && lane < 16)  // every row of accb holds the column sums
        static_for<TN>([&](auto J) {
            const int n = n0 + wn * WTN + J * 16 + lane;
            if (n < H.N) H.bias_slab[(long long)split * H.N + n] = accb[J][0];
        });
}

}  // namespace

// defined in gemm.hip
void kf_wgrad_reduce(const float *slab, const float *bias_slab, int splits, int M, int N, float *dW,
                     long long ldw, float *bias_grad, int accumulate, const float *cs = nullptr);
int kf_prof_start2(int cls, double flops, double bytes);
void kf_prof_stop(int idx);

// Returns 1 when launched, 0 when the operands are not a 3x3 conv im2col pair this
// kernel covers (the caller runs the im2col GEMM), -1 on error.
int kf_conv_wgrad_halo_try(int M, int N, int K, const OpD &a, const OpD &b, float *dW, long long ldw,
                           float *bias_grad, int accumulate) {
    kf_take_pending(__func__);
    if (a.nparts != WTAPS || a.pw % 64 || a.simple || a.edges || a.tclamp || a.hshift ||
        a.hmul < 1 || a.hmul > 2 || a.hout < 2 || a.ncols != WTAPS * a.pw || M != a.ncols ||
        a.nrows != K || !b.simple || b.nrows != K || b.ncols != N || N % 64)
        return 0;
    // 64-column tiles on 4-wave workgroups, two per CU, measured faster than 128-column
    // tiles on 8 waves for every layer (cnn6 1330 -> 1238 us, cnn4 690 -> 640 us)
    int BN = 64;
    int dtmin = 1 << 20, dtmax = -(1 << 20), dhmin = 1 << 20, dhmax = -(1 << 20);
    for (int p = 0; p < WTAPS; ++p) {
        dtmin = std::min(dtmin, a.dt[p]);
        dtmax = std::max(dtmax, a.dt[p]);
        dhmin = std::min(dhmin, a.dh[p]);
        dhmax = std::max(dhmax, a.dh[p]);
    }
    WHalo H;
    memset(&H, 0, sizeof H);
    H.x = a.base;
    H.ld = a.ld;
    H.T = a.T;
    H.hout = a.hout;
    H.hmul = a.hmul;
    H.hsrc = a.hsrc;
    H.fin = a.pw;
    H.pad = std::max(0, -dhmin);
    const int maxshp = (a.hout - 1) * a.hmul + dhmax + H.pad;
    const int HP = std::max(a.hsrc + H.pad, maxshp + 1);
    H.hpe = (HP + a.hmul - 1) / a.hmul;
    H.hpos = H.hpe * a.hmul;
    H.dtmin = dtmin;
    H.ts = a.tmul;
    H.toff = a.t0;
    // frames a 64-row K-step touches (its first row's frame + the rows' span, ts apart) + the
    // time taps
    H.nf = H.ts * ((BK - 1 + a.hout - 1) / a.hout) + 1 + (dtmax - dtmin);
    H.rows = H.nf * H.hpos;
    H.npieces = (H.rows + 7) / 8;
    H.halo_bytes = H.npieces * 1024;
    H.inv_hout = (65536u + a.hout - 1) / a.hout;
    if ((long long)(a.hout + 2 * BK) * a.hout >= 65536) return 0;  // the 16-bit division
    for (int p = 0; p < WTAPS; ++p) {
        const int x = a.dh[p] + H.pad;
        H.ctap[p] = (a.dt[p] - dtmin) * H.hpos + (x % a.hmul) * H.hpe + x / a.hmul;
    }
    H.mout = K;
    // BN = 64: 4-wave workgroups, two per CU; BN = 128: 8 waves, one per CU.
    // Stages: 3 where they fit in LDS, else 2.
    // a halo too large for 4 waves' registers (cnn3: 37 pieces) takes the 8-wave form
    if (BN == 64 && (H.npieces + 3) / 4 > HPW_MAX && N % 128 == 0) BN = 128;
    const int nw = BN == 64 ? 4 : 8;
    H.hpw = (H.npieces + nw - 1) / nw;
    if (H.hpw > HPW_MAX || H.nf >= 2048 || (long long)a.hsrc * a.pw * 2 >= (1 << 20)) return 0;
    const size_t stage = (size_t)H.halo_bytes + (size_t)BN * BK * 2;
    const size_t cap = BN == 64 ? 80 * 1024 : 160 * 1024;  // BN = 64: leave room for 2 per CU
    // (8-wave tiles: 2 stages, measured faster than 3)
    const int ns = BN == 64 && 3 * stage + 1024 <= cap ? 3 : 2;
    const size_t lds = ns * stage + 1024;
    if (lds > 160 * 1024 || (ns - 2) * (H.hpw + BN / 8 / nw) > 15) return 0;
    if (((long long)a.T * a.ld + (long long)a.hsrc * a.pw) * 2 >= (1LL << 32) - 64) return 0;
    H.ctiles = a.pw / 64;
    H.ntiles = N / BN;
    const int tiles = H.ctiles * H.ntiles;
    const int nks = (K + BK - 1) / BK;
    // one workgroup per CU: split the reduction so the grid is about one full wave of CUs
    // (KF_CWGRAD_TARGET: another workgroup target, A/B)
    static const int env_target = getenv("KF_CWGRAD_TARGET") ? atoi(getenv("KF_CWGRAD_TARGET")) : 0;
    const int target = env_target > 0 ? env_target : nw == 4 && lds <= 80 * 1024 ? 512 : 256;
    int splits = std::max(1, (target + tiles - 1) / tiles);
    splits = std::min(splits, std::max(1, nks / 8));
    H.kps = (nks + splits - 1) / splits;
    H.splits = (nks + H.kps - 1) / H.kps;
    H.Mtot = M;
    H.N = N;
    const size_t slab_bytes = (size_t)H.splits * M * N * 4;
    const size_t bias_bytes = bias_grad ? (size_t)H.splits * N * 4 : 0;
    char *ws = (char *)kf_workspace_stream(slab_bytes + bias_bytes + 256);
    if (!ws) {
        kf_report_error("conv wgrad: workspace allocation of %zu bytes failed", slab_bytes + bias_bytes);
        return -1;
    }
    H.slab = (float *)ws;
    H.bias_slab = bias_grad ? (float *)(ws + ((slab_bytes + 255) & ~(size_t)255)) : nullptr;
    const int prof = kf_prof_start2(5, 2.0 * M * N * (double)K,
                                    (double)a.T * a.hsrc * a.pw * 2.0 + (double)K * N * 2.0 + (double)M * N * 4.0);
    const dim3 grid(tiles * H.splits);
    if (BN == 128) {
        if (ns == 3) conv_wgrad_halo_kernel<128, 8, 3><<<grid, 512, lds, kf_stream()>>>(b, H);
        else conv_wgrad_halo_kernel<128, 8, 2><<<grid, 512, lds, kf_stream()>>>(b, H);
    } else {
        if (ns == 3) conv_wgrad_halo_kernel<64, 4, 3><<<grid, 256, lds, kf_stream()>>>(b, H);
        else conv_wgrad_halo_kernel<64, 4, 2><<<grid, 256, lds, kf_stream()>>>(b, H);
    }
    kf_prof_stop(prof);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        kf_report_error("conv wgrad halo launch (M=%d N=%d K=%d): %s", M, N, K, hipGetErrorString(e));
        return -1;
    }
    kf_wgrad_reduce(H.slab, H.bias_slab, H.splits, M, N, dW, ldw, bias_grad, accumulate);
    e = hipGetLastError();
    if (e != hipSuccess) {
        kf_report_error("conv wgrad reduce: %s", hipGetErrorString(e));
        return -1;
    }
    return 1;
}
