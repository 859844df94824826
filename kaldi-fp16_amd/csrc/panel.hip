// panel.hip — short-reduction, wide-output fused GEMMs with the A panel resident in LDS.
//
// The TDNN-F affine forward (K = 2 x 160, N = 1536) and the linear layer's input
// gradient (K = 2 x 160, N = 1536) — the reference's cublasGemmEx plus ~12 small
// kernels per layer (internal/nnet/forward.go:589-695, network_backward.go:336-463) —
// move 2-3 full-width fp16 tensors through the epilogue but only a 320-wide A row per
// output row: HBM-bound by the epilogue, with ~1/10 of the tile time in MFMA. The
// tiled gemm_kernel re-stages A and B for every 192 x 128 tile through a 2-stage ring
// and waits an L2 round trip per K-step; here one workgroup owns 128 output rows:
//   * the A panel (128 x K, K <= 512, spliced rows resolved by the LDS-DMA stager) is
//     loaded into LDS once, then every wave works on its own 32-column blocks with no
//     workgroup barrier: its epilogue overlaps the other waves' MFMA;
//   * B fragments come straight from global memory (16-byte loads of B^T rows, which
//     the host supplies k-contiguous: weights stay L2-resident, 1 MB per layer),
//     prefetched PD K-steps ahead in registers, the next block's first steps during
//     the current block's epilogue;
//   * the MFMAs produce C^T blocks (B^T fragment as the first operand), so each lane
//     holds 4 consecutive columns of one row: the epilogue (bias / ReLU + mask / BN /
//     bypass / second output, kf_ops.h) runs on the accumulators in place with 8-byte
//     stores and no LDS staging; the ReLU mask byte joins two lanes' nibbles; the
//     block's residual and input-mask bytes are prefetched while its MFMAs run.
#include "gemm_common.h"

namespace {

constexpr int PBM = 128;          // rows per workgroup panel
constexpr int PNW = 8;            // waves
constexpr int PWM = 64;           // rows per wave tile
constexpr int PWN = 64;           // columns per wave tile (128 bytes of an output row)
constexpr int PSTG = PWN + 4;     // epilogue staging row stride (floats)
constexpr int PD = 2;             // B prefetch depth (K-steps of 32)
constexpr int PCHUNK = PBM * BK * 2;  // one 64-column A image, 16 KB

}  // namespace

// KS = K / 32 reduction steps (K = 32 * KS <= 512)
template <int KS, int AM>
__global__ __launch_bounds__(64 * PNW, 1) void panel_kernel(int M, int N, OpD A, PanelB B, KfEpilogue E, int dbg,
                                                            int stagger) {
    extern __shared__ __attribute__((aligned(16))) char dsm[];
    constexpr int NCH = (KS + 1) / 2;  // 64-column A images
    constexpr int K = 32 * KS;
    constexpr int TI = PWM / 16, TJ = PWN / 16;  // 16 x 16 MFMA blocks per wave tile
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int m0 = blockIdx.x * PBM;

    // ---- the A panel: NCH images of [128][64] halves (kc_off layout), once
    {
        Stager<true, PBM, AM, PNW> sa;
        sa.init(A, m0, wave, lane);
        const __amdgpu_buffer_rsrc_t ra = make_rsrc(A.base);
        static_for<NCH>([&](auto C) {
            constexpr int c = decltype(C)::value;
            sa.issue(A, ra, c * BK, K, dsm + c * PCHUNK, wave, lane);
        });
    }
    float *stg = reinterpret_cast<float *>(dsm + NCH * PCHUNK) + wave * 16 * PSTG;

    // wave tiles: PBM / PWM row slices x N / PWN column blocks; a wave keeps one row slice
    const int nslice = PBM / PWM, nblk = (N / PWN) * nslice;
    const int rs = wave % nslice;  // (PNW is a multiple of nslice)
    int b = wave;
    // B^T fragment pointer: column block cb, fragment J, K-step q
    auto bptr = [&](int blk, int J, int q) -> const h16 * {
        if (dbg & 1) blk = 0, q = 0;
        const int k = 32 * q;
        const int p = B.nparts > 1 && k >= B.pw ? 1 : 0;
        const int n = (blk / nslice) * PWN + J * 16 + (lane & 15);
        return B.base + (long long)(n + B.roff[p]) * B.ld + (k - p * B.pw) + 8 * (lane >> 4);
    };
    half8 pre[PD][TJ];
    if (b < nblk) {
        static_for<PD>([&](auto Q) {
            constexpr int q = decltype(Q)::value;
            if constexpr (q < KS) static_for<TJ>([&](auto J) { pre[q][J] = load_h8(bptr(b, J, q)); });
        });
    }
    wait_vmcnt<0>();
    __syncthreads();  // the A panel has landed (every wave's LDS-DMA)
    // waves 4-7 (the second wave on each SIMD) may start later (KF_PANEL_STAGGER), so the
    // two waves of a SIMD alternate MFMA and epilogue phases
    if (wave >= PNW / 2 && stagger > 0)
        for (int i = 0; i < stagger; ++i) __builtin_amdgcn_s_sleep(127);

    // Output C^T per 16 x 16 MFMA block (the B^T fragment is the first operand): lane l
    // holds row m = 16 I + (l & 15), columns n = 16 J + 4 (l >> 4) + e, e = 0..3, so a
    // 16-row group stages through LDS with one ds_write_b128 per block, and the epilogue
    // reads 8 consecutive columns per lane: row r = l >> 3 (+ 8), columns 8 (l & 7).
    const int er = lane >> 3, ec = 8 * (lane & 7);
    for (; b < nblk; b += PNW) {
        const int n0 = (b / nslice) * PWN;
        int ne = n0 + ec;                  // this lane's 8 epilogue columns
        int mrow = m0 + rs * PWM + er;     // this lane's epilogue row in group 0, half 0
        // opaque per block: otherwise the 64-bit row addresses are hoisted out of the
        // block loop for every group and epilogue tensor and spill
        asm volatile("" : "+v"(mrow), "+v"(ne));
        // the block's row operands, in flight during the MFMAs
        half8 rres[TI][2];
        unsigned mb[TI][2];
        static_for<TI>([&](auto I) {
            static_for<2>([&](auto H) {
                const int m = mrow + 16 * I + 8 * H;
                rres[I][H] = half8{};
                mb[I][H] = 0xFFu;
                if (m < M) {
                    if (E.resid) rres[I][H] = load_h8((const h16 *)E.resid + (long long)m * E.ldr + ne);
                    if (E.mask_in) mb[I][H] = E.mask_in[((long long)m * E.ldo2 + ne) >> 3];
                }
            });
        });
        float4v acc[TI][TJ];
        static_for<TI>([&](auto I) {
            static_for<TJ>([&](auto J) { acc[I][J] = float4v{0.f, 0.f, 0.f, 0.f}; });
        });
        half8 fb[KS][TJ];
        static_for<PD>([&](auto Q) {
            constexpr int q = decltype(Q)::value;
            if constexpr (q < KS) static_for<TJ>([&](auto J) { fb[q][J] = pre[q][J]; });
        });
        static_for<KS>([&](auto Q) {
            constexpr int q = decltype(Q)::value;
            if constexpr (q + PD < KS)
                static_for<TJ>([&](auto J) { fb[q + PD][J] = load_h8(bptr(b, J, q + PD)); });
            const char *img = dsm + (q / 2) * PCHUNK;
            half8 fa[TI];
            static_for<TI>([&](auto I) { fa[I] = load_frag<true, PBM>(img, rs * PWM + I * 16, q & 1, lane); });
            static_for<TI>([&](auto I) {
                static_for<TJ>([&](auto J) {
                    acc[I][J] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fb[q][J], fa[I], acc[I][J], 0, 0, 0);
                });
            });
        });
        // the next block's first K-steps load during this block's epilogue
        const int bn = b + PNW;
        if (bn < nblk) {
            static_for<PD>([&](auto Q) {
                constexpr int q = decltype(Q)::value;
                if constexpr (q < KS) static_for<TJ>([&](auto J) { pre[q][J] = load_h8(bptr(bn, J, q)); });
            });
        }
        if (dbg & 2) {
            if (lane == 0 && acc[0][0][0] == 12345.f) ((float *)E.out)[b] = acc[TI - 1][TJ - 1][3];
            continue;
        }
        // per-column parameters of this lane's 8 columns (LDS slots of epilogue8: local 0..7)
        float bias[8], scale[8], shift[8], scale2[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            bias[e] = 0.f;
            scale[e] = 0.f;
            shift[e] = 0.f;
            scale2[e] = 1.f;
        }
        if (E.bias) {
            const half8 bv = load_h8((const h16 *)E.bias + ne);
#pragma unroll
            for (int e = 0; e < 8; ++e) bias[e] = (float)bv[e];
        }
        if (E.scale) {
            const float4v s0 = *reinterpret_cast<const float4v *>(E.scale + ne);
            const float4v s1 = *reinterpret_cast<const float4v *>(E.scale + ne + 4);
            const float4v h0 = *reinterpret_cast<const float4v *>(E.shift + ne);
            const float4v h1 = *reinterpret_cast<const float4v *>(E.shift + ne + 4);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                scale[e] = s0[e], scale[e + 4] = s1[e];
                shift[e] = h0[e], shift[e + 4] = h1[e];
            }
        }
        if (E.scale2) {
            const float4v s0 = *reinterpret_cast<const float4v *>(E.scale2 + ne);
            const float4v s1 = *reinterpret_cast<const float4v *>(E.scale2 + ne + 4);
#pragma unroll
            for (int e = 0; e < 4; ++e) scale2[e] = s0[e], scale2[e + 4] = s1[e];
        }
        const EpiCols P{bias, scale, shift, scale2};
        static_for<TI>([&](auto I) {
            // stage the 16 x PWN group: one 16-byte write per MFMA block
            static_for<TJ>([&](auto J) {
                *reinterpret_cast<float4v *>(stg + (lane & 15) * PSTG + 16 * J + 4 * (lane >> 4)) = acc[I][J];
            });
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            float4v x[2][2];
            static_for<2>([&](auto H) {
                x[H][0] = *reinterpret_cast<const float4v *>(stg + (er + 8 * H) * PSTG + ec);
                x[H][1] = *reinterpret_cast<const float4v *>(stg + (er + 8 * H) * PSTG + ec + 4);
            });
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            static_for<2>([&](auto H) {
                const int m = mrow + 16 * I + 8 * H;
                if (m < M) {
                    float v[8];
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        v[e] = x[H][0][e];
                        v[e + 4] = x[H][1][e];
                    }
                    epilogue8(E, P, m, ne, 0, v, half8{}, rres[I][H], mb[I][H]);
                }
            });
            __builtin_amdgcn_sched_barrier(0);
        });
    }
}

// KF_PANEL=0 disables the panel kernel (A/B); kf_gemm_debug_panel overrides it (tests)
static int g_panel_override = -1;
extern "C" void kf_gemm_debug_panel(int mode) { g_panel_override = mode < 0 ? -1 : (mode != 0); }
extern "C" int kf_panel_enabled(void) {
    // off by default: on the MI355X the tiled gemm_kernel with k-contiguous (transposed)
    // weights was as fast or faster for every TDNN-F shape measured
    static const int env = getenv("KF_PANEL") ? atoi(getenv("KF_PANEL")) : 0;
    return g_panel_override >= 0 ? g_panel_override : env != 0;
}

bool kf_panel_ok(int M, int N, int K, const OpD &a, const OpD &b, bool bkc, const KfEpilogue &E, PanelB *pb) {
    if (!kf_panel_enabled() || M <= 0 || !bkc || K > 512 || K % 32 || N % PWN || E.beta != 0.f || E.out8 || a.sc || b.sc)
        return false;
    switch (K / 32) {
        case 2: case 4: case 5: case 8: case 10: break;  // the instantiated reductions
        default: return false;
    }
    if (!a.simple && !(a.nparts <= 2 && a.hout == 1 && a.hmul == 0 && a.hshift == 0)) return false;  // OP_P2
    if (a.ncols != K || b.nrows < N) return false;
    memset(pb, 0, sizeof *pb);
    pb->base = b.base;
    pb->ld = b.ld;
    if (b.simple) {
        pb->nparts = 1;
        pb->pw = K;
        return b.ncols == K;
    }
    // op_wrows: part p = rows [dt_p, dt_p + N) of a plain matrix, all inside it
    if (b.nparts > 2 || b.hout != 1 || b.hmul != 0 || b.hshift || b.edges || b.pw % 32 || b.nparts * b.pw != K)
        return false;
    for (int p = 0; p < b.nparts; ++p) {
        if (b.dt[p] < 0 || b.dt[p] + N > b.T || b.dh[p] != 0) return false;
        pb->roff[p] = b.dt[p];
    }
    pb->nparts = b.nparts;
    pb->pw = b.pw;
    return true;
}

int kf_panel_launch(int M, int N, int K, const OpD &a, const PanelB &pb, const KfEpilogue &E) {
    const int nch = (K / 32 + 1) / 2;
    const size_t lds = (size_t)nch * PCHUNK + (size_t)PNW * 16 * PSTG * 4;
    const dim3 grid((M + PBM - 1) / PBM);
    const bool p2 = !a.simple;
    static const int dbg = getenv("KF_PANEL_DBG") ? atoi(getenv("KF_PANEL_DBG")) : 0;
    // s_sleep(127) units (~8k cycles each) by which waves 4-7 start late
    static const int stagger = getenv("KF_PANEL_STAGGER") ? atoi(getenv("KF_PANEL_STAGGER")) : 0;
#define KF_PANEL_L(KS_)                                                                              \
    case KS_:                                                                                         \
        if (p2)                                                                                       \
            panel_kernel<KS_, OP_P2><<<grid, 64 * PNW, lds, kf_stream()>>>(M, N, a, pb, E, dbg, stagger);            \
        else                                                                                          \
            panel_kernel<KS_, OP_SIMPLE><<<grid, 64 * PNW, lds, kf_stream()>>>(M, N, a, pb, E, dbg, stagger);        \
        break;
    switch (K / 32) {
        KF_PANEL_L(2)
        KF_PANEL_L(4)
        KF_PANEL_L(5)
        KF_PANEL_L(8)
        KF_PANEL_L(10)
        default:
            kf_report_error("panel: K=%d not instantiated", K);
            return -1;
    }
#undef KF_PANEL_L
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        kf_report_error("panel launch (M=%d N=%d K=%d): %s", M, N, K, hipGetErrorString(e));
        return -1;
    }
    return 0;
}
