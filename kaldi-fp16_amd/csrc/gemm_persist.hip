// gemm_persist.hip — persistent fused GEMM with a resident weight panel, register-streamed
// activations and store waves, for the short-K wide-N products whose epilogue moves more
// bytes than their K loop: the TDNN-F affine forward (K = 2 x 160 -> N = 1536, out + bypass
// residual + ReLU mask), the linear input gradient (K = 2 x 160 -> N = 1536, g + dz + residual
// + input mask) and the output / prefinal products (K = 256), forward.go:589-1001 and
// network_backward.go:336-463 on MI355X.
//
// The tiled kernel (gemm.hip) runs these at ~3 TB/s: every tile restages its weight slab
// and its rows through a two-stage LDS ring whose one step of lookahead cannot cover the
// L2 round trip, and the epilogue's HBM traffic only partly overlaps the next K loop
// (DESIGN.md §10). Here a workgroup owns one 128-column block of the output for the whole
// launch and walks its 128-row tiles:
//   * the weight panel of its columns (K x 128, at most 80 KB) is loaded into LDS once;
//   * 4 MFMA waves (2 x 2, 64 x 64 each) read their A fragments straight from global memory
//     in the MFMA layout (16 bytes per lane = 8 consecutive k of one row), three K steps
//     ahead in registers (96 KB in flight per CU), so the K loop has no barrier and no LDS
//     traffic for A; the fp32 accumulators go to an LDS staging tile;
//   * 4 store waves take the staging tile, apply the whole epilogue (epilogue8's arithmetic
//     and order) and write it while the MFMA waves compute the next tile. vmcnt is per
//     wave, so these stores never sit in front of the operand loads in a counter.
// Per tile both roles pass two barriers: "staging full" and "staging read".
#include <algorithm>

#include "gemm_common.h"

KF_DECLARE_ERR(gp)

namespace {

constexpr int PBM = 128, PBN = 128;          // tile
constexpr int PWM = 2, PWN = 2;              // MFMA waves (64 x 64 each, one per SIMD)
constexpr int PNW = PWM * PWN, PSW = 4;      // MFMA waves, store waves
constexpr int PTHREADS = 64 * (PNW + PSW);
constexpr int PWTM = PBM / PWM, PWTN = PBN / PWN;
constexpr int PTM = PWTM / 16, PTN = PWTN / 16;
constexpr int B_ST = PBN * BK * 2;           // one K step of the weight panel (kc_off image)
constexpr int MAXNK = 5;                     // K <= 320
constexpr int LDS_T = PBN + 4;               // staging row pitch (floats)
constexpr int STG_OFF = MAXNK * B_ST;
constexpr int LDS_BYTES = STG_OFF + PBM * LDS_T * 4;
constexpr int CGS = PBN / 8;                 // 8-column groups per row
constexpr int SROWS = 64 * PSW / CGS;        // rows per store-wave pass
constexpr int SPASS = PBM / SROWS;           // passes per tile
#ifndef KF_PERSIST_ADEPTH
#define KF_PERSIST_ADEPTH 2
#endif
constexpr int ADEPTH = KF_PERSIST_ADEPTH;                    // A K steps in flight per MFMA wave
static_assert(SROWS * CGS == 64 * PSW && SPASS * SROWS == PBM, "store-wave coverage");
static_assert(LDS_BYTES <= 160 * 1024, "LDS");

struct PersistArgs {
    int M, N, K;
    int mt, nt;          // M / N tiles
    int groups;          // workgroups per column block
};

typedef unsigned u4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t brs(const void *p) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)0x7FFFFFFF, 0x00020000);
}

template <int AM, int BMD, int NK>
__global__ __launch_bounds__(PTHREADS, 1) void gemm_persist_kernel(OpD A, OpD B, KfEpilogue E, PersistArgs P) {
    using SB = Stager<true, PBN, BMD, PNW>;
    static_assert(SB::EVEN, "uniform loads per MFMA wave");
    static_assert(NK >= 1 && NK <= MAXNK, "K steps");
    __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
    float *stg = reinterpret_cast<float *>(smem + STG_OFF);

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool mw = wave < PNW;  // MFMA wave (uniform)

    // column block nt = blockIdx % nt, rows every groups-th M tile from blockIdx / nt
    const int nt = blockIdx.x % P.nt, slot = blockIdx.x / P.nt;
    if (slot >= P.groups) return;  // the few workgroups past groups * nt (whole workgroup)
    const int n0 = nt * PBN;
    const int my = P.mt > slot ? (P.mt - slot + P.groups - 1) / P.groups : 0;
    auto m0_of = [&](int i) { return (slot + i * P.groups) * PBM; };

    // the weight panel, once: MFMA waves issue it, every wave waits at the barrier
    if (mw) {
        SB sb;
        sb.init(B, n0, wave, lane);
        const Rsrc rb = make_rsrc(B.base);
#pragma unroll
        for (int kk = 0; kk < NK; ++kk) sb.issue(B, rb, kk * BK, P.K, smem + kk * B_ST, wave, lane);
        wait_vmcnt<0>();
    }
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);

    if (mw) {
        const int wm = wave / PWN, wn = wave % PWN;
        const __amdgpu_buffer_rsrc_t ra = brs(A.base);
        // per fragment row I and part p: the byte offset of this lane's row (BAD: zeros),
        // for the tile being prefetched
        unsigned ab[PTM][2];
        int ab_tile = -1;
        auto set_rows = [&](int i) {
            const int m0 = m0_of(i);
            static_for<PTM>([&](auto I) {
                const int r = m0 + wm * PWTM + I * 16 + (lane & 15);
                const bool ok = r < A.nrows;
                if constexpr (AM == OP_SIMPLE) {
                    ab[I][0] = ok ? (unsigned)((long long)r * A.ld * 2) : BAD;
                    ab[I][1] = BAD;
                } else {
                    ab[I][0] = ok ? op_boff(A, r, 0, 0, A.dt[0], A.dh[0], A.et[0], A.er[0]) : BAD;
                    ab[I][1] = ok && A.nparts > 1 ? op_boff(A, r, 0, 0, A.dt[1], A.dh[1], A.et[1], A.er[1]) : BAD;
                }
            });
            ab_tile = i;
        };
        half8 abuf[ADEPTH][PTM][2];
        // A fragments of K step kk of tile i into ring slot SL
        auto load_step = [&](auto SL, int i, int kk) {
            constexpr int sl = decltype(SL)::value;
            if (i >= my) return;
            if (i != ab_tile) set_rows(i);
            static_for<2>([&](auto S) {
                constexpr int s = decltype(S)::value;
                const int k = kk * BK + s * 32 + 8 * (lane >> 4);  // this lane's 8 k
                const bool p1 = AM != OP_SIMPLE && k >= A.pw;
                const unsigned kb = (unsigned)((p1 ? k - A.pw : k) * 2);
                static_for<PTM>([&](auto I) {
                    const unsigned base = p1 ? ab[I][1] : ab[I][0];
                    const unsigned off = (base == BAD || k >= P.K) ? BAD : base + kb;
                    abuf[sl][I][s] = __builtin_bit_cast(half8, __builtin_amdgcn_raw_buffer_load_b128(ra, off, 0, 0));
                });
            });
        };
        float4v acc[PTM][PTN];
        static_for<PTM>([&](auto I) {
            static_for<PTN>([&](auto J) { acc[I][J] = float4v{0.f, 0.f, 0.f, 0.f}; });
        });
        // prologue: global steps 0 .. ADEPTH - 1 (tiles 0, 1 when NK < ADEPTH)
        static_for<ADEPTH>([&](auto G) {
            constexpr int g = decltype(G)::value;
            load_step(std::integral_constant<int, g % ADEPTH>{}, g / NK, g % NK);
        });
        // ADEPTH tiles per iteration, so the ring slot of step j of an iteration is j % ADEPTH
        for (int it = 0; it * ADEPTH < my; ++it) {
            static_for<ADEPTH * NK>([&](auto J) {
                constexpr int j = decltype(J)::value, t3 = j / NK, kk = j % NK, sl = j % ADEPTH;
                const int i = it * ADEPTH + t3;
                if (i >= my) return;
                const char *tb = smem + kk * B_ST;
                static_for<2>([&](auto S) {
                    constexpr int s = decltype(S)::value;
                    half8 fb[PTN];
                    static_for<PTN>([&](auto Jn) { fb[Jn] = load_frag<true, PBN>(tb, wn * PWTN + Jn * 16, s, lane); });
                    static_for<PTM>([&](auto I) {
                        static_for<PTN>([&](auto Jn) {
                            acc[I][Jn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(abuf[sl][I][s], fb[Jn], acc[I][Jn], 0, 0, 0);
                        });
                    });
                });
                // the slot is free again: step j + ADEPTH (possibly of the next iteration)
                constexpr int jn = j + ADEPTH;
                load_step(std::integral_constant<int, sl>{}, it * ADEPTH + jn / NK, jn % NK);
                if constexpr (kk == NK - 1) {
                    if (i > 0) __builtin_amdgcn_s_barrier();  // staging read (tile i - 1)
                    static_for<PTM>([&](auto I) {
                        static_for<PTN>([&](auto Jn) {
                            const int c = wn * PWTN + Jn * 16 + (lane & 15);
                            static_for<4>([&](auto EI) {
                                const int r = wm * PWTM + I * 16 + 4 * (lane >> 4) + EI;
                                stg[r * LDS_T + c] = acc[I][Jn][decltype(EI)::value];
                            });
                            acc[I][Jn] = float4v{0.f, 0.f, 0.f, 0.f};
                        });
                    });
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    __builtin_amdgcn_s_barrier();  // staging full (tile i)
                    __builtin_amdgcn_sched_barrier(0);
                }
            });
        }
        if (my > 0) __builtin_amdgcn_s_barrier();  // staging read (the last tile)
        return;
    }

    // ---- store waves
    const int sl = tid - 64 * PNW, cg = sl % CGS, r0 = sl / CGS;  // store lane: column group, first row
    const int n = n0 + 8 * cg;
    const bool ncol = n < P.N;
    float pb[8], ps[8], psh[8], ps2[8];  // per-column parameters (fixed for the launch)
#pragma unroll
    for (int e = 0; e < 8; ++e) pb[e] = 0.f, ps[e] = 0.f, psh[e] = 0.f, ps2[e] = 1.f;
    if (ncol) {
        if (E.bias) {
            const half8 b = __builtin_bit_cast(half8, __builtin_amdgcn_raw_buffer_load_b128(brs(E.bias), n * 2, 0, 0));
#pragma unroll
            for (int e = 0; e < 8; ++e) pb[e] = (float)b[e];
        }
        auto ld8 = [&](const float *p, float (&d)[8]) {
            const __amdgpu_buffer_rsrc_t r = brs(p);
            const float4v a = __builtin_bit_cast(float4v, __builtin_amdgcn_raw_buffer_load_b128(r, n * 4, 0, 0));
            const float4v b = __builtin_bit_cast(float4v, __builtin_amdgcn_raw_buffer_load_b128(r, n * 4 + 16, 0, 0));
#pragma unroll
            for (int e = 0; e < 4; ++e) d[e] = a[e], d[e + 4] = b[e];
        };
        if (E.scale) {
            ld8(E.scale, ps);
            ld8(E.shift, psh);
        }
        if (E.scale2) ld8(E.scale2, ps2);
    }
    half8 sres[SPASS];
    unsigned smk[SPASS];
    // residual / input-mask rows of tile i (store waves address every tensor through a
    // buffer resource and a 32-bit byte offset, host-checked)
    auto store_load = [&](int i) {
        const int m0 = m0_of(i);
        const __amdgpu_buffer_rsrc_t rr = brs(E.resid), rm = brs(E.mask_in);
        static_for<SPASS>([&](auto R) {
            constexpr int rp = decltype(R)::value;
            const int m = m0 + r0 + rp * SROWS;
            const bool live = ncol && m < P.M;
            sres[rp] = half8{};
            smk[rp] = 0xFFu;
            if (live && E.resid)
                sres[rp] = __builtin_bit_cast(
                    half8, __builtin_amdgcn_raw_buffer_load_b128(rr, (unsigned)(((long long)m * E.ldr + n) * 2), 0, 0));
            if (live && E.mask_in)
                smk[rp] = __builtin_amdgcn_raw_buffer_load_b8(rm, (unsigned)(((long long)m * E.ldo2 + n) >> 3), 0, 0);
        });
    };
    if (my > 0) store_load(0);
    const __amdgpu_buffer_rsrc_t ro = brs(E.out), ro2 = brs(E.out2), rmo = brs(E.mask_out);
    for (int i = 0; i < my; ++i) {
        __builtin_amdgcn_s_barrier();  // staging full (tile i)
        __builtin_amdgcn_sched_barrier(0);
        float hv[SPASS][8];
        static_for<SPASS>([&](auto R) {
            constexpr int rp = decltype(R)::value;
            const float *src = stg + (r0 + rp * SROWS) * LDS_T + 8 * cg;
            const float4v x0 = *reinterpret_cast<const float4v *>(src);
            const float4v x1 = *reinterpret_cast<const float4v *>(src + 4);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                hv[rp][e] = x0[e];
                hv[rp][e + 4] = x1[e];
            }
        });
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();  // staging read (tile i)
        __builtin_amdgcn_sched_barrier(0);
        wait_vmcnt<0>();  // tile i's residual / mask rows (issued a tile ago)
        const int m0 = m0_of(i);
        if (ncol)
            static_for<SPASS>([&](auto R) {  // epilogue8's arithmetic and order
                constexpr int rp = decltype(R)::value;
                const int m = m0 + r0 + rp * SROWS;
                if (m >= P.M) return;
                float v[8];
#pragma unroll
                for (int e = 0; e < 8; ++e) v[e] = hv[rp][e] * E.alpha;
                if (E.bias) {
#pragma unroll
                    for (int e = 0; e < 8; ++e) v[e] += pb[e];
                }
                if (E.relu) {
                    unsigned bits = 0;
#pragma unroll
                    for (int e = 0; e < 8; ++e) {
                        if (v[e] > 0.f) bits |= 1u << e;
                        else v[e] = 0.f;
                    }
                    if (E.mask_out)
                        __builtin_amdgcn_raw_buffer_store_b8((unsigned char)bits, rmo,
                                                             (unsigned)(((long long)m * E.ldo + n) >> 3), 0, 0);
                }
                if (E.scale) {
#pragma unroll
                    for (int e = 0; e < 8; ++e) v[e] = fmaf(v[e], ps[e], psh[e]);
                }
                if (E.resid) {
#pragma unroll
                    for (int e = 0; e < 8; ++e) v[e] = fmaf(E.resid_alpha, (float)sres[rp][e], v[e]);
                }
                if (E.out) {
                    half8 o;
#pragma unroll
                    for (int e = 0; e < 8; ++e) o[e] = f2h(v[e]);
                    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, o), ro,
                                                           (unsigned)(((long long)m * E.ldo + n) * 2), 0, 0);
                }
                if (E.out2) {
                    half8 o;
#pragma unroll
                    for (int e = 0; e < 8; ++e) {
                        float w = v[e];
                        if (E.scale2) w *= ps2[e];
                        if (E.mask_in && !((smk[rp] >> e) & 1u)) w = 0.f;
                        o[e] = f2h(w);
                    }
                    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, o), ro2,
                                                           (unsigned)(((long long)m * E.ldo2 + n) * 2), 0, 0);
                }
            });
        if (i + 1 < my) store_load(i + 1);
    }
}

}  // namespace

double kf_gemm_alg_bytes(const OpD &a, const OpD &b, const KfEpilogue &E, long long M, long long N);
int kf_prof_start2(int cls, double flops, double bytes);
void kf_prof_stop(int idx);
// compute units of the current device (one persistent workgroup each), cached per device
static int device_cus() {
    static int cached[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (!cached[dev]) {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
        cached[dev] = cus;
    }
    return cached[dev];
}

static int g_persist = 0;
// test / A-B hook (kf_ops.h): 1 takes the persistent kernel where it applies, 0 sends every
// fused GEMM to the tiled kernel; returns the previous setting
extern "C" int kf_gemm_debug_persist(int on) {
    const int prev = g_persist;
    g_persist = on != 0;
    return prev;
}

template <int AM, int BMD>
static void launch_persist(int nk, int grid, const OpD &a, const OpD &b, const KfEpilogue &E, const PersistArgs &P) {
    switch (nk) {
        case 3: gemm_persist_kernel<AM, BMD, 3><<<grid, PTHREADS, 0, kf_stream()>>>(a, b, E, P); break;
        case 4: gemm_persist_kernel<AM, BMD, 4><<<grid, PTHREADS, 0, kf_stream()>>>(a, b, E, P); break;
        default: gemm_persist_kernel<AM, BMD, 5><<<grid, PTHREADS, 0, kf_stream()>>>(a, b, E, P); break;
    }
}

// Returns 1 when launched, 0 when not applicable (the caller runs the tiled kernel), -1 on
// error. Taken for fp16 k-contiguous operands (A plain or a two-part time splice; B plain or
// op_wrows' two shifted parts) with K = 192, 256 or 320, N a multiple of 128, at least 1024
// tiles, beta = 0 and no MXFP8 copy.
int kf_gemm_persist_try(int M, int N, int K, const OpD &a, const OpD &b, int am, int bm, const KfEpilogue &E) {
    if (!g_persist || E.out8 || E.beta != 0.f) return 0;
    if ((am != OP_SIMPLE && am != OP_P2) || (bm != OP_SIMPLE && bm != OP_P2)) return 0;
    if (N % PBN || (K != 192 && K != 256 && K != 320)) return 0;
    if (am == OP_P2 && a.pw % 8) return 0;
    // the store waves' and the A loads' 32-bit byte offsets (buffer resources of 2^31 - 1 bytes)
    const long long lim = 0x7FFFFFF0LL;
    if ((E.out && ((long long)M * E.ldo * 2 >= lim)) || (E.out2 && (long long)M * E.ldo2 * 2 >= lim) ||
        (E.resid && (long long)M * E.ldr * 2 >= lim) || ((long long)(a.T + 2) * a.ld * 2 >= lim))
        return 0;
    const long long mt = (M + PBM - 1) / PBM, nt = N / PBN;
    if (mt * nt < 1024 || mt >= (1LL << 30)) return 0;
    const int cus = device_cus();
    const int groups = (int)std::max<long long>(1, cus / nt);
    PersistArgs P{M, N, K, (int)mt, (int)nt, groups};
    const int grid = (int)(groups * nt);
    const int prof = kf_prof_start2(0, 2.0 * M * N * (double)K, kf_gemm_alg_bytes(a, b, E, M, N));
    const int nk = K / BK;
    if (am == OP_SIMPLE && bm == OP_SIMPLE) launch_persist<OP_SIMPLE, OP_SIMPLE>(nk, grid, a, b, E, P);
    else if (am == OP_SIMPLE) launch_persist<OP_SIMPLE, OP_P2>(nk, grid, a, b, E, P);
    else if (bm == OP_SIMPLE) launch_persist<OP_P2, OP_SIMPLE>(nk, grid, a, b, E, P);
    else launch_persist<OP_P2, OP_P2>(nk, grid, a, b, E, P);
    kf_prof_stop(prof);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        kf_report_error("persistent gemm launch (M=%d N=%d K=%d): %s", M, N, K, hipGetErrorString(e));
        return -1;
    }
    return 1;
}
