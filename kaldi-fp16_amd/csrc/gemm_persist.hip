// gemm_persist.hip — persistent fused GEMM with store waves, for the short-K, wide-N
// products whose epilogue moves more bytes than the K loop reads: the TDNN-F affine forward
// (K = 2 x 160 -> N = 1536: out + bypass residual + ReLU mask) and the linear input gradient
// (K = 2 x 160 -> N = 1536: g + dz + residual + input mask), forward.go:589-695 and
// network_backward.go:336-463 on MI355X.
//
// The tiled kernel (gemm.hip) runs these at ~3 TB/s: a tile's K loop is L2-latency bound
// while its epilogue saturates the CU's HBM share, and the two co-resident workgroups
// overlap the phases only partly. Here one workgroup per CU walks its tiles
// with two roles:
//   * 4 MFMA waves (2 x 2, 64 x 64 each, one per SIMD) run the 128 x 128 tile's K loop through a
//     two-stage LDS-DMA ring that continues across tile boundaries (the next tile's first
//     stage is issued during the current tile's last step), then write the fp32
//     accumulators to an LDS staging tile;
//   * 4 store waves take the staging tile, apply the whole epilogue (bias, ReLU + mask,
//     BatchNorm scale / shift, residual, out, out2 with scale2 x mask_in — epilogue8's
//     arithmetic and order) and write it while the MFMA waves compute the next tile.
// vmcnt is per wave, so the stores never sit in front of the operand loads in a counter.
// Every wave passes the same barriers: per tile, one per K step and one "staging full".
// The store waves read the staging tile between "staging full" and the next K-step
// barrier, before the MFMA waves can write it again.
#include "gemm_common.h"

KF_DECLARE_ERR(gp)

namespace {

constexpr int PBM = 128, PBN = 128;          // tile
constexpr int PWM = 2, PWN = 2;              // MFMA waves (64 x 64 each)
constexpr int PNW = PWM * PWN, PSW = 4;      // MFMA waves, store waves
constexpr int PTHREADS = 64 * (PNW + PSW);
constexpr int PWTM = PBM / PWM, PWTN = PBN / PWN;
constexpr int PTM = PWTM / 16, PTN = PWTN / 16;
constexpr int A_ST = PBM * BK * 2, B_ST = PBN * BK * 2, STAGE = A_ST + B_ST;
constexpr int NSTG = 3;                      // operand ring stages (two in flight)
constexpr int LDS_T = PBN + 4;               // staging row pitch (floats)
constexpr int HROWS = PBM / PWM;             // staging holds one wave row (64 rows) at a time
constexpr int STG_OFF = NSTG * STAGE;
constexpr int LDS_BYTES = STG_OFF + HROWS * LDS_T * 4;
constexpr int CGS = PBN / 8;                 // 8-column groups per row
constexpr int SROWS = 64 * PSW / CGS;        // rows per store-wave pass
constexpr int SPASS = PBM / SROWS;           // passes per tile
constexpr int HPASS = HROWS / SROWS;         // passes per staged half
static_assert(SROWS * CGS == 64 * PSW && SPASS * SROWS == PBM && HPASS * PWM == SPASS, "store-wave coverage");
static_assert(LDS_BYTES <= 160 * 1024, "LDS");

struct PersistArgs {
    int M, N, K;
    int mt, nt;          // M / N tiles
    int ntiles;
    unsigned long long *trace;  // diagnostics (kf_gemm_persist_trace): block 0's barrier stamps, or null
};

template <int AM>
__global__ __launch_bounds__(PTHREADS, 1) void gemm_persist_kernel(OpD A, OpD B, KfEpilogue E, PersistArgs P) {
    using SA = Stager<true, PBM, AM, PNW>;
    using SB = Stager<true, PBN, OP_SIMPLE, PNW>;
    static_assert(SA::EVEN && SB::EVEN, "uniform loads per MFMA wave");
    __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
    float *stg = reinterpret_cast<float *>(smem + STG_OFF);

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool mw = wave < PNW;  // MFMA wave (uniform)
    const int wm = wave / PWN, wn = wave % PWN;

    // this workgroup's tiles: XCD x = blockIdx % 8 owns the contiguous tile range
    // [x * q, ...) (the N tiles of an M tile are consecutive, so their A rows meet in one
    // L2); its workgroups take every (G / 8)-th tile of it
    const int G = gridDim.x, xcd = blockIdx.x % 8, loc = blockIdx.x / 8;
    const int gx = G / 8 + (xcd < G % 8 ? 1 : 0);
    const int q = P.ntiles / 8, rmd = P.ntiles % 8;
    const int t0 = xcd < rmd ? xcd * (q + 1) : rmd * (q + 1) + (xcd - rmd) * q;
    const int tcount = q + (xcd < rmd ? 1 : 0);
    const int my = tcount > loc ? (tcount - loc + gx - 1) / gx : 0;  // tiles of this workgroup
    auto tile_of = [&](int i) { return t0 + loc + i * gx; };

    const int nk = (P.K + BK - 1) / BK;
    const Rsrc ra = make_rsrc(A.base), rb = make_rsrc(B.base);
    SA sa;
    SB sb;
    int cur_m0 = -1, cur_n0 = -1;
    // MFMA waves: the loads of step k of my tile i into `stage` (plain statements, not a
    // lambda: a lambda makes the stagers' offset arrays address-taken, i.e. scratch)
#define GP_ISSUE(i_, k_, stage_)                                                  \
    do {                                                                          \
        const int t_ = tile_of(i_), m0_ = (t_ / P.nt) * PBM, n0_ = (t_ % P.nt) * PBN; \
        if (m0_ != cur_m0) {                                                      \
            sa.init(A, m0_, wave, lane);                                          \
            cur_m0 = m0_;                                                         \
        }                                                                         \
        if (n0_ != cur_n0) {                                                      \
            sb.init(B, n0_, wave, lane);                                          \
            cur_n0 = n0_;                                                         \
        }                                                                         \
        char *base_ = smem + (stage_) * STAGE;                                    \
        sa.issue(A, ra, (k_) * BK, P.K, base_, wave, lane);                       \
        sb.issue(B, rb, (k_) * BK, P.K, base_ + A_ST, wave, lane);                \
    } while (0)

    float4v acc[PTM][PTN];
    // store waves: the residual / input-mask rows of the staged tile
    const int sl = tid - 64 * PNW, cg = sl % CGS, r0 = sl / CGS;  // store lane: column group, first row
    half8 sres[SPASS];
    unsigned smk[SPASS];
    int s_m0 = 0, s_n0 = 0;

    // store waves address every tensor through a buffer resource and a 32-bit byte offset
    // (host-checked), so no 64-bit address is kept per row
    auto brs = [](const void *p) {
        return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)0x7FFFFFFF, 0x00020000);
    };
    typedef unsigned u4 __attribute__((ext_vector_type(4)));
    float pb[8], ps[8], psh[8], ps2[8];  // the staged tile's per-column parameters
    // residual / input-mask rows and column parameters of the tile at (s_m0, s_n0)
    auto store_load = [&]() {
        const int n = s_n0 + 8 * cg;
        const bool ncol = n < P.N;
        const __amdgpu_buffer_rsrc_t rr = brs(E.resid), rm = brs(E.mask_in);
        static_for<SPASS>([&](auto R) {
            constexpr int rp = decltype(R)::value;  // half rp / HPASS, pass rp % HPASS
            const int m = s_m0 + (rp / HPASS) * HROWS + r0 + (rp % HPASS) * SROWS;
            const bool live = ncol && m < P.M;
            sres[rp] = half8{};
            smk[rp] = 0xFFu;
            if (live && E.resid)
                sres[rp] = __builtin_bit_cast(
                    half8, __builtin_amdgcn_raw_buffer_load_b128(rr, (unsigned)(((long long)m * E.ldr + n) * 2), 0, 0));
            if (live && E.mask_in)
                smk[rp] = __builtin_amdgcn_raw_buffer_load_b8(rm, (unsigned)(((long long)m * E.ldo2 + n) >> 3), 0, 0);
        });
        if (!ncol) return;
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
    };
    float hv[2][HPASS][8];  // store waves: the staged tile's two halves in registers
    auto read_half = [&](auto H) {
        constexpr int h = decltype(H)::value;
        static_for<HPASS>([&](auto R) {
            constexpr int rp = decltype(R)::value;
            const float *src = stg + (r0 + rp * SROWS) * LDS_T + 8 * cg;
            const float4v x0 = *reinterpret_cast<const float4v *>(src);
            const float4v x1 = *reinterpret_cast<const float4v *>(src + 4);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                hv[h][rp][e] = x0[e];
                hv[h][rp][e + 4] = x1[e];
            }
        });
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    };
    // epilogue8's arithmetic and stores for the passes [p0, p1) of the staged tile
    auto store_passes = [&](int p0, int p1) {
        const int n = s_n0 + 8 * cg;
        if (n >= P.N) return;
        const __amdgpu_buffer_rsrc_t ro = brs(E.out), ro2 = brs(E.out2), rmo = brs(E.mask_out);
        static_for<SPASS>([&](auto R) {
            constexpr int pr = decltype(R)::value, h = pr / HPASS, rp = pr % HPASS;
            if (pr < p0 || pr >= p1) return;
            const int m = s_m0 + h * HROWS + r0 + rp * SROWS;
            if (m >= P.M) return;
            float v[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = hv[h][rp][e] * E.alpha;
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
                for (int e = 0; e < 8; ++e) v[e] = fmaf(E.resid_alpha, (float)sres[pr][e], v[e]);
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
                    if (E.mask_in && !((smk[pr] >> e) & 1u)) w = 0.f;
                    o[e] = f2h(w);
                }
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, o), ro2,
                                                       (unsigned)(((long long)m * E.ldo2 + n) * 2), 0, 0);
            }
        });
    };

    // Global step g = (my tile g / nk, K step g % nk) uses ring slot g % NSTG; stages g and
    // g + 1 are in flight while g is consumed (counted wait: LPT loads per MFMA wave per
    // stage), and the ring runs on across tile boundaries. After its K loop a tile leaves
    // through the half-tile staging: "half 0 staged" (wave row 0 wrote rows 0-63), "half 0
    // read" (the store waves hold them in registers), "half 1 staged" (wave row 1 wrote
    // rows 64-127); the store waves read half 1 after the next tile's first K-step barrier
    // and write it out during that tile's K loop. The two roles run separate loops with the
    // same barrier sequence (per tile: nk K steps + 3), so their registers are allocated for
    // either role alone.
    constexpr int LPT = SA::NC + SB::NC;
    const bool tr = P.trace && blockIdx.x == 0 && lane == 0 && wave == 0;  // MFMA wave 0
    const bool trs = P.trace && blockIdx.x == 0 && lane == 0 && wave == PNW;  // store wave 0
    const int total = my * nk;
    if (mw) {
        int ii = 0, kk = 0, islot = 0;  // issue pointer: tile, step, ring slot
        auto issue_next = [&]() {
            if (ii < my) {
                GP_ISSUE(ii, kk, islot);
                if (++kk == nk) kk = 0, ++ii;
                islot = islot + 1 == NSTG ? 0 : islot + 1;
            }
        };
        issue_next();
        issue_next();
        int slot = 0, g = 0;
        for (int i = 0; i < my; ++i) {
            static_for<PTM>([&](auto I) {
                static_for<PTN>([&](auto J) { acc[I][J] = float4v{0.f, 0.f, 0.f, 0.f}; });
            });
            for (int k = 0; k < nk; ++k, ++g) {
                if (g + 1 < total) wait_vmcnt<LPT>();  // stage g landed, g + 1 in flight
                else wait_vmcnt<0>();
                if (tr && i < 8) P.trace[i * 16 + k] = wall_clock64();  // loads landed
                __builtin_amdgcn_s_barrier();
                __builtin_amdgcn_sched_barrier(0);
                issue_next();  // stage g + 2 into the slot step g - 1 used
                const char *ta = smem + slot * STAGE, *tb = ta + A_ST;
                static_for<BK / 32>([&](auto S) {
                    constexpr int s = decltype(S)::value;
                    half8 fa[PTM], fb[PTN];
                    static_for<PTM>([&](auto I) { fa[I] = load_frag<true, PBM>(ta, wm * PWTM + I * 16, s, lane); });
                    static_for<PTN>([&](auto J) { fb[J] = load_frag<true, PBN>(tb, wn * PWTN + J * 16, s, lane); });
                    static_for<PTM>([&](auto I) {
                        static_for<PTN>([&](auto J) {
                            acc[I][J] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[I], fb[J], acc[I][J], 0, 0, 0);
                        });
                    });
                });
                slot = slot + 1 == NSTG ? 0 : slot + 1;
                __builtin_amdgcn_sched_barrier(0);
            }
            auto stage_acc = [&]() {
                static_for<PTM>([&](auto I) {
                    static_for<PTN>([&](auto J) {
                        const int c = wn * PWTN + J * 16 + (lane & 15);
                        static_for<4>([&](auto EI) {
                            const int r = I * 16 + 4 * (lane >> 4) + EI;
                            stg[r * LDS_T + c] = acc[I][J][decltype(EI)::value];
                        });
                    });
                });
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            };
            if (tr && i < 8) P.trace[i * 16 + 8] = wall_clock64();  // K loop done
            if (wm == 0) stage_acc();
            __builtin_amdgcn_s_barrier();  // half 0 staged
            __builtin_amdgcn_s_barrier();  // half 0 read
            __builtin_amdgcn_sched_barrier(0);
            if (tr && i < 8) P.trace[i * 16 + 9] = wall_clock64();  // half 0 read
            if (wm == 1) stage_acc();
            __builtin_amdgcn_s_barrier();  // half 1 staged
            __builtin_amdgcn_sched_barrier(0);
            if (tr && i < 8) P.trace[i * 16 + 10] = wall_clock64();  // handoff done
        }
    } else {
        // store waves: the previous tile's passes spread over this tile's K steps 0 .. nk-2
        // (its half 0 was read at "half 0 staged", half 1 is read after step 0's barrier),
        // then at step nk-1 the loads for this tile (landing during the handoff barriers)
        const int ppk = (SPASS + nk - 2) / (nk - 1);
        for (int i = 0; i < my; ++i) {
            for (int k = 0; k < nk; ++k) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();
                __builtin_amdgcn_sched_barrier(0);
                if (trs && i < 8) P.trace[128 + i * 16 + k] = wall_clock64();  // step k began
                if (i > 0 && k < nk - 1) {
                    if (k == 0) {
                        read_half(std::integral_constant<int, 1>{});
                        wait_vmcnt<0>();  // its residual / mask rows and parameters
                        if (trs && i < 8) P.trace[128 + i * 16 + 8] = wall_clock64();  // loads landed
                    }
                    store_passes(k * ppk, (k + 1) * ppk);
                    if (trs && i < 8) P.trace[128 + i * 16 + 9 + k] = wall_clock64();  // passes issued
                }
                if (k == nk - 1) {
                    const int t = tile_of(i);
                    s_m0 = (t / P.nt) * PBM;
                    s_n0 = (t % P.nt) * PBN;
                    store_load();
                }
                __builtin_amdgcn_sched_barrier(0);
            }
            __builtin_amdgcn_s_barrier();  // half 0 staged
            __builtin_amdgcn_sched_barrier(0);
            read_half(std::integral_constant<int, 0>{});
            __builtin_amdgcn_s_barrier();  // half 0 read
            __builtin_amdgcn_s_barrier();  // half 1 staged
            __builtin_amdgcn_sched_barrier(0);
        }
        if (my > 0) {  // the last tile
            read_half(std::integral_constant<int, 1>{});
            wait_vmcnt<0>();
            store_passes(0, SPASS);
        }
    }
#undef GP_ISSUE
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
static unsigned long long *g_ptrace = nullptr;
// diagnostics: the next persistent launch stamps block 0's MFMA wave 0 and store wave 0
// (wall_clock64, 100 MHz) into buf (256 u64): [i*16 + k] loads of step k landed, [+8] K loop
// done, [+9] half 0 read, [+10] handoff done; store wave [128 + i*16 + k] step k began,
// [+8] previous tile's loads landed, [+9+k] passes of step k issued. null = off
extern "C" void kf_gemm_persist_trace(unsigned long long *buf) { g_ptrace = buf; }
// test / A-B hook (kf_ops.h): 1 takes the persistent kernel where it applies, 0 sends every
// fused GEMM to the tiled kernel; returns the previous setting
extern "C" int kf_gemm_debug_persist(int on) {
    const int prev = g_persist;
    g_persist = on != 0;
    return prev;
}

// Returns 1 when launched, 0 when not applicable (the caller runs the tiled kernel), -1 on
// error. Taken for fp16 k-contiguous operands (A plain or a two-part time splice, B plain)
// with K <= 640, N a multiple of 128 and at least 1024 tiles, no MXFP8 copy, beta = 0.
int kf_gemm_persist_try(int M, int N, int K, const OpD &a, const OpD &b, int am, int bm, const KfEpilogue &E) {
    if (!g_persist || E.out8 || E.beta != 0.f || bm != OP_SIMPLE || (am != OP_SIMPLE && am != OP_P2)) return 0;
    if (N % PBN || K > 640 || K % 8 || K <= 2 * BK) return 0;
    // the store waves' 32-bit byte offsets (buffer resources of 2^31 - 1 bytes)
    const long long lim = 0x7FFFFFF0LL;
    if ((E.out && ((long long)M * E.ldo * 2 >= lim)) || (E.out2 && (long long)M * E.ldo2 * 2 >= lim) ||
        (E.resid && (long long)M * E.ldr * 2 >= lim))
        return 0;
    const long long mt = (M + PBM - 1) / PBM, nt = N / PBN;
    if (mt * nt < 1024 || mt * nt >= (1LL << 30)) return 0;
    PersistArgs P{M, N, K, (int)mt, (int)nt, (int)(mt * nt), g_ptrace};
    g_ptrace = nullptr;
    int grid = device_cus();
    if (grid > P.ntiles) grid = P.ntiles;
    const int prof = kf_prof_start2(0, 2.0 * M * N * (double)K, kf_gemm_alg_bytes(a, b, E, M, N));
    if (am == OP_SIMPLE)
        gemm_persist_kernel<OP_SIMPLE><<<grid, PTHREADS, 0, kf_stream()>>>(a, b, E, P);
    else
        gemm_persist_kernel<OP_P2><<<grid, PTHREADS, 0, kf_stream()>>>(a, b, E, P);
    kf_prof_stop(prof);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        kf_report_error("persistent gemm launch (M=%d N=%d K=%d): %s", M, N, K, hipGetErrorString(e));
        return -1;
    }
    return 1;
}
