// rowpanel.hip — short-reduction, wide-output fused GEMMs with the A rows held in
// registers and the weights streamed per 64-column block.
//
// The TDNN-F affine forward and the linear layer's input gradient (K = 2 x 160,
// N = 1536; the reference's cublasGemmEx plus ~12 small kernels per layer,
// internal/nnet/forward.go:589-695, network_backward.go:336-463), and the prefinal big
// affine (K = 256) read a 320-wide A row per output row but write 2-3 full-width
// tensors: HBM-bound by the epilogue. The tiled gemm_kernel re-stages A and B through
// LDS for every 192 x 128 tile (205 KB of LDS fills per 15.7 MFLOP, a 2-stage ring
// that waits an L2 round trip per K-step). Here:
//   * a workgroup owns 128 output rows; every wave loads its 32 rows x K of A into
//     registers ONCE (20 16-byte fragments per lane at K = 320) and sweeps all N;
//   * per 64-column block the weights (64 x K, k-contiguous) land in LDS by LDS-DMA,
//     one block ahead (2 slots), and the epilogue's row operands (bypass residual,
//     input mask) two blocks ahead (3 slots), so nothing but LDS-DMA is in flight
//     across the barriers and each wait retires exactly the block it needs
//     (MI355X_MICROARCH.md: vmcnt counts loads, stores and LDS-DMA together in issue
//     order; every store below is an unconditional buffer store, so the counts hold);
//   * the MFMAs produce C^T blocks (the weight fragment is the first operand), so each
//     lane holds 4 consecutive columns of one row: the epilogue (bias / ReLU + mask /
//     BN / bypass / second output, kf_ops.h) runs in registers with 8-byte stores,
//     the ReLU mask byte joining two lanes' nibbles; column parameters sit in LDS.
#include "gemm_common.h"

namespace {

constexpr int RBM = 128;                 // rows per workgroup
constexpr int RBN = 32;                  // columns per block
constexpr int RNW = 4;                   // waves, one 32-row slice each; two workgroups per CU
constexpr int RTM = 2, RTN = 2;          // 16 x 16 MFMA blocks per wave (32 x 32)
constexpr int RB_CHUNK = RBN * BK * 2;   // one 64-deep weight image, 4 KB
constexpr int RR_BYTES = RBM * RBN * 2;  // residual block, 8 KB
constexpr int RM_BYTES = RBM * RBN / 8;  // mask block, 512 B

typedef unsigned int v2u_t __attribute__((ext_vector_type(2)));

// s_waitcnt vmcnt(n), n wave-uniform at run time
__device__ __forceinline__ void rp_wait(int n) {
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

// residual block image: row r (64 B) holds its 16-byte chunk c at slot c ^ ((r >> 2) & 3),
// so the epilogue's 8-byte reads (16 rows x 2 halves per lane group) hit distinct banks
__device__ __forceinline__ int rr_off(int r, int col) {
    return r * 64 + 16 * ((col >> 3) ^ ((r >> 2) & 3)) + 2 * (col & 7);
}

}  // namespace

// KS = K / 32 reduction slices (A fragments per row group); AM / BMODE: operand modes.
// LDS: column parameters [np][npad] f32 (only the epilogue's: bias, scale + shift,
// scale2), 2 weight slots, 2 residual slots, 2 input-mask slots, 2 output-mask stages.
template <int KS, int AM, int BMODE>
__global__ __launch_bounds__(64 * RNW, 2) void rowpanel_kernel(int M, int N, int K, OpD A, OpD B, KfEpilogue E,
                                                               int npad, unsigned long long *trace) {
    constexpr int KCH = (KS + 1) / 2;  // 64-deep weight images per block
    extern __shared__ __attribute__((aligned(16))) char dsm[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int m0 = blockIdx.x * RBM;
    const int nblk = N / RBN;
    // diagnostics (kf_rowpanel_trace): block 300, wave 0 stamps 4 phases per column block
    const bool tr = trace && blockIdx.x == 300 && threadIdx.x == 0;
#define RP_TP(nb, i) \
    if (tr && (nb) < 64) trace[(nb) * 4 + (i)] = wall_clock64();

    const int np = (E.bias ? 1 : 0) + (E.scale ? 2 : 0) + (E.scale2 ? 1 : 0);
    float *prm = reinterpret_cast<float *>(dsm);
    const float *pbias = prm, *pscale = prm + (E.bias ? npad : 0), *pshift = pscale + npad;
    const float *pscale2 = prm + ((E.bias ? 1 : 0) + (E.scale ? 2 : 0)) * npad;
    char *bring = dsm + 4 * (size_t)np * npad;               // 2 x KCH weight images
    char *rring = bring + 2 * KCH * RB_CHUNK;                 // 2 residual blocks
    char *mring = rring + 2 * RR_BYTES;                       // 2 input-mask blocks
    unsigned char *mstage = reinterpret_cast<unsigned char *>(mring + 2 * RM_BYTES);  // 2 output-mask blocks

    // ---- column parameters, and the A rows into registers
    for (int c = tid; c < npad; c += 64 * RNW) {
        const bool in = c < N;
        float *q = prm;
        if (E.bias) *(q + c) = in ? (float)((const h16 *)E.bias)[c] : 0.f, q += npad;
        if (E.scale) {
            q[c] = in ? E.scale[c] : 0.f;
            q[npad + c] = in ? E.shift[c] : 0.f;
            q += 2 * npad;
        }
        if (E.scale2) q[c] = in ? E.scale2[c] : 1.f;
    }
    // lane l of fragment (I, s): row m0 + wave*32 + I*16 + (l & 15), k = 32 s + 8 (l >> 4) .. + 8
    half8 afr[RTM][KS];
    static_for<RTM>([&](auto I) {
        const int m = m0 + wave * 32 + I * 16 + (lane & 15);
        static_for<KS>([&](auto S) {
            constexpr int s = decltype(S)::value;
            const int k = 32 * s + 8 * (lane >> 4);
            half8 v = half8{};
            if (m < M && k < A.ncols) {
                long long off;
                if constexpr (AM == OP_SIMPLE) {
                    off = (long long)m * A.ld + k;
                } else {
                    const int p = A.nparts > 1 && k >= A.pw ? 1 : 0;
                    off = op_off(A, m, 0, k - p * A.pw, A.dt[p], A.dh[p], A.et[p], A.er[p]);
                }
                if (off >= 0) v = load_h8(A.base + off);
            }
            afr[I][s] = v;
        });
    });
    // wait for the A rows HERE, and hand them to the loop as values the compiler sees as
    // defined after the wait: otherwise it re-waits vmcnt(0) at their first use inside
    // the loop, draining the LDS-DMA ring every block
    wait_vmcnt<0>();
    static_for<RTM>([&](auto I) {
        static_for<KS>([&](auto S) {
            typedef int v4i __attribute__((ext_vector_type(4)));
            v4i t = __builtin_bit_cast(v4i, afr[I][decltype(S)::value]);
            asm volatile("" : "+v"(t));
            afr[I][decltype(S)::value] = __builtin_bit_cast(half8, t);
        });
    });
    __syncthreads();  // parameters in LDS

    // ---- LDS-DMA producers
    const __amdgpu_buffer_rsrc_t rb = make_rsrc(B.base);
    const __amdgpu_buffer_rsrc_t rr = make_rsrc(E.resid ? E.resid : B.base);
    const __amdgpu_buffer_rsrc_t rmk = make_rsrc(E.mask_in ? (const void *)E.mask_in : (const void *)B.base);
    Stager<true, RBN, BMODE, RNW> sb;
    auto issue_b = [&](int nb) {  // weights of block nb into slot nb & 1 (KCH loads per lane)
        sb.init(B, nb * RBN, wave, lane);
        char *dst = bring + (nb & 1) * KCH * RB_CHUNK;
        static_for<KCH>([&](auto C) {
            constexpr int c = decltype(C)::value;
            sb.issue(B, rb, c * BK, K, dst + c * RB_CHUNK, wave, lane);
        });
    };
    const unsigned ldr2 = (unsigned)(E.ldr * 2);
    auto issue_r = [&](int nb) {  // row operands of block nb into slot nb & 1
        const int slot = nb & 1, n0 = nb * RBN;
        if (E.resid) {
            char *dst = rring + slot * RR_BYTES;
            static_for<2>([&](auto Q) {  // 8 pieces of 16 rows, two per wave
                const int q = wave * 2 + decltype(Q)::value;
                const int r = 16 * q + (lane >> 2);
                const int c = (lane & 3) ^ ((r >> 2) & 3);  // logical chunk of this slot
                const int m = m0 + r;
                const unsigned voff = m < M ? (unsigned)m * ldr2 + (unsigned)(n0 + 8 * c) * 2u : BAD;
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    rr, (__attribute__((address_space(3))) void *)(dst + q * 1024), 16, voff, 0, 0, 0);
            });
        }
        if (E.mask_in && wave < 2) {  // [128 rows][4 bytes]: one dword per lane on waves 0-1
            char *dst = mring + slot * RM_BYTES;
            const int r = wave * 64 + lane, m = m0 + r;
            const unsigned voff = m < M ? (unsigned)(((long long)m * E.ldo2 + n0) >> 3) : BAD;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                rmk, (__attribute__((address_space(3))) void *)(dst + wave * 256), 4, voff, 0, 0, 0);
        }
    };
    const int nst = RTM * RTN * ((E.out ? 1 : 0) + (E.out2 ? 1 : 0));  // epilogue stores per block
    const int nfl = E.mask_out && wave < 2 ? 1 : 0;                    // mask flush stores per block

    const __amdgpu_buffer_rsrc_t ro = make_rsrc(E.out ? E.out : B.base);
    const __amdgpu_buffer_rsrc_t ro2 = make_rsrc(E.out2 ? E.out2 : B.base);
    const __amdgpu_buffer_rsrc_t rmo = make_rsrc(E.mask_out ? (const void *)E.mask_out : (const void *)B.base);

    // output ReLU bits of block k, staged by its epilogue: one 4-byte row segment per lane
    // of waves 0-1 (one write per row and block instead of two 2-byte pieces)
    auto flush_mask = [&](int k) {
        if (nfl) {
            const int r = wave * 64 + lane, m = m0 + r;
            const unsigned w = *reinterpret_cast<const unsigned *>(mstage + (k & 1) * RM_BYTES + r * 4);
            const unsigned off = m < M ? (unsigned)(((long long)m * E.ldo + (long long)k * RBN) >> 3) : BAD;
            __builtin_amdgcn_raw_buffer_store_b32(w, rmo, off, 0, 0);
        }
    };

    issue_b(0);
    if (nblk > 0) issue_r(0);

    const int g = lane >> 4;  // this lane's 4-column group in a 16-column block
    for (int nb = 0; nb < nblk; ++nb) {
        // retire block nb's weights and row operands (issued in iteration nb - 1, before
        // block nb - 2's mask flush and block nb - 1's epilogue stores, which may stay in flight)
        RP_TP(nb, 0);
        rp_wait((nb >= 2 ? nfl : 0) + (nb >= 1 ? nst : 0));
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's staged mask bytes
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        RP_TP(nb, 1);
        if (nb + 1 < nblk) {
            issue_b(nb + 1);
            issue_r(nb + 1);
        }
        if (nb >= 1) flush_mask(nb - 1);  // after the loads, so the next wait may leave it in flight
        const char *tb = bring + (nb & 1) * KCH * RB_CHUNK;
        float4v acc[RTM][RTN];
        static_for<RTM>([&](auto I) {
            static_for<RTN>([&](auto J) { acc[I][J] = float4v{0.f, 0.f, 0.f, 0.f}; });
        });
        static_for<KS>([&](auto S) {
            constexpr int s = decltype(S)::value;
            half8 fb[RTN];
            static_for<RTN>([&](auto J) {
                fb[J] = load_frag<true, RBN>(tb + (s / 2) * RB_CHUNK, J * 16, s & 1, lane);
            });
            static_for<RTM>([&](auto I) {
                static_for<RTN>([&](auto J) {
                    acc[I][J] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fb[J], afr[I][s], acc[I][J], 0, 0, 0);
                });
            });
        });
        __builtin_amdgcn_sched_barrier(0);
        RP_TP(nb, 2);
        // ---- epilogue: lane holds rows m0 + wave*32 + I*16 + (l & 15), columns n..n+3
        const int n0 = nb * RBN, slot = nb & 1;
        const char *rimg = rring + slot * RR_BYTES;
        const unsigned char *mimg = reinterpret_cast<const unsigned char *>(mring + slot * RM_BYTES);
        unsigned char *mst = mstage + slot * RM_BYTES;
        static_for<RTM>([&](auto I) {
            const int rl = wave * 32 + I * 16 + (lane & 15);
            const int m = m0 + rl;
            static_for<RTN>([&](auto J) {
                const int cl = J * 16 + 4 * g;  // local column of this lane's 4
                const int n = n0 + cl;
                float v[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = acc[I][J][e] * E.alpha;
                if (E.bias) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] += pbias[n + e];
                }
                unsigned bits = 0xFu;
                if (E.relu) {
                    bits = 0;
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        if (v[e] > 0.f) bits |= 1u << e;
                        else v[e] = 0.f;
                    }
                }
                if (E.scale) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] = fmaf(v[e], pscale[n + e], pshift[n + e]);
                }
                if (E.resid) {
                    const half4 rv = *reinterpret_cast<const half4 *>(rimg + rr_off(rl, cl));
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] = fmaf(E.resid_alpha, (float)rv[e], v[e]);
                }
                const bool live = m < M;
                if (E.out) {
                    half4 o;
#pragma unroll
                    for (int e = 0; e < 4; ++e) o[e] = f2h(v[e]);
                    const unsigned off = live ? ((unsigned)m * (unsigned)E.ldo + (unsigned)n) * 2u : BAD;
                    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u_t, o), ro, off, 0, 0);
                }
                if (E.out2) {
                    unsigned mb = 0xFu;
                    if (E.mask_in) mb = (mimg[rl * 4 + (cl >> 3)] >> (4 * ((cl >> 2) & 1))) & 0xFu;
                    half4 o;
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        float w = v[e];
                        if (E.scale2) w *= pscale2[n + e];
                        if (!((mb >> e) & 1u)) w = 0.f;
                        o[e] = f2h(w);
                    }
                    const unsigned off = live ? ((unsigned)m * (unsigned)E.ldo2 + (unsigned)n) * 2u : BAD;
                    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u_t, o), ro2, off, 0, 0);
                }
                if (E.mask_out) {
                    // lanes g (columns n..n+3) and g ^ 1 (the other half of the byte)
                    const unsigned other = (unsigned)__shfl_xor((int)bits, 16);
                    if (!(g & 1)) mst[rl * 4 + (cl >> 3)] = (unsigned char)(bits | (other << 4));
                }
            });
        });
        __builtin_amdgcn_sched_barrier(0);
        RP_TP(nb, 3);
    }
    if (E.mask_out && nblk >= 1) {  // the last block's bits
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
        __builtin_amdgcn_s_barrier();
        flush_mask(nblk - 1);
    }
#undef RP_TP
}

static unsigned long long *g_rp_trace = nullptr;
extern "C" void kf_rowpanel_trace(unsigned long long *buf) { g_rp_trace = buf; }

int kf_prof_start2(int cls, double flops, double bytes);
void kf_prof_stop(int idx);
double kf_gemm_alg_bytes(const OpD &a, const OpD &b, const KfEpilogue &E, long long M, long long N);

// applicable: K = 160, 256 or 320; N % 64 == 0; A k-contiguous plain or time-spliced
// (parts on 32-column boundaries), B k-contiguous plain or op_wrows rows; no beta /
// MXFP8 copy; 32-bit byte offsets for every epilogue tensor
// Off by default: measured slower than the tiled gemm_kernel on every TDNN-F shape
// (scripts/rp_trace.py). KF_ROWPANEL=1 or kf_gemm_debug_rowpanel(1)
// turns it on (A/B, tests).
static int g_rp_override = -1;
extern "C" void kf_gemm_debug_rowpanel(int mode) { g_rp_override = mode < 0 ? -1 : (mode != 0); }
int kf_rowpanel_try(int M, int N, int K, const OpD &a, const OpD &b, int am, int bm, bool bkc,
                    const KfEpilogue &E) {
    static const int env = getenv("KF_ROWPANEL") ? atoi(getenv("KF_ROWPANEL")) : 0;
    const int on = g_rp_override >= 0 ? g_rp_override : env;
    if (!on || M <= 0 || !bkc || N % RBN || E.beta != 0.f || E.out8 || a.sc || b.sc) return 0;
    if (K != 160 && K != 256 && K != 320) return 0;
    if (am != OP_SIMPLE && am != OP_P2) return 0;
    if (bm != OP_SIMPLE && bm != OP_P2) return 0;
    if (am == OP_P2 && (a.pw % 32 || a.nparts * a.pw != K)) return 0;
    if (a.ncols != K || b.ncols != K || b.nrows < N) return 0;
    if (!E.out && !E.out2) return 0;
    const long long lim = (1LL << 32) - 64;
    if ((E.out && (long long)M * E.ldo * 2 >= lim) || (E.out2 && (long long)M * E.ldo2 * 2 >= lim) ||
        (E.resid && (long long)M * E.ldr * 2 >= lim) || (E.mask_out && (long long)M * E.ldo / 8 >= lim) ||
        (E.mask_in && (long long)M * E.ldo2 / 8 >= lim))
        return 0;
    if ((E.out && E.ldo % 8) || (E.out2 && E.ldo2 % 8) || (E.resid && E.ldr % 8)) return 0;
    const int npad = (N + RBN - 1) / RBN * RBN;
    const int KCH = (K / 32 + 1) / 2;
    const int np = (E.bias ? 1 : 0) + (E.scale ? 2 : 0) + (E.scale2 ? 1 : 0);
    const size_t lds = 4 * (size_t)np * npad + 2 * (size_t)KCH * RB_CHUNK + 2 * (size_t)RR_BYTES + 4 * (size_t)RM_BYTES;
    if (lds > 80 * 1024) return 0;  // two workgroups per CU
    const dim3 grid((M + RBM - 1) / RBM);
    const int prof = kf_prof_start2(0, 2.0 * M * N * (double)K, kf_gemm_alg_bytes(a, b, E, M, N));
#define KF_RP(KS_)                                                                                       \
    do {                                                                                                 \
        if (am == OP_SIMPLE && bm == OP_SIMPLE)                                                          \
            rowpanel_kernel<KS_, OP_SIMPLE, OP_SIMPLE><<<grid, 64 * RNW, lds, kf_stream()>>>(M, N, K, a, b, E, npad, g_rp_trace); \
        else if (am == OP_SIMPLE)                                                                        \
            rowpanel_kernel<KS_, OP_SIMPLE, OP_P2><<<grid, 64 * RNW, lds, kf_stream()>>>(M, N, K, a, b, E, npad, g_rp_trace);     \
        else if (bm == OP_SIMPLE)                                                                        \
            rowpanel_kernel<KS_, OP_P2, OP_SIMPLE><<<grid, 64 * RNW, lds, kf_stream()>>>(M, N, K, a, b, E, npad, g_rp_trace);     \
        else                                                                                             \
            rowpanel_kernel<KS_, OP_P2, OP_P2><<<grid, 64 * RNW, lds, kf_stream()>>>(M, N, K, a, b, E, npad, g_rp_trace);         \
    } while (0)
    if (K == 160) KF_RP(5);
    else if (K == 256) KF_RP(8);
    else KF_RP(10);
#undef KF_RP
    kf_prof_stop(prof);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        kf_report_error("rowpanel launch (M=%d N=%d K=%d): %s", M, N, K, hipGetErrorString(e));
        return -1;
    }
    return 1;
}
