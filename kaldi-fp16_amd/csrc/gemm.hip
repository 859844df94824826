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
void kf_report_error(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    kf_err_.set(fmt, ap);
    va_end(ap);
}

#include "gemm_common.h"

// ---------------------------------------------------------------------------
// the kernel
// ---------------------------------------------------------------------------
struct WgradArgs {
    float *slab;        // [splits][M][N] fp32 partials
    float *bias_slab;   // [splits][N] fp32 column sums of B, or nullptr
    int k_per_split;    // multiple of BK
    // > 0: A has two time-shifted parts of one source and part p's M tile j covers the
    // same source columns as tile pair_ps * p + j (N fits one tile). Each XCD then gets
    // whole (column chunk, split) pairs, so the two parts' reads of the same source rows
    // meet in one L2 instead of two
    int pair_ps;
    int kil;            // fused: 1 = alternate the K-steps of a two-part A (KF_GEMM_KIL, default 1)
    // diagnostics (kf_gemm_trace), null = off: [0..63] phase stamps of block trace_blk
    // (tid 0), then per block {start, end, hw id | xcc id << 32}
    unsigned long long *trace;
    int trace_blk;
    // fused MXFP8 only (kf_gemm_fused_edge): the last M tile's workgroups also write the fp16
    // row eo[j] = sum_c ex0[c] ew[j][c] + ex1[c] ew[N + j][c] for their columns j
    h16 *eo;
    const h16 *ex0, *ex1, *ew;
    int ecols;
};

template <int BM, int BN, int ST, int SCB = 0>
struct SmemSize {
    static constexpr int stage = (BM + BN) * BK * 2 + SCB;
    static constexpr int pipe = ST * stage;
    static constexpr int bytes = pipe;
};

// ---------------------------------------------------------------------------
// MXFP8 scale staging: per K-step of 128 fp8 elements every tile row needs the
// 4 E8M0 bytes of its 4 blocks, one dword. Slot s of [A rows | B rows | unused]
// is lane s%64 of LDS-DMA instruction s/64; each wave issues SPW of them, so
// the vmcnt bookkeeping stays uniform. Instructions never straddle A and B
// (BM % 64 == 0), so each has one buffer resource.
// ---------------------------------------------------------------------------
template <int BM, int BN, int NW, int AM>
struct ScaleStager {
    static constexpr int SLOTS = BM + BN;
    static constexpr int SPW = (SLOTS + 64 * NW - 1) / (64 * NW);
    static constexpr int BYTES = SPW * NW * 64 * 4;
    static_assert(BM % 64 == 0, "A scale rows fill whole instructions");
    unsigned b0[SPW], b1[SPW];  // A: part-0 / part-1 row offsets; B: row offset (b1 unused)
    __device__ __forceinline__ void init(const OpD &A, const OpD &B, int m0, int n0, int wave,
                                         int lane) {
        static_for<SPW>([&](auto I) {
            constexpr int i = decltype(I)::value;
            const int slot = (wave * SPW + i) * 64 + lane;
            b0[i] = b1[i] = BAD;
            if (slot < BM) {
                const int r = m0 + slot;
                if (r < A.nrows) {
                    if constexpr (AM == OP_SIMPLE) {
                        b0[i] = (unsigned)r * A.lds;
                    } else {
                        for (int p = 0; p < 2 && p < A.nparts; ++p) {
                            int st = r + A.dt[p];
                            bool ok = true;
                            if (A.tclamp) st = min(max(st, 0), A.T - 1);
                            else ok = (unsigned)st < (unsigned)A.T;
                            if (ok) (p ? b1[i] : b0[i]) = (unsigned)st * A.lds;
                        }
                    }
                }
            } else if (slot < SLOTS) {
                const int n = n0 + slot - BM;
                if (n < B.nrows) b0[i] = (unsigned)n * B.lds;
            }
        });
    }
    // k0 in 2-byte units (the fp16 stagers' unit): fp8 element 2*k0 starts the step
    __device__ __forceinline__ void issue(const OpD &A, const OpD &B, Rsrc ra,
                                          Rsrc rb, int k0, char *dst, int wave,
                                          int lane) {
        const int k8 = 2 * k0;
        static_for<SPW>([&](auto I) {
            constexpr int i = decltype(I)::value;
            const int ins = wave * SPW + i;  // wave-uniform
            const int slot = ins * 64 + lane;
            unsigned voff = BAD;
            const bool isA = ins * 64 < BM;
            if (isA) {
                if (k8 < 2 * A.ncols) {
                    if constexpr (AM == OP_SIMPLE) {
                        if (b0[i] != BAD) voff = b0[i] + (unsigned)(k8 >> 5);
                    } else {
                        const int p = k8 >= A.pw8 ? 1 : 0;
                        const unsigned b = p ? b1[i] : b0[i];
                        if (b != BAD) voff = b + (unsigned)((k8 - p * A.pw8) >> 5);
                    }
                }
            } else if (slot < SLOTS && k8 < 2 * B.ncols && b0[i] != BAD) {
                voff = b0[i] + (unsigned)(k8 >> 5);
            }
            // a wave-uniform branch, not a select: a selected 128-bit resource goes to scratch
            if (isA) lds_dma<4>(ra, dst + ins * 256, voff);
            else lds_dma<4>(rb, dst + ins * 256, voff);
        });
    }
};

// e4m3 (OCP) of 8 values already divided by the block scale; clamp at 448 first
// (v_cvt_pk_fp8_f32 rounds 464..479 to 448 but 480 and above to NaN)
__device__ __forceinline__ uint2 pack_e4m3x8(const float *v) {
    uint2 r;
    unsigned w[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        float c[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) c[e] = fminf(fmaxf(v[4 * h + e], -448.f), 448.f);
        unsigned x = __builtin_amdgcn_cvt_pk_fp8_f32(c[0], c[1], 0, false);
        x = __builtin_amdgcn_cvt_pk_fp8_f32(c[2], c[3], x, true);
        w[h] = x;
    }
    r.x = w[0];
    r.y = w[1];
    return r;
}

// E8M0 exponent of a block with max magnitude amax: floor(log2 amax) - 8,
// clamped so that 2^-e stays a normal float; amax = 0 -> 0
__device__ __forceinline__ int mx_exponent(float amax) {
    if (!(amax > 0.f)) return 0;
    const int ex = (int)((__float_as_uint(amax) >> 23) & 0xFF) - 127;
    return min(max(ex - 8, -126), 126);
}

// ---------------------------------------------------------------------------
// fused epilogue of a BM x BN tile held as 16x16 accumulators. Per-column
// parameters go to LDS once per workgroup; then every wave stages its
// accumulators through its own LDS region 32 rows at a time and each lane owns 8
// consecutive columns of a row (16-byte global I/O). `smem` must hold
// 4*BN + 32*EpiMap<BN/WN>::LDT*WM*WN floats; every LDS-DMA into it must have landed.
// ---------------------------------------------------------------------------
// the epilogue's per-column parameters of column n0 + tid, loaded before the K loop so
// their latency hides under it (KF_EPI_EARLY=0: loaded in the epilogue)
struct EpiPre {
    float b, s, sh, s2;
};
template <int BN, int NTH>
__device__ __forceinline__ EpiPre epi_params(const KfEpilogue &E, int N, int n0, int tid) {
    static_assert(BN <= NTH, "one column per thread");
    EpiPre p{0.f, 0.f, 0.f, 1.f};
    const int n = n0 + tid;
    if (tid < BN && n < N) {
        if (E.bias) p.b = (float)((const h16 *)E.bias)[n];
        if (E.scale) {
            p.s = E.scale[n];
            p.sh = E.shift[n];
        }
        if (E.scale2) p.s2 = E.scale2[n];
    }
    return p;
}

// Epilogue item map and fp32 staging layout of a wave's 32-row chunk. Item k of a lane is
// (row r, 8-column group cg); the lane reads columns 8cg .. 8cg+7 of row r as two 16-byte
// LDS reads and owns them for the global I/O (CG consecutive lanes cover a row's 16 * CG
// contiguous bytes). Rows of WTN + 4 dwords, except for WTN = 64 (the conv halo tiles and
// the 256x256 / 128x128 / 256x64 GEMM tiles): rows of 64 dwords with 16-byte unit u of row r
// at u ^ xr(r), which makes both the accumulator stores and the 16-byte reads bank-conflict
// free (scripts/epi_lds_check.py; the padded rows are 2-way conflicted on the reads: with
// 8-column items a row covers only every other 16-byte unit). For WTN = 32 / 48 (the 80 KB
// 192x128 / 128x192 tiles) the conflicts stay: r5 measured a conflict-free form (the MFMAs
// producing C^T, one 16-byte store per accumulator, rows of 48 dwords, 4-lane row runs) at
// +6 % on the TDNN-F input gradient (257 -> 272 us: its 32-byte global row runs for the last
// 16 columns cost more than the LDS cycles saved), and an XOR mixing lane and loop-index
// bits at 18 more VGPRs (the second workgroup per CU lost, +50 %).
template <int WTN>
struct EpiMap {
    static constexpr int CG = WTN / 8;
    static constexpr bool SWZ = WTN == 64;
    static constexpr int LDT = SWZ ? 64 : WTN + 4;
    __device__ __forceinline__ static int row(int k, int lane) { return (lane + 64 * k) / CG; }
    __device__ __forceinline__ static int cg(int k, int lane) { return (lane + 64 * k) % CG; }
    __device__ __forceinline__ static int xr(int r) { return ((r >> 1) & 1) | (((r >> 2) & 1) << 2); }
    // dword offset of column c of row r
    __device__ __forceinline__ static int off(int r, int c) {
        if constexpr (SWZ) return r * LDT + 4 * ((c >> 2) ^ xr(r)) + (c & 3);
        else return r * LDT + c;
    }
};

// RG: the epilogue honours KfEpilogue.row_group (the conv input-gradient halo kernels only:
// the row map's registers cost the 80 KB GEMM tiles their second workgroup per CU)
template <int BM, int BN, int WM, int WN, bool RG = false>
__device__ __forceinline__ void fused_epilogue(float4v (&acc)[BM / WM / 16][BN / WN / 16], char *smem,
                                               const KfEpilogue &E, int M, int N, int m0, int n0,
                                               int tid, int lane, int wave, const EpiPre *pre = nullptr) {
    constexpr int NW = WM * WN, NTH = 64 * NW;
    constexpr int WTM = BM / WM, WTN = BN / WN;
    constexpr int TM = WTM / 16, TN = WTN / 16;
    const int wm = wave / WN, wn = wave % WN;
    // grouped output rows (KfEpilogue.row_group): the address row of GEMM row m
    const int rg = RG ? E.row_group : 0;
    auto arow = [&](int m) -> long long {
        if (!RG || rg <= 0) return m;
        const int g = m / rg;
        return (long long)g * E.row_stride + (m - g * rg);
    };
    wait_vmcnt<0>();
    __syncthreads();
    float *prm = reinterpret_cast<float *>(smem);
    {
        const EpiPre p = pre ? *pre : epi_params<BN, NTH>(E, N, n0, tid);
        if (tid < BN) {
            prm[tid] = p.b;
            prm[BN + tid] = p.s;
            prm[2 * BN + tid] = p.sh;
            prm[3 * BN + tid] = p.s2;
        }
    }
    __syncthreads();
    const EpiCols P{prm, prm + BN, prm + 2 * BN, prm + 3 * BN};
    using EM = EpiMap<WTN>;
    constexpr int LDT = EM::LDT;
    float *st = prm + 4 * BN + wave * 32 * LDT;
    constexpr int CG = WTN / 8;
    constexpr int ITEMS = 32 * CG / 64;
    static_assert(ITEMS * 64 == 32 * CG, "items per lane");
    static_assert(TM % 2 == 0, "epilogue stages 32 rows");
    // Row operands (residual, old C, input mask) of the 32-row chunks. The residual rows
    // sit in a ring of NSL register slots, the others in two: chunk ic + NSL - 1 (ic + 1)
    // is issued while chunk ic is processed. When the whole wave tile fits (NSL = TM / 2,
    // small ITEMS), every chunk's residual loads are issued before the first chunk's
    // stores, so no chunk's wait queues behind an earlier chunk's stores (vmcnt is in
    // order): one memory round trip per tile for the bypass epilogue, not one per chunk.
    constexpr int NCH = TM / 2;
    constexpr int NSL = (NCH <= 4 && ITEMS * NCH <= 6) ? NCH : 2;
    half8 rres[NSL][ITEMS], cold[2][ITEMS];
    unsigned mb[2][ITEMS];
    auto prefetch_res = [&](auto ICc) {
        constexpr int icp = decltype(ICc)::value, sl = icp % NSL;
        static_for<ITEMS>([&](auto K) {
            constexpr int k = decltype(K)::value;
            const int r = EM::row(k, lane), cg = EM::cg(k, lane);
            const int m = m0 + wm * WTM + icp * 32 + r, n = n0 + wn * WTN + 8 * cg;
            rres[sl][k] = half8{};
            if (m < M && n < N && E.resid) rres[sl][k] = load_h8((const h16 *)E.resid + arow(m) * E.ldr + n);
        });
    };
    auto prefetch = [&](auto ICc) {
        constexpr int icp = decltype(ICc)::value, sl = icp & 1;
        static_for<ITEMS>([&](auto K) {
            constexpr int k = decltype(K)::value;
            const int r = EM::row(k, lane), cg = EM::cg(k, lane);
            const int m = m0 + wm * WTM + icp * 32 + r, n = n0 + wn * WTN + 8 * cg;
            const bool ok = m < M && n < N;
            cold[sl][k] = half8{};
            mb[sl][k] = 0xFFu;
            if (ok && E.beta != 0.f) cold[sl][k] = load_h8((const h16 *)E.out + arow(m) * E.ldo + n);
            if (ok && E.mask_in) mb[sl][k] = E.mask_in[(arow(m) * E.ldo2 + n) >> 3];
        });
    };
    static_for<NSL - 1>([&](auto IC) { prefetch_res(IC); });
    prefetch(std::integral_constant<int, 0>{});
    static_for<NCH>([&](auto IC) {
        constexpr int ic = decltype(IC)::value, sl = ic & 1, slr = ic % NSL;
        if constexpr (ic + NSL - 1 < NCH) prefetch_res(std::integral_constant<int, ic + NSL - 1>{});
        if constexpr (ic + 1 < NCH) prefetch(std::integral_constant<int, ic + 1>{});
        static_for<2>([&](auto I2) {
            static_for<TN>([&](auto J) {
                const int c = J * 16 + (lane & 15);
                static_for<4>([&](auto EI) {
                    const int r = I2 * 16 + 4 * (lane >> 4) + EI;
                    st[EM::off(r, c)] = acc[2 * ic + I2][J][decltype(EI)::value];
                });
            });
        });
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        static_for<ITEMS>([&](auto K) {
            constexpr int k = decltype(K)::value;
            const int r = EM::row(k, lane), cg = EM::cg(k, lane);
            const int nl = wn * WTN + 8 * cg;
            const int m = m0 + wm * WTM + ic * 32 + r, n = n0 + nl;
            const bool live = m < M && n < N;
            float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
            if (live) {
                float4v x0 = *reinterpret_cast<const float4v *>(st + EM::off(r, 8 * cg));
                float4v x1 = *reinterpret_cast<const float4v *>(st + EM::off(r, 8 * cg + 4));
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    v[e] = x0[e];
                    v[e + 4] = x1[e];
                }
                epilogue8(E, P, arow(m), n, nl, v, cold[sl][k], rres[slr][k], mb[sl][k]);
            }
            if constexpr (CG % 4 == 0) {
                // MXFP8 copy: the 4 lanes l..l+3 (l % 4 == 0) hold one 32-column block
                if (E.out8) {
                    float amax = 0.f;
#pragma unroll
                    for (int e = 0; e < 8; ++e) amax = fmaxf(amax, fabsf(v[e]));
                    amax = fmaxf(amax, __shfl_xor(amax, 1));
                    amax = fmaxf(amax, __shfl_xor(amax, 2));
                    const int ex = mx_exponent(amax);
                    const float inv = __uint_as_float((unsigned)(127 - ex) << 23);
                    float q[8];
#pragma unroll
                    for (int e = 0; e < 8; ++e) q[e] = v[e] * inv;
                    const uint2 pk = pack_e4m3x8(q);
                    if (live) {
                        const long long ma = arow(m);
                        *reinterpret_cast<uint2 *>((uint8_t *)E.out8 + ma * E.ldo8 + n) = pk;
                        if ((lane & 3) == 0) E.scale8[ma * (E.ldo8 >> 5) + (n >> 5)] = (uint8_t)(ex + 127);
                    }
                }
            }
        });
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    });
    // edge row (KfEpilogue.edge_out): the row tile that holds rows [edge_r0, edge_r1) sums the
    // values it just stored, per column in row order (kf_rows_sum's order and rounding), once
    // every wave's stores are visible to the workgroup. The host falls back to kf_rows_sum when
    // the rows span two tiles (launch<>). Visibility rests on CU mode with the write-through
    // L1 (the workgroup-scope release / acquire below) and on no earlier read of out / out2
    // in this kernel (a beta accumulation reads out, but only rows it then overwrites, and
    // edge_src = 1 sums out2, which nothing reads before); a change to either needs a
    // different source, e.g. the fp32 staging rounded as stored.
    if (E.edge_out && E.edge_r0 >= m0 && E.edge_r1 <= m0 + BM && E.edge_r1 <= M && E.edge_r0 < E.edge_r1) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __syncthreads();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        const h16 *src = (const h16 *)(E.edge_src ? E.out2 : E.out);
        const long long ld = E.edge_src ? E.ldo2 : E.ldo;
        for (int c = tid; c < BN; c += NTH) {
            const int n = n0 + c;
            if (n >= N) continue;
            float s = 0.f;
            for (int r = E.edge_r0; r < E.edge_r1; ++r) s += h2f(src[(long long)r * ld + n]);
            ((h16 *)E.edge_out)[n] = f2h(s);
        }
    }
}

template <int BM, int BN, int WM, int WN, bool AKC, bool BKC, bool WGRAD, int ST, int AM, int BMODE,
          int F8 = 0>
__global__ __launch_bounds__(64 * WM * WN, 1) void gemm_kernel(int M, int N, int K, OpD A, OpD B,
                                                               KfEpilogue E, WgradArgs G,
                                                               int n_mtiles, int n_ntiles) {
    constexpr int NW = WM * WN, NTH = 64 * NW;
    // operand modes; bit 3 (OP_MASKED) = the operand carries a bit mask (KfOperand.mask)
    constexpr int AMD = AM & 7, BMD = BMODE & 7;
    constexpr bool AMK = (AM & OP_MASKED) != 0, BMK = (BMODE & OP_MASKED) != 0, MK = AMK || BMK;
    static_assert(!MK || (ST == 2 && !F8), "masked operands: two-stage ring, fp16");
    using SCS = ScaleStager<F8 ? BM : 64, F8 ? BN : 64, NW, AMD>;  // used by MXFP8 only
    constexpr int SCB = F8 ? SCS::BYTES : 0;
    static_assert(!F8 || (AKC && BKC && !WGRAD && BMD == OP_SIMPLE && AMD != OP_GEN),
                  "MXFP8: k-contiguous plain / spliced A, plain B");
    static_assert(NW == 4 || NW == 8, "4 or 8 waves");
    constexpr int WTM = BM / WM, WTN = BN / WN;
    constexpr int TM = WTM / 16, TN = WTN / 16;
    static_assert(TM * 16 == WTM && TN * 16 == WTN, "wave tile multiple of 16");
    constexpr int A_STAGE = BM * BK * 2, B_STAGE = BN * BK * 2;
    constexpr int STAGE = A_STAGE + B_STAGE + SCB;
    using SA = Stager<AKC, BM, AMD, NW, AMK>;
    using SB = Stager<BKC, BN, BMD, NW, BMK>;
    constexpr int LPT = SA::NC + SB::NC + (F8 ? SCS::SPW : 0);  // LDS-DMA per thread per stage
    static_assert((SA::EVEN && SB::EVEN) || ST == 2, "uneven stagers need the vmcnt(0) ring");
    static_assert(ST >= 2 && ST <= 4, "stages");
    static_assert(WGRAD || 4 * BN * 4 + (32 * EpiMap<WTN>::LDT * 4) * NW <= SmemSize<BM, BN, ST, SCB>::bytes,
                  "epilogue staging");

    __shared__ __attribute__((aligned(16))) char smem[SmemSize<BM, BN, ST, SCB>::bytes + (MK ? 4096 : 0)];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / WN, wn = wave % WN;
    const int bid = blockIdx.x + blockIdx.y * gridDim.x;
    const bool trb = G.trace != nullptr && tid == 0, trp = trb && bid == G.trace_blk;
    if (trb) {
        G.trace[64 + 3 * bid] = wall_clock64();
        G.trace[64 + 3 * bid + 2] = (unsigned long long)__builtin_amdgcn_s_getreg((4) | (31 << 11)) |
                                    ((unsigned long long)__builtin_amdgcn_s_getreg((20) | (31 << 11)) << 32);
    }
#define GEMM_TP(slot) \
    if (trp) G.trace[slot] = wall_clock64();
    GEMM_TP(0);
    if (trb && bid == 0) {
        G.trace[60] = (unsigned long long)M | ((unsigned long long)N << 20) | ((unsigned long long)K << 40);
        G.trace[61] = (unsigned long long)BM | ((unsigned long long)BN << 16) | ((unsigned long long)gridDim.x << 32);
        G.trace[62] = gridDim.y;
    }

    // XCD-aware tile order: consecutive tile ids (the N tiles of one M tile, which
    // share the A rows) land on one XCD, whose L2 then serves the A re-reads.
    const int ntiles = n_mtiles * n_ntiles;
    int tile = blockIdx.x;
    if (ntiles >= 8) {
        const int q = ntiles / 8, rmd = ntiles % 8, xcd = tile % 8, loc = tile / 8;
        tile = (xcd < rmd ? xcd * (q + 1) : rmd * (q + 1) + (xcd - rmd) * q) + loc;
    }
    int split = blockIdx.y;
    if constexpr (WGRAD) {
        if (G.pair_ps > 0) {
            const int total = gridDim.x * gridDim.y, L = blockIdx.x + blockIdx.y * gridDim.x;
            const int q = total / 8, rmd = total % 8, xcd = L % 8, loc = L / 8;
            const int w = (xcd < rmd ? xcd * (q + 1) : rmd * (q + 1) + (xcd - rmd) * q) + loc;
            const int unit = w >> 1, chunk = unit / gridDim.y;
            split = unit - chunk * gridDim.y;
            tile = (w & 1) * G.pair_ps + chunk;  // n_ntiles == 1
        }
    }
    const int mt = tile / n_ntiles, nt = tile - mt * n_ntiles;
    const int m0 = mt * BM, n0 = nt * BN;
    int kbeg = 0, kend = K;
    if constexpr (WGRAD) {
        kbeg = split * G.k_per_split;
        kend = min(K, kbeg + G.k_per_split);
    }
    const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;

    SA sa;
    SB sb;
    SCS ss;
    sa.init(A, m0, wave, lane);
    sb.init(B, n0, wave, lane);
    if constexpr (F8) ss.init(A, B, m0, n0, wave, lane);
    const Rsrc ra = make_rsrc(A.base), rb = make_rsrc(B.base);
    Rsrc rsa = ra, rsb = rb;
    if constexpr (F8) {
        rsa = make_rsrc(A.sc);
        rsb = make_rsrc(B.sc);
    }
    auto issue = [&](int stage, int k0) {
        char *base = smem + stage * STAGE;
        sa.issue(A, ra, k0, kend, base, wave, lane);
        sb.issue(B, rb, k0, kend, base + A_STAGE, wave, lane);
        if constexpr (F8) ss.issue(A, B, rsa, rsb, k0, base + A_STAGE + B_STAGE, wave, lane);
    };

    float4v acc[TM][TN];
    static_for<TM>([&](auto I) {
        static_for<TN>([&](auto J) { acc[I][J] = float4v{0.f, 0.f, 0.f, 0.f}; });
    });

    const bool do_bsum = WGRAD && G.bias_slab != nullptr && mt == 0 && !BKC;
    float bsum = 0.f;

    // ST-stage LDS ring: stages kt .. kt+ST-2 are in flight while kt is consumed;
    // the counted wait retires only stage kt (never vmcnt(0) in steady state)
    // (plain statements: a lambda around `issue` makes the stager's offset arrays
    // address-taken and sends them to scratch)
    EpiPre epre{0.f, 0.f, 0.f, 1.f};
    if constexpr (!WGRAD) epre = epi_params<BN, 64 * NW>(E, N, n0, tid);
    // a two-part k-contiguous A ([x(t + d0) | x(t + d1)], K = 2 x part width): the K-steps
    // alternate between the parts, so each 64-column chunk of the source rows is fetched
    // for both parts while it is still in L2 (in part order the second pass misses)
    int kil = 0;
    if constexpr (!WGRAD && !F8 && AKC && AMD == OP_P2)
        // (wide parts only: a narrow part's second pass is a few K-steps away and still hits)
        kil = (A.nparts == 2 && A.pw % BK == 0 && A.pw >= 8 * BK && K == 2 * A.pw && G.kil) ? A.pw : 0;
    auto kofs = [&](int kt) { return kbeg + (kil ? (kt & 1) * kil + (kt >> 1) * BK : kt * BK); };
    uint4 *const mlut = reinterpret_cast<uint4 *>(smem + ST * STAGE);
    if constexpr (MK) {
        mask_lut_fill(mlut, tid, NTH);
        __syncthreads();
    }
    if (nk > 0) issue(0, kofs(0));
    if (ST >= 3 && nk > 1) issue(1, kofs(1));
    if (ST >= 4 && nk > 2) issue(2, kofs(2));
    GEMM_TP(1);
    for (int kt = 0; kt < nk; ++kt) {
        if (kt + ST - 2 < nk) wait_vmcnt<LPT * (ST - 2)>();
        else wait_vmcnt<0>();
        if constexpr (MK) {
            // ST == 2: the wait above retired this stage's chunks and mask bytes
            char *stg = smem + (kt % ST) * STAGE;
            if constexpr (AMK) sa.apply_mask(stg, mlut, wave, lane);
            if constexpr (BMK) sb.apply_mask(stg + A_STAGE, mlut, wave, lane);
            __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the masked chunks are in LDS
        }
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        if (kt < 40) GEMM_TP(2 + kt);
        if (kt + ST - 1 < nk) issue((kt + ST - 1) % ST, kofs(kt + ST - 1));
        const char *ta = smem + (kt % ST) * STAGE;
        const char *tb = ta + A_STAGE;
        if constexpr (F8) {
            // one v_mfma_scale_f32_16x16x128_f8f6f4 per (I, J) per K-step: lane l holds
            // bytes [16g, 16g+16) and [64+16g, 64+16g+16) of its row (g = l>>4) — the
            // chunks the fp16 fragment loads of s = 0, 1 return — and supplies the
            // E8M0 scale of block g of row l&15 (lane maps measured on the MI355X,
            // scripts/probe_mx.py)
            const unsigned *sct = reinterpret_cast<const unsigned *>(tb + B_STAGE);
            const int g8 = 8 * (lane >> 4);
            typedef int v8i __attribute__((ext_vector_type(8)));
            v8i fa[TM], fb[TN];
            int sca[TM], scb[TN];
            static_for<TM>([&](auto I) {
                const int r = wm * WTM + I * 16;
                half8 lo = load_frag<true, BM>(ta, r, 0, lane), hi = load_frag<true, BM>(ta, r, 1, lane);
                fa[I] = __builtin_shufflevector(__builtin_bit_cast(v4i_t, lo), __builtin_bit_cast(v4i_t, hi),
                                                0, 1, 2, 3, 4, 5, 6, 7);
                sca[I] = (int)((sct[r + (lane & 15)] >> g8) & 0xFF);
            });
            static_for<TN>([&](auto J) {
                const int c = wn * WTN + J * 16;
                half8 lo = load_frag<true, BN>(tb, c, 0, lane), hi = load_frag<true, BN>(tb, c, 1, lane);
                fb[J] = __builtin_shufflevector(__builtin_bit_cast(v4i_t, lo), __builtin_bit_cast(v4i_t, hi),
                                                0, 1, 2, 3, 4, 5, 6, 7);
                scb[J] = (int)((sct[BM + c + (lane & 15)] >> g8) & 0xFF);
            });
            static_for<TM>([&](auto I) {
                static_for<TN>([&](auto J) {
                    acc[I][J] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
                        fa[I], fb[J], acc[I][J], 0, 0, 0, sca[I], 0, scb[J]);
                });
            });
        } else
        static_for<BK / 32>([&](auto S) {
            constexpr int s = decltype(S)::value;
            half8 fa[TM], fb[TN];
            static_for<TM>([&](auto I) { fa[I] = load_frag<AKC, BM>(ta, wm * WTM + I * 16, s, lane); });
            static_for<TN>([&](auto J) { fb[J] = load_frag<BKC, BN>(tb, wn * WTN + J * 16, s, lane); });
            static_for<TM>([&](auto I) {
                static_for<TN>([&](auto J) {
                    acc[I][J] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[I], fb[J], acc[I][J], 0, 0, 0);
                });
            });
        });
        if constexpr (WGRAD && !BKC) {
            if (do_bsum && tid < BN) {
                for (int r = 0; r < BK; ++r) {
                    const char *p = tb + mn_off<BN>(r, tid >> 2) + 2 * (tid & 3);
                    bsum += (float)*reinterpret_cast<const h16 *>(p);
                }
            }
        }
        __builtin_amdgcn_sched_barrier(0);
    }

    if constexpr (WGRAD) {
        float *slab = G.slab + (long long)split * M * N;
        static_for<TM>([&](auto I) {
            static_for<TN>([&](auto J) {
                const int n = n0 + wn * WTN + J * 16 + (lane & 15);
                static_for<4>([&](auto EI) {
                    const int m = m0 + wm * WTM + I * 16 + 4 * (lane >> 4) + EI;
                    if (m < M && n < N) slab[(long long)m * N + n] = acc[I][J][decltype(EI)::value];
                });
            });
        });
        if (do_bsum && tid < BN && n0 + tid < N)
            G.bias_slab[(long long)split * N + n0 + tid] = bsum;
    } else {
        GEMM_TP(42);
        fused_epilogue<BM, BN, WM, WN>(acc, smem, E, M, N, m0, n0, tid, lane, wave, &epre);
        if constexpr (F8) {
            if (G.eo && mt == n_mtiles - 1) {
                // the clamped-edge row of the TDNN-F affine input gradient in fp16 (its second
                // part is a sum of rows, which the MXFP8 operand does not hold): one wave per
                // output column, 8-element chunks per lane, fixed-order wave reduction
                for (int j = n0 + wave; j < min(n0 + BN, N); j += NW) {
                    const h16 *w0 = G.ew + (long long)j * G.ecols, *w1 = G.ew + (long long)(N + j) * G.ecols;
                    float a = 0.f;
                    for (int c = 8 * lane; c < G.ecols; c += 8 * 64) {
                        const half8 x = load_h8(G.ex0 + c), y = load_h8(G.ex1 + c), u = load_h8(w0 + c),
                                    v = load_h8(w1 + c);
#pragma unroll
                        for (int e = 0; e < 8; ++e) a = fmaf((float)x[e], (float)u[e], fmaf((float)y[e], (float)v[e], a));
                    }
#pragma unroll
                    for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o);
                    if (lane == 0) G.eo[j] = f2h(a);
                }
            }
        }
    }
    GEMM_TP(43);
    if (trb) G.trace[64 + 3 * bid + 1] = wall_clock64();
#undef GEMM_TP
}

// ---------------------------------------------------------------------------
// Convolution with the input halo resident in LDS (forward, and the input gradient
// as a transposed convolution). The im2col GEMM above stages every tap's A rows
// through LDS separately, so a 3x3 conv moves each source element ~9x from L2;
// here a tile's source frames x heights x 64 channels land ONCE per channel chunk
// (one LDS-DMA sweep, zero rows for the time and height padding) and every tap's
// A fragment is read from that image at a per-tap row offset. The reduction runs
// chunk-major, tap-minor: K-step (c, p) = 64 channels of chunk c under tap p, so
// B (weights) still streams one 64-row slab per step through a 2-stage ring, and
// the halo of chunk c + 1 is issued in ntaps slices alongside, into the other of
// two halo buffers.
//
// Halo image: row R = f * hpos + pos holds source frame tbase + f and padded
// height shp = idx * hmul + par, where pos = par * hpe + idx (heights de-interleaved
// by parity when hmul = 2, so consecutive output heights read consecutive rows for
// every tap); 128 bytes per row. Row R's 16-byte chunk c sits at halo_off(R, c): 1 KiB
// piece R / 8, 16-byte slot (c + 2R) mod 16 of 256-byte block c / 2. A fragment read
// (16 lanes per ds_read_b128 group: eight rows at chunk c0, eight at c0 + 1, c0 even)
// then hits 16 distinct slots whenever its rows are consecutive halo rows, whatever the
// first row; with hpos = hout (mod 8) the rows of 16 consecutive output rows are
// consecutive modulo 8 across frame boundaries too (the host pads hpos when the LDS
// allows). The kc_off swizzle ((R >> 1) & 7) was 2-way conflicted for half of the
// starting rows and at every frame boundary (SQ_LDS_BANK_CONFLICT 0.30-0.40 of the
// LDS cycles).
// Output row m = (t, h) under tap p reads halo row
//     (t - tbase) * hpos + h + ctap[p]
// with ctap[p] = (dt_p - dtmin) * hpos + ((dh_p + pad) % hmul) * hpe + (dh_p + pad) / hmul.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int halo_off(int R, int c) {
    return (R >> 3) * 1024 + 256 * (c >> 1) + 16 * ((c + 2 * R) & 15);
}
struct HaloArgs {
    const h16 *x;           // source [T x ...] rows of ld elements, heights of pw channels
    long long ld;
    int T, hout, hmul, hsrc, pw, pad, hpe, hpos, nf, dtmin;
    int ntaps, nch;         // taps, 64-channel chunks per tap
    int ts, toff;           // output frame t reads source frames ts * t + toff + dt (1 / 0: plain)
    int rows;               // halo rows per chunk image (nf * hpos)
    int npieces;            // 1 KiB LDS-DMA pieces per image (ceil(rows / 8))
    int slice;              // pieces issued per step (ceil(npieces / ntaps))
    int halo_bytes;         // per image, 1 KiB multiple
    int nbuf;               // halo images (2 when nch > 1)
    int ctap[KF_MAX_PARTS];
    int bshift[KF_MAX_PARTS];  // BROW: row shift of tap p's weight block (op_wrows)
    unsigned mhpos;            // ceil(2^32 / hpos): R / hpos = umulhi(R, mhpos)
    unsigned long long *trace;  // diagnostics (kf_halo_trace): block 300 wave 0 stamps, else null
};

// s_waitcnt vmcnt(n) for a wave-uniform run-time n <= 15
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

// BROW: B is op_wrows' shifted weight rows (input gradient); the kernel then stages
// it as a plain 64-column operand whose base moves per step (scalar), instead of
// re-deriving every chunk's part offsets as the general stager would each step.
// ST: B ring stages. With ST > 2 the waits are counted (every wave knows how many
// loads it issued in each step: its share of that step's halo slice plus its B
// chunks), so ST - 2 weight stages stay in flight across each barrier.
template <int BM, int BN, int WM, int WN, bool BKC, int BMODE, bool BROW, int ST>
__global__ __launch_bounds__(64 * WM * WN, 1) void conv_halo_kernel(int M, int N, OpD B, KfEpilogue E,
                                                                    HaloArgs H, int n_mtiles,
                                                                    int n_ntiles) {
    constexpr int NW = WM * WN;
    constexpr int WTM = BM / WM, WTN = BN / WN;
    constexpr int TM = WTM / 16, TN = WTN / 16;
    constexpr int B_STAGE = BN * BK * 2;
    // Waves 0 .. NWB-1 stage B (weights, L2), the others the next chunk's halo slices
    // (HBM). vmcnt is per wave and loads retire in order, so a B wave's per-step wait no
    // longer queues behind halo loads, and a halo wave waits only at a chunk start: the
    // slices get the whole chunk to land instead of one step.
    constexpr int NWB = NW / 2;
    using SB = Stager<BKC, BN, BMODE, NWB>;
    static_assert(SB::EVEN, "uniform B loads per B wave");
    static_assert(ST == 2, "the split-wave waits are written for a two-stage B ring");
    extern __shared__ __attribute__((aligned(16))) char dsm[];
    char *bring = dsm + H.nbuf * H.halo_bytes;  // ST B stages after the halo images

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / WN, wn = wave % WN;

    // XCD-aware tile order (as gemm_kernel): the N tiles of one M tile share an XCD
    const int ntiles = n_mtiles * n_ntiles;
    int tile = blockIdx.x;
    if (ntiles >= 8) {
        const int q = ntiles / 8, rmd = ntiles % 8, xcd = tile % 8, loc = tile / 8;
        tile = (xcd < rmd ? xcd * (q + 1) : rmd * (q + 1) + (xcd - rmd) * q) + loc;
    }
    const int mt = tile / n_ntiles, nt = tile - mt * n_ntiles;
    const int m0 = mt * BM, n0 = nt * BN;
    const int tbase = H.ts * (m0 / H.hout) + H.toff + H.dtmin;

    const bool bwave = wave < NWB;
    SB sb;
    if (bwave) sb.init(B, n0, wave, lane);
    const Rsrc rx = make_rsrc(H.x), rb = make_rsrc(B.base);
    const int K = H.ntaps * H.pw;

    // halo pieces [q0, q1) of chunk c into image `img`, strided over waves w0 .. w0+nw-1
    auto halo_issue = [&](int c, int img, int q0, int q1, int w0, int nw) {
        char *dst = dsm + img * H.halo_bytes;
        // lane l fills 16-byte position l of the piece: chunk kc, row 8q + r with
        // halo_off(R, kc) = 1024 q + 16 l (block kc / 2 = l / 16, slot (kc + 2r) mod 16 = l mod 16)
        const int slot = lane & 15, kc = 2 * (lane >> 4) + (slot & 1), r = ((slot - kc) & 15) >> 1;
        if (wave < w0) return;
        for (int q = q0 + wave - w0; q < q1; q += nw) {
            const int R = 8 * q + r;
            unsigned voff = BAD;
            if (R < H.rows) {
                // f = R / hpos by multiply-high (exact for every R < rows: host-checked);
                // hmul <= 2, so the parity half is one compare
                const int f = (int)__umulhi((unsigned)R, H.mhpos), pos = R - f * H.hpos;
                const int par = pos >= H.hpe ? 1 : 0, idx = pos - par * H.hpe;
                const int sh = idx * H.hmul + par - H.pad, t = tbase + f;
                if ((unsigned)t < (unsigned)H.T && (unsigned)sh < (unsigned)H.hsrc)
                    voff = (unsigned)(((long long)t * H.ld + (long long)sh * H.pw + c * BK + kc * 8) * 2);
            }
            lds_dma<16>(rx, dst + q * 1024, voff);
        }
    };

    // per-lane halo row of each 16-row group's row for tap 0 offset 0
    int rb0[TM];
    static_for<TM>([&](auto I) {
        const int r = wm * WTM + I * 16 + (lane & 15);
        const int m = min(m0 + r, M - 1);
        const int t = m / H.hout, h = m - t * H.hout;
        rb0[I] = (H.ts * t + H.toff - tbase + H.dtmin) * H.hpos + h;
    });

    float4v acc[TM][TN];
    static_for<TM>([&](auto I) {
        static_for<TN>([&](auto J) { acc[I][J] = float4v{0.f, 0.f, 0.f, 0.f}; });
    });

    const int steps = H.nch * H.ntaps;
    auto issue_b = [&](int st1, char *dst) {
        const int c1 = st1 / H.ntaps, p1 = st1 - c1 * H.ntaps;
        if (!bwave) return;
        if constexpr (BROW) {
            const h16 *bb = B.base + (long long)H.bshift[p1] * B.ld + c1 * BK;
            sb.issue(B, make_rsrc(bb), 0, BK, dst, wave, lane);
        } else {
            sb.issue(B, rb, p1 * H.pw + c1 * BK, K, dst, wave, lane);
        }
    };
    const bool tr = H.trace && blockIdx.x == 300 && tid == 0;
#define HALO_TP(slot) \
    if (tr && (slot) < 128) H.trace[slot] = wall_clock64();
    HALO_TP(0);
    const EpiPre epre = epi_params<BN, 64 * NW>(E, N, n0, tid);
    halo_issue(0, 0, 0, H.npieces, 0, NW);
    if (steps > 0) issue_b(0, bring);
    int sb_st = 0;  // B stage of step st
    for (int st = 0; st < steps; ++st) {
        const int c = st / H.ntaps, p = st - c * H.ntaps;
        // B waves: B(st), issued in step st - 1; halo waves: the whole halo of chunk c at
        // its first step (its slices were issued over chunk c - 1's steps)
        if (bwave || p == 0) wait_vmcnt<0>();
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        HALO_TP(1 + 2 * st);
        if (H.nbuf == 1 && c > 0 && p == 0) {
            // one halo image (two do not fit beside the B ring): every wave is past the
            // previous chunk's last fragment reads, so reload it in place and wait
            halo_issue(c, 0, 0, H.npieces, 0, NW);
            wait_vmcnt<0>();
            __builtin_amdgcn_s_barrier();
            __builtin_amdgcn_sched_barrier(0);
        }
        // the halo slice first, then the B stage (the order the waits above count)
        if (H.nbuf > 1 && c + 1 < H.nch) {
            const int q0 = p * H.slice;
            halo_issue(c + 1, (c + 1) & 1, q0, min(H.npieces, q0 + H.slice), NWB, NW - NWB);
        }
        if (st + 1 < steps) issue_b(st + 1, bring + (sb_st ^ 1) * B_STAGE);
        const char *ta = dsm + (H.nbuf > 1 ? (c & 1) : 0) * H.halo_bytes;
        const char *tb = bring + sb_st * B_STAGE;
        sb_st = sb_st + 1 == ST ? 0 : sb_st + 1;
        const int ct = __builtin_amdgcn_readfirstlane(H.ctap[p]);
        static_for<BK / 32>([&](auto S) {
            constexpr int s = decltype(S)::value;
            half8 fa[TM], fb[TN];
            static_for<TM>([&](auto I) {
                const int R = rb0[I] + ct;
                fa[I] = *reinterpret_cast<const half8 *>(ta + halo_off(R, s * 4 + (lane >> 4)));
            });
            static_for<TN>([&](auto J) { fb[J] = load_frag<BKC, BN>(tb, wn * WTN + J * 16, s, lane); });
            static_for<TM>([&](auto I) {
                static_for<TN>([&](auto J) {
                    acc[I][J] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[I], fb[J], acc[I][J], 0, 0, 0);
                });
            });
        });
        __builtin_amdgcn_sched_barrier(0);
        HALO_TP(2 + 2 * st);
    }
    HALO_TP(126);
    fused_epilogue<BM, BN, WM, WN, BROW>(acc, dsm, E, M, N, m0, n0, tid, lane, wave, &epre);
    HALO_TP(127);
#undef HALO_TP
}

// split-K reduction: dst[m][n] (+)= sum_s slab[s][m][n], summed in split order (the
// result does not depend on the launch shape). Each thread owns 4 consecutive columns
// and keeps 8 slab loads in flight; the scalar form (one dependent load chain per
// element) ran at ~1.2 TB/s.
__device__ __forceinline__ void slab_reduce_body(const float *slab, int splits, int M, int N, float *dst,
                                                 long long ldw, int accumulate, int bid, int nblk,
                                                 const float *cs) {
    const long long total = (long long)M * N;
    const long long step = (long long)nblk * blockDim.x;
    if ((N & 3) == 0) {
        const long long t4 = total >> 2;
        const float4v *s4 = reinterpret_cast<const float4v *>(slab);
        for (long long i = (long long)bid * blockDim.x + threadIdx.x; i < t4; i += step) {
            float4v acc = {0.f, 0.f, 0.f, 0.f};
            int k = 0;
            for (; k + 8 <= splits; k += 8) {
                float4v v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) v[u] = __builtin_nontemporal_load(s4 + (k + u) * t4 + i);
#pragma unroll
                for (int u = 0; u < 8; ++u) acc += v[u];
            }
            for (; k < splits; ++k) acc += __builtin_nontemporal_load(s4 + k * t4 + i);
            const long long e = 4 * i, m = e / N, n = e - m * N;
            float *d = dst + m * ldw + n;
            if (cs) {
#pragma unroll
                for (int u = 0; u < 4; ++u) acc[u] *= cs[n + u];
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) d[u] = accumulate ? d[u] + acc[u] : acc[u];
        }
        return;
    }
    for (long long i = (long long)bid * blockDim.x + threadIdx.x; i < total; i += step) {
        float s = 0.f;
        for (int k = 0; k < splits; ++k) s += slab[k * total + i];
        const long long m = i / N, n = i - m * N;
        if (cs) s *= cs[n];
        float *d = dst + m * ldw + n;
        *d = accumulate ? *d + s : s;
    }
}

// bias column sums over the splits: 4 waves split the slabs of 64 columns, fixed-order
// combine (the one-thread-per-column form was latency bound: 27 us for 86 splits)
__device__ __forceinline__ void slab_reduce_cols_body(const float *slab, int splits, int N, float *dst,
                                                      int accumulate, int bid, const float *cs) {
    __shared__ float part[4][64];
    const int c = bid * 64 + (threadIdx.x & 63), g = threadIdx.x >> 6;
    float s = 0.f;
    if (c < N)
        for (int k = g; k < splits; k += 4) s += slab[(long long)k * N + c];
    part[g][threadIdx.x & 63] = s;
    __syncthreads();
    if (g == 0 && c < N) {
        const int l = threadIdx.x & 63;
        float t = (part[0][l] + part[1][l]) + (part[2][l] + part[3][l]);
        if (cs) t *= cs[c];
        dst[c] = accumulate ? dst[c] + t : t;
    }
}

__global__ __launch_bounds__(256) void k_slab_reduce(const float *slab, int splits, int M, int N,
                                                     float *dst, long long ldw, int accumulate,
                                                     const float *cs) {
    slab_reduce_body(slab, splits, M, N, dst, ldw, accumulate, blockIdx.x, gridDim.x, cs);
}
// both reduces in one launch: the first ncb blocks sum the bias columns, the rest the
// dW slabs (the column job alone is a few latency-bound blocks: 9.5 us per launch)
__global__ __launch_bounds__(256) void k_slab_reduce_both(const float *slab, int splits, int M, int N,
                                                          float *dst, long long ldw, int accumulate,
                                                          const float *bias_slab, float *bias_dst, int ncb,
                                                          const float *cs) {
    if ((int)blockIdx.x < ncb)
        slab_reduce_cols_body(bias_slab, splits, N, bias_dst, accumulate, blockIdx.x, cs);
    else
        slab_reduce_body(slab, splits, M, N, dst, ldw, accumulate, blockIdx.x - ncb, gridDim.x - ncb, cs);
}

__global__ void k_rows_sum(h16 *edge, const h16 *src, long long ld, int r0, int r1, int cols,
                           const uint8_t *mask) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= cols) return;
    float s = 0.f;
    for (int r = r0; r < r1; ++r) {
        const long long i = (long long)r * ld + c;
        if (!mask || ((mask[i >> 3] >> (i & 7)) & 1u)) s += h2f(src[i]);
    }
    edge[c] = f2h(s);
}

// ---------------------------------------------------------------------------
// optional per-launch HIP-event timing (kf_prof_*), used by bench.py to price
// the dominant kernel class over the timed region on the stream it runs on
// ---------------------------------------------------------------------------
#include <algorithm>
#include <vector>

#include <hip/hip_ext.h>
namespace {
struct ProfRec {
    hipEvent_t a, b;
    int cls;
    double flops;
    double bytes;  // algorithmic HBM bytes: unique operand sources + epilogue reads / writes
    int m, n, k;   // GEMM shape (0 when the bracket is not one launch)
    int tile;      // BM * 10000 + BN, or 0
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
// classes (kf_ops.h): 0 fused GEMM, 1 wgrad GEMM, 2 chain numerator, 3 chain den, 4 conv
// halo forward / input gradient, 5 conv halo weight gradient, 6 split-K slab reduce
enum { KF_PROF_FUSED = 0, KF_PROF_WGRAD = 1, KF_PROF_HALO = 4, KF_PROF_REDUCE = 6 };

// generic bracket for other kernel classes (kf_common.h): returns a record
// index, or -1 when profiling is off
int kf_prof_start(int cls, double work) {
    if (!g_prof) return -1;
    ProfRec rec{};
    rec.a = prof_event();
    rec.b = prof_event();
    rec.cls = cls;
    rec.flops = work;
    hipEventRecord(rec.a, kf_stream());
    g_prof_recs.push_back(rec);
    return (int)g_prof_recs.size() - 1;
}
int kf_prof_start2(int cls, double flops, double bytes) {
    const int i = kf_prof_start(cls, flops);
    if (i >= 0) g_prof_recs[i].bytes = bytes;
    return i;
}
void kf_prof_stop(int idx) {
    if (idx < 0 || idx >= (int)g_prof_recs.size()) return;
    hipEventRecord(g_prof_recs[idx].b, kf_stream());
}

extern "C" void kf_prof_enable(int on) { g_prof = on != 0; }
// pre-create events for n timed launches' worth of records (two per launch), so that no
// hipEventCreate falls inside a timed region
extern "C" int kf_prof_reserve(int n) {
    while ((int)g_prof_pool.size() < 2 * n) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return -1;
        g_prof_pool.push_back(e);
    }
    return 0;
}
// sums per class since the last collect: count, milliseconds, flops, algorithmic bytes
extern "C" int kf_prof_collect2(int cls, long long *count, double *ms, double *flops, double *bytes) {
    kf_take_pending(__func__);
    long long c = 0;
    double t = 0, f = 0, by = 0;
    for (auto &r : g_prof_recs) {
        if (r.cls != cls) continue;
        hipEventSynchronize(r.b);
        kf_take_pending("kf_prof_collect2: hipEventSynchronize");
        float e = 0.f;
        hipEventElapsedTime(&e, r.a, r.b);
        kf_take_pending("kf_prof_collect2: hipEventElapsedTime");
        c++;
        t += e;
        f += r.flops;
        by += r.bytes;
    }
    if (count) *count = c;
    if (ms) *ms = t;
    if (flops) *flops = f;
    if (bytes) *bytes = by;
    return 0;
}
// every record since the last reset, in issue order (diagnostics): class, milliseconds,
// flops, GEMM shape and tile (0 for non-GEMM brackets); returns the count written
extern "C" int kf_prof_records(int max, int *cls, float *ms, double *flops, int *mnkt) {
    int i = 0;
    for (auto &r : g_prof_recs) {
        if (i >= max) break;
        hipEventSynchronize(r.b);
        float e = 0.f;
        hipEventElapsedTime(&e, r.a, r.b);
        cls[i] = r.cls;
        ms[i] = e;
        flops[i] = r.flops;
        mnkt[4 * i] = r.m;
        mnkt[4 * i + 1] = r.n;
        mnkt[4 * i + 2] = r.k;
        mnkt[4 * i + 3] = r.tile;
        ++i;
    }
    return i;
}
extern "C" int kf_prof_collect(int cls, long long *count, double *ms, double *flops) {
    return kf_prof_collect2(cls, count, ms, flops, nullptr);
}

// Algorithmic HBM bytes of one GEMM launch: each operand's SOURCE tensor read once
// (an implicit splice / im2col operand reads its [T x hsrc x part] source, not the
// K-expanded view), the epilogue's tensors read / written once, the fp32 weight
// gradient written once. The floor a perfect-reuse kernel would move.
static double op_src_bytes(const OpD &o, int f8) {
    // geometry is in 2-byte units, also for MXFP8 (there: payload bytes)
    double b = o.simple ? (double)o.nrows * o.ncols * 2.0 : (double)o.T * (o.hsrc > 0 ? o.hsrc : 1) * o.pw * 2.0;
    if (f8) b += b / 32.0;  // one E8M0 scale per 32 e4m3 values
    if (o.mk) b += b / 16.0;  // one mask bit per fp16 element
    return b;
}
static double epi_bytes(const KfEpilogue &E, long long M, long long N) {
    const double mn = (double)M * N;
    double b = 0;
    if (E.out) b += mn * 2 * (E.beta != 0.f ? 2 : 1);
    if (E.out2) b += mn * 2;
    if (E.resid) b += mn * 2;
    if (E.mask_out) b += mn / 8;
    if (E.mask_in) b += mn / 8;
    if (E.out8) b += mn + mn / 32;
    return b;
}
double kf_gemm_alg_bytes(const OpD &a, const OpD &b, const KfEpilogue &E, long long M, long long N) {
    return op_src_bytes(a, 0) + op_src_bytes(b, 0) + epi_bytes(E, M, N);
}
// (no hipEventSynchronize here: a record of a stream destroyed since, e.g. a closed network's
// weight-gradient stream, made it fail with hipErrorStreamCaptureUnsupported; re-recording an
// event, also one still in flight, is what the next launch does anyway)
extern "C" void kf_prof_reset(void) {
    kf_take_pending(__func__);
    for (auto &r : g_prof_recs) {
        g_prof_pool.push_back(r.a);
        g_prof_pool.push_back(r.b);
    }
    g_prof_recs.clear();
}

// ---------------------------------------------------------------------------
// host side: operand conversion, tile selection and launch
// ---------------------------------------------------------------------------
static bool to_dev(const KfOperand &d, OpD &o, const char *name) {
    if (!d.base) {
        kf_set_error("operand %s: null base", name);
        return false;
    }
    if (d.nparts < 1 || d.nparts > KF_MAX_PARTS || d.part_width <= 0 || d.hout < 1 || d.hdiv < 1 ||
        (d.hdiv & (d.hdiv - 1)) || d.hdiv > 8) {
        kf_set_error("operand %s: bad addressing (nparts=%d width=%d hout=%d hdiv=%d)", name,
                     d.nparts, d.part_width, d.hout, d.hdiv);
        return false;
    }
    if (d.part_width % 8 != 0 || d.ncols % 8 != 0 || d.ld % 8 != 0 || ((uintptr_t)d.base & 15)) {
        kf_set_error("operand %s: columns / ld / base must be 16-byte granular", name);
        return false;
    }
    if (d.hout > 1 && (long long)(d.hout + BK) * d.hout >= 65536) {
        kf_set_error("operand %s: hout %d too large", name, d.hout);
        return false;
    }
    const bool f8 = d.fmt == KF_FMT_MXFP8;
    if (d.fmt != KF_FMT_FP16 && !f8) {
        kf_set_error("operand %s: unknown format %d", name, d.fmt);
        return false;
    }
    if (f8 && (!d.kcontig || d.hout != 1 || d.ncols % 128 || d.part_width % 128 || d.ld % 16 ||
               !d.scales || d.lds <= 0 || d.nparts > 2)) {
        kf_set_error("operand %s: MXFP8 needs a k-contiguous operand with hout 1, <= 2 parts, "
                     "ncols / part_width multiples of 128, ld multiple of 16 and scales", name);
        return false;
    }
    memset(&o, 0, sizeof o);
    o.base = (const h16 *)d.base;
    // MXFP8: 2-byte units for the byte movers (ld, ncols, part width halved)
    const int u = f8 ? 2 : 1;
    o.ld = d.ld / u;
    o.nrows = d.nrows;
    o.ncols = d.ncols / u;
    o.nparts = d.nparts;
    o.pw = d.part_width / u;
    o.sc = f8 ? d.scales : nullptr;
    o.lds = f8 ? (unsigned)d.lds : 0;
    o.pw8 = f8 ? d.part_width : 0;
    o.T = d.T;
    o.hout = d.hout;
    o.hsrc = d.hsrc;
    o.hmul = d.hmul;
    o.hshift = d.hdiv == 1 ? 0 : d.hdiv == 2 ? 1 : d.hdiv == 4 ? 2 : 3;
    o.tclamp = d.tpolicy == KF_CLAMP;
    o.p64 = o.pw % BK == 0;
    o.inv_hout = (65536u + d.hout - 1) / d.hout;
    bool edges = false;
    for (int i = 0; i < KF_MAX_PARTS; ++i) {
        o.dt[i] = d.dt[i];
        o.dh[i] = d.dh[i];
        o.et[i] = i < d.nparts ? d.edge_t[i] : -1;
        o.er[i] = d.edge_row[i];
        if (i < d.nparts && d.edge_t[i] >= 0) edges = true;
    }
    o.simple = d.nparts == 1 && d.hout == 1 && d.dt[0] == 0 && !edges;
    o.edges = edges;
    if (d.mask) {
        if (f8 || d.hout != 1 || d.mask_rows < 0) {
            kf_set_error("operand %s: a mask needs an fp16 operand with hout 1", name);
            return false;
        }
        o.mk = d.mask;
        const long long lim = (long long)d.mask_rows * d.ld * 2;
        o.mlim = lim > 0xFFFFFFF0LL ? 0xFFFFFFF0u : (unsigned)lim;
    }
    if (d.tmul < 0 || d.t0 < 0 || (d.tmul > 1 && (f8 || d.hout < 2))) {
        kf_set_error("operand %s: time-strided rows (tmul=%d t0=%d) need an fp16 conv operand", name, d.tmul, d.t0);
        return false;
    }
    o.tmul = d.tmul > 1 ? d.tmul : 1;
    o.t0 = d.t0;
    o.ldb = (unsigned)(d.ld * 2 / u);
    o.pwb = (unsigned)(d.part_width * 2 / u);
    // 32-bit byte offsets (buffer addressing): the largest source row must fit
    long long rows = d.nrows;
    if (!o.simple) {
        rows = d.T + 2;
        for (int i = 0; i < d.nparts; ++i)
            if (d.edge_t[i] >= 0 && d.edge_row[i] + 1 > rows) rows = d.edge_row[i] + 1;
    }
    if (rows * d.ld * 2 / u >= (1LL << 32) - 64 || (f8 && rows * d.lds >= (1LL << 32) - 64)) {
        kf_set_error("operand %s: %lld x %lld elements exceed 32-bit buffer addressing", name, rows,
                     d.ld);
        return false;
    }
    return true;
}

static int op_mode(const OpD &o) {
    if (o.simple) return OP_SIMPLE;
    if (o.nparts <= 2 && o.hout == 1 && o.hmul == 0 && o.hshift == 0) return OP_P2;
    return OP_GEN;
}
// the reduction-major general stager has no edge-row path
static bool mn_gen_ok(const OpD &o, const char *name) {
    if (op_mode(o) == OP_GEN && o.edges) {
        kf_set_error("operand %s: edge rows need a time-only (<= 2 part) reduction-major operand", name);
        return false;
    }
    return true;
}

// diagnostics: stamp the gemm_kernel launch number `at` (fused and wgrad launches, counted
// from this call): phase stamps of block `blk` and {start, end, hw id} of every block
// (wall_clock64 ticks, 100 MHz). buf holds 64 + 3 * blocks words; null = off
static unsigned long long *g_gemm_trace = nullptr;
static int g_gemm_trace_at = -1, g_gemm_trace_blk = 0, g_gemm_launches = 0;
extern "C" void kf_gemm_trace(unsigned long long *buf, int at, int blk) {
    g_gemm_trace = buf;
    g_gemm_trace_at = at;
    g_gemm_trace_blk = blk;
    g_gemm_launches = 0;
}

template <int BM, int BN, int WM, int WN, bool AKC, bool BKC, bool WGRAD, int ST, int AM, int BMODE,
          int F8 = 0>
static int launch(int M, int N, int K, const OpD &A, const OpD &B, const KfEpilogue &E,
                  const WgradArgs &G0, int splits) {
    kf_take_pending(__func__);
    const int mt = (M + BM - 1) / BM, nt = (N + BN - 1) / BN;
    dim3 grid(mt * nt, WGRAD ? splits : 1);
    WgradArgs G = G0;
    G.trace = nullptr;
    if (g_gemm_trace && g_gemm_launches++ == g_gemm_trace_at) {
        G.trace = g_gemm_trace;
        G.trace_blk = g_gemm_trace_blk;
    }
    ProfRec rec{};
    if (g_prof) {
        rec.a = prof_event();
        rec.b = prof_event();
        rec.cls = WGRAD ? KF_PROF_WGRAD : KF_PROF_FUSED;
        rec.flops = 2.0 * M * N * (double)K * (F8 ? 2 : 1);  // K counts 2-byte units
        rec.m = M;
        rec.n = N;
        rec.k = K;
        rec.tile = BM * 10000 + BN;
        // A is [M x K] (or its K-major view), B is [K x N]; wgrad writes fp32 dW [M x N]
        rec.bytes = op_src_bytes(A, F8) + op_src_bytes(B, F8) + (WGRAD ? (double)M * N * 4 : epi_bytes(E, M, N));
        // the dispatch packet itself carries the start / stop timestamps: no marker
        // packets between kernels (event records cost ~1 ms per step of gaps)
        hipExtLaunchKernelGGL(gemm_kernel<BM, BN, WM, WN, AKC, BKC, WGRAD, ST, AM, BMODE, F8>, grid,
                              dim3(64 * WM * WN), 0, kf_stream(), rec.a, rec.b, 0, M, N, K, A, B, E, G, mt, nt);
        g_prof_recs.push_back(rec);
    } else {
        gemm_kernel<BM, BN, WM, WN, AKC, BKC, WGRAD, ST, AM, BMODE, F8>
            <<<grid, 64 * WM * WN, 0, kf_stream()>>>(M, N, K, A, B, E, G, mt, nt);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        kf_set_error("gemm launch (M=%d N=%d K=%d): %s", M, N, K, hipGetErrorString(e));
        return -1;
    }
    if (!WGRAD && E.edge_out && E.edge_r0 < E.edge_r1 &&
        (E.edge_r0 / BM != (E.edge_r1 - 1) / BM || E.edge_r1 > M || E.edge_r0 < 0))
        return kf_rows_sum_mask(E.edge_out, E.edge_src ? E.out2 : E.out, E.edge_src ? E.ldo2 : E.ldo, E.edge_r0,
                                E.edge_r1, N, nullptr);
    return 0;
}


// ---------------------------------------------------------------------------
// conv_halo_kernel dispatch: A must be a conv im2col / col2im operand (k-contiguous,
// 64-channel parts, zero time padding, no edge rows, hdiv 1, hmul 1 or 2). Returns
// 1 when launched, 0 when not applicable (the caller runs the im2col GEMM), -1 on error.
// ---------------------------------------------------------------------------
static unsigned long long *g_halo_trace = nullptr;
static int g_halo_trace_at = -1, g_halo_launches = 0;
// diagnostics: stamp block 300 of the conv-halo launch number `at` (counted from this call)
extern "C" void kf_halo_trace(unsigned long long *buf, int at) {
    g_halo_trace = buf;
    g_halo_trace_at = at;
    g_halo_launches = 0;
}
template <int BM, int BN, int WM, int WN, bool BKC, int BMODE, bool BROW, int ST>
static int launch_halo(int M, int N, const OpD &B, const KfEpilogue &E, const HaloArgs &H0, size_t lds) {
    kf_take_pending(__func__);
    const int mt = (M + BM - 1) / BM, nt = (N + BN - 1) / BN;
    HaloArgs H = H0;
    H.trace = g_halo_trace && g_halo_launches++ == g_halo_trace_at ? g_halo_trace : nullptr;
    ProfRec rec{};
    if (g_prof) {
        rec.a = prof_event();
        rec.b = prof_event();
        rec.cls = KF_PROF_HALO;
        rec.flops = 2.0 * M * N * (double)H.ntaps * H.pw;
        rec.m = M;
        rec.n = N;
        rec.k = H.ntaps * H.pw;
        rec.tile = BM * 10000 + BN;
        rec.bytes = (double)H.T * H.hsrc * H.pw * 2.0 + (double)H.ntaps * H.pw * N * 2.0 + epi_bytes(E, M, N);
        hipExtLaunchKernelGGL(conv_halo_kernel<BM, BN, WM, WN, BKC, BMODE, BROW, ST>, dim3(mt * nt),
                              dim3(64 * WM * WN), (std::uint32_t)lds, kf_stream(), rec.a, rec.b, 0, M, N, B, E, H,
                              mt, nt);
        g_prof_recs.push_back(rec);
    } else {
        conv_halo_kernel<BM, BN, WM, WN, BKC, BMODE, BROW, ST>
            <<<dim3(mt * nt), 64 * WM * WN, lds, kf_stream()>>>(M, N, B, E, H, mt, nt);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        kf_set_error("conv halo launch (M=%d N=%d): %s", M, N, hipGetErrorString(e));
        return -1;
    }
    return 1;
}

static int conv_halo_try(int M, int N, int K, const OpD &a, const OpD &b, int bm, bool bkc,
                         const KfEpilogue &E) {
    if (op_mode(a) != OP_GEN || !a.p64 || a.edges || a.tclamp || a.hshift ||
        a.hmul < 1 || a.hmul > 2 || a.hout < 2 || a.ncols != K || a.nparts * a.pw != K)
        return 0;
    if (bkc ? bm != OP_GEN : bm != OP_SIMPLE) return 0;
    if (E.edge_out) return 0;  // the edge-row sum is the tiled kernel's (launch<> has its fallback)
    // shifted weight rows (op_wrows): every tap's block lies inside the matrix
    bool brow = bkc && b.hout == 1 && b.hmul == 0 && !b.hshift && !b.edges && !b.tclamp &&
                b.nparts == a.nparts && b.pw == a.pw;
    for (int p = 0; brow && p < b.nparts; ++p) brow = b.dt[p] >= 0 && b.dt[p] + b.nrows <= b.T;
    if (bkc && !brow) return 0;
    if (E.row_group && !brow) return 0;  // grouped rows: the input-gradient (BROW) kernels only
    OpD bp = b;
    if (brow) {  // one 64-column chunk of a plain [nrows x ld] matrix, rebased per step
        bp.simple = 1;
        bp.nparts = 1;
        bp.ncols = BK;
        bp.pw = BK;
        bp.T = b.nrows;
        for (int p = 0; p < KF_MAX_PARTS; ++p) bp.dt[p] = bp.dh[p] = 0;
    }
    int dtmin = 1 << 20, dtmax = -(1 << 20), dhmin = 1 << 20, dhmax = -(1 << 20);
    for (int p = 0; p < a.nparts; ++p) {
        dtmin = std::min(dtmin, a.dt[p]);
        dtmax = std::max(dtmax, a.dt[p]);
        dhmin = std::min(dhmin, a.dh[p]);
        dhmax = std::max(dhmax, a.dh[p]);
    }
    HaloArgs H;
    memset(&H, 0, sizeof H);
    H.x = a.base;
    H.ld = a.ld;
    H.T = a.T;
    H.hout = a.hout;
    H.hmul = a.hmul;
    H.hsrc = a.hsrc;
    H.pw = a.pw;
    H.pad = std::max(0, -dhmin);
    const int maxshp = (a.hout - 1) * a.hmul + dhmax + H.pad;
    const int HP = std::max(a.hsrc + H.pad, maxshp + 1);
    const int hpe0 = (HP + a.hmul - 1) / a.hmul;
    H.dtmin = dtmin;
    H.ntaps = a.nparts;
    H.nch = a.pw / BK;
    // 32-bit source offsets: the largest byte offset the halo can form
    if (((long long)a.T * a.ld + (long long)a.hsrc * a.pw) * 2 >= (1LL << 32) - 64) return 0;
    const int BN_ = N <= 64 ? 64 : N <= 128 ? 128 : 256;
    // 256-row tiles, except 128-row tiles for the strided convs' per-residue input
    // gradients (3 or 6 taps; two workgroups per CU): cnn3 461 -> 332 and 588 -> 460 us,
    // cnn5 370 -> 317 and 536 -> 468 us
    static const int env_rbm = getenv("KF_HALO_RES_BM") ? atoi(getenv("KF_HALO_RES_BM")) : 128;
    const bool residue = a.nparts < 9 && env_rbm != 256;  // (B as shifted weight rows or a transposed copy)
    // time-strided rows (a.tmul > 1): a tile's output frames read tmul times the source
    // frames, so 128-row tiles keep the image in LDS
    // (KF_HALO_BM=128: 128-row tiles for every halo conv, A/B)
    static const int env_hbm = getenv("KF_HALO_BM") ? atoi(getenv("KF_HALO_BM")) : 256;
    const int BM_ = residue || a.tmul > 1 || env_hbm == 128 ? 128 : 256;
    H.ts = a.tmul;
    H.toff = a.t0;
    H.nf = H.ts * ((BM_ - 1 + a.hout - 1) / a.hout) + 1 + (dtmax - dtmin);
    const int nw = BN_ == 64 ? 4 : 8;
    const size_t epi = 16 * BN_ + 32 * EpiMap<64>::LDT * 4 * nw;
    // LDS of a halo geometry: two images when there are several channel chunks, else one
    // (two too large, e.g. cnn5's stride-2 forward: 80 KB each beside a 64 KB B ring: one
    // image, reloaded between channel chunks)
    auto geometry = [&](int hpe, int &nbuf, int &halo_bytes) {
        halo_bytes = (H.nf * hpe * a.hmul + 7) / 8 * 1024;
        nbuf = H.nch > 1 ? 2 : 1;
        size_t l = std::max((size_t)nbuf * halo_bytes + 2 * BN_ * BK * 2, epi);
        if (l > 160 * 1024 && nbuf == 2) {
            nbuf = 1;
            l = std::max((size_t)halo_bytes + 2 * BN_ * BK * 2, epi);
        }
        return l;
    };
    int nb0, hb0;
    const size_t lds0 = geometry(hpe0, nb0, hb0);
    // hpos = hout (mod 8): conflict-free fragment reads across frame boundaries (halo_off),
    // taken when it keeps the image count and the workgroups per CU (80 KB: two)
    // (bounded: with hmul = 2 and an odd hout no pitch qualifies, so no pad is taken)
    int hpe = hpe0;
    while (hpe < hpe0 + 8 && (hpe * a.hmul - a.hout) % 8) ++hpe;
    const bool found8 = (hpe * a.hmul - a.hout) % 8 == 0;
    int nb1 = nb0, hb1 = hb0;
    const size_t lds1 = found8 ? geometry(hpe, nb1, hb1) : lds0;
    const bool pad8 = found8 && lds1 <= 160 * 1024 && nb1 == nb0 && (lds0 > 80 * 1024 || lds1 <= 80 * 1024);
    if (!pad8) hpe = hpe0;
    H.hpe = hpe;
    H.hpos = hpe * a.hmul;
    H.nbuf = pad8 ? nb1 : nb0;
    H.halo_bytes = pad8 ? hb1 : hb0;
    const size_t lds = pad8 ? lds1 : lds0;
    if (lds > 160 * 1024) return 0;
    H.rows = H.nf * H.hpos;
    H.npieces = (H.rows + 7) / 8;
    H.mhpos = (unsigned)((0x100000000ULL + H.hpos - 1) / H.hpos);
    if (a.hmul > 2) return 0;
    for (unsigned R = 0; R < (unsigned)(8 * H.npieces); ++R)
        if ((unsigned)(((unsigned long long)R * H.mhpos) >> 32) != R / (unsigned)H.hpos) return 0;
    H.slice = (H.npieces + H.ntaps - 1) / H.ntaps;
    for (int p = 0; p < a.nparts; ++p) {
        const int x = a.dh[p] + H.pad;
        H.ctap[p] = (a.dt[p] - dtmin) * H.hpos + (x % a.hmul) * H.hpe + x / a.hmul;
        H.bshift[p] = brow ? b.dt[p] : 0;
    }
    // (measured and dropped: a 4-stage weight ring at one workgroup per CU, cnn2 517 ->
    // 884 us; 64-column tiles on two 128x64-tile waves, cnn2 529 -> 781 us)
#define KF_HALO(BKC_, BMODE_, BROW_)                                                                     \
    do {                                                                                                 \
        if (BN_ == 64)                                                                                   \
            return BM_ == 128 ? launch_halo<128, 64, 4, 1, BKC_, BMODE_, BROW_, 2>(M, N, bp, E, H, lds)  \
                              : launch_halo<256, 64, 4, 1, BKC_, BMODE_, BROW_, 2>(M, N, bp, E, H, lds); \
        if (BN_ == 128)                                                                                  \
            return BM_ == 128 ? launch_halo<128, 128, 4, 2, BKC_, BMODE_, BROW_, 2>(M, N, bp, E, H, lds) \
                              : launch_halo<256, 128, 4, 2, BKC_, BMODE_, BROW_, 2>(M, N, bp, E, H, lds); \
        return BM_ == 128 ? launch_halo<128, 256, 2, 4, BKC_, BMODE_, BROW_, 2>(M, N, bp, E, H, lds)     \
                          : launch_halo<256, 256, 2, 4, BKC_, BMODE_, BROW_, 2>(M, N, bp, E, H, lds);    \
    } while (0)
    if (bkc) KF_HALO(true, OP_SIMPLE, true);
    KF_HALO(false, OP_SIMPLE, false);
#undef KF_HALO
    return 0;
}


// K-step interleave of two-part spliced A operands (WgradArgs::kil): 1 = on (default),
// 0 = part order. Test hook: kf_gemm_debug_kil (kf_ops.h) compares the two orders.
static int g_kil = 1;
extern "C" void kf_gemm_debug_kil(int on) { g_kil = on != 0; }

static int fused_impl(int M, int N, int K, const KfOperand *A, const KfOperand *B, const KfEpilogue *epi,
                      const WgradArgs *edge);
extern "C" int kf_gemm_fused(int M, int N, int K, const KfOperand *A, const KfOperand *B,
                             const KfEpilogue *epi) {
    return fused_impl(M, N, K, A, B, epi, nullptr);
}
extern "C" int kf_gemm_fused_edge(int M, int N, int K, const KfOperand *A, const KfOperand *B,
                                  const KfEpilogue *epi, void *edge_out, const void *x0, const void *x1,
                                  const void *W, int cols) {
    if (!edge_out || !x0 || !x1 || !W || cols <= 0 || cols % 8 || ((uintptr_t)x0 | (uintptr_t)x1 | (uintptr_t)W) & 15 ||
        A->fmt != KF_FMT_MXFP8 || M <= 0) {
        kf_set_error("kf_gemm_fused_edge: an MXFP8 product with M > 0, an edge row and 16-byte aligned fp16 "
                     "operands, cols %% 8 == 0 (cols=%d)", cols);
        return -1;
    }
    WgradArgs g{};
    g.eo = (h16 *)edge_out;
    g.ex0 = (const h16 *)x0;
    g.ex1 = (const h16 *)x1;
    g.ew = (const h16 *)W;
    g.ecols = cols;
    return fused_impl(M, N, K, A, B, epi, &g);
}
static int fused_impl(int M, int N, int K, const KfOperand *A, const KfOperand *B, const KfEpilogue *epi,
                      const WgradArgs *edge) {
    if (M <= 0 || N <= 0) return 0;
    OpD a, b;
    if (!to_dev(*A, a, "A") || !to_dev(*B, b, "B")) return -1;
    if (N % 8 != 0) {
        kf_set_error("kf_gemm_fused: N=%d must be a multiple of 8", N);
        return -1;
    }
    if (!A->kcontig) {
        kf_set_error("kf_gemm_fused: A must be k-contiguous");
        return -1;
    }
    if (!B->kcontig && !mn_gen_ok(b, "B")) return -1;
    const KfEpilogue &E = *epi;
    if ((E.out && E.ldo % 8) || (E.out2 && E.ldo2 % 8) || (E.resid && E.ldr % 8) ||
        (E.mask_out && E.ldo % 8)) {
        kf_set_error("kf_gemm_fused: leading dimensions must be multiples of 8");
        return -1;
    }
    if (E.out8 && E.out8_src && !E.out2) {
        kf_set_error("kf_gemm_fused: out8_src = 1 needs out2");
        return -1;
    }
    if (E.row_group < 0 || (E.row_group > 0 && (E.row_stride < E.row_group || E.edge_out || edge))) {
        kf_set_error("kf_gemm_fused: row_group %d / row_stride %d (row_stride >= row_group > 0, no edge row)",
                     E.row_group, E.row_stride);
        return -1;
    }
    if (E.out8 && (N % 32 || E.ldo8 % 32 || !E.scale8)) {
        kf_set_error("kf_gemm_fused: out8 needs N and ldo8 multiples of 32 and scale8");
        return -1;
    }
    WgradArgs G{nullptr, nullptr, 0, 0, g_kil};
    if (edge) {
        G.eo = edge->eo;
        G.ex0 = edge->ex0;
        G.ex1 = edge->ex1;
        G.ew = edge->ew;
        G.ecols = edge->ecols;
    }
    const int am = op_mode(a), bm = op_mode(b);
    const bool f8 = A->fmt == KF_FMT_MXFP8;
    if (f8 != (B->fmt == KF_FMT_MXFP8)) {
        kf_set_error("kf_gemm_fused: both operands must be MXFP8, or neither");
        return -1;
    }
    if (E.row_group && (f8 || a.mk || b.mk)) {
        kf_set_error("kf_gemm_fused: grouped output rows (row_group) need an fp16 conv input gradient");
        return -1;
    }
    if (f8) {
        if (K % 128 || am == OP_GEN || a.edges || bm != OP_SIMPLE) {
            kf_set_error("kf_gemm_fused: MXFP8 needs K %% 128 == 0, a plain or time-spliced A and a "
                         "plain B (K=%d)", K);
            return -1;
        }
        const int K2 = K / 2;  // the kernel counts the reduction in 2-byte units
        if (N % 160 == 0 && N <= 320 && !E.out8) {  // TDNN-F linear (N = bottleneck): no idle columns
            if (am == OP_SIMPLE)
                return launch<384, 160, 4, 2, true, true, false, 2, OP_SIMPLE, OP_SIMPLE, 1>(M, N, K2, a, b, E, G, 1);
            return launch<384, 160, 4, 2, true, true, false, 2, OP_P2, OP_SIMPLE, 1>(M, N, K2, a, b, E, G, 1);
        }
        if (N >= 256) {
            if (am == OP_SIMPLE)
                return launch<256, 256, 2, 4, true, true, false, 2, OP_SIMPLE, OP_SIMPLE, 1>(M, N, K2, a, b, E, G, 1);
            return launch<256, 256, 2, 4, true, true, false, 2, OP_P2, OP_SIMPLE, 1>(M, N, K2, a, b, E, G, 1);
        }
        if (am == OP_SIMPLE)
            return launch<128, 128, 2, 2, true, true, false, 2, OP_SIMPLE, OP_SIMPLE, 1>(M, N, K2, a, b, E, G, 1);
        return launch<128, 128, 2, 2, true, true, false, 2, OP_P2, OP_SIMPLE, 1>(M, N, K2, a, b, E, G, 1);
    }
    if (a.mk || b.mk) {
        // masked A (the TDNN-F affine input gradient on the implicit dz, N = bottleneck):
        // 384x160 tiles for N = 160 / 320, 256x64 for N <= 64, else 128x128
        if (!b.mk && B->kcontig && !E.out8 && ((am == OP_P2 && bm == OP_P2) || (am == OP_SIMPLE && bm == OP_SIMPLE))) {
            const int mt = N % 160 == 0 && N <= 320 ? 5 : N <= 64 ? 2 : 0;
#define KF_MASKED(AM_, BM_)                                                                                    \
    do {                                                                                                       \
        if (mt == 5) return launch<384, 160, 4, 2, true, true, false, 2, AM_ | OP_MASKED, BM_>(M, N, K, a, b, E, G, 1); \
        if (mt == 2) return launch<256, 64, 4, 1, true, true, false, 2, AM_ | OP_MASKED, BM_>(M, N, K, a, b, E, G, 1);  \
        return launch<128, 128, 2, 2, true, true, false, 2, AM_ | OP_MASKED, BM_>(M, N, K, a, b, E, G, 1);               \
    } while (0)
            if (am == OP_P2) KF_MASKED(OP_P2, OP_P2);
            KF_MASKED(OP_SIMPLE, OP_SIMPLE);
#undef KF_MASKED
        }
        kf_set_error("kf_gemm_fused: a masked operand must be A (plain or two-part time splice, with a "
                     "k-contiguous B of the same kind, no MXFP8 copy) (M=%d N=%d K=%d)", M, N, K);
        return -1;
    }
    {  // the halo kernel shares fused_epilogue, MXFP8 copy included (BN >= 64)
        const int hr = conv_halo_try(M, N, K, a, b, bm, B->kcontig != 0, E);
        if (hr != 0) return hr < 0 ? -1 : 0;
    }
    if (a.tmul > 1 || a.t0 || b.tmul > 1 || b.t0 || E.row_group) {
        kf_set_error("kf_gemm_fused: time-strided rows (tmul / t0) and grouped output rows (row_group) need a "
                     "conv on the halo kernel (M=%d N=%d K=%d)", M, N, K);
        return -1;
    }
    // Tiles: 384x160 8-wave for N = 160 / 320; 256x64 for N <= 64; for
    // N >= 256 192x128 (or 128x192, below) 8-wave tiles (80 KB of LDS: two workgroups share a CU and one's
    // epilogue overlaps the other's MFMA loop; the wide K = 320 products write 2-3
    // full-width fp16 tensors; their 32-column wave tiles hold the MXFP8 copy's blocks);
    // 128x128 otherwise.
    int tile = 0;
    if (N % 160 == 0 && N <= 320 && !E.out8) tile = 5;
    else if (N <= 64) tile = 2;
    else if (N >= 256) tile = 6;  // 192x128: 32-column wave tiles, so out8 blocks fit
    // short-K wide products with N % 192 == 0: 128x192 tiles (same 80 KB, two per CU; 12 -> 8
    // column tiles per row block): TDNN-F linear input gradient 281 -> 257 us, affine forward
    // 215 -> 207 us (rocprof A/B/A/B). Not with an MXFP8 copy: its 48-column wave tiles do
    // not hold whole 32-column blocks (and 32x96 wave tiles overflow the epilogue's LDS).
    if (tile == 6 && K <= 640 && N % 192 == 0 && !E.out8) tile = 7;
    // N = 160 / 320 with few row blocks (the row-subsampled TDNN-F stack: M = T / 3): 128x160
    // 4-wave tiles, two workgroups per CU, so that the launch fills the CUs (384x160 at
    // M = 32,020 is 84 workgroups)
    if (tile == 5 && (long long)((M + 383) / 384) * ((N + 159) / 160) < 192) tile = 8;
    // (64x160 tiles instead measured 25.21 against 25.05 ms, same box: not used)
#define KF_FUSED(BKC_, AM_, BM_)                                                                 \
    do {                                                                                         \
        if (tile == 8) return launch<128, 160, 2, 2, true, BKC_, false, 2, AM_, BM_>(M, N, K, a, b, E, G, 1); \
        if (tile == 7) return launch<128, 192, 2, 4, true, BKC_, false, 2, AM_, BM_>(M, N, K, a, b, E, G, 1); \
        if (tile == 6) return launch<192, 128, 2, 4, true, BKC_, false, 2, AM_, BM_>(M, N, K, a, b, E, G, 1); \
        if (tile == 5) return launch<384, 160, 4, 2, true, BKC_, false, 2, AM_, BM_>(M, N, K, a, b, E, G, 1); \
        if (tile == 2) return launch<256, 64, 4, 1, true, BKC_, false, 2, AM_, BM_>(M, N, K, a, b, E, G, 1);  \
        return launch<128, 128, 2, 2, true, BKC_, false, 2, AM_, BM_>(M, N, K, a, b, E, G, 1);               \
    } while (0)
    if (!B->kcontig) {
        if (bm == OP_SIMPLE) {
            if (am == OP_SIMPLE) KF_FUSED(false, OP_SIMPLE, OP_SIMPLE);
            if (am == OP_P2) KF_FUSED(false, OP_P2, OP_SIMPLE);
            KF_FUSED(false, OP_GEN, OP_SIMPLE);
        }
        KF_FUSED(false, OP_GEN, OP_GEN);
    }
    if (am == OP_SIMPLE && bm == OP_SIMPLE) KF_FUSED(true, OP_SIMPLE, OP_SIMPLE);
    if (am == OP_P2 && bm == OP_SIMPLE) KF_FUSED(true, OP_P2, OP_SIMPLE);
    if (am == OP_P2 && bm == OP_P2) KF_FUSED(true, OP_P2, OP_P2);
    KF_FUSED(true, OP_GEN, OP_GEN);
#undef KF_FUSED
}

// split-K reduce of kf_gemm_wgrad's slabs (also used by conv_wgrad.hip)
void kf_wgrad_reduce(const float *slab, const float *bias_slab, int splits, int M, int N, float *dW,
                     long long ldw, float *bias_grad, int accumulate, const float *cs) {
    const int nb = kf_blocks((long long)M * N / 4 + 1, 256, 4096);
    const int ncb = bias_grad ? (N + 63) / 64 : 0;
    ProfRec rec{};
    hipEvent_t ea = nullptr, eb = nullptr;
    if (g_prof) {  // timestamps in the dispatch packet, as for the GEMMs
        ea = rec.a = prof_event();
        eb = rec.b = prof_event();
        rec.cls = KF_PROF_REDUCE;
        // the slabs read once, dW (and the bias) written once (+ read when accumulating)
        rec.bytes = ((double)splits * (M + (bias_grad ? 1 : 0)) + (accumulate ? 2.0 : 1.0) * (M + 1)) * N * 4.0;
        g_prof_recs.push_back(rec);
    }
    if (bias_grad && g_prof)
        hipExtLaunchKernelGGL(k_slab_reduce_both, dim3(ncb + nb), dim3(256), 0, kf_stream(), ea, eb, 0, slab, splits,
                              M, N, dW, ldw, accumulate, bias_slab, bias_grad, ncb, cs);
    else if (bias_grad)
        k_slab_reduce_both<<<ncb + nb, 256, 0, kf_stream()>>>(slab, splits, M, N, dW, ldw, accumulate, bias_slab,
                                                             bias_grad, ncb, cs);
    else if (g_prof)
        hipExtLaunchKernelGGL(k_slab_reduce, dim3(nb), dim3(256), 0, kf_stream(), ea, eb, 0, slab, splits, M, N, dW,
                              ldw, accumulate, cs);
    else
        k_slab_reduce<<<nb, 256, 0, kf_stream()>>>(slab, splits, M, N, dW, ldw, accumulate, cs);
}

int kf_conv_wgrad_halo_try(int M, int N, int K, const OpD &a, const OpD &b, float *dW, long long ldw,
                           float *bias_grad, int accumulate);

// workgroups per weight-gradient launch (split-K target): 512 alone on the device; nnet's
// backward sets 256 while its weight gradients run on their own stream beside the
// input-gradient chain (half the CUs each, half the fp32 slab bytes)
static thread_local int g_wgrad_target = 512;
extern "C" int kf_gemm_wgrad_target(int wgs) {
    const int old = g_wgrad_target;
    if (wgs > 0) g_wgrad_target = wgs;
    return old;
}

static int wgrad_impl(int M, int N, int K, const KfOperand *A, const KfOperand *B, float *dW, long long ldw,
                      float *bias_grad, int accumulate, const float *cs) {
    kf_take_pending(__func__);
    if (M <= 0 || N <= 0) return 0;
    OpD a, b;
    if (!to_dev(*A, a, "A") || !to_dev(*B, b, "B")) return -1;
    if (b.tmul > 1 || b.t0) {
        kf_set_error("kf_gemm_wgrad: time-strided rows (tmul / t0) only on the conv im2col operand A");
        return -1;
    }
    if (A->kcontig || B->kcontig) {
        kf_set_error("kf_gemm_wgrad: A and B must be reduction-major");
        return -1;
    }
    if (!mn_gen_ok(a, "A") || !mn_gen_ok(b, "B")) return -1;
    if (a.mk || (b.mk && (op_mode(b) != OP_SIMPLE || op_mode(a) == OP_GEN))) {
        kf_set_error("kf_gemm_wgrad: a masked operand must be a plain B (A plain or a two-part time splice)");
        return -1;
    }
    // 3x3 convolutions: the source halo in LDS instead of nine im2col slabs
    if (!b.mk) {
        const int hr = kf_conv_wgrad_halo_try(M, N, K, a, b, dW, ldw, bias_grad, accumulate);
        if (hr != 0) return hr < 0 ? -1 : 0;
    }
    if (a.tmul > 1 || a.t0) {
        kf_set_error("kf_gemm_wgrad: time-strided rows (tmul / t0) need a 3x3 conv on the halo kernel");
        return -1;
    }
    // tiles: 384x160 for N = 160 / 320 (TDNN-F linear); otherwise 64-, 128- or 256-column
    // tiles whose row count (192, 256 or 320) wastes the fewest padded rows of M
    int BMc = 256, BNc = (N % 160 == 0 && N <= 320) ? 160 : N <= 64 ? 64 : N <= 128 ? 128 : 256;
    if (BNc == 160) {
        BMc = 384;
    } else {
        const int cands[3] = {256, BNc == 256 ? 320 : 256, 192};
        long long bw = (long long)(M + 255) / 256 * 256;
        for (int c : cands) {
            const long long w = (long long)(M + c - 1) / c * c;
            if (w < bw) bw = w, BMc = c;
        }
    }
    // (r5: two workgroups per CU for the TDNN-F weight gradients, 160x128 / 128x160 tiles at
    // 72 KB, a quarter of the fp32 slab bytes: affine 121 -> 311 us, linear 126 -> 171 us per
    // launch, the reduce 25 -> 13 us; the bigger tiles' operand reuse is worth more)
    const int tiles = ((M + BMc - 1) / BMc) * ((N + BNc - 1) / BNc);
    // workgroups per launch: every split writes an M x N fp32 slab that the reduce
    // reads back, so the target trades CU fill against slab traffic
    // (targets of 256 / 384 / 768 / 1024 measured slower)
    // at most the target (rounding the split count down): beside the input-gradient chain a
    // launch with a few workgroups more than fit at once holds them pending until a whole
    // workgroup's K range retires, and the chain's launches queue behind them (a 4-row
    // edge sum took 128 us instead of 6.5; bench 36.90-37.02 -> 36.57-36.65 ms, r5)
    int splits = std::max(1, g_wgrad_target / tiles);
    const int maxsplit = (K + 4 * BK - 1) / (4 * BK);  // at least 4 K-steps per split
    if (splits > maxsplit) splits = maxsplit;
    if (splits < 1) splits = 1;
    int kps = (K + splits - 1) / splits;
    kps = (kps + BK - 1) / BK * BK;
    splits = (K + kps - 1) / kps;
    size_t slab_bytes = (size_t)splits * M * N * 4;
    size_t bias_bytes = bias_grad ? (size_t)splits * N * 4 : 0;
    char *ws = (char *)kf_workspace_stream(slab_bytes + bias_bytes + 256);
    if (!ws) {
        kf_set_error("kf_gemm_wgrad: workspace allocation of %zu bytes failed",
                     slab_bytes + bias_bytes);
        return -1;
    }
    WgradArgs G{(float *)ws,
                bias_grad ? (float *)(ws + ((slab_bytes + 255) & ~(size_t)255)) : nullptr, kps, 0, 0};
    KfEpilogue E{};
    const int am = op_mode(a), bm = op_mode(b);
    // the TDNN-F linear's [x(t - s) | x(t)]: pair the parts' tiles per XCD
    if (am == OP_P2 && A->nparts == 2 && N <= BNc && A->part_width % BMc == 0 &&
        M == 2 * A->part_width)
        G.pair_ps = A->part_width / BMc;
    int rc;
#define KF_WG(AM_, BM_)                                                                          \
    do {                                                                                         \
        if (BMc == 320 && BNc == 256)                                                            \
            rc = launch<320, 256, 2, 4, false, false, true, 2, AM_, BM_>(M, N, K, a, b, E, G, splits); \
        else if (BMc == 192 && BNc == 256)                                                       \
            rc = launch<192, 256, 2, 4, false, false, true, 2, AM_, BM_>(M, N, K, a, b, E, G, splits); \
        else if (BMc == 192 && BNc == 128)                                                       \
            rc = launch<192, 128, 4, 2, false, false, true, 2, AM_, BM_>(M, N, K, a, b, E, G, splits); \
        else if (BMc == 192 && BNc == 64)                                                        \
            rc = launch<192, 64, 4, 1, false, false, true, 2, AM_, BM_>(M, N, K, a, b, E, G, splits); \
        else if (BMc == 256 && BNc == 256)                                                       \
            rc = launch<256, 256, 2, 4, false, false, true, 2, AM_, BM_>(M, N, K, a, b, E, G, splits); \
        else if (BMc == 256 && BNc == 128)                                                       \
            rc = launch<256, 128, 4, 2, false, false, true, 2, AM_, BM_>(M, N, K, a, b, E, G, splits); \
        else if (BNc == 160)                                                                     \
            rc = launch<384, 160, 4, 2, false, false, true, 2, AM_, BM_>(M, N, K, a, b, E, G, splits); \
        else                                                                                     \
            rc = launch<256, 64, 4, 1, false, false, true, 2, AM_, BM_>(M, N, K, a, b, E, G, splits); \
    } while (0)
    if (b.mk) {
        // masked B (the TDNN-F affine weight gradient on the implicit dz, N = layer width)
        if (BNc != 256) {
            kf_set_error("kf_gemm_wgrad: masked B needs N > 128 (M=%d N=%d)", M, N);
            return -1;
        }
#define KF_WGM(AM_)                                                                                      \
    do {                                                                                                 \
        if (BMc == 320)                                                                                  \
            rc = launch<320, 256, 2, 4, false, false, true, 2, AM_, OP_SIMPLE | OP_MASKED>(M, N, K, a, b, E, G, splits); \
        else if (BMc == 192)                                                                             \
            rc = launch<192, 256, 2, 4, false, false, true, 2, AM_, OP_SIMPLE | OP_MASKED>(M, N, K, a, b, E, G, splits); \
        else                                                                                             \
            rc = launch<256, 256, 2, 4, false, false, true, 2, AM_, OP_SIMPLE | OP_MASKED>(M, N, K, a, b, E, G, splits); \
    } while (0)
        if (am == OP_SIMPLE) KF_WGM(OP_SIMPLE);
        else KF_WGM(OP_P2);
#undef KF_WGM
    } else if (bm == OP_SIMPLE && am == OP_SIMPLE) KF_WG(OP_SIMPLE, OP_SIMPLE);
    else if (bm == OP_SIMPLE && am == OP_P2) KF_WG(OP_P2, OP_SIMPLE);
    else if (bm == OP_SIMPLE) KF_WG(OP_GEN, OP_SIMPLE);
    else KF_WG(OP_GEN, OP_GEN);
#undef KF_WG
    if (rc) return rc;
    kf_wgrad_reduce(G.slab, G.bias_slab, splits, M, N, dW, ldw, bias_grad, accumulate, cs);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        kf_set_error("wgrad reduce: %s", hipGetErrorString(e));
        return -1;
    }
    return 0;
}

extern "C" int kf_gemm_wgrad(int M, int N, int K, const KfOperand *A, const KfOperand *B,
                             float *dW, long long ldw, float *bias_grad, int accumulate) {
    return wgrad_impl(M, N, K, A, B, dW, ldw, bias_grad, accumulate, nullptr);
}
extern "C" int kf_gemm_wgrad_scaled(int M, int N, int K, const KfOperand *A, const KfOperand *B, float *dW,
                                    long long ldw, float *bias_grad, int accumulate, const float *col_scale) {
    if (!col_scale) {
        kf_set_error("kf_gemm_wgrad_scaled: null col_scale");
        return -1;
    }
    return wgrad_impl(M, N, K, A, B, dW, ldw, bias_grad, accumulate, col_scale);
}

extern "C" int kf_rows_sum_mask(void *edge, const void *src, long long ld, int r0, int r1, int cols,
                                const uint8_t *mask) {
    kf_take_pending(__func__);
    if (cols <= 0) return 0;
    k_rows_sum<<<(cols + 255) / 256, 256, 0, kf_stream()>>>((h16 *)edge, (const h16 *)src, ld,
                                                            r0, r1, cols, mask);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        kf_set_error("rows_sum: %s", hipGetErrorString(e));
        return -1;
    }
    return 0;
}
extern "C" int kf_rows_sum(void *edge, const void *src, long long ld, int r0, int r1, int cols) {
    return kf_rows_sum_mask(edge, src, ld, r0, r1, cols, nullptr);
}

// out[j] = rne_fp16(x0 . W[j] + x1 . W[rows + j]) for j < rows (W [2*rows x cols], fp32
// accumulation): one row of a two-part product, e.g. the clamped-edge row T-1 of the MXFP8
// affine input gradient (network.cpp). A workgroup per output element: a one-row GEMM would
// walk K on two workgroups.
__global__ __launch_bounds__(256) void k_dot2_rows(h16 *out, const h16 *x0, const h16 *x1, const h16 *W, int rows,
                                                   int cols) {
    __shared__ float part[4];
    const int j = blockIdx.x;
    const h16 *w0 = W + (long long)j * cols, *w1 = W + (long long)(rows + j) * cols;
    float acc = 0.f;
    for (int c = 8 * threadIdx.x; c < cols; c += 8 * blockDim.x) {
        const half8 a = load_h8(x0 + c), b = load_h8(x1 + c), u = load_h8(w0 + c), v = load_h8(w1 + c);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc = fmaf((float)a[e], (float)u[e], fmaf((float)b[e], (float)v[e], acc));
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) out[j] = f2h(part[0] + part[1] + part[2] + part[3]);
}

extern "C" int kf_dot2_rows(void *out, const void *x0, const void *x1, const void *W, int rows, int cols) {
    kf_take_pending(__func__);
    if (rows <= 0) return 0;
    if (cols % 8 || ((uintptr_t)x0 | (uintptr_t)x1 | (uintptr_t)W) & 15) {
        kf_set_error("kf_dot2_rows: cols %% 8 and 16-byte aligned operands required (cols=%d)", cols);
        return -1;
    }
    k_dot2_rows<<<rows, 256, 0, kf_stream()>>>((h16 *)out, (const h16 *)x0, (const h16 *)x1, (const h16 *)W, rows,
                                              cols);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        kf_set_error("kf_dot2_rows: %s", hipGetErrorString(e));
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

// short-K products on 8-column vectors (K <= 8: AddBias is ops_gemm with K = 1 against a
// ones column, internal/gpu/ops.go:335-351): a thread owns one 8-column vector of C for
// all its rows and keeps B's K x 8 block in registers; A's K values of a row are the same
// for every thread of that row (one cached line). Same arithmetic and order as
// k_gemm_small: s = sum_k a*b in fp32, v = alpha * s (+ beta * C), one RNE store.
constexpr int kSmallK = 8;
template <int KS>
__global__ __launch_bounds__(256) void k_gemm_smallk_v8(int M, int ncv, int K, long long R, float alpha,
                                                        const h16 *A, int lda, const h16 *B, int ldb,
                                                        float beta, h16 *C, int ldc) {
    const long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= (long long)ncv * R) return;
    const int cv = (int)(g % ncv);
    float b[KS][8];
#pragma unroll
    for (int k = 0; k < KS; ++k) {
        if (k < K) {
            const half8 v = *reinterpret_cast<const half8 *>(B + (long long)k * ldb + 8 * cv);
#pragma unroll
            for (int e = 0; e < 8; ++e) b[k][e] = (float)v[e];
        }
    }
    // four rows in flight per thread (AddBias: K = 1, C's rows are the HBM stream). Every
    // load of a group is issued before its first store: vmcnt also counts stores, so a load
    // issued behind a store would wait for that store's acknowledgement.
    auto row = [&](long long m, const float (&a)[KS], const half8 &c0) {
        half8 out;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            float s = 0.f;
#pragma unroll
            for (int k = 0; k < KS; ++k)
                if (k < K) s += a[k] * b[k][e];
            float v = alpha * s;
            if (beta != 0.f) v += beta * (float)c0[e];
            out[e] = f2h(v);
        }
        *reinterpret_cast<half8 *>(C + m * ldc + 8 * cv) = out;
    };
    auto load = [&](long long m, float (&a)[KS], half8 &c0) {
#pragma unroll
        for (int k = 0; k < KS; ++k) a[k] = k < K ? h2f(A[m * lda + k]) : 0.f;
        c0 = beta != 0.f ? *reinterpret_cast<const half8 *>(C + m * ldc + 8 * cv) : half8{};
    };
    long long m = g / ncv;
    for (; m + 3 * R < M; m += 4 * R) {
        float a[4][KS];
        half8 c0[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) load(m + u * R, a[u], c0[u]);
#pragma unroll
        for (int u = 0; u < 4; ++u) row(m + u * R, a[u], c0[u]);
    }
    for (; m < M; m += R) {
        float a[KS];
        half8 c0;
        load(m, a, c0);
        row(m, a, c0);
    }
}

// ---------------------------------------------------------------------------
// MXFP8 quantisation (kf_ops.h): one thread per (row, 32-element block)
// ---------------------------------------------------------------------------
__global__ void k_quant_mxfp8(const h16 *src, long long ld_src, int rows, int cols, int cols_pad,
                              int transpose, uint8_t *q, long long ldq, uint8_t *scales,
                              long long lds) {
    const int nblk = cols_pad / 32;
    const long long total = (long long)rows * nblk;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        // transposed source (weights): consecutive threads take consecutive rows r, so each
        // of the 32 loads of a block is one coalesced source row; else consecutive blocks
        int r, b;
        if (transpose) {
            b = (int)(i / rows);
            r = (int)(i - (long long)b * rows);
        } else {
            r = (int)(i / nblk);
            b = (int)(i - (long long)r * nblk);
        }
        float v[32];
        float amax = 0.f;
#pragma unroll
        for (int j = 0; j < 32; ++j) {
            const int c = 32 * b + j;
            float x = 0.f;
            if (c < cols) x = h2f(transpose ? src[(long long)c * ld_src + r] : src[(long long)r * ld_src + c]);
            v[j] = x;
            amax = fmaxf(amax, fabsf(x));
        }
        const int ex = mx_exponent(amax);
        const float inv = __uint_as_float((unsigned)(127 - ex) << 23);
#pragma unroll
        for (int j = 0; j < 32; ++j) v[j] *= inv;
        uint8_t *qr = q + (long long)r * ldq + 32 * b;
#pragma unroll
        for (int w = 0; w < 4; ++w) *reinterpret_cast<uint2 *>(qr + 8 * w) = pack_e4m3x8(v + 8 * w);
        scales[(long long)r * lds + b] = (uint8_t)(ex + 127);
    }
}

// Row quantisation on 16-byte vectors (source rows 16-byte aligned, cols % 8 == 0): four
// lanes per 32-element block, eight elements each, the block's amax by two lane swaps as in
// the GEMM epilogue's copy, so a wave reads 1 KB of contiguous row bytes per load.
__global__ __launch_bounds__(256) void k_quant_mxfp8_rows_v8(const h16 *src, long long ld_src, int rows, int cols,
                                                             int nblk, uint8_t *q, long long ldq, uint8_t *scales,
                                                             long long lds) {
    const long long total = (long long)rows * nblk * 4;
    const long long S = (long long)gridDim.x * blockDim.x;
    // total is a multiple of 4 and S of 64, so a block's four lanes are live together
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += S) {
        const long long rb = i >> 2;
        const int r = (int)(rb / nblk), b = (int)(rb - (long long)r * nblk), c0 = 32 * b + 8 * (int)(i & 3);
        float v[8];
        if (c0 < cols) {
            const half8 x = *reinterpret_cast<const half8 *>(src + (long long)r * ld_src + c0);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = (float)x[e];
        } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = 0.f;
        }
        float amax = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) amax = fmaxf(amax, fabsf(v[e]));
        amax = fmaxf(amax, __shfl_xor(amax, 1));
        amax = fmaxf(amax, __shfl_xor(amax, 2));
        const int ex = mx_exponent(amax);
        const float inv = __uint_as_float((unsigned)(127 - ex) << 23);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] *= inv;
        *reinterpret_cast<uint2 *>(q + (long long)r * ldq + c0) = pack_e4m3x8(v);
        if ((i & 3) == 0) scales[(long long)r * lds + b] = (uint8_t)(ex + 127);
    }
}

// Weight quantisation of many matrices in one launch (kf_quant_mxfp8_batch): job j owns
// threads [t0[j], t0[j+1]) of the grid, one per (row, 32-element block), rows fastest.
struct QuantJobs {
    KfQuantJob job[KF_QUANT_MAX];
    long long t0[KF_QUANT_MAX + 1];
    int n;
};
__global__ __launch_bounds__(256) void k_quant_mxfp8_batch(QuantJobs J) {
    const long long S = (long long)gridDim.x * blockDim.x;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < J.t0[J.n]; i += S) {
        int j = 0;
        while (j + 1 < J.n && i >= J.t0[j + 1]) ++j;
        const KfQuantJob &Q = J.job[j];
        const long long l = i - J.t0[j];
        const h16 *src = (const h16 *)Q.src;
        int r, b;
        if (Q.transpose) {
            b = (int)(l / Q.rows);
            r = (int)(l - (long long)b * Q.rows);
        } else {
            const int nblk = (Q.cols + 127) / 128 * 4;
            r = (int)(l / nblk);
            b = (int)(l - (long long)r * nblk);
        }
        float v[32];
        float amax = 0.f;
#pragma unroll
        for (int e = 0; e < 32; ++e) {
            const int c = 32 * b + e;
            float x = 0.f;
            if (c < Q.cols) x = h2f(Q.transpose ? src[(long long)c * Q.ld_src + r] : src[(long long)r * Q.ld_src + c]);
            v[e] = x;
            amax = fmaxf(amax, fabsf(x));
        }
        const int ex = mx_exponent(amax);
        const float inv = __uint_as_float((unsigned)(127 - ex) << 23);
#pragma unroll
        for (int e = 0; e < 32; ++e) v[e] *= inv;
        uint8_t *qr = (uint8_t *)Q.q + (long long)r * Q.ldq + 32 * b;
#pragma unroll
        for (int w = 0; w < 4; ++w) *reinterpret_cast<uint2 *>(qr + 8 * w) = pack_e4m3x8(v + 8 * w);
        Q.scales[(long long)r * Q.lds + b] = (uint8_t)(ex + 127);
    }
}

// Row jobs on 16-byte vectors (cols % 8 == 0, ld_src % 8 == 0, aligned source: host-checked),
// as k_quant_mxfp8_rows_v8: four lanes per 32-element block; J.t0 counts lanes
__global__ __launch_bounds__(256) void k_quant_mxfp8_vbatch(QuantJobs J) {
    const long long S = (long long)gridDim.x * blockDim.x;
    // every job's lane count is a multiple of 4 and S of 64: a block's four lanes are live together
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < J.t0[J.n]; i += S) {
        int j = 0;
        while (j + 1 < J.n && i >= J.t0[j + 1]) ++j;
        const KfQuantJob &Q = J.job[j];
        const long long l = i - J.t0[j], rb = l >> 2;
        const int nblk = (Q.cols + 127) / 128 * 4;
        const int r = (int)(rb / nblk), b = (int)(rb - (long long)r * nblk), c0 = 32 * b + 8 * (int)(l & 3);
        float v[8];
        if (c0 < Q.cols) {
            const half8 x = load_h8((const h16 *)Q.src + (long long)r * Q.ld_src + c0);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = (float)x[e];
        } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = 0.f;
        }
        float amax = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) amax = fmaxf(amax, fabsf(v[e]));
        amax = fmaxf(amax, __shfl_xor(amax, 1));
        amax = fmaxf(amax, __shfl_xor(amax, 2));
        const int ex = mx_exponent(amax);
        const float inv = __uint_as_float((unsigned)(127 - ex) << 23);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] *= inv;
        *reinterpret_cast<uint2 *>((uint8_t *)Q.q + (long long)r * Q.ldq + c0) = pack_e4m3x8(v);
        if ((l & 3) == 0) Q.scales[(long long)r * Q.lds + b] = (uint8_t)(ex + 127);
    }
}

// Transposed jobs (weights W[K][N] -> W8[N][K]) through LDS: a workgroup owns 64 output rows
// r (source columns) x 256 k (8 blocks): the source tile is read as 256 row segments of 128
// bytes, and each output row's 256 bytes are written by 32 consecutive lanes (4 per block,
// the block amax by two lane swaps), so both sides are coalesced.
struct QuantTJobs {
    KfQuantJob job[KF_QUANT_MAX];
    int wg0[KF_QUANT_MAX + 1];  // first workgroup of each job
    int rt[KF_QUANT_MAX];       // 64-row tiles of each job
    int n;
};
__global__ __launch_bounds__(256) void k_quant_mxfp8_tbatch(QuantTJobs J) {
    __shared__ float tile[256][65];
    int j = 0;
    while (j + 1 < J.n && (int)blockIdx.x >= J.wg0[j + 1]) ++j;
    const KfQuantJob &Q = J.job[j];
    const int w = blockIdx.x - J.wg0[j];
    const int r0 = (w % J.rt[j]) * 64, k0 = (w / J.rt[j]) * 256;
    const h16 *src = (const h16 *)Q.src;
    // 2048 16-byte source vectors (8 per 64-row tile row), all loads issued before the LDS
    // writes (rows % 8 == 0, ld_src % 8 == 0, 16-byte aligned source: host-checked)
    half8 xs[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
        const int i = threadIdx.x + 256 * u, k = k0 + (i >> 3), r = r0 + 8 * (i & 7);
        xs[u] = (k < Q.cols && r < Q.rows) ? load_h8(src + (long long)k * Q.ld_src + r) : half8{};
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
        const int i = threadIdx.x + 256 * u, kk = i >> 3, rr = 8 * (i & 7);
#pragma unroll
        for (int e = 0; e < 8; ++e) tile[kk][rr + e] = (float)xs[u][e];
    }
    __syncthreads();
    const int kpad = (Q.cols + 127) / 128 * 128;
    for (int i = threadIdx.x; i < 64 * 32; i += 256) {  // i = output row * 32 + block * 4 + quarter
        const int rr = i >> 5, b = (i >> 2) & 7, qq = i & 3, r = r0 + rr, c0 = 32 * b + 8 * qq;
        float v[8];
        float amax = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            v[e] = tile[c0 + e][rr];
            amax = fmaxf(amax, fabsf(v[e]));
        }
        amax = fmaxf(amax, __shfl_xor(amax, 1));
        amax = fmaxf(amax, __shfl_xor(amax, 2));
        const int ex = mx_exponent(amax);
        const float inv = __uint_as_float((unsigned)(127 - ex) << 23);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] *= inv;
        if (r < Q.rows && k0 + c0 < kpad) {
            *reinterpret_cast<uint2 *>((uint8_t *)Q.q + (long long)r * Q.ldq + k0 + c0) = pack_e4m3x8(v);
            if (qq == 0) Q.scales[(long long)r * Q.lds + (k0 >> 5) + b] = (uint8_t)(ex + 127);
        }
    }
}

static bool quant_args_ok(const void *src, int rows, int cols, const void *q, long long ldq, const uint8_t *scales,
                          long long lds) {
    const int cols_pad = (cols + 127) / 128 * 128;
    return src && q && scales && ldq >= cols_pad && ldq % 16 == 0 && lds >= cols_pad / 32 && !((uintptr_t)q & 7);
}

extern "C" int kf_quant_mxfp8_batch(int n, const KfQuantJob *jobs) {
    kf_take_pending(__func__);
    if (n < 0 || n > KF_QUANT_MAX || (n && !jobs)) {
        kf_set_error("kf_quant_mxfp8_batch: %d jobs (at most %d)", n, KF_QUANT_MAX);
        return -1;
    }
    QuantJobs J{}, VJ{};
    QuantTJobs TJ{};
    long long tot = 0, vtot = 0;
    int twg = 0;
    for (int j = 0; j < n; ++j) {
        const KfQuantJob &Q = jobs[j];
        if (Q.rows < 0 || Q.cols < 0 || ((Q.rows && Q.cols) && !quant_args_ok(Q.src, Q.rows, Q.cols, Q.q, Q.ldq,
                                                                                Q.scales, Q.lds))) {
            kf_set_error("kf_quant_mxfp8_batch: bad job %d (rows=%d cols=%d ldq=%lld lds=%lld)", j, Q.rows, Q.cols,
                         Q.ldq, Q.lds);
            return -1;
        }
        if (!Q.rows || !Q.cols) continue;
        if (Q.transpose && Q.rows % 8 == 0 && Q.ld_src % 8 == 0 && !((uintptr_t)Q.src & 15)) {
            // LDS-tiled: 64 rows x 256 k per workgroup
            TJ.job[TJ.n] = Q;
            TJ.wg0[TJ.n] = twg;
            TJ.rt[TJ.n] = (Q.rows + 63) / 64;
            twg += TJ.rt[TJ.n] * ((Q.cols + 127) / 128 * 128 + 255) / 256;
            ++TJ.n;
        } else if (!Q.transpose && Q.cols % 8 == 0 && Q.ld_src % 8 == 0 && !((uintptr_t)Q.src & 15)) {
            VJ.job[VJ.n] = Q;  // row jobs on 16-byte vectors
            VJ.t0[VJ.n] = vtot;
            vtot += (long long)Q.rows * ((Q.cols + 127) / 128 * 4) * 4;
            ++VJ.n;
        } else {
            J.job[J.n] = Q;
            J.t0[J.n] = tot;
            tot += (long long)Q.rows * ((Q.cols + 127) / 128 * 4);
            ++J.n;
        }
    }
    J.t0[J.n] = tot;
    VJ.t0[VJ.n] = vtot;
    TJ.wg0[TJ.n] = twg;
    if (tot > 0) k_quant_mxfp8_batch<<<kf_blocks(tot, 256, 16384), 256, 0, kf_stream()>>>(J);
    if (vtot > 0) k_quant_mxfp8_vbatch<<<kf_blocks(vtot, 256, 16384), 256, 0, kf_stream()>>>(VJ);
    if (twg > 0) k_quant_mxfp8_tbatch<<<twg, 256, 0, kf_stream()>>>(TJ);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        kf_set_error("kf_quant_mxfp8_batch: %s", hipGetErrorString(e));
        return -1;
    }
    return 0;
}

extern "C" int kf_quant_mxfp8(const void *src, long long ld_src, int rows, int cols, int transpose,
                              void *q, long long ldq, uint8_t *scales, long long lds) {
    kf_take_pending(__func__);
    if (rows <= 0 || cols <= 0) return 0;
    const int cols_pad = (cols + 127) / 128 * 128;
    if (!src || !q || !scales || ldq < cols_pad || ldq % 16 || lds < cols_pad / 32 ||
        ((uintptr_t)q & 7)) {
        kf_set_error("kf_quant_mxfp8: bad arguments (rows=%d cols=%d ldq=%lld lds=%lld)", rows,
                     cols, ldq, lds);
        return -1;
    }
    const long long total = (long long)rows * (cols_pad / 32);
    if (!transpose && cols % 8 == 0 && ld_src % 8 == 0 && !((uintptr_t)src & 15))
        k_quant_mxfp8_rows_v8<<<kf_blocks(4 * total, 256, 16384), 256, 0, kf_stream()>>>(
            (const h16 *)src, ld_src, rows, cols, cols_pad / 32, (uint8_t *)q, ldq, scales, lds);
    else
        k_quant_mxfp8<<<kf_blocks(total, 256, 16384), 256, 0, kf_stream()>>>(
            (const h16 *)src, ld_src, rows, cols, cols_pad, transpose, (uint8_t *)q, ldq, scales, lds);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        kf_set_error("kf_quant_mxfp8: %s", hipGetErrorString(e));
        return -1;
    }
    return 0;
}

int kf_ops_gemm_impl(int M, int N, int K, float alpha, const void *A, int lda, const void *B,
                     int ldb, float beta, void *C, int ldc, char *err, size_t errlen) {
    kf_take_pending(__func__);
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
    const bool smallk_vec = K <= kSmallK && N % 8 == 0 && ldb % 8 == 0 && ldc % 8 == 0 &&
                            !(((uintptr_t)B | (uintptr_t)C) & 15);
    if (smallk_vec) {
        const int ncv = N / 8;
        long long R = 524288 / ncv;
        if (R < 1) R = 1;
        if (R > M) R = M;
        const unsigned grid = (unsigned)((ncv * R + 255) / 256);
        if (K == 1)  // AddBias (ops.go:335-351): one column of B in registers
            k_gemm_smallk_v8<1><<<grid, 256, 0, kf_stream()>>>(M, ncv, K, R, alpha, (const h16 *)A, lda,
                                                                (const h16 *)B, ldb, beta, (h16 *)C, ldc);
        else
            k_gemm_smallk_v8<kSmallK><<<grid, 256, 0, kf_stream()>>>(M, ncv, K, R, alpha, (const h16 *)A, lda,
                                                                      (const h16 *)B, ldb, beta, (h16 *)C, ldc);
    } else if (!fast || K == 0) {
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
