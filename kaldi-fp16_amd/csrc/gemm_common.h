// gemm_common.h — device pieces shared by the MFMA GEMM kernels (gemm.hip, conv_wgrad.hip):
// operand addressing (the device form of KfOperand), the LDS images and fragment
// loads of v_mfma_f32_16x16x32_f16, the LDS-DMA operand stager and the 8-column
// epilogue. gfx950 only.
#pragma once
#include <utility>

#include "kf_common.h"
#include "../../include/kf_ops.h"

// ---------------------------------------------------------------------------
// operand addressing (device form of KfOperand, see kf_ops.h)
// ---------------------------------------------------------------------------
struct OpD {
    const h16 *base;
    long long ld;
    int nrows, ncols;
    int nparts, pw;
    int T, hout, hsrc, hmul, hshift;
    int tclamp, simple, p64;
    unsigned inv_hout;  // ceil(2^16 / hout): exact t = h/hout for h*hout < 2^16
    unsigned ldb, pwb;  // ld and part_width in bytes (32-bit addressing is checked on the host)
    int edges;          // any edge rows
    int dt[KF_MAX_PARTS], dh[KF_MAX_PARTS], et[KF_MAX_PARTS], er[KF_MAX_PARTS];
    // MXFP8: geometry above is in 2-byte units (so the fp16 stagers move the bytes),
    // the E8M0 scales are addressed per source row (lds bytes) and element / 32
    const uint8_t *sc;
    unsigned lds;
    int pw8;            // part width in fp8 elements
    // masked operand (KfOperand.mask): element i of the source (linear index, ld-strided)
    // reads as zero unless bit i of mk is set; source bytes >= mlim (rows past the mask,
    // e.g. an edge row) are unmasked
    const uint8_t *mk;
    unsigned mlim;
    int tmul, t0;       // time-strided rows (KfOperand.tmul / t0; conv halo forward only)
};

// compile-time loop: body(I) with I a std::integral_constant (forces full unrolling,
// so register arrays are never indexed dynamically and never fall to scratch)
#include <utility>
template <typename F, int... Is>
__device__ __forceinline__ void static_for_impl(F &&f, std::integer_sequence<int, Is...>) {
    (f(std::integral_constant<int, Is>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F &&f) {
    static_for_impl(f, std::make_integer_sequence<int, N>{});
}

template <typename T>
__device__ __forceinline__ T sel9(const T (&a)[KF_MAX_PARTS], int p, int nparts) {
    if (nparts <= 2) return p ? a[1] : a[0];
    T v = a[0];
#pragma unroll
    for (int i = 1; i < KF_MAX_PARTS; ++i)
        if (p == i) v = a[i];
    return v;
}

// element offset of Op row (t, h), part p, in-part column kk; -1 = reads as zero
__device__ __forceinline__ long long op_off(const OpD &d, int t, int h, int kk, int dtp, int dhp,
                                            int etp, int erp) {
    int st;
    if (t == etp) {
        st = erp;
    } else {
        st = t + dtp;
        if (d.tclamp) st = min(max(st, 0), d.T - 1);
        else if ((unsigned)st >= (unsigned)d.T) return -1;
    }
    int sh = h * d.hmul + dhp;
    if (d.hshift) {
        if (sh & ((1 << d.hshift) - 1)) return -1;
        sh >>= d.hshift;
    }
    if ((unsigned)sh >= (unsigned)d.hsrc) return -1;
    return (long long)st * d.ld + (long long)sh * d.pw + kk;
}

// ---------------------------------------------------------------------------
// LDS images (both bank-conflict free for the 16x16x32 fragment maps; the
// swizzles were checked offline against the ds_read lane groups of
// MI355X_MICROARCH §LDS). BK is fixed at 64 halves.
// ---------------------------------------------------------------------------
constexpr int BK = 64;
// k-contiguous [rows][64] halves: 16-byte chunk c of row r at slot c ^ ((r>>1)&7)
__device__ __forceinline__ int kc_off(int r, int c) { return r * 128 + 16 * (c ^ ((r >> 1) & 7)); }
// reduction-major [64][W] halves: 8-byte unit u of row r at u ^ swz(r). One
// ds_read_b64_tr_b16 reads rows {8g + q (+4)} x 4 units in each 32-lane group; the
// swizzle spreads those 8 rows over all 64 banks for the row stride's residue:
// W/2 dwords = 0 (mod 64) needs 8 distinct 4-unit blocks, 32 (mod 64) 4 distinct 4-unit
// blocks per half-bank set, 16 (mod 32) one block flip (checked offline for every tile
// width in use: 64 ... 384; the W = 192 / 320 / 384 wgrad tiles were 2-4-way conflicted
// under the W % 32 rule, SQ_LDS_BANK_CONFLICT 0.31-0.62 of their LDS cycles)
template <int W>
__device__ __forceinline__ int mn_swz(int r) {
    if constexpr (W % 128 == 0) return ((r & 3) << 2) ^ (((r >> 3) & 1) << 4);
    else if constexpr (W % 64 == 0) return ((r & 2) << 1) ^ (((r >> 3) & 1) << 3);
    else if constexpr (W % 32 == 0) return ((r >> 3) & 1) << 2;
    else return 0;
}
template <int W>
__device__ __forceinline__ int mn_off(int r, int u) {
    return r * (W * 2) + 8 * (u ^ mn_swz<W>(r));
}

typedef __attribute__((address_space(3))) short4v lds_s4;
typedef int v4i_t __attribute__((ext_vector_type(4)));

// v_mfma_f32_16x16x32_f16 fragment: lane l holds Op[idx0 + (l&15)][k = 32s + 8(l>>4) + j]
template <bool KC, int W>
__device__ __forceinline__ half8 load_frag(const char *tile, int idx0, int s, int lane) {
    if constexpr (KC) {
        const int r = idx0 + (lane & 15);
        const int c = s * 4 + (lane >> 4);
        return *reinterpret_cast<const half8 *>(tile + kc_off(r, c));
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
// per-thread LDS-DMA staging of one operand tile
//   KC: tile [TR][64], rows fixed per chunk, columns advance with k
//   MN: tile [64][TR], columns fixed per chunk, rows advance with k
// Each wave owns NC consecutive 1 KiB pieces; lane l fills bytes 16l..16l+15
// of a piece, so the swizzle is applied to the SOURCE address (rule 21).
// ---------------------------------------------------------------------------
// operand kinds, chosen on the host: the stager keeps only the state its kind needs
enum { OP_SIMPLE = 0, OP_P2 = 1, OP_GEN = 2 };
// or-ed into a gemm_kernel operand mode: the operand is masked (Stager MK)
constexpr int OP_MASKED = 8;
constexpr unsigned BAD = 0xFFFFFFFFu;  // byte offset that reads as zero (buffer range check)

// buffer resource (SGPR quad): base, stride 0, 2^32 - 1 records (an offset of BAD reads
// as zero through the range check), the raw-buffer flags word
typedef unsigned Rsrc __attribute__((ext_vector_type(4)));
__device__ __forceinline__ Rsrc make_rsrc(const void *base) {
    const unsigned long long b = (unsigned long long)base;
    return Rsrc{(unsigned)__builtin_amdgcn_readfirstlane((unsigned)b),
                (unsigned)__builtin_amdgcn_readfirstlane((unsigned)(b >> 32)) & 0xFFFFu, 0xFFFFFFFFu, 0x00020000u};
}

// LDS-DMA: lane l's BYTES (16 or 4) at buffer offset voff land at lds_dst + BYTES * l
// (lds_dst wave-uniform). Issued from inline asm so that hipcc does not track it: as a
// tracked LDS write (__builtin_amdgcn_raw_ptr_buffer_load_lds) it made hipcc emit
// s_waitcnt vmcnt(0) before every ds_read_b64_tr_b16 after it — the next stage's loads
// drained before the current stage's fragment reads, in every kernel with a
// reduction-major operand (the wgrads, the halo forward, N-major B). Every wait on these
// loads is explicit: wait_vmcnt<N>() / wait_vmcnt_rt() before the barrier that precedes
// the reads of a stage (cdna_hip_programming.md, "What hipcc does not do", LDS-DMA recipe).
template <int BYTES>
__device__ __forceinline__ void lds_dma(Rsrc rs, const void *lds_dst, unsigned voff) {
    // the low dword of a flat pointer into LDS is the LDS offset (the shared aperture is the
    // high dword); no address-space cast, which hipcc miscompiles inside some wave branches
    const unsigned m0v = (unsigned)__builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)lds_dst);
    unsigned keep;
    if constexpr (BYTES == 16)
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\t"
                     "s_mov_b32 m0, %0"
                     : "=&s"(keep)
                     : "v"(voff), "s"(rs), "s"(m0v)
                     : "memory");
    else
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dword %1, %2, 0 offen lds\n\t"
                     "s_mov_b32 m0, %0"
                     : "=&s"(keep)
                     : "v"(voff), "s"(rs), "s"(m0v)
                     : "memory");
}

// byte offset of (row t,h ; part p ; in-part column kk) or BAD
__device__ __forceinline__ unsigned op_boff(const OpD &d, int t, int h, int kk, int dtp, int dhp,
                                            int etp, int erp) {
    const long long off = op_off(d, t, h, kk, dtp, dhp, etp, erp);
    return off < 0 ? BAD : (unsigned)(off * 2);
}

template <bool KC, int TR, int MODE, int NW, bool MK = false>
struct Stager {
    // 1 KiB pieces (= chunks) per thread; when TR / 8 pieces do not split evenly over
    // the waves (160-row tiles on 8 waves) the last wave issues fewer (wave-uniform skip)
    static constexpr int NP = TR / 8;
    static constexpr int NC = (NP + NW - 1) / NW;
    static constexpr bool EVEN = NC * NW == NP;
    static_assert(NP * 8 == TR, "tile rows must be a multiple of 8");
    unsigned o0[NC];                    // KC: part-0 row byte offset; MN: fixed byte offset base
    unsigned o1[MODE == OP_P2 && KC ? NC : 1];  // KC/P2: part-1 row byte offset
    int th[MODE == OP_GEN ? NC : 1];    // GEN: KC packed (t<<8)|h ; MN packed part info
    int dt1[!KC && MODE != OP_SIMPLE ? NC : 1];  // MN: dt of the chunk's part
    unsigned mbv[MK ? NC : 1];          // MK: the mask byte of each chunk of the last issue
    int curp;

    __device__ __forceinline__ static int kc_row(int q, int lane) { return q * 8 + (lane >> 3); }
    __device__ __forceinline__ static int kc_col(int q, int lane) {
        return 8 * ((lane & 7) ^ ((kc_row(q, lane) >> 1) & 7));
    }
    __device__ __forceinline__ static int mn_row(int q, int lane) {
        return (q * 1024 + 16 * lane) / (2 * TR);
    }
    __device__ __forceinline__ static int mn_col(int q, int lane) {  // column in tile
        const int P = q * 1024 + 16 * lane, row = P / (2 * TR), within = P - row * (2 * TR);
        return 4 * ((within >> 3) ^ mn_swz<TR>(row));
    }

    __device__ __forceinline__ void init(const OpD &d, int tile0, int wave, int lane) {
        curp = -1;
        static_for<NC>([&](auto J) {
            constexpr int j = decltype(J)::value;
            const int q = wave * NC + j;
            if constexpr (KC) {
                const int r = tile0 + kc_row(q, lane);
                const bool ok = r < d.nrows;
                if constexpr (MODE == OP_SIMPLE) {
                    o0[j] = ok ? (unsigned)((long long)r * d.ld * 2) : BAD;
                } else if constexpr (MODE == OP_P2) {
                    o0[j] = ok ? op_boff(d, r, 0, 0, d.dt[0], d.dh[0], d.et[0], d.er[0]) : BAD;
                    o1[j] = ok && d.nparts > 1 ? op_boff(d, r, 0, 0, d.dt[1], d.dh[1], d.et[1], d.er[1])
                                               : BAD;
                } else {
                    const int t = d.hout > 1 ? r / d.hout : r;
                    th[j] = ok ? (t << 8) | (r - t * d.hout) : -1;
                    o0[j] = BAD;
                }
            } else {
                const int col = tile0 + mn_col(q, lane);
                const int rrel = mn_row(q, lane);
                const bool ok = col < d.ncols;
                if constexpr (MODE == OP_SIMPLE) {
                    o0[j] = ok ? (unsigned)(((long long)rrel * d.ld + col) * 2) : BAD;
                } else {
                    const int p = d.nparts > 1 ? col / d.pw : 0;
                    const int kk = col - p * d.pw;
                    o0[j] = ok ? (unsigned)(kk * 2) : BAD;
                    dt1[j] = sel9(d.dt, p, d.nparts);
                    if constexpr (MODE == OP_GEN)
                        th[j] = ((sel9(d.dh, p, d.nparts) + 128) & 0xFF) | (p << 8);
                }
            }
        });
    }

    // issue the NC LDS-DMA loads of the tile at reduction offset k0 into `dst`
    __device__ __forceinline__ void issue(const OpD &d, Rsrc rs, int k0, int kend,
                                          char *dst, int wave, int lane) {
        const int klim = min(kend, KC ? d.ncols : d.nrows);
        if constexpr (KC && MODE == OP_GEN) {
            // part of this K step is uniform when part_width % 64 == 0
            if (d.p64) {
                const int pu = k0 / d.pw;
                if (pu != curp) {
                    curp = pu;
                    const int dtp = sel9(d.dt, pu, d.nparts), dhp = sel9(d.dh, pu, d.nparts);
                    const int etp = sel9(d.et, pu, d.nparts), erp = sel9(d.er, pu, d.nparts);
                    static_for<NC>([&](auto J) {
                        constexpr int j = decltype(J)::value;
                        o0[j] = th[j] < 0 ? BAD
                                          : op_boff(d, th[j] >> 8, th[j] & 0xFF, 0, dtp, dhp, etp, erp);
                    });
                }
            }
        }
        int t0 = 0, h0 = 0;
        if constexpr (!KC && MODE == OP_GEN) {
            t0 = k0 / d.hout;
            h0 = k0 - t0 * d.hout;
        }
        static_for<NC>([&](auto J) {
            constexpr int j = decltype(J)::value;
            const int q = wave * NC + j;
            unsigned voff = BAD;
            if constexpr (KC) {
                const int col = k0 + kc_col(q, lane);
                if (col < klim) {
                    if constexpr (MODE == OP_SIMPLE) {
                        if (o0[j] != BAD) voff = o0[j] + col * 2;
                    } else if constexpr (MODE == OP_P2) {
                        const bool p1 = col >= d.pw;
                        const unsigned b = p1 ? o1[j] : o0[j];
                        if (b != BAD) voff = b + (col - (p1 ? d.pw : 0)) * 2;
                    } else {
                        if (d.p64) {
                            if (o0[j] != BAD) voff = o0[j] + (col - curp * d.pw) * 2;
                        } else if (th[j] >= 0) {  // general (tests): part per chunk
                            const int p = col / d.pw;
                            voff = op_boff(d, th[j] >> 8, th[j] & 0xFF, col - p * d.pw,
                                           sel9(d.dt, p, d.nparts), sel9(d.dh, p, d.nparts),
                                           sel9(d.et, p, d.nparts), sel9(d.er, p, d.nparts));
                        }
                    }
                }
            } else {
                const int r = k0 + mn_row(q, lane);
                if (r < klim && o0[j] != BAD) {
                    if constexpr (MODE == OP_SIMPLE) {
                        voff = o0[j] + (unsigned)k0 * d.ldb;
                    } else if constexpr (MODE == OP_P2) {
                        int st = r + dt1[j];
                        bool ok = true;
                        if (d.tclamp) st = min(max(st, 0), d.T - 1);
                        else ok = (unsigned)st < (unsigned)d.T;
                        if (ok) voff = (unsigned)st * d.ldb + o0[j];
                    } else {
                        // conv im2col rows (t, h): no edge rows on this path (host-checked)
                        const int hx = h0 + mn_row(q, lane);
                        const int qd = (int)(((unsigned)hx * d.inv_hout) >> 16);
                        const int st = t0 + qd + dt1[j];
                        int sh = (hx - qd * d.hout) * d.hmul + ((th[j] & 0xFF) - 128);
                        bool ok = (unsigned)st < (unsigned)d.T;
                        if (d.hshift) {
                            ok = ok && !(sh & ((1 << d.hshift) - 1));
                            sh >>= d.hshift;
                        }
                        ok = ok && (unsigned)sh < (unsigned)d.hsrc;
                        if (ok) voff = (unsigned)st * d.ldb + (unsigned)sh * d.pwb + o0[j];
                    }
                }
            }
            if constexpr (MK) {
                // a 16-byte chunk is 8 consecutive source elements at an 8-aligned linear
                // index: one mask byte, loaded ahead of the chunk itself
                mbv[j] = 0xFFu;
                if ((EVEN || q < NP) && voff < d.mlim) mbv[j] = d.mk[voff >> 4];
            }
            if (EVEN || q < NP) lds_dma<16>(rs, dst + q * 1024, voff);
        });
    }

    // MK: zero the masked elements of this thread's chunks of the stage at `dst` once they
    // have landed (after the stage's vmcnt wait, before the barrier that publishes it).
    // lut: 256 x 16-byte AND masks in LDS (byte b -> fp16 lane e kept iff bit e of b)
    __device__ __forceinline__ void apply_mask(char *dst, const uint4 *lut, int wave, int lane) const {
        static_for<NC>([&](auto J) {
            constexpr int j = decltype(J)::value;
            const int q = wave * NC + j;
            if (EVEN || q < NP) {
                uint4 *p = reinterpret_cast<uint4 *>(dst + q * 1024 + 16 * lane);
                const uint4 m = lut[mbv[j] & 0xFFu];
                uint4 v = *p;
                v.x &= m.x;
                v.y &= m.y;
                v.z &= m.z;
                v.w &= m.w;
                *p = v;
            }
        });
    }
};

// the 256-entry AND-mask table of Stager::apply_mask, filled by the whole workgroup
__device__ __forceinline__ void mask_lut_fill(uint4 *lut, int tid, int nth) {
    for (int b = tid; b < 256; b += nth) {
        unsigned w[4];
#pragma unroll
        for (int d = 0; d < 4; ++d)
            w[d] = (((b >> (2 * d)) & 1u) ? 0x0000FFFFu : 0u) | (((b >> (2 * d + 1)) & 1u) ? 0xFFFF0000u : 0u);
        lut[b] = uint4{w[0], w[1], w[2], w[3]};
    }
}

// s_waitcnt vmcnt(N) only (gfx9 encoding: vmcnt[3:0], vmcnt[5:4] at 15:14)
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    static_assert(N >= 0 && N < 64, "vmcnt");
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}

// ---------------------------------------------------------------------------
// epilogue on 8 consecutive columns of one row. Per-column parameters come from
// LDS (staged once per workgroup); the row operands (residual, input mask, old C)
// were prefetched by the caller, so no global load sits between two stores.
// ---------------------------------------------------------------------------
struct EpiCols {
    const float *bias, *scale, *shift, *scale2;  // LDS, indexed by local column
};

__device__ __forceinline__ void epilogue8(const KfEpilogue &E, const EpiCols &P, long long m, int n,
                                          int nl, float v[8], half8 cold, half8 rres,
                                          unsigned mbits) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] *= E.alpha;
    if (E.beta != 0.f) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += E.beta * (float)cold[e];
    }
    if (E.bias) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += P.bias[nl + e];
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
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = fmaf(v[e], P.scale[nl + e], P.shift[nl + e]);
    }
    if (E.resid) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = fmaf(E.resid_alpha, (float)rres[e], v[e]);
    }
    if (E.out) {
        half8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = f2h(v[e]);
        store_h8((h16 *)E.out + (long long)m * E.ldo + n, o);
    }
    if (E.out2) {
        half8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            float w = v[e];
            if (E.scale2) w *= P.scale2[nl + e];
            if (E.mask_in && !((mbits >> e) & 1u)) w = 0.f;
            o[e] = f2h(w);
            if (E.out8_src) v[e] = w;  // the MXFP8 copy after this call quantises out2's value
        }
        store_h8((h16 *)E.out2 + (long long)m * E.ldo2 + n, o);
    }
}
