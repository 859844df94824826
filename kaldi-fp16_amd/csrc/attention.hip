// attention.hip — restricted (local-context) self-attention of attention-relu-batchnorm
// layers on the MI355X. The reference runs this on the CPU
// (internal/nnet/forward.go:795-909, the per-head loop at :850-893) after a GPU affine.
//
// Per frame t and head h the affine output row holds [key (kd) | value (vd) | query key
// (kd) | query context (ctx)]; for o in [0, ctx) the attended row is
// r_o = t + (o - nleft) * stride, zero when outside [0, T) (the reference zero-pads):
//     b_o = qctx[o] + key_scale * <qkey(t), key(r_o)>,  w = softmax(b)
//     out(t, h) = [ sum_o w_o value(r_o) (vd) | w (ctx) ]
// followed by ReLU and the frozen BatchNorm (scale / shift), fused here.
//
// Layout: one wave per frame t, all heads: the softmax weights of the H heads sit in a
// wave-private LDS slice, and the output row is produced in 64-column chunks whose ReLU
// bits are packed with one ballot per chunk (so no two waves share a mask byte). The
// affine rows are re-read ctx times from L2; the layer is latency-bound, off the
// CNN-TDNN hot path.
//
// Backward (exact; the reference reuses its conv backward for this layer,
// network_backward.go:539-544, which is not a gradient of this function):
//   dw_o = dz_w[o] + <dz_v, value(r_o)>,  db_o = w_o (dw_o - sum_j w_j dw_j)
//   d qctx[o] = db_o,  d qkey = s sum_o db_o key(r_o)                       (k_att_bwd_q)
//   d key(r) = s sum_o db_o(t_o) qkey(t_o),  d value(r) = sum_o w_o(t_o) dz_v(t_o),
//   t_o = r - (o - nleft) * stride                                          (k_att_bwd_kv)
// The second kernel gathers instead of scattering, so the result is deterministic.
#include "kf_common.h"
#include "../../include/kf_ops.h"

namespace {

constexpr int kWaves = 4;
constexpr int kMaxHC = 1024;  // H * ctx floats of LDS per wave

struct AttD {
    const h16 *proj;
    long long ldp;
    int T, H, kd, vd, ctx, nleft, stride;
    float key_scale;
    int A;  // per-head affine width 2 kd + vd + ctx
};

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

__device__ __forceinline__ const h16 *row_ptr(const AttD &d, int r, int h) {
    return d.proj + (long long)r * d.ldp + (long long)h * d.A;
}
// context position o of frame t: inside the sequence? and element `col` of its head-h
// row, loaded unconditionally (row clamped into [0, T), o clamped to ctx - 1) so that
// a group of loads can be in flight together; callers select with ctx_live
__device__ __forceinline__ bool ctx_live(const AttD &d, int t, int o) {
    const int r = t + (o - d.nleft) * d.stride;
    return r >= 0 && r < d.T;
}
__device__ __forceinline__ float ctx_load(const AttD &d, int t, int h, int o, int col) {
    const int r = t + (min(o, d.ctx - 1) - d.nleft) * d.stride;
    return (float)row_ptr(d, min(max(r, 0), d.T - 1), h)[col];
}

// The ctx dot products of a frame (length kd or vd) are split over the wave: 2^lg lanes
// per context position (2^lg * ctx <= 64), each summing a strided part, then a
// butterfly within the lane group. Returns, in lane o < ctx, <a, row(r_o) + off>.
__device__ __forceinline__ int att_lg(int ctx) {
    int lg = 6;
    while ((ctx << lg) > 64) --lg;
    return lg;
}
__device__ __forceinline__ float split_dot(const AttD &d, int t, int h, int lane, int lg, const h16 *a, int off,
                                           int n) {
    const int G = 1 << lg, o = lane >> lg, sub = lane & (G - 1);
    float dot = 0.f;
    if (o < d.ctx) {
        const int r = t + (o - d.nleft) * d.stride;
        if (r >= 0 && r < d.T) {
            const h16 *k = row_ptr(d, r, h) + off;
            for (int j = sub; j < n; j += G) dot += (float)a[j] * (float)k[j];
        }
    }
    for (int m = G >> 1; m > 0; m >>= 1) dot += __shfl_xor(dot, m);
    return __shfl(dot, min(lane, d.ctx - 1) << lg);
}

// softmax weights of (t, h) into w[ctx] (lane o holds w_o; also returned); lanes >= ctx: 0
__device__ __forceinline__ float att_weights(const AttD &d, int t, int h, int lane) {
    const h16 *q = row_ptr(d, t, h) + d.kd + d.vd;  // query key part, then query context
    const float dot = split_dot(d, t, h, lane, att_lg(d.ctx), q, 0, d.kd);
    float b = -INFINITY;
    if (lane < d.ctx) b = (float)q[d.kd + lane] + d.key_scale * dot;
    const float mx = wave_max(b);
    const float e = lane < d.ctx ? expf(b - mx) : 0.f;
    const float s = wave_sum(e);
    return e / s;
}

__global__ __launch_bounds__(64 * kWaves) void k_att_fwd(AttD d, h16 *out, long long ldo, uint8_t *mask,
                                                         const float *scale, const float *shift) {
    __shared__ float wsh[kWaves][kMaxHC];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int t = blockIdx.x * kWaves + wave;
    if (t >= d.T) return;  // whole wave
    float *w = wsh[wave];
    for (int h = 0; h < d.H; ++h) {
        const float wv = att_weights(d, t, h, lane);
        if (lane < d.ctx) w[h * d.ctx + lane] = wv;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int od = d.vd + d.ctx, width = d.H * od;
    for (int c0 = 0; c0 < width; c0 += 64) {
        const int c = c0 + lane;
        float y = 0.f;
        if (c < width) {
            const int h = c / od, j = c - h * od;
            if (j < d.vd) {
                for (int o0 = 0; o0 < d.ctx; o0 += 8) {  // 8 row loads in flight, same order
                    float v[8];
#pragma unroll
                    for (int i = 0; i < 8; ++i) v[i] = ctx_load(d, t, h, o0 + i, d.kd + j);
#pragma unroll
                    for (int i = 0; i < 8; ++i)
                        if (o0 + i < d.ctx && ctx_live(d, t, o0 + i)) y += w[h * d.ctx + o0 + i] * v[i];
                }
            } else {
                y = w[h * d.ctx + (j - d.vd)];
            }
        }
        const bool pos = c < width && y > 0.f;
        const unsigned long long bits = __ballot(pos);
        if (c < width) {
            const float v = (pos ? y : 0.f) * scale[c] + shift[c];
            out[(long long)t * ldo + c] = (h16)v;
        }
        // width % 8 == 0 (checked on the host): row t's bits start on a byte boundary
        if (mask && lane < 8 && c0 + 8 * lane < width)
            mask[(((long long)t * width) >> 3) + (c0 >> 3) + lane] = (uint8_t)(bits >> (8 * lane));
    }
}

// d query parts of row t; w / db of (t, h, o) to the fp32 scratch for k_att_bwd_kv
__global__ __launch_bounds__(64 * kWaves) void k_att_bwd_q(AttD d, const h16 *dz, long long ldz, h16 *dproj,
                                                           float *wst, float *dbst) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int t = blockIdx.x * kWaves + wave;
    if (t >= d.T) return;
    const int od = d.vd + d.ctx;
    for (int h = 0; h < d.H; ++h) {
        const float w = att_weights(d, t, h, lane);
        const h16 *g = dz + (long long)t * ldz + (long long)h * od;  // [dz_v (vd) | dz_w (ctx)]
        const float gv = split_dot(d, t, h, lane, att_lg(d.ctx), g, d.kd, d.vd);  // <dz_v, value(r_o)>
        float dw = 0.f;
        if (lane < d.ctx) dw = (float)g[d.vd + lane] + gv;
        const float wdw = wave_sum(lane < d.ctx ? w * dw : 0.f);
        const float db = lane < d.ctx ? w * (dw - wdw) : 0.f;
        h16 *dq = dproj + (long long)t * d.ldp + (long long)h * d.A + d.kd + d.vd;
        if (lane < d.ctx) {
            dq[d.kd + lane] = (h16)db;
            const long long s = ((long long)t * d.H + h) * d.ctx + lane;
            wst[s] = w;
            dbst[s] = db;
        }
        for (int j0 = 0; j0 < d.kd; j0 += 64) {
            const int j = j0 + lane;
            float acc = 0.f;
            const int jc = min(j, d.kd - 1);
            for (int o0 = 0; o0 < d.ctx; o0 += 8) {  // 8 row loads in flight, same order
                float v[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) v[i] = ctx_load(d, t, h, o0 + i, jc);
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const float dbo = __shfl(db, min(o0 + i, 63));
                    if (j < d.kd && o0 + i < d.ctx && ctx_live(d, t, o0 + i)) acc += dbo * v[i];
                }
            }
            if (j < d.kd) dq[j] = (h16)(d.key_scale * acc);
        }
    }
}

// d key / d value parts of row r, gathered from the frames that attend to it
__global__ __launch_bounds__(64 * kWaves) void k_att_bwd_kv(AttD d, const h16 *dz, long long ldz, h16 *dproj,
                                                            const float *wst, const float *dbst) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = blockIdx.x * kWaves + wave;
    if (r >= d.T) return;
    const int od = d.vd + d.ctx;
    for (int h = 0; h < d.H; ++h) {
        h16 *dk = dproj + (long long)r * d.ldp + (long long)h * d.A;
        for (int j0 = 0; j0 < d.kd + d.vd; j0 += 64) {
            const int j = j0 + lane;
            float acc = 0.f;
            if (j < d.kd + d.vd) {
                for (int o0 = 0; o0 < d.ctx; o0 += 8) {  // 8 gathers in flight, same order
                    float c[8], v[8];
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        const int oc = min(o0 + i, d.ctx - 1);
                        const int tc = min(max(r - (oc - d.nleft) * d.stride, 0), d.T - 1);
                        const long long s = ((long long)tc * d.H + h) * d.ctx + oc;
                        if (j < d.kd) {  // key: s * db_o(t) * qkey(t)
                            c[i] = dbst[s];
                            v[i] = (float)row_ptr(d, tc, h)[d.kd + d.vd + j];
                        } else {         // value: w_o(t) * dz_v(t)
                            c[i] = wst[s];
                            v[i] = (float)dz[(long long)tc * ldz + (long long)h * od + (j - d.kd)];
                        }
                    }
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        const int t = r - (o0 + i - d.nleft) * d.stride;
                        if (o0 + i < d.ctx && t >= 0 && t < d.T) acc += c[i] * v[i];
                    }
                }
                if (j < d.kd) acc *= d.key_scale;
                dk[j] = (h16)acc;
            }
        }
    }
}

bool att_check(const KfAttention &a, const char *what) {
    if (!a.proj || a.T <= 0 || a.num_heads <= 0 || a.key_dim <= 0 || a.value_dim < 0 || a.context <= 0 ||
        a.context > 64 || a.num_heads * a.context > kMaxHC || a.stride <= 0 || a.num_left < 0 ||
        a.num_left >= a.context || a.ldp < (long long)a.num_heads * (2 * a.key_dim + a.value_dim + a.context)) {
        kf_report_error("%s: bad attention shape (T %d heads %d key %d value %d ctx %d stride %d left %d)", what,
                        a.T, a.num_heads, a.key_dim, a.value_dim, a.context, a.stride, a.num_left);
        return false;
    }
    return true;
}

AttD att_dev(const KfAttention &a) {
    AttD d;
    d.proj = (const h16 *)a.proj;
    d.ldp = a.ldp;
    d.T = a.T;
    d.H = a.num_heads;
    d.kd = a.key_dim;
    d.vd = a.value_dim;
    d.ctx = a.context;
    d.nleft = a.num_left;
    d.stride = a.stride;
    d.key_scale = a.key_scale;
    d.A = 2 * a.key_dim + a.value_dim + a.context;
    return d;
}

}  // namespace

extern "C" int kf_attention_forward(const KfAttention *a, void *out, long long ldo, uint8_t *mask,
                                    const float *scale, const float *shift) {
    kf_take_pending(__func__);
    if (!a || !att_check(*a, "kf_attention_forward")) return -1;
    const int width = a->num_heads * (a->value_dim + a->context);
    if (!out || !scale || !shift || ldo < width || (mask && (width % 8))) {
        kf_report_error("kf_attention_forward: bad output (width %d ldo %lld, mask needs width %% 8 == 0)", width,
                        ldo);
        return -1;
    }
    k_att_fwd<<<(a->T + kWaves - 1) / kWaves, 64 * kWaves, 0, kf_stream()>>>(att_dev(*a), (h16 *)out, ldo, mask,
                                                                              scale, shift);
    return hipGetLastError() == hipSuccess ? 0 : (kf_report_error("kf_attention_forward: launch failed"), -1);
}

extern "C" int kf_attention_backward(const KfAttention *a, const void *dz, long long ldz, void *dproj,
                                     float *scratch) {
    kf_take_pending(__func__);
    if (!a || !att_check(*a, "kf_attention_backward")) return -1;
    const int width = a->num_heads * (a->value_dim + a->context);
    if (!dz || !dproj || !scratch || ldz < width) {
        kf_report_error("kf_attention_backward: bad arguments");
        return -1;
    }
    const AttD d = att_dev(*a);
    float *wst = scratch, *dbst = scratch + (size_t)a->T * a->num_heads * a->context;
    const int grid = (a->T + kWaves - 1) / kWaves;
    k_att_bwd_q<<<grid, 64 * kWaves, 0, kf_stream()>>>(d, (const h16 *)dz, ldz, (h16 *)dproj, wst, dbst);
    k_att_bwd_kv<<<grid, 64 * kWaves, 0, kf_stream()>>>(d, (const h16 *)dz, ldz, (h16 *)dproj, wst, dbst);
    return hipGetLastError() == hipSuccess ? 0 : (kf_report_error("kf_attention_backward: launch failed"), -1);
}
