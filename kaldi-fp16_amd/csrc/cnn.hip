// cnn.hip — the generic CNN launch wrappers of include/cnn_fp16.h.
//
// Behaviour of cpp/cuda/cnn_kernels.cu:19-830 and backward_wrappers.cu:87-102 /
// :212-225 (conv1d, pooling, stats pooling, batch/layer norm, depthwise /
// pointwise conv), with the defect fixes listed in the header. These calls sit
// off the CNN-TDNN training path, so the kernels are plain one-output-per-thread
// loops with fp32 accumulation and one RNE fp16 store. Every reduction over
// frames is a block reduction in a fixed order (no atomics), so results repeat
// bit for bit.
#include "kf_common.h"
#include "../../include/cnn_fp16.h"

namespace {

hipStream_t pick(void *s) { return s ? (hipStream_t)s : kf_stream(); }

void check(const char *what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) kf_report_error("%s: %s", what, hipGetErrorString(e));
}

// fixed-order sum over a 256-thread block (wave shuffles, then waves in order)
__device__ float block_sum256(float v, float *sh) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
    __syncthreads();
    return ((sh[0] + sh[1]) + sh[2]) + sh[3];
}

// ---------------------------------------------------------------- conv1d
// out[b][t][oc] = bias[oc] + sum_{k, ic} in[b][t*stride - pad + k*dil][ic] * w[oc][ic][k]
// (cnn_kernels.cu:19-59); oc is the fastest thread index so stores coalesce
__global__ void k_conv1d_fwd(const h16 *in, const h16 *w, const h16 *bias, h16 *out, int B,
                             int Ti, int Ci, int Co, int K, int stride, int pad, int dil, int To) {
    const long long total = (long long)B * To * Co;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const int oc = (int)(i % Co);
        const long long bt = i / Co;
        const int t = (int)(bt % To), b = (int)(bt / To);
        float s = 0.f;
        for (int k = 0; k < K; ++k) {
            const int ti = t * stride - pad + k * dil;
            if (ti < 0 || ti >= Ti) continue;
            const h16 *x = in + ((long long)b * Ti + ti) * Ci;
            const h16 *wk = w + (long long)oc * Ci * K + k;
            for (int ic = 0; ic < Ci; ++ic) s += h2f(x[ic]) * h2f(wk[(long long)ic * K]);
        }
        if (bias) s += h2f(bias[oc]);
        out[i] = f2h(s);
    }
}

// gin[b][ti][ic] = sum_{oc, k : ti + pad - k*dil = to*stride} gout[b][to][oc] * w[oc][ic][k]
// (cnn_kernels.cu:127-162; the range test is on `to`, after the division)
__global__ void k_conv1d_bwd_in(const h16 *gout, const h16 *w, h16 *gin, int B, int Ti, int Ci,
                                int Co, int K, int stride, int pad, int dil, int To) {
    const long long total = (long long)B * Ti * Ci;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const int ic = (int)(i % Ci);
        const long long bt = i / Ci;
        const int ti = (int)(bt % Ti), b = (int)(bt / Ti);
        float s = 0.f;
        for (int k = 0; k < K; ++k) {
            const int tt = ti + pad - k * dil;
            if (tt < 0 || tt % stride) continue;
            const int to = tt / stride;
            if (to >= To) continue;
            const h16 *g = gout + ((long long)b * To + to) * Co;
            for (int oc = 0; oc < Co; ++oc) s += h2f(g[oc]) * h2f(w[((long long)oc * Ci + ic) * K + k]);
        }
        gin[i] = f2h(s);
    }
}

// one block per weight (oc, ic, k): gw = sum_{b, to} in[b][ti][ic] * gout[b][to][oc]
// (cnn_kernels.cu:165-205, minus the float atomic into fp16)
__global__ void k_conv1d_bwd_w(const h16 *in, const h16 *gout, h16 *gw, int B, int Ti, int Ci,
                               int Co, int K, int stride, int pad, int dil, int To) {
    __shared__ float sh[4];
    const int widx = blockIdx.x;  // (oc*Ci + ic)*K + k
    const int k = widx % K, ic = (widx / K) % Ci, oc = widx / (K * Ci);
    float s = 0.f;
    for (long long n = threadIdx.x; n < (long long)B * To; n += blockDim.x) {
        const int to = (int)(n % To), b = (int)(n / To);
        const int ti = to * stride - pad + k * dil;
        if (ti < 0 || ti >= Ti) continue;
        s += h2f(in[((long long)b * Ti + ti) * Ci + ic]) * h2f(gout[n * Co + oc]);
    }
    s = block_sum256(s, sh);
    if (threadIdx.x == 0) gw[widx] = f2h(s);
}

// one block per channel: sum over (b, t) of x[b][t][c] (cnn_kernels.cu:208-229)
__global__ void k_col_sum(const h16 *x, h16 *out, long long rows, int C) {
    __shared__ float sh[4];
    const int c = blockIdx.x;
    float s = 0.f;
    for (long long r = threadIdx.x; r < rows; r += blockDim.x) s += h2f(x[r * C + c]);
    s = block_sum256(s, sh);
    if (threadIdx.x == 0) out[c] = f2h(s);
}

// ---------------------------------------------------------------- pooling
// cnn_kernels.cu:320-351: first strictly greater value from -1e10 wins
__global__ void k_maxpool_fwd(const h16 *in, h16 *out, int32_t *idx, int B, int Ti, int C, int K,
                              int stride, int To) {
    const long long total = (long long)B * To * C;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const int c = (int)(i % C);
        const long long bt = i / C;
        const int t = (int)(bt % To), b = (int)(bt / To);
        float mx = -1e10f;
        int at = 0;
        for (int k = 0; k < K; ++k) {
            const int ti = t * stride + k;
            const float v = h2f(in[((long long)b * Ti + ti) * C + c]);
            if (v > mx) {
                mx = v;
                at = ti;
            }
        }
        out[i] = f2h(mx);
        idx[i] = at;
    }
}

// one thread per (b, c) walks its outputs in time order: gin[max] += gout
// (backward_wrappers.cu:87-102 without the float atomic on fp16)
__global__ void k_maxpool_bwd(const h16 *gout, const int32_t *idx, h16 *gin, int B, int Ti,
                              int To, int C) {
    const long long total = (long long)B * C;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const int c = (int)(i % C), b = (int)(i / C);
        for (int t = 0; t < To; ++t) {
            const long long o = ((long long)b * To + t) * C + c;
            const int ti = idx[o];
            if (ti < 0 || ti >= Ti) continue;
            h16 *g = gin + ((long long)b * Ti + ti) * C + c;
            *g = f2h(h2f(*g) + h2f(gout[o]));
        }
    }
}

// cnn_kernels.cu:423-454: mean, then sqrt(var + 1e-10) (two passes)
__global__ void k_stats_pool(const h16 *in, h16 *out, int B, int T, int C) {
    const long long total = (long long)B * C;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const int c = (int)(i % C), b = (int)(i / C);
        const h16 *x = in + (long long)b * T * C + c;
        float s = 0.f;
        for (int t = 0; t < T; ++t) s += h2f(x[(long long)t * C]);
        const float mean = s / T;
        float v = 0.f;
        for (int t = 0; t < T; ++t) {
            const float d = h2f(x[(long long)t * C]) - mean;
            v += d * d;
        }
        out[(long long)b * 2 * C + c] = f2h(mean);
        out[(long long)b * 2 * C + C + c] = f2h(sqrtf(v / T + 1e-10f));
    }
}

// ---------------------------------------------------------------- normalisation
// one block per channel (cnn_kernels.cu:236-312)
__global__ void k_bn1d(const h16 *in, const h16 *gamma, const h16 *beta, h16 *rmean, h16 *rvar,
                       h16 *out, h16 *smean, h16 *sinv, long long rows, int C, float momentum,
                       float eps, int training) {
    __shared__ float sh[4];
    const int c = blockIdx.x;
    float mean, invstd;
    if (training) {
        float s = 0.f;
        for (long long r = threadIdx.x; r < rows; r += blockDim.x) s += h2f(in[r * C + c]);
        mean = block_sum256(s, sh) / rows;
        float v = 0.f;
        for (long long r = threadIdx.x; r < rows; r += blockDim.x) {
            const float d = h2f(in[r * C + c]) - mean;
            v += d * d;
        }
        const float var = block_sum256(v, sh) / rows;
        invstd = rsqrtf(var + eps);
        if (threadIdx.x == 0) {
            if (smean) smean[c] = f2h(mean);
            if (sinv) sinv[c] = f2h(invstd);
            rmean[c] = f2h(h2f(rmean[c]) * (1 - momentum) + mean * momentum);
            rvar[c] = f2h(h2f(rvar[c]) * (1 - momentum) + var * momentum);
        }
    } else {
        mean = h2f(rmean[c]);
        invstd = rsqrtf(h2f(rvar[c]) + eps);
    }
    const float g = h2f(gamma[c]), bt = h2f(beta[c]);
    for (long long r = threadIdx.x; r < rows; r += blockDim.x)
        out[r * C + c] = f2h((h2f(in[r * C + c]) - mean) * invstd * g + bt);
}

// one block per (b, t) row: var = E[x^2] - mean^2 (cnn_kernels.cu:461-510)
__global__ void k_layernorm(const h16 *in, const h16 *gamma, const h16 *beta, h16 *out, int C,
                            float eps) {
    __shared__ float sh[4];
    const h16 *x = in + (long long)blockIdx.x * C;
    h16 *y = out + (long long)blockIdx.x * C;
    float s = 0.f, q = 0.f;
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
        const float v = h2f(x[c]);
        s += v;
        q += v * v;
    }
    s = block_sum256(s, sh);
    q = block_sum256(q, sh);
    const float mean = s / C, invstd = rsqrtf(q / C - mean * mean + eps);
    for (int c = threadIdx.x; c < C; c += blockDim.x)
        y[c] = f2h((h2f(x[c]) - mean) * invstd * h2f(gamma[c]) + h2f(beta[c]));
}

// ---------------------------------------------------------------- separable conv
__global__ void k_depthwise(const h16 *in, const h16 *w, const h16 *bias, h16 *out, int B, int Ti,
                            int C, int K, int stride, int pad, int To) {
    const long long total = (long long)B * To * C;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const int c = (int)(i % C);
        const long long bt = i / C;
        const int t = (int)(bt % To), b = (int)(bt / To);
        float s = 0.f;
        for (int k = 0; k < K; ++k) {
            const int ti = t * stride - pad + k;
            if (ti >= 0 && ti < Ti) s += h2f(in[((long long)b * Ti + ti) * C + c]) * h2f(w[c * K + k]);
        }
        if (bias) s += h2f(bias[c]);
        out[i] = f2h(s);
    }
}

__global__ void k_pointwise(const h16 *in, const h16 *w, const h16 *bias, h16 *out, long long rows,
                            int Ci, int Co) {
    const long long total = rows * Co;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const int oc = (int)(i % Co);
        const long long r = i / Co;
        const h16 *x = in + r * Ci, *wr = w + (long long)oc * Ci;
        float s = 0.f;
        for (int ic = 0; ic < Ci; ++ic) s += h2f(x[ic]) * h2f(wr[ic]);
        if (bias) s += h2f(bias[oc]);
        out[i] = f2h(s);
    }
}

bool positive(const char *what, std::initializer_list<int> v) {
    for (int x : v)
        if (x <= 0) {
            kf_report_error("%s: non-positive dimension", what);
            return false;
        }
    return true;
}

}  // namespace

extern "C" {

void launch_conv1d_forward_fp16(const void *input, const void *weight, const void *bias,
                                void *output, int B, int Ti, int Ci, int Co, int K, int stride,
                                int pad, int dil, void *stream) {
    kf_take_pending(__func__);
    if (!positive("conv1d_forward", {B, Ti, Ci, Co, K, stride, dil})) return;
    const int To = conv1d_output_size(Ti, K, stride, pad, dil);
    if (To <= 0) return;
    const long long n = (long long)B * To * Co;
    k_conv1d_fwd<<<kf_blocks(n, 256, 65536), 256, 0, pick(stream)>>>(
        (const h16 *)input, (const h16 *)weight, (const h16 *)bias, (h16 *)output, B, Ti, Ci, Co, K,
        stride, pad, dil, To);
    check("conv1d_forward");
}

void launch_conv1d_backward_fp16(const void *input, const void *grad_output, const void *weight,
                                 void *grad_input, void *grad_weight, void *grad_bias, int B,
                                 int Ti, int Ci, int Co, int K, int stride, int pad, int dil,
                                 void *stream) {
    kf_take_pending(__func__);
    if (!positive("conv1d_backward", {B, Ti, Ci, Co, K, stride, dil})) return;
    const int To = conv1d_output_size(Ti, K, stride, pad, dil);
    if (To <= 0) return;
    hipStream_t s = pick(stream);
    if (grad_input) {
        const long long n = (long long)B * Ti * Ci;
        k_conv1d_bwd_in<<<kf_blocks(n, 256, 65536), 256, 0, s>>>(
            (const h16 *)grad_output, (const h16 *)weight, (h16 *)grad_input, B, Ti, Ci, Co, K,
            stride, pad, dil, To);
    }
    if (grad_weight)
        k_conv1d_bwd_w<<<Co * Ci * K, 256, 0, s>>>((const h16 *)input, (const h16 *)grad_output,
                                                   (h16 *)grad_weight, B, Ti, Ci, Co, K, stride,
                                                   pad, dil, To);
    if (grad_bias)
        k_col_sum<<<Co, 256, 0, s>>>((const h16 *)grad_output, (h16 *)grad_bias, (long long)B * To,
                                     Co);
    check("conv1d_backward");
}

void launch_maxpool1d_forward_fp16(const void *input, void *output, void *indices, int B, int Ti,
                                   int C, int K, int stride, void *stream) {
    kf_take_pending(__func__);
    if (!positive("maxpool1d_forward", {B, Ti, C, K, stride})) return;
    const int To = pool1d_output_size(Ti, K, stride);
    if (To <= 0) return;
    const long long n = (long long)B * To * C;
    k_maxpool_fwd<<<kf_blocks(n, 256, 65536), 256, 0, pick(stream)>>>(
        (const h16 *)input, (h16 *)output, (int32_t *)indices, B, Ti, C, K, stride, To);
    check("maxpool1d_forward");
}

void launch_maxpool1d_backward_fp16(const void *grad_output, const void *indices, void *grad_input,
                                    int B, int Ti, int To, int C, void *stream) {
    kf_take_pending(__func__);
    if (!positive("maxpool1d_backward", {B, Ti, To, C})) return;
    k_maxpool_bwd<<<kf_blocks((long long)B * C, 256, 65536), 256, 0, pick(stream)>>>(
        (const h16 *)grad_output, (const int32_t *)indices, (h16 *)grad_input, B, Ti, To, C);
    check("maxpool1d_backward");
}

void launch_stats_pooling_fp16(const void *input, void *output, int B, int T, int C,
                               void *stream) {
    kf_take_pending(__func__);
    if (!positive("stats_pooling", {B, T, C})) return;
    k_stats_pool<<<kf_blocks((long long)B * C, 256, 65536), 256, 0, pick(stream)>>>(
        (const h16 *)input, (h16 *)output, B, T, C);
    check("stats_pooling");
}

void launch_batchnorm1d_forward_fp16(const void *input, const void *gamma, const void *beta,
                                     void *running_mean, void *running_var, void *output,
                                     void *save_mean, void *save_invstd, int B, int T, int C,
                                     float momentum, float eps, bool training, void *stream) {
    kf_take_pending(__func__);
    if (!positive("batchnorm1d_forward", {B, T, C})) return;
    k_bn1d<<<C, 256, 0, pick(stream)>>>((const h16 *)input, (const h16 *)gamma, (const h16 *)beta,
                                        (h16 *)running_mean, (h16 *)running_var, (h16 *)output,
                                        (h16 *)save_mean, (h16 *)save_invstd, (long long)B * T, C,
                                        momentum, eps, training ? 1 : 0);
    check("batchnorm1d_forward");
}

void launch_layernorm_forward_fp16(const void *input, const void *gamma, const void *beta,
                                   void *output, int B, int T, int C, float eps, void *stream) {
    kf_take_pending(__func__);
    if (!positive("layernorm_forward", {B, T, C})) return;
    k_layernorm<<<B * T, 256, 0, pick(stream)>>>((const h16 *)input, (const h16 *)gamma,
                                                 (const h16 *)beta, (h16 *)output, C, eps);
    check("layernorm_forward");
}

void launch_depthwise_conv1d_fp16(const void *input, const void *weight, const void *bias,
                                  void *output, int B, int Ti, int C, int K, int stride, int pad,
                                  void *stream) {
    kf_take_pending(__func__);
    if (!positive("depthwise_conv1d", {B, Ti, C, K, stride})) return;
    const int To = (Ti + 2 * pad - K) / stride + 1;
    if (To <= 0) return;
    const long long n = (long long)B * To * C;
    k_depthwise<<<kf_blocks(n, 256, 65536), 256, 0, pick(stream)>>>(
        (const h16 *)input, (const h16 *)weight, (const h16 *)bias, (h16 *)output, B, Ti, C, K,
        stride, pad, To);
    check("depthwise_conv1d");
}

void launch_pointwise_conv1d_fp16(const void *input, const void *weight, const void *bias,
                                  void *output, int B, int T, int Ci, int Co, void *stream) {
    kf_take_pending(__func__);
    if (!positive("pointwise_conv1d", {B, T, Ci, Co})) return;
    const long long rows = (long long)B * T;
    k_pointwise<<<kf_blocks(rows * Co, 256, 65536), 256, 0, pick(stream)>>>(
        (const h16 *)input, (const h16 *)weight, (const h16 *)bias, (h16 *)output, rows, Ci, Co);
    check("pointwise_conv1d");
}

}  // extern "C"
