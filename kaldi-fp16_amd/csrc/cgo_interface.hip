// cgo_interface.hip — libkaldi_fp16_cgo.so: the go/kaldibridge C-ABI (include/kaldi_bridge.h).
//
// Behaviour of cpp/src/cgo_interface.cu:20-451: opaque fp16 tensors, a GEMM on
// them, in-place activations, element-wise add/scale and the dynamic loss
// scaler. GEMMs go to the MFMA kernels of libkaldi_fp16.so (kf_gemm_fused), with
// the transposes expressed as operand orientation; shapes the MFMA tiles cannot
// address (dimensions not multiples of 8) take a plain fp32-accumulating kernel.
#include "kf_common.h"
#include "../../include/kaldi_bridge.h"
#include "../../include/kf_ops.h"

KF_DECLARE_ERR(kaldi)

extern "C" const char *kaldi_get_last_error(void) { return kaldi_err_.get(); }
extern "C" void kaldi_clear_error(void) { kaldi_err_.clear(); }

namespace {

// same field order as the reference's TensorFP16 (cgo_interface.cu:81-86)
struct Tensor {
    h16 *data;
    int rows, cols;
    size_t size;
};

constexpr unsigned kCtxMagic = 0x6b663136u;  // "kf16"
struct GemmCtx {
    unsigned magic;
    int tensor_cores;
};

bool hip_ok(hipError_t e, const char *what) {
    if (e == hipSuccess) return true;
    kaldi_set_error("%s: %s", what, hipGetErrorString(e));
    return false;
}

// fp32 staging for host copies (grown on demand, never shrunk)
float *g_stage = nullptr;
size_t g_stage_n = 0;
float *stage(size_t n) {
    if (n <= g_stage_n) return g_stage;
    if (g_stage) hipFree(g_stage);
    g_stage = nullptr;
    g_stage_n = 0;
    if (!hip_ok(hipMalloc(&g_stage, n * sizeof(float)), "staging buffer")) return nullptr;
    g_stage_n = n;
    return g_stage;
}

#define GRID_LOOP(i, n)                                                                      \
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < (long long)(n); \
         i += (long long)gridDim.x * blockDim.x)

__global__ void k_f32_to_f16(const float *s, h16 *d, long long n) { GRID_LOOP(i, n) d[i] = f2h(s[i]); }
__global__ void k_f16_to_f32(const h16 *s, float *d, long long n) { GRID_LOOP(i, n) d[i] = h2f(s[i]); }
__global__ void k_fill(h16 *d, long long n, float v) { GRID_LOOP(i, n) d[i] = f2h(v); }

enum { A_RELU, A_SIGMOID, A_TANH, A_SCALE };
__global__ void k_act(h16 *d, long long n, int op, float a) {
    GRID_LOOP(i, n) {
        const float x = h2f(d[i]);
        float y;
        if (op == A_RELU) y = x > 0.f ? x : 0.f;
        else if (op == A_SIGMOID) y = 1.f / (1.f + expf(-x));
        else if (op == A_TANH) y = tanhf(x);
        else y = x * a;
        d[i] = f2h(y);
    }
}
__global__ void k_add(h16 *a, const h16 *b, long long n) { GRID_LOOP(i, n) a[i] = f2h(h2f(a[i]) + h2f(b[i])); }

// row softmax with the reference's two rounding points (cgo_interface.cu:283-336):
// e = fp16(exp(x - max)) is stored, the sum is of the unrounded exps, and the
// result is fp16(e / sum)
__global__ void k_softmax_rows(h16 *data, int cols) {
    __shared__ float sh[4];
    h16 *row = data + (long long)blockIdx.x * cols;
    float mx = -1e10f;
    for (int c = threadIdx.x; c < cols; c += blockDim.x) mx = fmaxf(mx, h2f(row[c]));
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = mx;
    __syncthreads();
    mx = fmaxf(fmaxf(sh[0], sh[1]), fmaxf(sh[2], sh[3]));
    __syncthreads();
    float s = 0.f;
    for (int c = threadIdx.x; c < cols; c += blockDim.x) {
        const float e = expf(h2f(row[c]) - mx);
        row[c] = f2h(e);
        s += e;
    }
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s;
    __syncthreads();
    s = ((sh[0] + sh[1]) + sh[2]) + sh[3];
    for (int c = threadIdx.x; c < cols; c += blockDim.x) row[c] = f2h(h2f(row[c]) / s);
}

// C[m][n] = alpha * sum_k opA(m,k) opB(k,n) + beta * C[m][n], any shape / orientation
__global__ void k_gemm_any(int M, int N, int K, float alpha, const h16 *A, int lda, int ta,
                           const h16 *B, int ldb, int tb, float beta, h16 *C, int ldc) {
    GRID_LOOP(i, (long long)M * N) {
        const int m = (int)(i / N), n = (int)(i % N);
        float s = 0.f;
        for (int k = 0; k < K; ++k) {
            const float a = h2f(ta ? A[(long long)k * lda + m] : A[(long long)m * lda + k]);
            const float b = h2f(tb ? B[(long long)n * ldb + k] : B[(long long)k * ldb + n]);
            s += a * b;
        }
        h16 *c = C + (long long)m * ldc + n;
        float v = alpha * s;
        if (beta != 0.f) v += beta * h2f(*c);
        *c = f2h(v);
    }
}

// A^T staged k-contiguous for the MFMA path: dst[m][k] = src[k][m]
__global__ void k_transpose(const h16 *src, h16 *dst, int R, int Cc) {
    GRID_LOOP(i, (long long)R * Cc) {
        const int r = (int)(i / Cc), c = (int)(i % Cc);
        dst[(long long)c * R + r] = src[i];
    }
}

int blocks(long long n) { return kf_blocks(n, 256, 65536); }

Tensor *as_tensor(TensorHandle h) { return (Tensor *)h; }

KfOperand plain(const void *p, long long ld, int rows, int cols, int kcontig) {
    KfOperand d;
    memset(&d, 0, sizeof d);
    d.base = p;
    d.ld = ld;
    d.nrows = rows;
    d.ncols = cols;
    d.kcontig = kcontig;
    d.nparts = 1;
    d.part_width = cols;
    d.T = rows;
    d.hout = d.hsrc = d.hdiv = 1;
    d.tpolicy = KF_ZERO;
    for (int i = 0; i < KF_MAX_PARTS; ++i) d.edge_t[i] = -1;
    return d;
}

void launch_act(TensorHandle h, int op, float a, const char *what) {
    kf_take_pending(__func__);
    Tensor *t = as_tensor(h);
    if (!t || !t->size) return;
    k_act<<<blocks(t->size), 256, 0, kf_stream()>>>(t->data, (long long)t->size, op, a);
    hip_ok(hipGetLastError(), what);
}

}  // namespace

extern "C" {

CuBLASHandlePtr kaldi_cublas_create(void) { return new GemmCtx{kCtxMagic, 0}; }
void kaldi_cublas_destroy(CuBLASHandlePtr h) {
    GemmCtx *c = (GemmCtx *)h;
    if (c && c->magic == kCtxMagic) {
        c->magic = 0;
        delete c;
    }
}
void kaldi_cublas_enable_tensor_cores(CuBLASHandlePtr h) {
    GemmCtx *c = (GemmCtx *)h;
    if (c && c->magic == kCtxMagic) c->tensor_cores = 1;
}

TensorHandle kaldi_tensor_create(int rows, int cols) {
    if (rows < 0 || cols < 0) {
        kaldi_set_error("tensor_create: negative shape %d x %d", rows, cols);
        return nullptr;
    }
    Tensor *t = new Tensor{nullptr, rows, cols, (size_t)rows * (size_t)cols};
    if (t->size && !hip_ok(hipMalloc(&t->data, t->size * sizeof(h16)), "tensor_create")) {
        delete t;
        return nullptr;
    }
    return t;
}

TensorHandle kaldi_tensor_zeros(int rows, int cols) {
    Tensor *t = as_tensor(kaldi_tensor_create(rows, cols));
    if (t && t->size) hip_ok(hipMemsetAsync(t->data, 0, t->size * sizeof(h16), kf_stream()), "tensor_zeros");
    return t;
}

TensorHandle kaldi_tensor_ones(int rows, int cols) {
    kf_take_pending(__func__);
    Tensor *t = as_tensor(kaldi_tensor_create(rows, cols));
    if (t && t->size) {
        k_fill<<<blocks(t->size), 256, 0, kf_stream()>>>(t->data, (long long)t->size, 1.f);
        hip_ok(hipGetLastError(), "tensor_ones");
    }
    return t;
}

void kaldi_tensor_free(TensorHandle h) {
    Tensor *t = as_tensor(h);
    if (!t) return;
    if (t->data) {
        hipStreamSynchronize(kf_stream());
        hipFree(t->data);
    }
    delete t;
}

int kaldi_tensor_rows(TensorHandle h) { return h ? as_tensor(h)->rows : 0; }
int kaldi_tensor_cols(TensorHandle h) { return h ? as_tensor(h)->cols : 0; }
size_t kaldi_tensor_size(TensorHandle h) { return h ? as_tensor(h)->size : 0; }
void *kaldi_tensor_data(TensorHandle h) { return h ? (void *)as_tensor(h)->data : nullptr; }

void kaldi_tensor_copy_from_host_fp32(TensorHandle h, const float *data, size_t count) {
    kf_take_pending(__func__);
    Tensor *t = as_tensor(h);
    if (!t || !data) return;
    if (count > t->size) count = t->size;
    if (!count) return;
    // the staging buffer may still feed a previous conversion
    if (!hip_ok(hipStreamSynchronize(kf_stream()), "copy_from_host_fp32")) return;
    float *s = stage(count);
    if (!s) return;
    if (!hip_ok(hipMemcpy(s, data, count * sizeof(float), hipMemcpyHostToDevice), "copy_from_host_fp32"))
        return;
    k_f32_to_f16<<<blocks(count), 256, 0, kf_stream()>>>(s, t->data, (long long)count);
    hip_ok(hipGetLastError(), "copy_from_host_fp32");
}

void kaldi_tensor_copy_to_host_fp32(TensorHandle h, float *data, size_t count) {
    kf_take_pending(__func__);
    Tensor *t = as_tensor(h);
    if (!t || !data) return;
    if (count > t->size) count = t->size;
    if (!count) return;
    float *s = stage(count);
    if (!s) return;
    k_f16_to_f32<<<blocks(count), 256, 0, kf_stream()>>>(t->data, s, (long long)count);
    if (!hip_ok(hipGetLastError(), "copy_to_host_fp32")) return;
    if (!hip_ok(hipStreamSynchronize(kf_stream()), "copy_to_host_fp32")) return;
    hip_ok(hipMemcpy(data, s, count * sizeof(float), hipMemcpyDeviceToHost), "copy_to_host_fp32");
}

void kaldi_gemm(CuBLASHandlePtr handle, TensorHandle hA, TensorHandle hB, TensorHandle hC,
                float alpha, float beta, int transA, int transB) {
    kf_take_pending(__func__);
    Tensor *A = as_tensor(hA), *B = as_tensor(hB), *Cm = as_tensor(hC);
    if (!handle || !A || !B || !Cm) {
        kaldi_set_error("null pointer in GEMM");
        return;
    }
    const int M = transA ? A->cols : A->rows, K = transA ? A->rows : A->cols;
    const int Kb = transB ? B->cols : B->rows, N = transB ? B->rows : B->cols;
    if (K != Kb || Cm->rows != M || Cm->cols != N) {
        kaldi_set_error("GEMM shape mismatch: op(A) %dx%d, op(B) %dx%d, C %dx%d", M, K, Kb, N,
                        Cm->rows, Cm->cols);
        return;
    }
    if (!M || !N) return;
    // cublasHgemm takes half alpha / beta (cgo_interface.cu:226-227)
    alpha = (float)(h16)alpha;
    beta = (float)(h16)beta;
    const bool aligned = K % 8 == 0 && N % 8 == 0 && M % 8 == 0 && K > 0;
    if (!aligned) {
        k_gemm_any<<<blocks((long long)M * N), 256, 0, kf_stream()>>>(
            M, N, K, alpha, A->data, A->cols, transA, B->data, B->cols, transB, beta, Cm->data, N);
        hip_ok(hipGetLastError(), "gemm");
        return;
    }
    const h16 *a = A->data;
    if (transA) {  // stage A^T k-contiguous: [M][K]
        h16 *at = (h16 *)kf_workspace((size_t)M * K * sizeof(h16), 3);
        if (!at) {
            kaldi_set_error("gemm: workspace for A^T (%d x %d) unavailable", M, K);
            return;
        }
        k_transpose<<<blocks((long long)M * K), 256, 0, kf_stream()>>>(A->data, at, K, M);
        a = at;
    }
    // operands in the kf_ops.h addressing rule: A is [M][K] k-contiguous; B is the
    // logical [K][N] (row-major, reduction-major) or, transposed, stored [N][K]
    KfOperand oa = plain(a, K, M, K, 1);
    KfOperand ob = transB ? plain(B->data, B->cols, N, K, 1) : plain(B->data, B->cols, K, N, 0);
    KfEpilogue E;
    memset(&E, 0, sizeof E);
    E.out = Cm->data;
    E.ldo = N;
    E.alpha = alpha;
    E.beta = beta;
    if (kf_gemm_fused(M, N, K, &oa, &ob, &E) != 0)
        kaldi_set_error("gemm: %s", kf_last_error() ? kf_last_error() : "launch failed");
}

void kaldi_relu(TensorHandle t) { launch_act(t, A_RELU, 0.f, "relu"); }
void kaldi_sigmoid(TensorHandle t) { launch_act(t, A_SIGMOID, 0.f, "sigmoid"); }
void kaldi_tanh(TensorHandle t) { launch_act(t, A_TANH, 0.f, "tanh"); }
void kaldi_scale(TensorHandle t, float alpha) { launch_act(t, A_SCALE, alpha, "scale"); }

void kaldi_softmax(TensorHandle h) {
    kf_take_pending(__func__);
    Tensor *t = as_tensor(h);
    if (!t || !t->rows || !t->cols) return;
    k_softmax_rows<<<t->rows, 256, 0, kf_stream()>>>(t->data, t->cols);
    hip_ok(hipGetLastError(), "softmax");
}

void kaldi_add(TensorHandle ha, TensorHandle hb) {
    kf_take_pending(__func__);
    Tensor *a = as_tensor(ha), *b = as_tensor(hb);
    if (!a || !b) return;
    if (b->size < a->size) {  // the reference reads past b here (cgo_interface.cu:357-365)
        kaldi_set_error("add: b has %zu elements, a has %zu", b->size, a->size);
        return;
    }
    if (!a->size) return;
    k_add<<<blocks(a->size), 256, 0, kf_stream()>>>(a->data, b->data, (long long)a->size);
    hip_ok(hipGetLastError(), "add");
}

// cgo_interface.cu:379-445
struct LossScaler {
    float scale, growth, backoff;
    int interval, since;
};

LossScalerHandle kaldi_loss_scaler_create(float initial_scale) {
    return new LossScaler{initial_scale, 2.f, 0.5f, 2000, 0};
}
void kaldi_loss_scaler_free(LossScalerHandle h) { delete (LossScaler *)h; }
float kaldi_loss_scaler_get_scale(LossScalerHandle h) { return h ? ((LossScaler *)h)->scale : 1.f; }
void kaldi_loss_scaler_update(LossScalerHandle h, int overflow) {
    LossScaler *ls = (LossScaler *)h;
    if (!ls) return;
    if (overflow) {
        ls->scale *= ls->backoff;
        ls->since = 0;
    } else if (++ls->since >= ls->interval) {
        ls->scale *= ls->growth;
        ls->since = 0;
    }
    ls->scale = fminf(fmaxf(ls->scale, 1.f), 65536.f);
}

}  // extern "C"
