/*
 * ops.h — compute half of the kaldi-fp16 C-ABI, MI355X build.
 *
 * Drop-in for the reference's cpp/include/ops.h:16-188 (implemented there in
 * cpp/cuda/ops.cu:336-643 and cpp/cuda/backward_wrappers.cu:151-291, bound
 * from Go by internal/gpu/ops.go:21-366 and internal/gpu/backward_ops.go).
 *
 * Conventions kept from the reference:
 *   - matrices are row-major and contiguous; fp16 is raw IEEE binary16 bits;
 *   - every fp16 result is computed in fp32 and rounded to nearest-even once;
 *   - 0 = success, -1 = failure with the text in ops_last_error() (thread-local);
 *   - ops_subsample_rows is void and silent (ops.cu:632-643).
 *
 * What differs behind the same signatures (documented in DESIGN.md):
 *   - ops_gemm / ops_gemm_strided run hand-written gfx950 MFMA kernels
 *     (v_mfma_f32_16x16x32_f16, fp32 accumulation) instead of cuBLAS. lda/ldb/ldc
 *     are honoured (the reference ignores them, ops.cu:386-389); passing the
 *     contiguous values (K, N, N) reproduces the reference exactly.
 *   - ops_cublas_create keeps its name and returns an opaque GEMM context.
 *   - library temporaries come from a persistent per-device workspace.
 */
#ifndef KALDI_FP16_AMD_OPS_H
#define KALDI_FP16_AMD_OPS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* dst[r] = src[row_offset + r*stride], r < (in_rows-row_offset+stride-1)/stride (ops.cu:632) */
void ops_subsample_rows(void *dst, const void *src, int in_rows, int cols, int stride,
                        int row_offset);

/* GEMM context (ops.cu:336-354) */
void *ops_cublas_create(void);
void ops_cublas_destroy(void *handle);

/* C[MxN] = alpha*A[MxK]*B[KxN] + beta*C (ops.cu:366-400) */
int ops_gemm(void *handle, int M, int N, int K, float alpha, const void *A, int lda,
             const void *B, int ldb, float beta, void *C, int ldc);
/* batched with element strides, B may be shared via strideB = 0 (ops.cu:402-426) */
int ops_gemm_strided(void *handle, int M, int N, int K, float alpha, const void *A, int lda,
                     int64_t strideA, const void *B, int ldb, int64_t strideB, float beta,
                     void *C, int ldc, int64_t strideC, int batch_count);

/* in-place activations on count fp16 values (ops.cu:26-67, :439-477) */
int ops_relu(void *data, int count);
int ops_sigmoid(void *data, int count);
int ops_tanh_act(void *data, int count);
int ops_clipped_relu(void *data, int count, float ceiling);

/* per-row (log-)softmax on [rows x cols] (ops.cu:70-166, :483-509).
 * The reference's int-atomicMax row max is wrong for all-negative rows; this
 * build computes the true row max. */
int ops_softmax(void *data, int rows, int cols);
int ops_log_softmax(void *data, int rows, int cols);

/* inference BatchNorm with frozen statistics, in place on x[T x D] (ops.cu:171-204) */
int ops_batchnorm_forward(void *x, int T, int D, const float *mean, const float *var,
                          const float *gamma, const float *beta, float epsilon);
int ops_batchnorm_forward_rms(void *x, int T, int D, const float *mean, const float *var,
                              float target_rms, float epsilon);

/* element-wise (ops.cu:207-237, :546-580) */
int ops_add_scaled(void *dst, const void *src, int count, float alpha, float beta);
int ops_add(void *dst, const void *src, int count);
int ops_copy(void *dst, const void *src, int count);
int ops_fill(void *dst, int count, float val);

/* column placement / extraction (ops.cu:241-254, :308-320) */
int ops_concat_cols(void *dst, int T, int dst_cols, const void *src, int src_cols,
                    int dst_col_offset);
int ops_slice_cols(const void *src, int T, int src_cols, void *dst, int dst_cols,
                   int src_col_offset);
/* [T x (H*F1 | H*F2)] -> [T x H*(F1+F2)] in place (ops.cu:258-287, :590-626) */
int ops_combine_feature_maps(void *data, int T, int total_dim, int height, int num_filters1,
                             int num_filters2);

const char *ops_last_error(void);
void ops_clear_error(void);

/* backward element-wise (backward_wrappers.cu:41-115, :151-253) */
int ops_relu_backward(const void *x, void *grad, int count);
int ops_sigmoid_backward(const void *output, void *grad, int count);
int ops_tanh_backward(const void *output, void *grad, int count);
int ops_transpose(const void *src, void *dst, int M, int N);
int ops_batchnorm_backward(const void *grad_out, void *grad_in, const float *gamma,
                           const float *variance, float eps, int rows, int cols);

/* optimiser pieces (backward_wrappers.cu:118-142, :255-291):
 * v = momentum*v + g; w32 -= lr*v; w16 = rne(w32) */
int ops_fp16_to_fp32(const void *src, float *dst, int count);
int ops_sgd_update(float *w_fp32, void *w_fp16, const void *grad_fp16, float *velocity,
                   float lr, float momentum, int count);

#ifdef __cplusplus
}
#endif
#endif
