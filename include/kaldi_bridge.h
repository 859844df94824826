/*
 * kaldi_bridge.h — the go/kaldibridge C-ABI (libkaldi_fp16_cgo.so), rebuilt for MI355X.
 *
 * Replaces the declarations of go/kaldibridge/bridge.go:10-53, implemented by
 * cpp/src/cgo_interface.cu:20-451. Same names, argument meaning and error
 * convention: void functions, NULL handles on failure, and a thread-local
 * kaldi_get_last_error() that returns NULL when clear.
 *
 * Differences behind the same calls:
 *  - "cublas" handles are opaque GEMM contexts of this build (no cuBLAS exists);
 *    kaldi_cublas_enable_tensor_cores is accepted and changes nothing, since every
 *    GEMM runs on the fp16 MFMA kernels.
 *  - kaldi_gemm accumulates in fp32 and rounds once to fp16 (RNE); the reference's
 *    cublasHgemm accumulates in fp16 (cgo_interface.cu:229-238). alpha and beta are
 *    rounded to fp16 first, as the reference does.
 *  - kaldi_tensor_data returns the device pointer of a tensor. The reference's
 *    cnn_bridge.go passes the address of the C struct instead (cnn_bridge.go:174-183),
 *    SURVEY §8b(5); a Go caller uses this accessor for launch_* arguments.
 *  - Calls run on the library's current stream (kf_set_stream, default the null
 *    stream); kaldi_tensor_copy_to_host_fp32 synchronises it.
 */
#ifndef KALDI_FP16_AMD_KALDI_BRIDGE_H
#define KALDI_FP16_AMD_KALDI_BRIDGE_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void *TensorHandle;
typedef void *CuBLASHandlePtr;
typedef void *LossScalerHandle;

CuBLASHandlePtr kaldi_cublas_create(void);
void kaldi_cublas_destroy(CuBLASHandlePtr handle);
void kaldi_cublas_enable_tensor_cores(CuBLASHandlePtr handle);

/* fp16 [rows x cols] row-major device tensors */
TensorHandle kaldi_tensor_create(int rows, int cols);
TensorHandle kaldi_tensor_zeros(int rows, int cols);
TensorHandle kaldi_tensor_ones(int rows, int cols);
void kaldi_tensor_free(TensorHandle t);
int kaldi_tensor_rows(TensorHandle t);
int kaldi_tensor_cols(TensorHandle t);
size_t kaldi_tensor_size(TensorHandle t);
void *kaldi_tensor_data(TensorHandle t);

/* count is clamped to the tensor size; fp32 -> fp16 is RNE */
void kaldi_tensor_copy_from_host_fp32(TensorHandle t, const float *data, size_t count);
void kaldi_tensor_copy_to_host_fp32(TensorHandle t, float *data, size_t count);

/* C = alpha * op(A) * op(B) + beta * C, op = transpose when trans != 0 */
void kaldi_gemm(CuBLASHandlePtr handle, TensorHandle A, TensorHandle B, TensorHandle C,
                float alpha, float beta, int transA, int transB);
void kaldi_relu(TensorHandle t);
void kaldi_sigmoid(TensorHandle t);
void kaldi_tanh(TensorHandle t);
void kaldi_softmax(TensorHandle t); /* per row */
void kaldi_add(TensorHandle a, TensorHandle b); /* a += b */
void kaldi_scale(TensorHandle t, float alpha);

/* dynamic loss scale: x0.5 on overflow, x2 after 2000 clean steps, clamped to [1, 65536] */
LossScalerHandle kaldi_loss_scaler_create(float initial_scale);
void kaldi_loss_scaler_free(LossScalerHandle ls);
float kaldi_loss_scaler_get_scale(LossScalerHandle ls);
void kaldi_loss_scaler_update(LossScalerHandle ls, int overflow);

const char *kaldi_get_last_error(void);
void kaldi_clear_error(void);

#ifdef __cplusplus
}
#endif
#endif
