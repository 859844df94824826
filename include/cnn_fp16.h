/*
 * cnn_fp16.h — the reference's generic CNN launch wrappers, rebuilt for MI355X.
 *
 * Replaces cpp/include/cnn_fp16.h:24-160 (kernels cpp/cuda/cnn_kernels.cu:19-830)
 * and launch_maxpool1d_backward_fp16 (cpp/cuda/backward_wrappers.cu:212-225).
 * Callers: go/kaldibridge/cnn_bridge.go:14-72 and internal/gpu/backward_ops.go:19-28.
 * These wrappers are off the CNN-TDNN training path (the path's convolutions are
 * the implicit-im2col GEMMs of kf_ops.h); they are correct, simple HIP kernels.
 *
 * Layouts as in the reference: activations [batch][time][channels] fp16,
 * conv weights [out_channels][in_channels][kernel_size] fp16, biases fp16.
 * `stream` is a hipStream_t (NULL = the library's current stream, kf_set_stream).
 *
 * Deviations from the reference, each a fix of a defect:
 *  - gradients are plain fp16 stores of an fp32 sum: the reference adds float
 *    atomics into fp16 buffers (cnn_kernels.cu:204, :384; backward_wrappers.cu:100);
 *    grad_weight/grad_bias/grad_input are OVERWRITTEN, maxpool backward adds into
 *    the (caller-zeroed) grad_input in a fixed order;
 *  - conv1d input gradient tests the output index after the stride division
 *    (cnn_kernels.cu:148 compares it before); identical for stride 1;
 *  - launch_conv1d_backward_fp16 skips grad_input / grad_weight / grad_bias when NULL.
 * The functions are void, as in the reference; launch errors are reported through
 * kf_last_error().
 */
#ifndef KALDI_FP16_AMD_CNN_FP16_H
#define KALDI_FP16_AMD_CNN_FP16_H

#ifndef __cplusplus
#include <stdbool.h>
#endif

#ifdef __cplusplus
extern "C" {
#endif

void launch_conv1d_forward_fp16(const void *input, const void *weight, const void *bias,
                                void *output, int batch_size, int time_in, int in_channels,
                                int out_channels, int kernel_size, int stride, int padding,
                                int dilation, void *stream);

void launch_conv1d_backward_fp16(const void *input, const void *grad_output, const void *weight,
                                 void *grad_input, void *grad_weight, void *grad_bias,
                                 int batch_size, int time_in, int in_channels, int out_channels,
                                 int kernel_size, int stride, int padding, int dilation,
                                 void *stream);

/* indices: int32 [batch][time_out][channels], absolute input time of each max */
void launch_maxpool1d_forward_fp16(const void *input, void *output, void *indices,
                                   int batch_size, int time_in, int channels, int kernel_size,
                                   int stride, void *stream);

void launch_maxpool1d_backward_fp16(const void *grad_output, const void *indices,
                                    void *grad_input, int batch_size, int time_in, int time_out,
                                    int channels, void *stream);

/* output [batch][2*channels]: mean then sqrt(var + 1e-10) over time */
void launch_stats_pooling_fp16(const void *input, void *output, int batch_size, int time_steps,
                               int channels, void *stream);

/* gamma/beta/running stats/save buffers are fp16 [channels]; biased variance */
void launch_batchnorm1d_forward_fp16(const void *input, const void *gamma, const void *beta,
                                     void *running_mean, void *running_var, void *output,
                                     void *save_mean, void *save_invstd, int batch_size,
                                     int time_steps, int channels, float momentum, float eps,
                                     bool training, void *stream);

void launch_layernorm_forward_fp16(const void *input, const void *gamma, const void *beta,
                                   void *output, int batch_size, int time_steps, int channels,
                                   float eps, void *stream);

/* weight [channels][kernel_size] */
void launch_depthwise_conv1d_fp16(const void *input, const void *weight, const void *bias,
                                  void *output, int batch_size, int time_in, int channels,
                                  int kernel_size, int stride, int padding, void *stream);

/* weight [out_channels][in_channels] */
void launch_pointwise_conv1d_fp16(const void *input, const void *weight, const void *bias,
                                  void *output, int batch_size, int time_steps, int in_channels,
                                  int out_channels, void *stream);

static inline int conv1d_output_size(int time_in, int kernel_size, int stride, int padding,
                                     int dilation) {
    return (time_in + 2 * padding - dilation * (kernel_size - 1) - 1) / stride + 1;
}
static inline int pool1d_output_size(int time_in, int kernel_size, int stride) {
    return (time_in - kernel_size) / stride + 1;
}

#ifdef __cplusplus
}
#endif
#endif
