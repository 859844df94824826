/*
 * chain_backward_api.h — objective-assembly half of the kaldi-fp16 C-ABI,
 * MI355X build. Drop-in for the reference's cpp/include/chain_backward_api.h
 * :45-143 (implemented in cpp/cuda/chain_backward.cu:27-410, called from
 * internal/nnet/backward.go:224-371). All arrays are device arrays; FP32 unless
 * named otherwise.
 */
#ifndef KALDI_FP16_AMD_CHAIN_BACKWARD_API_H
#define KALDI_FP16_AMD_CHAIN_BACKWARD_API_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* FP32 nnet_output -> FP16 -> log-domain forward-backward -> num_post [T x P];
 * start state 0; returns the total log-prob or -1e30 (chain_backward.cu:341-410) */
float chain_num_forward_backward(const int *fst_row_ptr, const int *fst_col_idx,
                                 const float *fst_weights, const int *fst_pdf_ids,
                                 const int *fst_final_states, const float *fst_final_weights,
                                 int num_states, int num_arcs, int num_final,
                                 const float *nnet_output, float *num_post, int T, int num_pdfs,
                                 void *stream);
/* grad_output FP16 = weight * (num_post - den_post) (chain_backward.cu:91-104, :186-205) */
int chain_combine_gradient(const float *num_post, const float *den_post, float weight, int T,
                           int num_pdfs, void *grad_output);
/* even frames: deriv += (+-limit - x) * scale outside [-limit, limit]; returns the
 * count (chain_backward.cu:27-67, :215-240) */
int chain_penalize_out_of_range(const float *nnet_output, float *grad_output, float limit,
                                float scale, int T, int num_pdfs);
/* grad -= l2_scale * x; returns -0.5 * l2_scale * sum(x^2) (chain_backward.cu:111-148) */
float chain_l2_regularize(const float *nnet_output, float *grad_output, float l2_scale,
                          int total_elements);
/* (chain_backward.cu:153-160, :276-288) */
int chain_grad_fp32_to_fp16(const float *grad_fp32, void *grad_fp16, int total_elements);
/* grad += weight * (num_post - den_post) (chain_backward.cu:168-180, :292-313) */
int chain_add_posterior_gradient(const float *num_post, const float *den_post, float *grad,
                                 float weight, int total_elements);

#ifdef __cplusplus
}
#endif
#endif
