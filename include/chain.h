/*
 * chain.h — log-domain chain forward-backward half of the kaldi-fp16 C-ABI,
 * MI355X build. Drop-in for the reference's cpp/include/chain.h:23-159
 * (implemented there in cpp/cuda/chain.cu:368-612 and chain_det.cu:293-477,
 * bound from Go by internal/nnet/chain_loss.go:33-213).
 *
 * Same names, struct layouts and conventions: int 0 / -1 with a thread-local
 * chain_last_error(); float entry points return -1e30 on failure. FST pointers
 * are device pointers; labels are 1-indexed pdf ids (0 = epsilon, skipped);
 * weights are log weights. nnet_output is FP16 unless named otherwise.
 *
 * MI355X differences: every forward-backward is one
 * workgroup-resident kernel that keeps its own fixed arc order, so the plain
 * and the *_det entry points return identical, deterministic results; the
 * `stream` arguments are honoured (NULL = the library's current stream).
 */
#ifndef KALDI_FP16_AMD_CHAIN_H
#define KALDI_FP16_AMD_CHAIN_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* chain.h:23-35 */
typedef struct {
    int32_t *row_ptr;      /* [num_states + 1] */
    int32_t *col_idx;      /* [num_arcs] destination states */
    int32_t *labels;       /* [num_arcs] pdf ids, 1-indexed */
    float *weights;        /* [num_arcs] log weights */
    int32_t *final_states; /* [num_final] */
    float *final_weights;  /* [num_final] log weights */
    int num_states;
    int num_arcs;
    int num_final;
    int start_state;
} ChainFstGPU;

/* chain.h:38-44 */
typedef struct {
    float num_logprob;
    float den_logprob;
    float loss; /* -(num_logprob - den_logprob) */
} ChainLossResult;

/* alpha/beta: caller-owned [(T+1) x num_states] FP32 (chain.cu:368-438) */
int chain_forward_backward(const void *nnet_output, const ChainFstGPU *fst, int T, int num_pdfs,
                           float *alpha, float *beta, float *total_logprob);
/* posteriors [T x num_pdfs] FP32, overwritten (chain.cu:440-473) */
int chain_compute_posteriors(const void *nnet_output, const ChainFstGPU *fst, int T, int num_pdfs,
                             const float *alpha, const float *beta, float total_logprob,
                             float *posteriors);
/* both FSTs in the log semiring; grad_output FP16 [T x num_pdfs] = clamp(den-num, +-30),
 * NULL to skip (chain.cu:475-612) */
int chain_compute_loss(const void *nnet_output, const ChainFstGPU *num_fst,
                       const ChainFstGPU *den_fst, int T, int num_pdfs, void *grad_output,
                       ChainLossResult *result);

/* deterministic variants (chain_det.cu:293-477) */
int chain_forward_backward_det(const void *nnet_output, const ChainFstGPU *fst, int T,
                               int num_pdfs, float *alpha, float *beta, float *total_logprob);
int chain_compute_posteriors_det(const void *nnet_output, const ChainFstGPU *fst, int T,
                                 int num_pdfs, const float *alpha, const float *beta,
                                 float total_logprob, float *posteriors);
/* FP32 nnet_output, converted to FP16 first (chain_det.cu:412-477) */
float chain_num_forward_backward_det(const int *fst_row_ptr, const int *fst_col_idx,
                                     const float *fst_weights, const int *fst_pdf_ids,
                                     const int *fst_final_states, const float *fst_final_weights,
                                     int num_states, int num_arcs, int num_final,
                                     const float *nnet_output, float *num_post, int T,
                                     int num_pdfs, void *stream);

/* 2 * (T+1) * num_states * sizeof(float) (chain.cu:361-366) */
size_t chain_workspace_bytes(int T, int num_states);

const char *chain_last_error(void);
void chain_clear_error(void);

#ifdef __cplusplus
}
#endif
#endif
