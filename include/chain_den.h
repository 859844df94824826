/*
 * chain_den.h — probability-space denominator half of the kaldi-fp16 C-ABI,
 * MI355X build. Drop-in for the reference's cpp/include/chain_den.h:28-80
 * (implemented in cpp/cuda/chain_den.cu:295-706, bound from Go by
 * internal/nnet/denominator.go:98-283).
 *
 * Same contract: transitions are uploaded once (SoA, pdf ids 0-indexed,
 * tp = exp(-weight)); den_forward / den_forward_backward take HOST nnet output
 * [T x num_pdfs] FP32 and HOST initial probs, return the log-prob (-1e30 on
 * failure, den_last_error()) and, for the latter, HOST posteriors.
 * One sequence per call, as denominator.go:226-228 requires.
 *
 * MI355X: den_fst_upload also builds the sliced, degree-sorted arc tables the
 * workgroup-resident kernel streams (kept beside the struct, released by
 * den_fst_free); one launch runs all frames with no host round trip.
 */
#ifndef KALDI_FP16_AMD_CHAIN_DEN_H
#define KALDI_FP16_AMD_CHAIN_DEN_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* chain_den.h:28-37 */
typedef struct {
    int32_t *src_states;
    int32_t *dst_states;
    int32_t *pdf_ids;
    float *transition_probs;
    int num_transitions;
    int num_states;
    int num_pdfs;
} DenFstGPU;

int den_fst_upload(DenFstGPU *fst, const int32_t *src, const int32_t *dst, const int32_t *pdf,
                   const float *trans_probs, int num_trans, int num_states, int num_pdfs);
void den_fst_free(DenFstGPU *fst);

float den_forward(const DenFstGPU *fst, const float *nnet_output, const float *initial_probs,
                  int T, float leaky_hmm_coeff);
float den_forward_backward(const DenFstGPU *fst, const float *nnet_output,
                           const float *initial_probs, int T, float leaky_hmm_coeff,
                           float *grad_output);

const char *den_last_error(void);
void den_clear_error(void);

#ifdef __cplusplus
}
#endif
#endif
