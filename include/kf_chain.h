/*
 * kf_chain.h — MI355X batched chain LF-MMI objective (the device-resident form of
 * the reference's per-sequence objective).
 *
 * Replaces, for a whole minibatch in two kernel launches:
 *   ComputeChainObjfAndDeriv      internal/nnet/backward.go:224-371 (per sequence)
 *   ComputeChainLossBatch's loop  internal/nnet/chain_loss.go:221-294 (subsampling)
 *   NativeDenominator             internal/nnet/denominator.go:47-283
 *   den_forward_backward          cpp/cuda/chain_den.cu:496-706
 *   chain_num_forward_backward    cpp/cuda/chain_backward.cu:341-410 (det. order of
 *                                 chain_det.cu:55-237)
 * The reference runs one sequence per call with ~10 launches and ~3 blocking
 * device->host copies per frame; here one workgroup owns one sequence for all
 * its frames, state vectors stay in LDS and nothing returns to the host until
 * kf_chain_result() is asked for the statistics.
 *
 * Output gradient convention: out_grad = d(-objf)/d(nnet_output), i.e. the
 * negated Kaldi derivative, so that the SGD step w -= lr*v (backward_wrappers.cu
 * :129-142) ascends the objective — the same sign chain_compute_loss hands to
 * the reference's TrainStep (chain.cu:330-352, train_step.go:196-212).
 * Frame k of sequence i is row seq_row0[i] + k*stride of nnet_output/out_grad;
 * every such row is written on every call (zeros when the sequence's objective
 * is not finite, backward.go:356-363); no other row is touched.
 *
 * Errors: int 0 / -1 (NULL for constructors) and kf_chain_last_error().
 */
#ifndef KF_CHAIN_H
#define KF_CHAIN_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct KfDenGraph KfDenGraph;
typedef struct KfNumBatch KfNumBatch;
typedef struct KfChain KfChain;

/* Mirrors ChainTrainingOpts, backward.go:114-140 (xent_regularize is accepted and
 * unused: the xent branch is out of scope). */
typedef struct {
    float l2_regularize;
    float out_of_range_regularize;
    float leaky_hmm_coefficient;
    float xent_regularize;
    float supervision_weight;
} KfChainOpts;

/* Sums over the sequences of the last kf_chain_compute (backward.go:142-180). */
typedef struct {
    double objf;          /* sum_i w*(num_i - den_i), or -10*w*frames_i for bad ones */
    double l2_term;
    double total_weight;  /* sum_i w*frames_i */
    double num_logprob;   /* sum_i num_i */
    double den_logprob;   /* sum_i den_i */
    int frames;
    int out_of_range;
    int num_ok;           /* sequences whose objective was finite */
    int num_seqs;
} KfChainResult;

/* Denominator graph from its transitions (denominator.go:68-117): src/dst states,
 * pdf0 = label-1 (0-indexed), tp = exp(-tropical weight). initial_probs NULL ->
 * computed by the 100-iteration rule from start_state (denominator.go:131-171). */
KfDenGraph *kf_den_graph_create(int num_states, int num_pdfs, int num_transitions,
                                const int32_t *src, const int32_t *dst, const int32_t *pdf0,
                                const float *tp, int start_state, const float *initial_probs);
int kf_den_graph_initial_probs(const KfDenGraph *g, float *out /* host [S] */);
void kf_den_graph_free(KfDenGraph *g);

/* Numerator FSTs of one minibatch, host CSR arrays concatenated over sequences
 * (the layout of sparse.CSR, internal/sparse/sparse.go:20-91):
 *   seq i owns states [state_off[i], state_off[i+1]) and arcs [arc_off[i], arc_off[i+1]);
 *   row_ptr has state_off[nseq] + nseq entries: seq i's S_i+1 entries start at
 *   state_off[i] + i and hold LOCAL arc indices; dst holds LOCAL state ids;
 *   pdf1 are 1-indexed labels (0 = epsilon, skipped); logw = negated tropical weight;
 *   finals [final_off[i], final_off[i+1]) with LOCAL state ids and log weights.
 * The start state is 0 (chain_backward.cu:370). */
KfNumBatch *kf_num_batch_create(int nseq, const int32_t *state_off, const int32_t *arc_off,
                                const int32_t *row_ptr, const int32_t *dst, const int32_t *pdf1,
                                const float *logw, const int32_t *final_off,
                                const int32_t *final_state, const float *final_logw);
/* Re-fill an existing batch with the next minibatch's FSTs (same arrays as
 * kf_num_batch_create), TrainStep's per-minibatch upload (chain_loss.go:44-97) without a
 * device-wide stall: host preparation into pinned staging and one asynchronous copy on
 * `stream` (NULL: kf_get_stream()) into device buffers that only grow (a growth waits for
 * the device once). The caller orders the copy after every kernel still reading the batch's
 * previous contents; kf_chain_compute waits for the copy itself. 0 / -1. */
int kf_num_batch_refill(KfNumBatch *b, int nseq, const int32_t *state_off, const int32_t *arc_off,
                        const int32_t *row_ptr, const int32_t *dst, const int32_t *pdf1,
                        const float *logw, const int32_t *final_off, const int32_t *final_state,
                        const float *final_logw, void *stream);
void kf_num_batch_free(KfNumBatch *b);

/* Workspace for up to max_seqs sequences of up to max_frames frames each. */
KfChain *kf_chain_create(const KfDenGraph *den, int max_seqs, int max_frames);
void kf_chain_free(KfChain *c);

/* One objective + derivative for the minibatch, asynchronous on kf_get_stream().
 * nnet_output / out_grad: fp16 device matrices of num_rows rows, leading dims ld / ldg
 * (>= P). seq_row0 / seq_frames: host arrays [nseq]; every supervised row must lie
 * inside the matrix. */
int kf_chain_compute(KfChain *c, const KfNumBatch *num, const KfChainOpts *opts,
                     const void *nnet_output, long long ld, long long num_rows, int nseq,
                     const int32_t *seq_row0, const int32_t *seq_frames, int stride,
                     void *out_grad, long long ldg);
/* Device array of per-sequence statistics of the last compute:
 * float[8] per sequence {num_lp, den_lp, objf, l2_term, weight*frames, frames, oor, ok}. */
const float *kf_chain_seq_stats(const KfChain *c);
/* Synchronises the stream and sums the per-sequence statistics of the last compute.
 * Fails (-1) when a den exchange timed out in any compute since the previous call. */
int kf_chain_result(KfChain *c, KfChainResult *out);

/* diagnostics: phase timestamps of the den forward kernel (sequence 0, block 0,
 * frames 16..47, 8 u64 each, 100 MHz wall clock), then the arc-phase end of every wave
 * of blocks 0 and 1 (32 x 2 x 16 u64) into a device buffer; NULL = off */
void kf_chain_trace(KfChain *c, unsigned long long *dev_buf);
/* diagnostics (tests): polls a den exchange wait makes before it declares the
 * partner blocks non-resident (default 2^21; 0 forces the timeout path;
 * 0xFFFFFFFF restores the default). A timeout in ANY compute since the last
 * kf_chain_result makes that call fail (the count is sticky across launches). */
void kf_chain_debug_spin_limit(KfChain *c, unsigned polls);
/* Diagnostics (tests): force != 0 makes the den exchange use agent scope (through to
 * memory) even where all blocks of a sequence share an XCD; 0 restores the default. */
void kf_chain_debug_exchange_sys(KfChain *c, int force);
/* Diagnostics (tests): pairs == 0 runs the den recursions one sequence per workgroup set
 * even where two sequences could share each record (the default, pairs == 1). */
void kf_chain_debug_den_pairs(KfChain *c, int pairs);
/* Diagnostics (tests): the XCD census of the last compute's den launch. *units = exchange
 * units per direction, *G = workgroups per unit; *local_fwd / *local_bwd = units whose G
 * workgroups all ran on one XCD (those take the L2-local exchange unless *forced = 1,
 * kf_chain_debug_exchange_sys). Any out pointer may be NULL. */
int kf_chain_debug_census(KfChain *c, int *units, int *local_fwd, int *local_bwd, int *forced, int *G);

const char *kf_chain_last_error(void);
void kf_chain_clear_error(void);

#ifdef __cplusplus
}
#endif
#endif
