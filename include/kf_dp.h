/*
 * kf_dp.h — data-parallel gradient exchange of the training step over RCCL
 * (BASELINE configs[3]: 8 x MI355X, one process per GPU, xGMI).
 *
 * The reference is single-device (cpp/cuda/bridge.cu:38-47: bridge_gpu_init
 * selects one device; no NCCL anywhere), so this header has no reference
 * counterpart: it is the entry point a Go (or C/C++) host binds to run the
 * reference's TrainStep (internal/nnet/train_step.go:142-283) data-parallel.
 *
 * Protocol (one process per GPU):
 *   rank 0: kf_dp_unique_id(id)              -> distribute the 128 bytes out of band
 *   every rank: dp = kf_dp_create(rank, world, id, device)   (collective)
 *               nnet_bind_dp(net, dp, bucket_bytes)          (kf_nnet.h)
 *   per step:   nnet_forward / kf_chain_compute / nnet_backward / nnet_sgd
 * With a network bound, nnet_backward issues one ncclAllReduce(avg) per gradient
 * bucket on the communicator's own stream as soon as the weight-gradient GEMMs
 * of the layers in that bucket have been enqueued (an event recorded on the
 * compute stream gates it), in reverse layer order, so the exchange overlaps the
 * rest of the backward; the compute stream waits for the last bucket before
 * nnet_backward returns, so nnet_sgd sees the averaged gradient.
 *
 * All calls are stream-ordered on kf_get_stream() (kf_ops.h) and return
 * 0 / -1 (NULL for the constructor) with the text in kf_dp_last_error().
 */
#ifndef KALDI_FP16_AMD_KF_DP_H
#define KALDI_FP16_AMD_KF_DP_H
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KF_DP_ID_BYTES 128

typedef struct KfDp KfDp;

/* ncclGetUniqueId: called on rank 0 only */
int kf_dp_unique_id(unsigned char id[KF_DP_ID_BYTES]);
/* ncclCommInitRank on `device` (collective over all ranks) plus a high-priority
 * communication stream */
KfDp *kf_dp_create(int rank, int world, const unsigned char id[KF_DP_ID_BYTES], int device);
void kf_dp_free(KfDp *dp);
int kf_dp_rank(const KfDp *dp);
int kf_dp_world(const KfDp *dp);

/* in-place average over ranks of `count` fp32 values, on the communication stream,
 * gated by the work already enqueued on kf_get_stream(); does NOT join: call
 * kf_dp_join before the compute stream reads `buf` */
int kf_dp_allreduce_mean_async(KfDp *dp, float *buf, size_t count);
/* kf_get_stream() waits for every exchange issued so far */
int kf_dp_join(KfDp *dp);
/* the two above back to back */
int kf_dp_allreduce_mean(KfDp *dp, float *buf, size_t count);
/* in-place sum over ranks of `count` fp64 values (objective statistics), joined */
int kf_dp_allreduce_sum_f64(KfDp *dp, double *buf, size_t count);
/* number of all-reduce launches and fp32 values exchanged since kf_dp_create */
int kf_dp_stats(const KfDp *dp, long long *launches, long long *values);

/* Test hooks (one GPU can then check what N ranks depend on). While a mode is on, every
 * bucket issued by kf_dp_allreduce_mean_async must lie inside [grad_base, grad_base + count)
 * and also does, on the communication stream:
 *   KF_DP_DEBUG_SNAPSHOT:  before the all-reduce, copies the bucket to the same offset
 *                          of aux_base: the values the exchange started from, so a test
 *                          can compare them with the finished gradient (a bucket issued
 *                          before its producers finished differs);
 *   KF_DP_DEBUG_PEER_MEAN: after the all-reduce, buf = (buf + aux) * 0.5 at the same
 *                          offset: a two-rank average whose other rank's gradient is
 *                          aux_base (a test supplies a second shard's gradient), so the
 *                          gates, the bucket coverage and kf_dp_join all change results.
 * count: fp32 values of grad_base (and of aux_base). While a mode is on, an exchange of a
 * bucket outside [grad_base, grad_base + count) fails instead of touching aux out of range.
 * mode 0 turns them off. The two modes are exclusive. -1: bad arguments. */
#define KF_DP_DEBUG_SNAPSHOT 1
#define KF_DP_DEBUG_PEER_MEAN 2
int kf_dp_debug(KfDp *dp, int mode, const float *grad_base, float *aux_base, size_t count);

/* Bucket plan of a flat gradient buffer (host only, no device work).
 * steps: the backward visits nsteps parameter groups in order; group i occupies
 * [lo[i], hi[i]) of the flat buffer (lo = hi: no parameters). total: buffer length.
 * A bucket is cut after group i when the not-yet-exchanged tail [lo[i], top) holds
 * at least bucket_elems values; whatever is left, [0, top), goes after the last group.
 * Writes after_step[j], begin[j], end[j] for each bucket j (after_step = nsteps for
 * the final one) and returns the number of buckets. Groups that are not in
 * descending buffer order (a group reaching above the exchanged boundary) make the
 * plan one bucket [0, total) after the backward. At most max_buckets buckets are
 * written: when the limit is reached, everything not yet exchanged goes into the final
 * bucket (after the last group). -1: bad arguments (a group outside [0, total],
 * max_buckets < 1). */
int kf_dp_plan(int nsteps, const long long *lo, const long long *hi, long long total,
               long long bucket_elems, int max_buckets, int *after_step, long long *begin,
               long long *end);

const char *kf_dp_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
