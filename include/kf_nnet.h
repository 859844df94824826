/*
 * kf_nnet.h — C-ABI of this build's host layer: the C++ restatement of the
 * reference's Go packages internal/nnet (xconfig.go, layers.go, model.go,
 * forward.go, network_backward.go, train_step.go) and internal/gpu
 * (optimize.go), running on the MI355X kernels of kf_ops.h.
 *
 * The reference's host code is Go; no Go toolchain exists in this image, so the
 * host layer is C++. The entry points below are the
 * Network / Trainer API of internal/nnet flattened into C:
 *   nnet_create        <- BuildModelFromString (model.go:31) + NewNetwork (forward.go:111)
 *   nnet_forward       <- Network.Forward (forward.go:148)
 *   nnet_backward      <- Network.Backward (network_backward.go:94)
 *   nnet_sgd           <- SGDOptimizer.Update for every parameter (optimize.go:95)
 *   nnet_train_step    <- TrainStep (train_step.go:142) with the chain objective
 * Errors: NULL / -1 with the text in nnet_last_error() (thread-local).
 */
#ifndef KALDI_FP16_AMD_KF_NNET_H
#define KALDI_FP16_AMD_KF_NNET_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct KfNet KfNet;

/* layer type codes reported by nnet_layer_info (xconfig.go:18-30 order) */
enum {
    NNET_INPUT = 0, NNET_IDCT, NNET_LINEAR, NNET_BATCHNORM, NNET_SPECAUGMENT,
    NNET_COMBINE_FEATURE_MAPS, NNET_CONV_RELU_BN, NNET_TDNNF, NNET_ATTENTION,
    NNET_PREFINAL, NNET_OUTPUT
};

const char *nnet_last_error(void);

/* parse + resolve an xconfig and allocate weights/activations for max_frames */
KfNet *nnet_create(const char *xconfig_text, int max_frames);
/* the same network without device storage (no GPU needed): layers, the flat
 * parameter layout and the data-parallel bucket plan can be queried; forward,
 * backward, sgd and the parameter setters fail on it. The MI355X kernels' shape
 * constraints (dims multiples of 8 / 32) are not enforced here. */
KfNet *nnet_create_layout(const char *xconfig_text, int max_frames);
/* parse + resolve only, no device work: "name type in out" per layer, then
 * "params N"; returns the bytes needed (incl. NUL) or -1 */
int nnet_parse_summary(const char *xconfig_text, char *out, int outlen);
void nnet_free(KfNet *net);

int nnet_num_layers(const KfNet *net);  /* excluding input layers */
int nnet_layer_info(const KfNet *net, int idx, char *name, int namelen, int *type, int *in_dim,
                    int *out_dim);
/* trainable parameters: flat fp32 master / fp16 working / fp32 grad / fp32 velocity */
long long nnet_num_params(const KfNet *net);
int nnet_num_param_tensors(const KfNet *net);
int nnet_param_info(const KfNet *net, int idx, char *name, int namelen, int *rows, int *cols,
                    long long *offset);
/* host fp32 values in the flat layout; stored fp16 by truncation
 * (internal/gpu/tensor.go:158-173) and the master copy = that fp16 value
 * (optimize.go:52-70 via ops_fp16_to_fp32) */
int nnet_set_params(KfNet *net, const float *host_flat);
int nnet_get_params(const KfNet *net, float *host_flat); /* fp32 master */
/* which = 0: the layer's (first) BatchNorm, 1: prefinal's second BatchNorm;
 * target_rms <= 0: the layer's configured target-rms (a batchnorm-component's, else 1) */
int nnet_set_bn(KfNet *net, const char *layer, int which, const float *mean, const float *var,
                const float *gamma, const float *beta, float eps, float target_rms);

/* replace an idct-layer's matrix: host fp32 [dim x dim], y = x . m (weight_loader.go:88-97) */
int nnet_set_idct(KfNet *net, const char *layer, const float *m, int rows, int cols);
/* attention layer key scale (> 0); default 1/sqrt(key-dim) or the xconfig key-scale */
int nnet_set_key_scale(KfNet *net, const char *layer, float key_scale);

/* forward with the ivector input (an input layer named "ivector", read through
 * ReplaceIndex(ivector, t, 0)): ivectors fp16 [B x ivector-dim] on the device, one row per
 * sequence; seq_row0 host int[B+1] with the frame offsets (0 ... T). */
int nnet_forward_ivector(KfNet *net, const void *features_dev, int T, const void *ivectors_dev, int B,
                         const int *seq_row0);
/* forward on T frames of fp16 features already in device memory */
int nnet_forward(KfNet *net, const void *features_dev, int T);
/* device pointer of a layer's output activation (fp16 [rows x cols]) */
const void *nnet_activation(const KfNet *net, const char *layer, int *rows, int *cols);
/* backward from the fp16 gradient of the chain output [T x num_pdfs] */
int nnet_backward(KfNet *net, const void *out_grad_dev);
float *nnet_grad_buffer(KfNet *net);   /* device fp32 [num_params] */
/* use caller-owned device memory (>= num_params fp32) as the gradient buffer */
int nnet_bind_grad_buffer(KfNet *net, float *dev);
float *nnet_master_buffer(KfNet *net); /* device fp32 [num_params] */
/* device fp16 [num_params]. A host that writes weights through this pointer (a
 * checkpoint restore, a weight broadcast) calls nnet_weights_changed afterwards, at
 * every such write: the forward of the TDNN-F affine and prefinal big layers reads
 * transposed copies and the fp8 mode MXFP8 copies, both derived from these weights. */
void *nnet_weight_buffer(KfNet *net);
/* the fp16 weights were written from outside: refresh the derived copies (transposed
 * copies at the next forward, MXFP8 copies now) */
int nnet_weights_changed(KfNet *net);
int nnet_sgd(KfNet *net, float lr, float momentum);
/* MXFP8 train step (BASELINE configs[4]): 1 = every TDNN-F / linear / prefinal / output
 * GEMM whose input has an MXFP8 copy runs on the fp8 MFMA (kf_ops.h MXFP8 operands);
 * the producing epilogues write those copies, weights are re-quantised on every
 * parameter change; in the backward the strided TDNN-F affine input gradients run on
 * e4m3 copies of dz (written by the layer above's input-gradient epilogue) and of W2,
 * everything else stays fp16. 2 = the same forward with an all-fp16 backward (a test
 * knob). 0 = off. */
int nnet_set_fp8(KfNet *net, int on);

/* Data parallel (kf_dp.h). nnet_bind_dp: nnet_backward exchanges the
 * gradient in buckets of >= bucket_bytes, each all-reduced (average over ranks) on
 * the communicator's stream as soon as the backward has enqueued the weight-gradient
 * kernels of every parameter in it, in reverse layer order; it returns with the
 * compute stream waiting for the last bucket. dp = NULL unbinds.
 * nnet_dp_plan: that bucket plan (kf_dp_plan's outputs; works on a layout-only net). */
typedef struct KfDp KfDp;
int nnet_bind_dp(KfNet *net, KfDp *dp, long long bucket_bytes);
int nnet_dp_plan(const KfNet *net, long long bucket_bytes, int max_buckets, int *after_step,
                 long long *begin, long long *end);
/* nnet_bind_dp plans at most 256 buckets (the rest merges into the final one).
 * Test hook: on != 0 issues every bucket at the start of nnet_backward, before any
 * gradient exists: the negative control of the overlap tests (kf_dp_debug). */
int nnet_dp_debug_early(KfNet *net, int on);

/* Weight gradients on a second stream (default on): nnet_backward launches every dW / db
 * GEMM (and the data-parallel bucket gates) on a stream of its own, ordered by events after
 * the producers on the caller's stream, so they overlap the input-gradient chain; the
 * caller's stream waits for them before nnet_backward returns. 0 = everything on the
 * caller's stream (the r4 order, A/B and tests). */
int nnet_set_wgrad_stream(KfNet *net, int on);

/* Row-subsampled train step (r6; default off). stride = 3 declares that the caller reads the
 * output, and writes output gradients, on rows 0 (mod 3) only (the chain objective with
 * frame-subsampling-factor 3 and every eg's first supervised row at 0 mod 3, as
 * chain_layout / TrainStep lay them out). The layers at the top of the output chain whose
 * row t depends only on rows t and t +- 3 of the layer below (TDNN-F with time stride 0 or
 * 3, linear, prefinal, output, above a conv-relu-batchnorm layer) then run on the rows
 * those outputs depend on — Kaldi nnet3's computation of only the indexes an output needs:
 * the rows 0 (mod 3) and, through the splices' clamp at T - 1, a tail of rows
 * T-1, T-4, ... — so each of those layers' forward and backward does a third of the work.
 * Output rows of the set, the objective, every weight gradient and the gradient into the
 * conv stack are those of the full computation (weight gradients up to the split-K
 * summation order). After nnet_forward, nnet_row_set gives the compact rows tc (0 = this
 * forward ran on full rows: fp8, implicit dz or a short T) and tc0: compact row c holds
 * source row 3c for c < tc0, else (T-1) - 3(tc-1-c); those layers' activations
 * (nnet_activation: rows = tc) and the output gradient nnet_backward reads are in compact
 * rows. stride 0 / 1: off. */
int nnet_set_row_subsampling(KfNet *net, int stride);
int nnet_row_set(const KfNet *net, int *tc, int *tc0);

/* Implicit dz (default off; fp16 steps): the input-gradient GEMM that produces a TDNN-F
 * layer's output gradient g (layers with a bypass, which store g anyway) does not also
 * store dz = rne(g * bnscale * relu_mask). The layer's affine weight gradient and input
 * gradient read g through the forward's ReLU mask (masked operands, kf_ops.h); the BN scale
 * multiplies the weight gradient's columns in its split-K reduction and is folded into a
 * scaled fp16 copy of W2 for the input gradient. Rounding points change accordingly (the
 * oracle's OrcNet.implicit_dz follows them). Measured step-neutral, hence
 * off: 0 = store dz (the default). */
int nnet_set_implicit_dz(KfNet *net, int on);

/* diagnostics (tests) of the two-stream backward: main_aff chooses where the TDNN-F
 * affine weight gradients run (-1 = KF_BWD_MAIN_AFF / the default 0: all on the
 * weight-gradient stream; 1 = every other one on the input-gradient chain; 2 = all on the
 * chain);
 * stall_cycles > 0 queues a spin kernel of that many GPU clock cycles (kf_debug_spin) on
 * the weight-gradient stream before each of its batches of work, so that stream runs far
 * behind the chain and any missing order shows as a wrong gradient. */
int nnet_debug_backward(KfNet *net, int main_aff, long long stall_cycles);

/* diagnostics (tests): back-propagate through the top n layers only; device
 * pointer of an internal tensor ("dz0" .. "dz2", "g0" .. "g2": the backward's gradient ring,
 * "dzlast": the ring buffer the last step wrote, "dbott" (the buffer of the last
 * TDNN-F / prefinal step), "aux", "mask",
 * "bn_scale", "bn2_scale", "dproj" (attention: the gradient of its affine output), and with fp8 on "x8q" / "x8s": the e4m3 values
 * [T x pad128(in_dim)] and E8M0 scales [T x pad128(in_dim)/32] of the MXFP8 input copy
 * the layer's GEMM reads; "w8dq" / "w8ds": a strided TDNN-F layer's e4m3 affine weight rows
 * for its MXFP8 input gradient [bottleneck x 2*pad128(out_dim)]; "dz8q" / "dz8s" with
 * layer = 0 .. 2: the e4m3 copy of dz0 .. dz2, and "dz8layer": 1 + the layer that copy is
 * for, as the returned pointer value (NULL: none); `layer` selects the per-layer ones),
 * NULL if unknown */
int nnet_backward_n(KfNet *net, const void *out_grad_dev, int n);
const void *nnet_debug_tensor(KfNet *net, const char *what, int layer);

#ifdef __cplusplus
}
#endif
#endif
