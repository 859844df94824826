/*
 * kf_oracle.h — CPU restatement of the reference's CNN-TDNN hot path.
 *
 * TEST INFRASTRUCTURE ONLY. Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the checker
 * (or the timed CPU baseline) — never as the product path.
 *
 * Plain C, float32 arithmetic (fp32 accumulation, as cublasGemmEx with
 * CUBLAS_COMPUTE_32F in cpp/cuda/ops.cu:381-392), with fp16 rounding applied at
 * tensor boundaries. Two rounding modes:
 *   ORC_ROUND_FUSED (F): round to fp16 once per stored tensor, where the MI355X
 *                        build stores fp16 tensors;
 *   ORC_ROUND_REF   (R): round after every reference op, as the reference's
 *                        chain of cuBLAS + element-wise kernels does
 *                        (internal/nnet/forward.go:589-695, ops.cu:26-228).
 * Parity pinning: see oracle/README in DESIGN.md §Oracle.
 */
#ifndef KF_ORACLE_H
#define KF_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* fp16 conversions */
uint16_t orc_f32_to_f16_rne(float f);     /* internal/fp16/fp16.go:12-70 */
uint16_t orc_f32_to_f16_trunc(float f);   /* internal/gpu/tensor.go:158-173 */
float orc_f16_to_f32(uint16_t h);         /* internal/fp16/fp16.go:73-110 */
void orc_round_f16(float *x, long long n); /* x = f32(rne(x)) in place */
void orc_set_threads(int n);
int orc_get_threads(void);

/* C[MxN] = A[MxK] . B[KxN] (fp32), rows split over threads (go/gotorch/ops.go:49-81) */
void orc_matmul(int M, int N, int K, const float *A, const float *B, float *C);

enum {
    ORC_IDCT = 1,
    ORC_BATCHNORM = 2,
    ORC_CONV = 3,
    ORC_TDNNF = 4,
    ORC_LINEAR = 5,
    ORC_PREFINAL = 6,
    ORC_OUTPUT = 7,
    ORC_ATTENTION = 8,
    ORC_COMBINE = 9,  /* combine-feature-maps of Append(input, input2) */
};
enum { ORC_ROUND_NONE = 0, ORC_ROUND_FUSED = 1, ORC_ROUND_REF = 2 };

typedef struct {
    const float *mean, *var, *gamma, *beta; /* [dim] */
    float eps, target_rms;
} OrcBN;

typedef struct {
    int type;
    int input;        /* index of input layer, -1 = features */
    int in_dim, out_dim;
    /* conv (forward.go:418-524 with Kaldi cross-product offsets) */
    int hin, hout, sub, fin, fout, noff;
    int toff[9], hoff[9];
    /* tdnnf (forward.go:589-695) */
    int bn_dim, stride;
    float bypass;
    /* prefinal (forward.go:912-968): big then small */
    int small_dim, big_dim;
    /* parameters (host fp32, values already fp16-representable) */
    const float *W;   /* conv [noff*fin x fout]; tdnnf LinearW; linear/output W; prefinal BigW; idct M */
    const float *b;   /* conv / output bias; prefinal BigBias */
    const float *W2;  /* tdnnf AffineW; prefinal SmallW */
    const float *b2;  /* tdnnf AffineBias */
    OrcBN bn;         /* conv / tdnnf / batchnorm-component / prefinal BN1 */
    OrcBN bn2;        /* prefinal BN2 (small dim); mean==NULL -> none */
    int log_softmax;  /* output-layer include-log-softmax=true (forward.go:991-997) */
    /* attention-relu-batchnorm (forward.go:795-909): W [din x heads*(2kd+vd+ctx)], b */
    int heads, kd, vd, ctx, nleft, astride;
    float key_scale;
    /* ivector path: input -2 = the ivector input; per_seq layers run on the B sequence
     * rows (ReplaceIndex(ivector, t, 0)); combine: second input, height, filters */
    int input2, per_seq, height, nf1, nf2;
} OrcLayer;

typedef struct {
    int nlayers;
    const OrcLayer *layers;
    int T;            /* frames */
    int feat_dim;
    int round_mode;
    /* outputs, allocated by the oracle (orc_net_free) */
    float **act;      /* [nlayers] forward outputs [T x out_dim] */
    uint8_t **mask;   /* [nlayers] relu masks (1 byte per element) */
    float **aux;      /* [nlayers] tdnnf bottleneck / prefinal big */
    float **gW, **gb, **gW2, **gb2; /* [nlayers] parameter gradients (fp32) */
    float **gact;     /* [nlayers] gradient w.r.t. each layer's output */
    /* optional: per-layer ReLU decisions to replay instead of recomputing
     * (1 byte per element, NULL = compute). Parity tests use it to compare
     * gradients without the sqrt(flip-fraction) noise of near-zero
     * pre-activations that two fp16 paths legitimately decide differently. */
    const uint8_t **force_mask;
    /* MXFP8 emulation of the GPU's nnet_set_fp8 forward (kf_nnet.h): the dense GEMMs
     * of TDNN-F / linear / prefinal / output layers read quantise-dequantised
     * (OCP MX, blocks of 32 along K) inputs and weights; act8 holds the
     * quantised copies of producer outputs (taken before the fp16 rounding). 1 also
     * emulates the MXFP8 affine input gradients of the strided TDNN-F layers in the
     * backward (mx_dgrad_layer), 2 does not (nnet_set_fp8(net, 2)). */
    int mx8;
    float **act8;
    /* ivector input: [B x ivec_dim] rows, frames of sequence s = [seq_off[s], seq_off[s+1]) */
    const float *ivec;
    int B, ivec_dim;
    const int *seq_off;
    /* MXFP8 copy of the features (dequantised, [T x feat_dim]) for a layer reading the
     * input directly: lets a test run one layer on the GPU's own fp8 input (mx8 only) */
    const float *feat8;
    /* F mode: emulate the GPU's implicit dz (kf_nnet.h nnet_set_implicit_dz, network.cpp
     * dx_epilogue): for a TDNN-F layer with a bypass whose gradient comes from the layer
     * above, dz is the stored g = rne(v) under the ReLU mask, the affine weight / bias
     * gradients are scaled by the BN scale after the reduction and the affine input
     * gradient uses rne(W2 * bnscale). Not with mx8 (the GPU's fp8 steps store dz). */
    int implicit_dz;
} OrcNet;

/* OCP MXFP8 quantise-dequantise of rows of `cols` (cols % 32 == 0) values:
 * the rule of kf_quant_mxfp8 (include/kf_ops.h) */
void orc_mx_qdq_rows(const float *x, float *y, long long rows, int cols);

int orc_net_forward(OrcNet *net, const float *features);
/* out_grad [T x out_dim(last)], already fp16-representable */
int orc_net_backward(OrcNet *net, const float *features, const float *out_grad);
/* the same seeded at layer `top` (Model.ChainOutput, network_backward.go:102-115):
 * layers off its input path get no gradient */
int orc_net_backward_top(OrcNet *net, const float *features, const float *out_grad, int top);
void orc_net_free(OrcNet *net);

/* v = mom*v + g; w32 -= lr*v (backward_wrappers.cu:129-142) */
void orc_sgd(float *w32, const float *g, float *v, float lr, float mom, long long n);

/* ------------------------------------------------------------------------- */
/* Chain LF-MMI objective (kf_oracle_chain.c)                                */
/* ------------------------------------------------------------------------- */
/* Denominator graph, prob space (cpp/cuda/chain_den.cu, internal/nnet/denominator.go). */
typedef struct {
    int S, P, A;
    const int *src, *dst, *pdf0;   /* pdf0: 0-indexed (label - 1, denominator.go:83) */
    const float *tp;               /* exp(-tropical weight) (denominator.go:87) */
    const float *init;             /* [S] initial probs (orc_den_initial_probs) */
} OrcDen;

/* Numerator FST in CSR, log domain (internal/sparse/sparse.go:54-91, chain.h:23-35). */
typedef struct {
    int S, A, nfinal, start;
    const int *row_ptr, *dst, *pdf1;  /* pdf1: 1-indexed, 0 = epsilon (skipped) */
    const float *logw;                /* negated tropical weights */
    const int *final_state;
    const float *final_w;
} OrcNum;

/* Mirrors ChainTrainingOpts (internal/nnet/backward.go:114-140). */
typedef struct {
    float l2_regularize, out_of_range_regularize, leaky_hmm_coefficient, xent_regularize,
        supervision_weight;
} OrcChainOpts;

typedef struct {
    double objf, l2_term, total_weight, num_logprob, den_logprob;
    int frames, out_of_range, ok;
} OrcChainResult;

/* 100 float64 iterations from the start state, averaged (denominator.go:131-171). */
void orc_den_initial_probs(int S, int A, const int *src, const int *dst, const float *tp,
                           int start, float *init_out);
/* den_forward / den_forward_backward (chain_den.cu:371-472, :496-706). nnet [T x P];
 * post [T x P] (NULL = forward only). Returns the log-prob. */
float orc_den_forward_backward(const OrcDen *den, const float *nnet, int T, float leaky,
                               float *post);
/* Deterministic log-domain numerator (chain_det.cu:55-237): nnet values are used as
 * given (the caller rounds to fp16, as chain_backward.cu:372-379 does). post [T x P]
 * is overwritten (NULL = skip). Returns the total log-prob. */
float orc_num_forward_backward(const OrcNum *num, const float *nnet, int T, int P, float *post);
/* ComputeChainObjfAndDeriv for one sequence (backward.go:224-371): deriv [T x P]. */
int orc_chain_objf(const OrcChainOpts *opts, const OrcDen *den, const OrcNum *num,
                   const float *nnet, int T, float *deriv, OrcChainResult *res);

#ifdef __cplusplus
}
#endif
#endif
