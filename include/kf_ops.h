/*
 * kf_ops.h — MI355X extension of the kaldi-fp16 C-ABI: fused, implicitly
 * addressed FP16 MFMA GEMMs and the few multi-tensor kernels the CNN-TDNN
 * training step needs. Nothing here replaces a reference symbol; these entry
 * points are what this build's host layer (the C++ mirror of internal/nnet and
 * internal/gpu, see kf_nnet.h) calls so that the splice / im2col / epilogue
 * work the reference does as separate kernels and host round trips
 * (internal/nnet/forward.go:418-790, internal/gpu/backward_ops.go:162-253)
 * happens inside one GEMM launch. Plain C types only; no torch, no HIP types.
 *
 * Operand addressing (KfOperand). An operand is a logical row-major matrix
 * Op[r][c] (r < nrows, c < ncols) whose 8-element column chunks are fetched
 * from memory by this rule (all counts in elements):
 *   part p = c / part_width, kk = c % part_width      (nparts parts)
 *   t = r / hout, h = r % hout                         (hout = 1 for TDNN rows)
 *   if edge_t[p] >= 0 and t == edge_t[p]: st = edge_row[p] (a spare row of the
 *      same buffer, e.g. row T, holding a precomputed sum; no range checks)
 *   else st = t + dt[p]; outside [0, T): clamp (tpolicy=KF_CLAMP) or zero (KF_ZERO)
 *   shn = h*hmul + dh[p]; zero unless shn % hdiv == 0; sh = shn / hdiv,
 *   zero unless 0 <= sh < hsrc
 *   value = base[st*ld + sh*part_width + kk]
 * With nparts=1, hout=1, dt=0 this is a plain [nrows x ncols] matrix with
 * leading dimension ld. The same rule expresses the TDNN time splice
 * (forward.go:699-790: dt = {-s, 0} clamp, or {0, +s} clamp), the conv im2col
 * (forward.go:435-456: dt x dh cross product, hmul = subsample, zero pad),
 * and their transposes used by the input-gradient GEMMs.
 *
 * Orientation: an operand is "k-contiguous" when its columns run along the
 * GEMM reduction index (row-major A[M][K], or B stored [N][K]); otherwise its
 * rows run along the reduction (A stored [K][M], B stored [K][N]).
 *
 * MXFP8 operands (fmt = KF_FMT_MXFP8, the OCP microscaling format): elements are
 * OCP e4m3 bytes and every 32 consecutive elements of a source row share one
 * E8M0 scale byte (value 2^(byte-127)) at scales[st*lds + c/32], st and c the
 * source row and column of the rule above. Only k-contiguous operands with
 * hout = 1 are accepted, ncols and part_width multiples of 128, ld multiple of
 * 16; both operands of a GEMM must then be MXFP8 (kf_gemm_fused runs the CDNA4
 * v_mfma_scale_f32_16x16x128_f8f6f4, twice the fp16 MFMA rate).
 *
 * Masked operands (mask != NULL, fp16 only): with i = st*ld + sh*part_width + kk the
 * linear source index of the rule above, the element reads as zero unless bit i of mask
 * (bit i % 8 of byte i / 8) is set; rows st >= mask_rows (e.g. an edge row) are not
 * masked. This is how the TDNN-F backward reads dz = g * bnscale * relu_mask without
 * storing it: g with the forward's ReLU mask, the BN scale folded into the other operand
 * (kf_scale_cols on W2) or into the weight gradient (kf_gemm_wgrad_scaled). Accepted on the A
 * operand of kf_gemm_fused (k-contiguous plain or two-part time splice, N = 160 / 320,
 * k-contiguous B) and the B operand of kf_gemm_wgrad(_scaled) (plain, reduction-major).
 */
#ifndef KALDI_FP16_AMD_KF_OPS_H
#define KALDI_FP16_AMD_KF_OPS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KF_MAX_PARTS 9
#define KF_ZERO 0
#define KF_CLAMP 1

typedef struct {
    const void *base;  /* fp16 */
    long long ld;      /* elements between consecutive source rows */
    int nrows, ncols;  /* logical shape of Op */
    int kcontig;       /* 1: columns are the reduction index */
    int nparts, part_width;
    int T, hout, hsrc, hmul, hdiv, tpolicy;
    int dt[KF_MAX_PARTS];
    int dh[KF_MAX_PARTS];
    int edge_t[KF_MAX_PARTS];
    int edge_row[KF_MAX_PARTS];
    int fmt;                   /* KF_FMT_FP16 (0) or KF_FMT_MXFP8 (1) */
    const uint8_t *scales;     /* MXFP8: E8M0 block scales */
    long long lds;             /* MXFP8: bytes between the scale rows of consecutive source rows */
    const uint8_t *mask;       /* masked operand (above), or NULL */
    int mask_rows;             /* source rows the mask covers */
    /* time-strided rows (a conv evaluated on a subset of its output frames, the row-
     * subsampled step's last conv): st = t0 + t*tmul + dt[p] in the rule above. 0 / 0 =
     * the plain rule. Only the A operand of a kf_gemm_fused convolution that runs on the
     * halo kernel takes it; other uses fail. */
    int tmul, t0;
} KfOperand;

#define KF_FMT_FP16 0
#define KF_FMT_MXFP8 1

/*
 * Fused epilogue, applied per output element (m, n) to the fp32 accumulator:
 *   v = alpha*acc (+ beta*out[m][n]) (+ bias[n])
 *   if relu: mask_out bit (m*ldo+n) = v > 0; v = max(v, 0)
 *   if scale: v = v*scale[n] + shift[n]          (frozen BatchNorm, folded)
 *   if resid: v += resid_alpha * resid[m][n]     (TDNN-F bypass / grad bypass)
 *   out[m][n] = rne_fp16(v)                       (when out != NULL)
 *   if out2: out2[m][n] = rne_fp16(v * scale2[n] * bit(mask_in, m*ldo2+n))
 *   if out8: MXFP8 copy (kf_quant_mxfp8's rule, 32-column blocks) of the unrounded v, or
 *            with out8_src = 1 of the unrounded out2 value
 *   if edge_out: edge_out[n] = rne_fp16(sum over rows m in [edge_r0, edge_r1) of the stored
 *            out[m][n] (edge_src = 0) or out2[m][n] (edge_src = 1)), in row order: kf_rows_sum
 *            of the result, written by the workgroups of the row tile holding those rows (a
 *            separate sum kernel after the GEMM when the rows span two tiles)
 * Masks are bit-packed in the linear element order of the tensor they describe
 * (bit i of byte i/8), so producer and consumer may tile differently.
 */
typedef struct {
    void *out;
    long long ldo;
    float alpha, beta;
    const void *bias;      /* fp16 [N] or NULL */
    int relu;
    uint8_t *mask_out;     /* or NULL */
    const float *scale;    /* fp32 [N] or NULL */
    const float *shift;    /* fp32 [N] (required with scale) */
    const void *resid;     /* fp16, or NULL */
    long long ldr;
    float resid_alpha;
    void *out2;            /* fp16, or NULL */
    long long ldo2;
    const float *scale2;   /* fp32 [N] or NULL (= 1) */
    const uint8_t *mask_in;/* or NULL (= all ones) */
    void *out8;            /* e4m3 [M x ldo8], or NULL */
    long long ldo8;
    uint8_t *scale8;       /* E8M0 [M x ldo8/32] (required with out8) */
    int out8_src;          /* 0: out8 quantises v (out's value); 1: out2's value (needs out2) */
    void *edge_out;        /* fp16 [N], or NULL: column sums of rows [edge_r0, edge_r1) (above) */
    int edge_r0, edge_r1, edge_src;
    /* grouped output rows: with row_group > 0, GEMM row m addresses row
     * (m / row_group) * row_stride + m % row_group of every row operand above (out, out2,
     * resid, mask_out, mask_in, out8): a transposed conv evaluated on every third frame
     * writes its frames in place. 0 = rows as they are. Not with edge_out. */
    int row_group, row_stride;
} KfEpilogue;

/* current stream for every launch made by this library on the calling thread
 * (NULL = legacy default stream, the reference's behaviour) */
void kf_set_stream(void *hip_stream);
void *kf_get_stream(void);
/* streams and events for host layers built without HIP headers (libkaldi_fp16_nnet's
 * weight-gradient stream): a non-blocking stream (NULL on failure), a timing-disabled
 * event; record / wait return 0 or -1 */
void *kf_stream_new(void);
void *kf_stream_new_high(void);  /* the device's highest stream priority */
void kf_stream_free(void *hip_stream);
void *kf_event_new(void);
void kf_event_free(void *hip_event);
int kf_event_record(void *hip_event, void *hip_stream);
int kf_stream_wait(void *hip_stream, void *hip_event);

/* C[M x N] = epilogue(A . B^T-style contraction over K) */
int kf_gemm_fused(int M, int N, int K, const KfOperand *A, const KfOperand *B,
                  const KfEpilogue *epi);

/*
 * Weight-gradient GEMM with the reduction split over workgroups:
 *   dW[M x N] (fp32, leading dim ldw) (+)= sum_r A(r, m) * B(r, n)
 * bias_grad[N] (fp32, optional) (+)= sum_r B(r, n).
 * accumulate=0 overwrites, 1 adds. Deterministic (slab reduction, no atomics).
 */
int kf_gemm_wgrad(int M, int N, int K, const KfOperand *A, const KfOperand *B, float *dW,
                  long long ldw, float *bias_grad, int accumulate);
/* kf_gemm_wgrad, then dW[:, n] and bias_grad[n] scaled by col_scale[n] (fp32 [N]) in the
 * split-K reduction: the TDNN-F affine weight gradient on the implicit dz (a masked B
 * operand g with the BN scale applied here) */
int kf_gemm_wgrad_scaled(int M, int N, int K, const KfOperand *A, const KfOperand *B, float *dW,
                         long long ldw, float *bias_grad, int accumulate, const float *col_scale);
/* split-K workgroup target of kf_gemm_wgrad on the calling thread (default 512); returns
 * the previous value (wgs <= 0: query only) */
int kf_gemm_wgrad_target(int wgs);

/*
 * MXFP8 quantisation (OCP MX): per block of 32 consecutive values of a row,
 * amax = max |v|, scale = 2^(floor(log2 amax) - 8) (E8M0 byte = exponent + 127,
 * clamped to [1, 253]; amax = 0 gives byte 127), q = e4m3_rne(clamp(v / scale, +-448)).
 *   transpose = 0: src [rows x cols] fp16 (ld_src); transpose = 1: q row r is
 *   column r of src [cols x rows] (weights W[K][N] -> W8[N][K]).
 * q: [rows x ldq] bytes, scales: [rows][lds]; columns cols .. roundup(cols, 128)-1
 * of q and their scale bytes are written as zero / 127 (padding read by the GEMM).
 */
int kf_quant_mxfp8(const void *src, long long ld_src, int rows, int cols, int transpose,
                   void *q, long long ldq, uint8_t *scales, long long lds);

/* Up to KF_QUANT_MAX kf_quant_mxfp8 calls in one launch (the weight copies after each
 * update: ~80 small matrices per step, each too small to fill the GPU on its own). Same
 * arguments and results as kf_quant_mxfp8, per job. */
#define KF_QUANT_MAX 32
typedef struct KfQuantJob {
    const void *src;
    long long ld_src;
    int rows, cols, transpose;
    void *q;
    long long ldq;
    uint8_t *scales;
    long long lds;
} KfQuantJob;
int kf_quant_mxfp8_batch(int n, const KfQuantJob *jobs);

/* out[j] = rne_fp16(sum_c x0[c] W[j][c] + x1[c] W[rows + j][c]), j < rows, W [2*rows x cols]
 * fp16 row-major, fp32 accumulation; cols % 8 == 0, 16-byte aligned pointers (out is not
 * required to be: it is written per element). One row of a two-part product. */
int kf_dot2_rows(void *out, const void *x0, const void *x1, const void *W, int rows, int cols);
/* kf_gemm_fused of an MXFP8 product (rows 0 .. M-1), whose last row tile's workgroups also
 * compute kf_dot2_rows(edge_out, x0, x1, W, N, cols): the TDNN-F affine input gradient's
 * clamped-edge row T - 1 (M = T - 1) in the same launch. As a separate one-row kernel beside
 * the weight-gradient stream it waited ~340 us per layer for CU slots (3072 model). */
int kf_gemm_fused_edge(int M, int N, int K, const KfOperand *A, const KfOperand *B, const KfEpilogue *epi,
                       void *edge_out, const void *x0, const void *x1, const void *W, int cols);

/* edge[c] = rne_fp16(sum_{r in [r0, r1)} src[r*ld + c]) for c < cols
 * (edge may be a spare row of src's own allocation) */
int kf_rows_sum(void *edge, const void *src, long long ld, int r0, int r1, int cols);
/* the same over the masked source: element r*ld + c counts only when its bit in mask is set */
int kf_rows_sum_mask(void *edge, const void *src, long long ld, int r0, int r1, int cols,
                     const uint8_t *mask);

/* ---- non-MFMA layer pieces (csrc/layers.hip) ---- */
/* y[T x N] = x[T x K] . M[K x N], K <= 64, N % 8 == 0 (IDCT, forward.go:317-330) */
int kf_small_gemm(const void *x, int ldx, const void *M, void *y, int ldy, int T, int K, int N);
/* y = rne(x*scale[d] + shift[d]) on [rows x D] (frozen BatchNorm, folded) */
int kf_bn_apply(const void *x, void *y, long long rows, int D, const float *scale,
                const float *shift);
/* conv-relu-batchnorm with one input filter (im2col K = noff), fused epilogue;
 * y [(T*hout) x fout], mask bits in the same element order */
int kf_conv_c1_forward(int T, int hin, int hout, int sub, int fout, int noff, const int *dt,
                       const int *dh, const void *x, const void *W, const void *bias,
                       const float *scale, const float *shift, void *y, uint8_t *mask);
/* its weight / bias gradient (fp32, overwritten), deterministic */
int kf_conv_c1_wgrad(int T, int hin, int hout, int sub, int fout, int noff, const int *dt,
                     const int *dh, const void *x, const void *dz, float *dW, float *db);
/* one-launch SGD over a flat parameter set: v = mom*v + g; w32 -= lr*v; w16 = rne(w32) */
int kf_sgd_flat(float *w32, void *w16, const float *g, float *v, float lr, float mom,
                long long n);
int kf_f32_to_f16_flat(const float *src, void *dst, long long n);
/* row sets of the row-subsampled train step (kf_nnet.h nnet_set_row_subsampling): compact
 * row c is source row 3c for c < tc0, else (T-1) - 3(tc-1-c). row_bytes % 16 == 0.
 * gather: dst[c] = src[row(c)] for c < tc; scatter: every full row t < T of dst gets the
 * compact row of src whose source row is t, or zeros */
int kf_gather_rows(void *dst, const void *src, long long row_bytes, int T, int tc0, int tc);
int kf_scatter_rows(void *dst, const void *src, long long row_bytes, int T, int tc0, int tc);
/* kf_scatter_rows for the full rows r0 .. T-1 only, dst row 0 = full row r0 */
int kf_scatter_rows_from(void *dst, const void *src, long long row_bytes, int T, int tc0, int tc, int r0);
/* dst block b (block_bytes each, % 16) = src block map[b], or zeros where map[b] < 0;
 * nblocks <= 32, map a host array (the merged weight rows of a strided conv's input gradient) */
int kf_copy_blocks(void *dst, const void *src, long long block_bytes, const int *map, int nblocks);
/* edge[c] = rne(sum over rows[0..n) in that order of src[rows[i] * ld + c]), n <= 4 (host array) */
int kf_rows_sum_list(void *edge, const void *src, long long ld, const int *rows, int n, int cols);
const char *kf_layers_last_error(void);

/* Kaldi compressed-matrix expansion (egs input, kf_egs.h). One descriptor per stored
 * matrix; payload_off = byte offset of its payload in the device blob (2-byte aligned,
 * 4 for FM); rows land at out rows [out_row, out_row + rows). cols <= 256. */
enum { KF_CM_ONEBYTE_COLHDR = 1, KF_CM_TWOBYTE = 2, KF_CM_ONEBYTE = 3, KF_CM_FLOAT = 4 };
typedef struct {
    int format, rows, cols, out_row;
    float min_value, range;
    long long payload_off;
} KfCmDesc;
int kf_cm_expand(const KfCmDesc *dev_desc, int nmat, int max_rows, int max_cols,
                 const void *dev_blob, void *dev_out, int ldo);
/* Same from host arrays: every descriptor is bounds-checked against blob_bytes, then
 * descriptors + blob travel in one pinned, stream-ordered H2D copy (kf_get_stream())
 * ahead of the launch. The host arrays may be freed on return. */
int kf_cm_expand_host(const KfCmDesc *desc, int nmat, int max_rows, int max_cols,
                      const void *blob, size_t blob_bytes, void *dev_out, int ldo);

/* Restricted self-attention of attention-relu-batchnorm layers (csrc/attention.hip;
 * forward.go:795-909 runs it on the CPU). proj: fp16 [T x ldp] affine output, per head
 * [key kd | value vd | query key kd | query context ctx]; frame t attends to rows
 * t + (o - num_left) * stride, o < context, zero outside [0, T). */
typedef struct {
    const void *proj;
    long long ldp;
    int T, num_heads, key_dim, value_dim, context, num_left, stride;
    float key_scale;
} KfAttention;
/* out: fp16 [T x ldo], width num_heads * (value_dim + context); y = bn(relu(att));
 * mask (may be NULL): ReLU bits, row-major over width (width % 8 == 0). */
int kf_attention_forward(const KfAttention *a, void *out, long long ldo, uint8_t *mask, const float *scale,
                         const float *shift);
/* dz: fp16 gradient at the attention output (pre-ReLU) [T x ldz]; dproj: fp16, same
 * layout and ld as proj (every element written); scratch: fp32 [2 x T x heads x context]. */
int kf_attention_backward(const KfAttention *a, const void *dz, long long ldz, void *dproj, float *scratch);

/* ivector input path (csrc/ivector.hip). dev_seq_off: device int[B+1] frame offsets of
 * the sequences (seq_off[B] = T); NULL in kf_combine_feature_maps = b is frame-level.
 * combine: out[t][h*(nf1+nf2) + f] = f < nf1 ? a[t][h*nf1 + f] : b[seq(t)][h*nf2 + f-nf1] */
int kf_combine_feature_maps(const void *a, long long lda, const void *b, long long ldb, const int *dev_seq_off,
                            int B, void *out, long long ldo, int T, int height, int nf1, int nf2);
/* db[s][h*nf2 + g] = sum over the frames t of sequence s of dy[t][h*(nf1+nf2) + nf1 + g] */
int kf_combine_feature_maps_backward(const void *dy, long long ldy, const int *dev_seq_off, int B, void *db,
                                     long long ldb, int height, int nf1, int nf2);
/* small num-filters-in convolution as im2col + GEMM: P [T*hout x kp], column tap*fin + c
 * = x[t + dt[tap]][ho*sub + dh[tap]][c] (zero outside), columns >= ntaps*fin zero */
int kf_im2col_small(const void *x, long long ldx, int T, int hin, int hout, int sub, int fin, int ntaps,
                    const int *dt, const int *dh, void *P, int kp);
/* its transpose, gather form: dx [T x hin*fin] */
int kf_col2im_small(const void *dP, int T, int hin, int hout, int sub, int fin, int ntaps, const int *dt,
                    const int *dh, int kp, void *dx, long long ldx);
/* per-sequence linear-component on R rows, any dims: y = x . W (fp32 accumulation) and
 * its weight gradient dW = x^T . g (fp32, overwritten, summed in row order) */
int kf_rows_gemm(const void *x, long long ldx, const void *W, long long ldw, void *y, long long ldy, int R, int K,
                 int N);
int kf_rows_wgrad(const void *x, long long ldx, const void *g, long long ldg, float *dW, long long ldd, int R, int M,
                  int N);
/* y[r][c] = rne_fp16(fp32(x[r][c] * scale[c])) (fp16 in / out, fp32 scale; x may be y) */
int kf_scale_cols(const void *x, long long ldx, const float *scale, void *y, long long ldy, int rows, int cols);

/* optional HIP-event timing of the step's kernel classes on the stream each runs on;
 * collect sums since reset. Classes: 0 = kf_gemm_fused on the tiled GEMM, 1 = kf_gemm_wgrad
 * GEMM, 2 = chain numerator (flops = arc updates), 3 = chain den (flops = algorithmic
 * L2/HBM bytes), 4 = kf_gemm_fused on the 3x3 conv halo kernel, 5 = the conv halo weight
 * gradient, 6 = the split-K slab reduce (bytes only) */
void kf_prof_enable(int on);
/* pre-create the timing events of n profiled launches (no event creation in timed code) */
int kf_prof_reserve(int n);
int kf_prof_collect(int cls, long long *count, double *ms, double *flops);
/* the same plus the algorithmic HBM bytes of those launches (GEMM classes: each
 * operand's source tensor read once, epilogue tensors read / written once) */
int kf_prof_collect2(int cls, long long *count, double *ms, double *flops, double *bytes);
void kf_prof_reset(void);

/* test hook: the fused GEMM's K-step interleave of a two-part spliced A with parts of
 * >= 512 columns (the TDNN-F linear forward / affine input gradient). 1 (default):
 * the K-steps alternate between the parts; 0: part order. Only the fp32 accumulation
 * order differs. */
void kf_gemm_debug_kil(int on);
/* n <= KF_TRANSPOSE_MAX fp16 transposes in one launch: dst[j] [N[j] x M[j]] = src[j]^T
 * (src[j] [M[j] x N[j]] row-major); the network's transposed weight copies */
#define KF_TRANSPOSE_MAX 48
int kf_transpose_batch(int n, const void *const *src, void *const *dst, const int *M, const int *N);
/* diagnostics: wall-clock stamps (100 MHz) of block 300, wave 0 of the conv-halo launch
 * number `at` counted from this call: [0] start, [1 + 2s] after step s's wait and barrier,
 * [2 + 2s] after its MFMAs, [126] before the epilogue, [127] end; buf NULL disarms */
void kf_halo_trace(unsigned long long *buf, int at);
/* diagnostics: phase stamps of block `blk` and {start, end, hw id | xcc << 32} of every
 * block of gemm_kernel launch number `at` (counted from this call), wall_clock64 ticks
 * (100 MHz); buf holds 64 + 3 * blocks words; null = off */
void kf_gemm_trace(unsigned long long *buf, int at, int blk);

const char *kf_last_error(void);
void kf_clear_error(void);
/* diagnostics: the kf_prof records since the last kf_prof_reset in issue order (class,
 * milliseconds, flops, and per record 4 ints: M, N, K, BM * 10000 + BN; zeros for
 * brackets that are not one GEMM launch); returns the count written (at most max) */
int kf_prof_records(int max, int *cls, float *ms, double *flops, int *mnkt);

/* Error hygiene across the C-ABI. HIP keeps one pending error per host
 * thread, read and reset by hipGetLastError(). Every entry point of this library that
 * checks its own launches with hipGetLastError() first calls kf_take_pending(its name):
 * an error some earlier HIP call left pending (another library, the caller's own HIP
 * calls, or a runtime call whose status nobody read) is consumed there and logged as
 * "pending before <where>: <error>" instead of being reported as that entry's failure.
 * kf_take_pending returns the consumed hipError_t (0 = none). kf_pending_log returns
 * the log since the last kf_pending_clear (NULL if empty; at most the last 16 notes,
 * plus the total count); kf_peek_error returns the pending error without consuming
 * it. With KF_ERR_VERBOSE=1 in the environment every note is also printed to stderr. */
int kf_take_pending(const char *where);
const char *kf_pending_log(void);
void kf_pending_clear(void);
int kf_peek_error(void);
/* diagnostics (tests): one workgroup spinning for `cycles` GPU clock cycles on `stream` */
int kf_debug_spin(void *stream, long long cycles);

#ifdef __cplusplus
}
#endif
#endif
