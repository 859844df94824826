/*
 * kf_egs.h — Kaldi chain egs input: binary-ark reader, FST/CSR conversion, minibatch
 * loader, and the MI355X-side feature decompression.
 *
 * Replaces (the reference is pure Go here; these are the entry points its packages
 * would bind through cgo):
 *   parser.NewReader / DetectFormat / ReadExample   internal/parser/parser.go:36-160
 *   parser.ReadFst (compact_acceptor, vector)       internal/parser/fst.go:18-160
 *   ReadCompressedMatrix{,2,3} / ReadFullMatrix     internal/parser/matrix.go:10-180
 *   ReadSparseMatrix                                internal/parser/matrix.go:182-245
 *   readIndexVector                                 internal/parser/parser.go:470-548
 *   sparse.FstToCSR / FstToCOO / COOToCSR / MergeCOO / LabelDim / Validate
 *                                                   internal/sparse/sparse.go:54-320
 *   loader.EgsIterator                              internal/loader/loader.go:12-170
 *   loader.DataLoader.NextBatch / TrainingBatch     internal/loader/dataloader.go:15-277
 *   batch.NewBatch (features + ivectors merge)      internal/batch/batch.go:43-123
 * plus, MI355X-native: the minibatch's feature matrices travel to HBM still
 * compressed (CM: 1 byte/value + 8 B/column) and one kernel expands them into the
 * fp16 network-input matrix (kf_egs_batch_features), instead of the reference's
 * host decompression -> fp32 merge -> host fp32->fp16 -> H2D of 2 B/value
 * (batch.go:97-104, bridge.go:123-366).
 *
 * Conventions: int 0 / -1 or NULL on error with a thread-local kf_egs_last_error()
 * (the reference returns Go errors); all arrays are host memory unless named dev_*.
 * Returned pointers stay valid until the owning object is freed.
 */
#ifndef KF_EGS_H
#define KF_EGS_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* matrix storage types, parser/types.go:27 ("CM", "CM2", "CM3", "FM") */
enum { KF_MAT_NONE = 0, KF_MAT_CM = 1, KF_MAT_CM2 = 2, KF_MAT_CM3 = 3, KF_MAT_FM = 4 };

/* One NnetIo block (parser/types.go:19-25 IoBlock + MatrixInfo). The matrix is kept
 * in its stored form: payload = the bytes after the global header, i.e.
 *   CM : cols x {u16 p0,p25,p75,p100} then rows*cols bytes COLUMN-major
 *   CM2: rows*cols u16 row-major;  CM3: rows*cols u8 row-major;  FM: rows*cols f32. */
typedef struct {
    const char *name;
    int num_indexes;
    const int32_t *indexes;    /* [num_indexes][3] = (n, t, x) */
    int format;                /* KF_MAT_* */
    int rows, cols;
    float min_value, range;    /* global header (CM/CM2/CM3) */
    const uint8_t *payload;
    size_t payload_bytes;
} KfEgsIo;

/* Chain supervision FST (parser/types.go:107-125) as arc arrays in state order. */
typedef struct {
    int64_t start, num_states, num_arcs;
    uint64_t properties;
    const int32_t *arc_off;    /* [num_states+1] */
    const int32_t *label;      /* [num_arcs] */
    const float *weight;       /* [num_arcs] tropical (-log p) */
    const int32_t *next_state; /* [num_arcs] */
    const float *final_weight; /* [num_states], +inf = not final */
} KfEgsFst;

/* One NnetChainExample (parser/types.go:3-9, SupervisionBlock :52-63). */
typedef struct {
    const char *key;
    int num_inputs, num_outputs;   /* <NumInputs>, <NumOutputs> */
    int num_io;
    const KfEgsIo *io;             /* in file order */
    const char *sup_name;
    int sup_num_indexes;
    const int32_t *sup_indexes;    /* [sup_num_indexes][3] */
    float weight;
    int num_sequences, frames_per_seq, label_dim, end2end;
    int has_fst;
    KfEgsFst fst;
    int num_deriv_weights;
    const float *deriv_weights;
} KfEgsExample;

typedef struct KfEgsReader KfEgsReader;
typedef struct KfEgsLoader KfEgsLoader;
typedef struct KfEgsBatch KfEgsBatch;

/* ---------------------------------------------------------------- reader */
/* parser.DetectFormat (parser.go:82-116): 0 = binary ark ("\0B" in the first 256 B),
 * -1 otherwise (text ark / too small / unreadable; reason in kf_egs_last_error). */
int kf_egs_detect_format(const char *path);
/* parser.NewReader (parser.go:36-72): ".gz" paths are gunzipped and skip the format
 * check; other paths must pass kf_egs_detect_format. */
KfEgsReader *kf_egs_open(const char *path);
/* ReadExample (parser.go:119-131): 1 = *out holds the next example (owned by the
 * reader, valid until the next call), 0 = end of file, -1 = error. */
int kf_egs_next(KfEgsReader *r, const KfEgsExample **out);
void kf_egs_close(KfEgsReader *r);
/* Example.Validate / IsUsable (parser.go:448-466): input 40 cols + ivector 1x100,
 * usable = valid, weight > 0, label_dim 3080. */
int kf_egs_example_valid(const KfEgsExample *ex);
int kf_egs_example_usable(const KfEgsExample *ex);

/* Host decompression of one matrix to fp32 row-major (matrix.go:10-180, bit-exact
 * restatement of its float arithmetic). */
int kf_egs_io_to_float(const KfEgsIo *io, float *out);

/* Byte-buffer entry points (the reference's unit-test surface). Each reads from the
 * start of buf and reports the bytes consumed in *used (may be NULL). */
/* readIndexVector (parser.go:470-548): count <= 0 -> -1; short input -> -1 with
 * *n_read = indexes decoded before the end. out: [count][3]. */
int kf_egs_parse_index_vector(const uint8_t *buf, size_t len, int count, int32_t *out,
                              int *n_read, size_t *used);
/* ReadFst (fst.go:18-40) into a caller-freed KfEgsFst (kf_egs_fst_free); NULL on a
 * bad magic, an unknown fst/arc type or truncation. */
KfEgsFst *kf_egs_parse_fst(const uint8_t *buf, size_t len, size_t *used);
void kf_egs_fst_free(KfEgsFst *f);
/* ReadSparseMatrix (matrix.go:182-245), buf starting after the "SM" token. Writes
 * row_dim[num_rows], row_off[num_rows+1] and (index, value) pairs; returns num_rows or
 * -1. Call with NULL outputs to size: *num_pairs gets the total pair count. */
int kf_egs_parse_sparse_matrix(const uint8_t *buf, size_t len, int32_t *row_dim,
                               int32_t *row_off, int32_t *pair_index, float *pair_value,
                               int *num_pairs, size_t *used);

/* ---------------------------------------------------------------- CSR (sparse.go) */
/* FstToCSR (sparse.go:54-100): arcs in state order, weights NEGATED (tropical ->
 * log-prob), finals in state order with negated weights. Sizes: row_ptr[S+1],
 * col/label/logw[A], final_state/final_logw[*num_finals <= S]. -1 for an FST with no
 * states. */
int kf_egs_fst_to_csr(const KfEgsFst *f, int32_t *row_ptr, int32_t *col, int32_t *label,
                      float *logw, int32_t *final_state, float *final_logw, int *num_finals);

/* ---------------------------------------------------------------- loader */
/* DataLoaderConfig (dataloader.go:56-62): glob pattern (or a '\n'-separated path list
 * when the string contains '\n'), batch size > 0, shuffle with seed, drop_last. */
KfEgsLoader *kf_egs_loader_create(const char *pattern, int batch_size, int shuffle,
                                  unsigned long long seed, int drop_last);
/* NextBatch (dataloader.go:100-184): 1 = *out holds a new batch (caller frees with
 * kf_egs_batch_free), 0 = exhausted, -1 = error. Examples failing validateExample
 * (dataloader.go:236-258) are skipped; unreadable files are skipped (loader.go). */
int kf_egs_loader_next(KfEgsLoader *l, KfEgsBatch **out);
/* Reset for a new epoch (dataloader.go:187-193). */
void kf_egs_loader_reset(KfEgsLoader *l);
/* Stats (dataloader.go:203-226): batches served, examples read, total seconds. */
void kf_egs_loader_stats(const KfEgsLoader *l, int *batches, int *examples, double *seconds);
int kf_egs_loader_num_files(const KfEgsLoader *l);
void kf_egs_loader_free(KfEgsLoader *l);

/* TrainingBatch (dataloader.go:15-40). */
typedef struct {
    int batch_size;
    int total_frames, feat_dim;      /* merged features [total_frames x feat_dim] */
    int ivector_dim;                 /* 0 = no ivectors */
    int label_dim;                   /* max label + 1 over the merged CSR (sparse.go:264) */
    int num_sequences;               /* of the first example */
    float weight;                    /* of the first example */
    const int32_t *frame_offsets;    /* [B] */
    const int32_t *num_frames;       /* [B] */
    const int32_t *frames_per_seq;   /* [B] supervision frames per example */
    const int32_t *state_offsets;    /* [B] offset of each FST in the merged CSR */
    /* merged CSR (MergeCOO + COOToCSR, sparse.go:161-258) */
    int num_states, num_arcs, num_finals;
    const int32_t *row_ptr, *col, *label;
    const float *logw;
    const int32_t *final_state;
    const float *final_logw;
    /* per-example CSRs concatenated in the kf_num_batch_create layout (kf_chain.h):
     * state_off/arc_off/final_off [B+1], per_row_ptr [num_states + B] local arc ids,
     * per_col [num_arcs] and per_final_state [num_finals] local state ids; labels,
     * log weights and final log weights are the merged arrays above (same order). */
    const int32_t *state_off, *arc_off, *final_off, *per_row_ptr, *per_col, *per_final_state;
} KfEgsBatchInfo;

int kf_egs_batch_info(const KfEgsBatch *b, KfEgsBatchInfo *out);
const char *kf_egs_batch_key(const KfEgsBatch *b, int i);
/* Host reference merge: fp32 features / ivectors as batch.NewBatch builds them. */
int kf_egs_batch_features_host(const KfEgsBatch *b, float *out /* [total_frames x feat_dim] */);
int kf_egs_batch_ivectors_host(const KfEgsBatch *b, float *out /* [B x ivector_dim] */);
/* MI355X path: upload the still-compressed feature matrices (one packed H2D copy)
 * and expand them on the GPU into the fp16 row-major matrix dev_out [total_frames x
 * ldo] (ldo >= feat_dim), fp32 decompression identical to kf_egs_io_to_float, then
 * fp16 round-to-nearest-even (fp16.FromFloat32, fp16.go:12-70). Asynchronous on
 * kf_get_stream(); the staging copy is stream-ordered. dev_ivec (may be NULL)
 * receives the ivectors [B x ivector_dim] in fp16 the same way. */
int kf_egs_batch_features(KfEgsBatch *b, void *dev_out, int ldo, void *dev_ivec);
/* bytes of the packed compressed feature upload of the last kf_egs_batch_features */
size_t kf_egs_batch_upload_bytes(const KfEgsBatch *b);
void kf_egs_batch_free(KfEgsBatch *b);

/* Build a batch from already-read examples (the TrainingBatch assembly of
 * dataloader.go:143-178, used by tests and by callers that own their reader). The
 * examples are deep-copied. */
KfEgsBatch *kf_egs_batch_from_examples(const KfEgsExample *const *ex, int n);

const char *kf_egs_last_error(void);
void kf_egs_clear_error(void);

#ifdef __cplusplus
}
#endif
#endif
