/*
 * kf_model.h — Kaldi nnet3 model import, in libkaldi_fp16_nnet.so.
 *
 * Replaces (internal/nnet/weight_loader.go; Go is absent from the image, the
 * entry points are what a cgo binding of that file would call):
 *   KaldiComponent                        weight_loader.go:28-61
 *   ParseNnet3Text                        weight_loader.go:608-727  -> kf_nnet3_parse_text
 *   ExportModelText (nnet3-copy, exec)    weight_loader.go:596-605  -> kf_nnet3_export
 *   NewNetworkFromKaldi / allocWeights    weight_loader.go:65-437   -> nnet_load_kaldi(KF_LOAD_NEW)
 *   LoadWeights / replaceMatrix/BN        weight_loader.go:750-1104 -> nnet_load_kaldi(KF_LOAD_REPLACE)
 *
 * Kaldi stores affine matrices [out x in]; they are transposed to the build's
 * [in x out] (transposeF32, :920-928) and enter the fp16 weights by truncation like
 * every other weight (nnet_set_params). Conv BatchNorm statistics are per filter and
 * tile over heights in the build's height-major layout (Kaldi's), not the reference's
 * filter-major tiling (makeBlockBN :490-530).
 *
 * Conventions: NULL / -1 on error with kf_nnet3_last_error() (thread-local).
 */
#ifndef KALDI_FP16_AMD_KF_MODEL_H
#define KALDI_FP16_AMD_KF_MODEL_H
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct KfNnet3Model KfNnet3Model;
typedef struct KfNet KfNet;

/* One parsed component (KaldiComponent). Arrays are owned by the model; NULL with a
 * zero length when the component has none. linear_* covers <LinearParams> and <Params>. */
typedef struct {
    const char *name;
    const char *type;            /* e.g. "TdnnComponent" (brackets stripped) */
    const float *linear;
    int linear_rows, linear_cols;
    const float *bias;
    int bias_dim;
    const float *stats_mean;
    int mean_dim;
    const float *stats_var;
    int var_dim;
    double count;
    float epsilon, target_rms;
    int num_filters_in, num_filters_out, height_in, height_out;
    int num_heads, key_dim, value_dim;
    float key_scale;
    float learning_rate, max_change, l2_regularize;
} KfNnet3Component;

const char *kf_nnet3_last_error(void);

/* ParseNnet3Text: the text nnet3-copy --binary=false writes. A component name seen
 * twice keeps the last one (Go map assignment). */
KfNnet3Model *kf_nnet3_parse_text(const char *text, size_t len);
/* the same text read from a file */
KfNnet3Model *kf_nnet3_read_text_file(const char *path);
/* ExportModelText + parse: runs `nnet3-copy --binary=false <mdl> -` (must be on PATH;
 * Kaldi is not part of this build) */
KfNnet3Model *kf_nnet3_export(const char *mdl_path);
void kf_nnet3_free(KfNnet3Model *m);

int kf_nnet3_num_components(const KfNnet3Model *m);
/* components in first-appearance order */
int kf_nnet3_component(const KfNnet3Model *m, int idx, KfNnet3Component *out);
/* index of a component by name, -1 if absent */
int kf_nnet3_find(const KfNnet3Model *m, const char *name);

/* BatchNorm semantics of the two reference entry points:
 *   KF_LOAD_NEW     makeBN / makeBlockBN: gamma = target_rms, beta = 0 over the
 *                   running statistics (Kaldi's test-mode BatchNorm); empty affine
 *                   biases become zeros; prefinal batchnorm2 is loaded.
 *   KF_LOAD_REPLACE replaceBN: gamma = target_rms / sqrt(var + eps), beta = -mean*gamma
 *                   AND the statistics, i.e. the reference's double normalisation
 *                   (SURVEY §8f row 2); empty biases keep the current values;
 *                   batchnorm2 is not loaded; attention layers are skipped. */
enum { KF_LOAD_NEW = 0, KF_LOAD_REPLACE = 1 };

typedef struct {
    int layers_loaded, layers_skipped;
    long long params;  /* the reference's totalParams count */
} KfLoadStats;

/* Loads every layer of `net` from the model's components (component names of the
 * reference: idct, <name>, <name>.conv/.batchnorm, <name>.linear/.affine/.batchnorm,
 * prefinal-chain|prefinal-xent.affine/.linear/.batchnorm1/.batchnorm2,
 * <name>.affine). A missing component or a shape that differs from the layer's is an
 * error and leaves the network unchanged. */
int nnet_load_kaldi(KfNet *net, const KfNnet3Model *m, int mode, KfLoadStats *stats);

#ifdef __cplusplus
}
#endif
#endif
