/*
 * bridge.h — device/memory/transfer half of the kaldi-fp16 C-ABI, MI355X build.
 *
 * Drop-in for the reference's cpp/include/bridge.h:13-60 (implemented there in
 * cpp/cuda/bridge.cu:38-334 and bound from Go by internal/gpu/bridge.go:45-436).
 * Same symbol names, argument meaning and error convention:
 *   - int-returning calls give 0 on success, -1 on failure;
 *   - pointer-returning calls give NULL on failure;
 *   - the failure text is kept per OS thread and read with bridge_last_error()
 *     (NULL when no error is pending), cleared with bridge_clear_error().
 * All copies are synchronous with respect to the host, as in the reference.
 * Device work is ordered on the library's current stream (kf_set_stream in
 * kf_ops.h; the default is the null stream, as in the reference).
 */
#ifndef KALDI_FP16_AMD_BRIDGE_H
#define KALDI_FP16_AMD_BRIDGE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* errors (bridge.cu:11-33) */
const char *bridge_last_error(void);
void bridge_clear_error(void);

/* device selection / info / sync (bridge.cu:38-72) */
int bridge_gpu_init(int device_id);
int bridge_gpu_get_free_memory(size_t *free_bytes, size_t *total_bytes);
int bridge_gpu_sync(void);

/* memory (bridge.cu:75-113); host_alloc returns page-locked memory */
void *bridge_gpu_malloc(size_t bytes);
void bridge_gpu_free(void *ptr);
void *bridge_host_alloc(size_t bytes);
void bridge_host_free(void *ptr);

/* host <-> device copies; counts are in elements (bridge.cu:117-173) */
int bridge_transfer_fp16(void *dst_device, const uint16_t *src_host, size_t count);
int bridge_read_fp16(uint16_t *dst_host, const void *src_device, size_t count);
int bridge_transfer_int32(void *dst_device, const int32_t *src_host, size_t count);
int bridge_transfer_float32(void *dst_device, const float *src_host, size_t count);
/* MI355X addition: float32 device -> host, synchronous on the library stream. Replaces the
 * direct cudaMemcpy D2H of internal/nnet/denominator_gpu.go:78-86. */
int bridge_read_float32(float *dst_host, const void *src_device, size_t count);

/*
 * One-allocation minibatch buffer (bridge.h:34-50, bridge.cu:177-267).
 * Sections, each rounded up to 256 bytes, in this order:
 *   features fp16 [total_frames x feat_dim] | ivectors fp16 [batch x ivec_dim] |
 *   CSR row_ptr int32 [num_states+1] | col_idx int32 [num_arcs] |
 *   labels int32 [num_arcs] | weights f32 [num_arcs]
 * The struct layout is read field-by-field by cgo and must not change.
 */
typedef struct {
    void *d_features;
    void *d_ivectors;
    void *d_csr_row_ptr;
    void *d_csr_col_idx;
    void *d_csr_labels;
    void *d_csr_weights;
    void *d_buffer;
    size_t total_bytes;
    size_t features_bytes;
    size_t ivectors_bytes;
    size_t csr_rowptr_bytes;
    size_t csr_colidx_bytes;
    size_t csr_labels_bytes;
    size_t csr_weights_bytes;
} GPUBatchPtrs;

int bridge_batch_alloc(int total_frames, int feat_dim, int batch_size, int ivec_dim,
                       int num_states, int num_arcs, GPUBatchPtrs *out);
int bridge_batch_transfer(const GPUBatchPtrs *ptrs, const void *host_buf, size_t total_bytes);
void bridge_batch_free(GPUBatchPtrs *ptrs);
void bridge_gpu_memset(void *ptr, int value, size_t bytes);

/* on-device conversions, RNE for fp32->fp16 (bridge.cu:288-334) */
int bridge_fp16_to_fp32_gpu(float *dst_device, const void *src_device, size_t count);
int bridge_fp32_to_fp16_gpu(void *dst_device, const float *src_device, size_t count);

#ifdef __cplusplus
}
#endif
#endif
