// bridge.hip — device / memory / transfer entry points (include/bridge.h).
// Behaviour follows the reference's cpp/cuda/bridge.cu:38-334; device work is
// issued on the library's current stream (kf_set_stream) and every call that
// hands data back to the host synchronises, as the reference's blocking
// cudaMemcpy calls do.
#include "kf_common.h"
#include <stdlib.h>
#include <string>
#include "../../include/bridge.h"
#include "../../include/kf_ops.h"

KF_DECLARE_ERR(bridge)

// ---------------------------------------------------------------------------
// stream + workspace shared by all modules of the library
// ---------------------------------------------------------------------------
static __thread hipStream_t g_stream = nullptr;
hipStream_t kf_stream() { return g_stream; }
extern "C" void kf_set_stream(void *s) { g_stream = (hipStream_t)s; }
extern "C" void *kf_stream_new(void) {
    hipStream_t s = nullptr;
    return hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess ? (void *)s : nullptr;
}
extern "C" void *kf_stream_new_high(void) {
    int least = 0, greatest = 0;
    hipStream_t s = nullptr;
    if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) return nullptr;
    return hipStreamCreateWithPriority(&s, hipStreamNonBlocking, greatest) == hipSuccess ? (void *)s : nullptr;
}
extern "C" void kf_stream_free(void *s) {
    if (s) hipStreamDestroy((hipStream_t)s);
}
extern "C" void *kf_event_new(void) {
    hipEvent_t e = nullptr;
    return hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess ? (void *)e : nullptr;
}
extern "C" void kf_event_free(void *e) {
    if (e) hipEventDestroy((hipEvent_t)e);
}
extern "C" int kf_event_record(void *e, void *s) {
    return hipEventRecord((hipEvent_t)e, (hipStream_t)s) == hipSuccess ? 0 : -1;
}
extern "C" int kf_stream_wait(void *s, void *e) {
    return hipStreamWaitEvent((hipStream_t)s, (hipEvent_t)e, 0) == hipSuccess ? 0 : -1;
}
extern "C" void *kf_get_stream(void) { return (void *)g_stream; }

// ---------------------------------------------------------------------------
// error hygiene (include/kf_ops.h: kf_take_pending). HIP's pending error is per host
// thread, and so is this log.
// ---------------------------------------------------------------------------
namespace {
struct PendingLog {
    enum { kKeep = 16 };
    char note[kKeep][192];
    int total = 0;
    std::string text;
};
__thread PendingLog *g_pending = nullptr;
PendingLog &pending_log() {
    if (!g_pending) g_pending = new PendingLog();  // per thread, lives as long as the thread
    return *g_pending;
}
bool pending_verbose() {
    static int v = -1;
    if (v < 0) {
        const char *e = getenv("KF_ERR_VERBOSE");
        v = e && *e && *e != '0';
    }
    return v;
}
}  // namespace

extern "C" int kf_take_pending(const char *where) {
    const hipError_t e = hipGetLastError();
    if (e == hipSuccess) return 0;
    PendingLog &L = pending_log();
    char *n = L.note[L.total % PendingLog::kKeep];
    snprintf(n, sizeof(L.note[0]), "pending before %s: %s (%s)", where ? where : "?", hipGetErrorName(e),
             hipGetErrorString(e));
    ++L.total;
    if (pending_verbose()) fprintf(stderr, "kfp16: HIP error %s\n", n);
    return (int)e;
}
extern "C" const char *kf_pending_log(void) {
    PendingLog &L = pending_log();
    if (!L.total) return nullptr;
    L.text = std::to_string(L.total) + " pending error(s)";
    const int first = L.total > PendingLog::kKeep ? L.total - PendingLog::kKeep : 0;
    for (int i = first; i < L.total; ++i) {
        L.text += "; ";
        L.text += L.note[i % PendingLog::kKeep];
    }
    return L.text.c_str();
}
extern "C" void kf_pending_clear(void) { pending_log().total = 0; }
extern "C" int kf_peek_error(void) { return (int)hipPeekAtLastError(); }

__global__ void k_spin(long long cycles, int *sink) {
    const long long t0 = clock64();
    long long n = 0;
    while (clock64() - t0 < cycles) {
        __builtin_amdgcn_s_sleep(8);
        ++n;
    }
    if (n < 0) *sink = 1;  // never: keeps the loop
}
extern "C" int kf_debug_spin(void *stream, long long cycles) {
    kf_take_pending(__func__);
    if (cycles <= 0) return 0;
    k_spin<<<1, 64, 0, (hipStream_t)stream>>>(cycles, nullptr);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

namespace {
struct Slot {
    void *ptr = nullptr;
    size_t bytes = 0;
};
constexpr int kMaxDev = 16, kMaxSlot = 8;
Slot g_ws[kMaxDev][kMaxSlot];
}  // namespace

void *kf_workspace(size_t bytes, int slot) {
    int dev = 0;
    hipGetDevice(&dev);
    if (dev < 0 || dev >= kMaxDev || slot < 0 || slot >= kMaxSlot) return nullptr;
    Slot &s = g_ws[dev][slot];
    if (s.bytes >= bytes && s.ptr) return s.ptr;
    // growing a slot is an allocation point: never inside a captured region
    if (s.ptr) {
        hipStreamSynchronize(g_stream);
        hipFree(s.ptr);
        s.ptr = nullptr;
        s.bytes = 0;
    }
    size_t want = bytes < (1u << 20) ? (1u << 20) : bytes;
    if (hipMalloc(&s.ptr, want) != hipSuccess) {
        s.ptr = nullptr;
        return nullptr;
    }
    s.bytes = want;
    return s.ptr;
}

// Per-stream scratch for the weight gradients' split-K fp32 slabs (kf_common.h). One
// backward runs weight gradients on two streams at once (the input-gradient chain's and
// the weight-gradient stream), and a slab lives from its GEMM to its reduce,
// so each stream gets a buffer of its own: two streams never share one. Up to kStreams
// streams per device keep a buffer; another stream takes the least recently used one
// after a device-wide sync (only when streams are new, e.g. a new network's).
namespace {
constexpr int kStreams = 4;
struct StreamSlot {
    hipStream_t s = nullptr;
    bool used = false;
    unsigned long long last = 0;
    void *ptr = nullptr;
    size_t bytes = 0;
};
StreamSlot g_sws[kMaxDev][kStreams];
unsigned long long g_sws_tick = 0;
}  // namespace

void *kf_workspace_stream(size_t bytes) {
    int dev = 0;
    hipGetDevice(&dev);
    if (dev < 0 || dev >= kMaxDev) return nullptr;
    const hipStream_t st = g_stream;
    StreamSlot *row = g_sws[dev], *s = nullptr;
    for (int i = 0; i < kStreams && !s; ++i)
        if (row[i].used && row[i].s == st) s = &row[i];
    if (!s) {
        for (int i = 0; i < kStreams && !s; ++i)
            if (!row[i].used) s = &row[i];
        if (!s) {  // evict the least recently used stream's buffer: its work may be queued
            s = &row[0];
            for (int i = 1; i < kStreams; ++i)
                if (row[i].last < s->last) s = &row[i];
            hipDeviceSynchronize();
        }
        s->s = st;
        s->used = true;
    }
    s->last = ++g_sws_tick;
    if (s->bytes >= bytes && s->ptr) return s->ptr;
    if (s->ptr) {  // growing: this stream's queued work may still read the old buffer
        hipStreamSynchronize(st);
        hipFree(s->ptr);
        s->ptr = nullptr;
        s->bytes = 0;
    }
    const size_t want = bytes < (1u << 20) ? (1u << 20) : bytes;
    if (hipMalloc(&s->ptr, want) != hipSuccess) {
        s->ptr = nullptr;
        return nullptr;
    }
    s->bytes = want;
    return s->ptr;
}

__global__ void k_f16_to_f32(float *dst, const h16 *src, size_t n) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    size_t stride = (size_t)gridDim.x * blockDim.x;
    for (; i < n; i += stride) dst[i] = h2f(src[i]);
}
__global__ void k_f32_to_f16(h16 *dst, const float *src, size_t n) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    size_t stride = (size_t)gridDim.x * blockDim.x;
    for (; i < n; i += stride) dst[i] = f2h(src[i]);
}

static size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }

static int copy_sync(void *dst, const void *src, size_t bytes, hipMemcpyKind kind,
                     const char *what, size_t count) {
    hipError_t e = hipMemcpyAsync(dst, src, bytes, kind, g_stream);
    if (e == hipSuccess) e = hipStreamSynchronize(g_stream);
    if (e != hipSuccess) {
        bridge_set_error("hipMemcpy %s (%zu): %s", what, count, hipGetErrorString(e));
        return -1;
    }
    return 0;
}

extern "C" {

const char *bridge_last_error(void) { return bridge_err_.get(); }
void bridge_clear_error(void) { bridge_err_.clear(); }

int bridge_gpu_init(int device_id) {
    hipError_t e = hipSetDevice(device_id);
    if (e != hipSuccess) {
        bridge_set_error("hipSetDevice(%d): %s", device_id, hipGetErrorString(e));
        return -1;
    }
    return 0;
}

int bridge_gpu_get_free_memory(size_t *free_bytes, size_t *total_bytes) {
    hipError_t e = hipMemGetInfo(free_bytes, total_bytes);
    if (e != hipSuccess) {
        bridge_set_error("hipMemGetInfo: %s", hipGetErrorString(e));
        return -1;
    }
    return 0;
}

int bridge_gpu_sync(void) {
    hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess) {
        bridge_set_error("hipDeviceSynchronize: %s", hipGetErrorString(e));
        return -1;
    }
    return 0;
}

void *bridge_gpu_malloc(size_t bytes) {
    void *p = nullptr;
    hipError_t e = hipMalloc(&p, bytes);
    if (e != hipSuccess) {
        bridge_set_error("hipMalloc(%zu): %s", bytes, hipGetErrorString(e));
        return nullptr;
    }
    return p;
}

void bridge_gpu_free(void *ptr) {
    if (ptr) hipFree(ptr);
}

void *bridge_host_alloc(size_t bytes) {
    void *p = nullptr;
    hipError_t e = hipHostMalloc(&p, bytes, hipHostMallocDefault);
    if (e != hipSuccess) {
        bridge_set_error("hipHostMalloc(%zu): %s", bytes, hipGetErrorString(e));
        return nullptr;
    }
    return p;
}

void bridge_host_free(void *ptr) {
    if (ptr) hipHostFree(ptr);
}

int bridge_transfer_fp16(void *dst_device, const uint16_t *src_host, size_t count) {
    return copy_sync(dst_device, src_host, count * 2, hipMemcpyHostToDevice, "FP16 H2D", count);
}
int bridge_read_fp16(uint16_t *dst_host, const void *src_device, size_t count) {
    return copy_sync(dst_host, src_device, count * 2, hipMemcpyDeviceToHost, "FP16 D2H", count);
}
int bridge_read_float32(float *dst_host, const void *src_device, size_t count) {
    return copy_sync(dst_host, src_device, count * 4, hipMemcpyDeviceToHost, "float32 D2H",
                     count);
}
int bridge_transfer_int32(void *dst_device, const int32_t *src_host, size_t count) {
    return copy_sync(dst_device, src_host, count * 4, hipMemcpyHostToDevice, "int32 H2D", count);
}
int bridge_transfer_float32(void *dst_device, const float *src_host, size_t count) {
    return copy_sync(dst_device, src_host, count * 4, hipMemcpyHostToDevice, "float32 H2D",
                     count);
}

int bridge_batch_alloc(int total_frames, int feat_dim, int batch_size, int ivec_dim,
                       int num_states, int num_arcs, GPUBatchPtrs *out) {
    memset(out, 0, sizeof(*out));
    out->features_bytes = align256((size_t)total_frames * feat_dim * 2);
    out->ivectors_bytes = align256((size_t)batch_size * ivec_dim * 2);
    out->csr_rowptr_bytes = align256((size_t)(num_states + 1) * 4);
    out->csr_colidx_bytes = align256((size_t)num_arcs * 4);
    out->csr_labels_bytes = align256((size_t)num_arcs * 4);
    out->csr_weights_bytes = align256((size_t)num_arcs * 4);
    out->total_bytes = out->features_bytes + out->ivectors_bytes + out->csr_rowptr_bytes +
                       out->csr_colidx_bytes + out->csr_labels_bytes + out->csr_weights_bytes;
    hipError_t e = hipMalloc(&out->d_buffer, out->total_bytes);
    if (e != hipSuccess) {
        bridge_set_error("hipMalloc combined (%zu bytes): %s", out->total_bytes,
                         hipGetErrorString(e));
        out->d_buffer = nullptr;
        return -1;
    }
    char *b = (char *)out->d_buffer;
    size_t off = 0;
    out->d_features = b + off;
    off += out->features_bytes;
    out->d_ivectors = b + off;
    off += out->ivectors_bytes;
    out->d_csr_row_ptr = b + off;
    off += out->csr_rowptr_bytes;
    out->d_csr_col_idx = b + off;
    off += out->csr_colidx_bytes;
    out->d_csr_labels = b + off;
    off += out->csr_labels_bytes;
    out->d_csr_weights = b + off;
    return 0;
}

int bridge_batch_transfer(const GPUBatchPtrs *ptrs, const void *host_buf, size_t total_bytes) {
    return copy_sync(ptrs->d_buffer, host_buf, total_bytes, hipMemcpyHostToDevice, "batch",
                     total_bytes);
}

void bridge_batch_free(GPUBatchPtrs *ptrs) {
    if (ptrs && ptrs->d_buffer) {
        hipFree(ptrs->d_buffer);
        memset(ptrs, 0, sizeof(*ptrs));
    }
}

void bridge_gpu_memset(void *ptr, int value, size_t bytes) {
    hipMemsetAsync(ptr, value, bytes, g_stream);
}

int bridge_fp16_to_fp32_gpu(float *dst_device, const void *src_device, size_t count) {
    kf_take_pending(__func__);
    if (count == 0) return 0;
    k_f16_to_f32<<<kf_blocks(count, 256, 8192), 256, 0, g_stream>>>(dst_device,
                                                                    (const h16 *)src_device, count);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        bridge_set_error("fp16_to_fp32 kernel: %s", hipGetErrorString(e));
        return -1;
    }
    return 0;
}

int bridge_fp32_to_fp16_gpu(void *dst_device, const float *src_device, size_t count) {
    kf_take_pending(__func__);
    if (count == 0) return 0;
    k_f32_to_f16<<<kf_blocks(count, 256, 8192), 256, 0, g_stream>>>((h16 *)dst_device,
                                                                    src_device, count);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        bridge_set_error("fp32_to_fp16 kernel: %s", hipGetErrorString(e));
        return -1;
    }
    return 0;
}

}  // extern "C"
