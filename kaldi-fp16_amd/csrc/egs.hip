// egs.hip — MI355X expansion of Kaldi compressed feature matrices into the fp16
// network-input matrix (kf_egs.h: kf_egs_batch_features).
//
// The reference decompresses every eg on the host (internal/parser/matrix.go:10-180),
// merges fp32 rows (internal/batch/batch.go:97-104), converts to fp16 on the host
// (internal/fp16/fp16.go:12-70) and copies 2 B/value over PCIe (bridge.go:123-366).
// Here the stored bytes (CM: 1 B/value + 8 B/column) go to HBM as one packed blob
// and this kernel does the rest in one launch for the whole minibatch.
//
// Arithmetic is the reference's, op for op, with no contraction: Go on amd64 evaluates
// each float32 operation separately. HIP's __f*_rn are plain operators that the
// default -ffp-contract=fast would fuse into FMAs, so contraction is switched off for
// this file (pragma below) — found by the bit-exact GPU test.
//   uint16ToFloat  matrix.go:11-14   min + (range * f32(1/65535)) * f32(v)
//   charToFloat    matrix.go:17-27   three pieces; the last divides in float64
//   CM2            matrix.go:106-130 min + f32(v) * (range / 65535)
//   CM3            matrix.go:134-158 min + f32(v) * (range / 255)
// followed by fp16 round-to-nearest-even (fp16.FromFloat32).
//
// Layout: workgroup = one 64-row slab of one matrix. CM bytes are column-major, so
// the slab is read as `cols` coalesced 64-byte runs, transposed through LDS, and
// written as 64 contiguous fp16 rows. HBM-bound: 1 B read + 2 B written per value.
#include <mutex>

#include "kf_common.h"
#include "../../include/kf_ops.h"

#pragma clang fp contract(off)

namespace {

constexpr int kRows = 64;      // rows per workgroup
constexpr int kMaxCols = 256;  // LDS tile bound (Kaldi features: 40; ivectors: 100)

// Own single-rounding helpers: the operators below carry no 'contract' flag under the
// pragma above (HIP's __fmul_rn / __fadd_rn live in a header compiled with contraction).
__device__ __forceinline__ float mul_rn(float a, float b) { return a * b; }
__device__ __forceinline__ float add_rn(float a, float b) { return a + b; }
__device__ __forceinline__ float sub_rn(float a, float b) { return a - b; }

__device__ __forceinline__ float u16_to_float(float mn, float rg, unsigned v) {
    const float inv65535 = 1.52590218966964e-05f;
    return add_rn(mn, mul_rn(mul_rn(rg, inv65535), (float)v));
}

__device__ __forceinline__ float char_to_float(float p0, float p25, float p75, float p100,
                                               unsigned v) {
    if (v <= 64u)
        return add_rn(p0, mul_rn(mul_rn(sub_rn(p25, p0), (float)v), 1.0f / 64.0f));
    if (v <= 192u)
        return add_rn(p25, mul_rn(mul_rn(sub_rn(p75, p25), (float)(v - 64u)),
                                        1.0f / 128.0f));
    const float prod = mul_rn(sub_rn(p100, p75), (float)(v - 192u));
    return (float)__dadd_rn((double)p75, __ddiv_rn((double)prod, 63.0));
}

__global__ void __launch_bounds__(256) k_cm_expand(const KfCmDesc *__restrict__ desc,
                                                   const uint8_t *__restrict__ blob,
                                                   h16 *__restrict__ out, int ldo,
                                                   int slabs_per_mat) {
    __shared__ h16 tile[kRows * kMaxCols];
    __shared__ float colp[4 * kMaxCols];
    const int m = blockIdx.x / slabs_per_mat;
    const int r0 = (blockIdx.x % slabs_per_mat) * kRows;
    const KfCmDesc d = desc[m];
    if (r0 >= d.rows) return;  // whole workgroup leaves together
    const int nr = min(kRows, d.rows - r0);
    const int cols = d.cols;
    const uint8_t *p = blob + d.payload_off;
    h16 *o = out + (long long)(d.out_row + r0) * ldo;

    if (d.format == KF_CM_ONEBYTE_COLHDR) {
        const uint16_t *hdr = reinterpret_cast<const uint16_t *>(p);
        for (int i = threadIdx.x; i < 4 * cols; i += 256)
            colp[i] = u16_to_float(d.min_value, d.range, hdr[i]);
        __syncthreads();
        const uint8_t *bytes = p + (size_t)cols * 8;
        for (int i = threadIdx.x; i < kRows * cols; i += 256) {
            const int c = i / kRows, r = i % kRows;
            if (r < nr) {
                const unsigned v = bytes[(size_t)c * d.rows + r0 + r];
                tile[r * cols + c] =
                    (h16)char_to_float(colp[4 * c], colp[4 * c + 1], colp[4 * c + 2], colp[4 * c + 3], v);
            }
        }
        __syncthreads();
        for (int i = threadIdx.x; i < nr * cols; i += 256) {
            const int r = i / cols, c = i % cols;
            o[(long long)r * ldo + c] = tile[r * cols + c];
        }
        return;
    }
    // row-major formats: element i of the slab is row r0 + i / cols
    const long long base = (long long)r0 * cols;
    if (d.format == KF_CM_TWOBYTE) {
        const float inc = __fdiv_rn(d.range, 65535.0f);
        const uint16_t *v = reinterpret_cast<const uint16_t *>(p);
        for (int i = threadIdx.x; i < nr * cols; i += 256)
            o[(long long)(i / cols) * ldo + i % cols] =
                (h16)add_rn(d.min_value, mul_rn((float)v[base + i], inc));
    } else if (d.format == KF_CM_ONEBYTE) {
        const float inc = __fdiv_rn(d.range, 255.0f);
        for (int i = threadIdx.x; i < nr * cols; i += 256)
            o[(long long)(i / cols) * ldo + i % cols] =
                (h16)add_rn(d.min_value, mul_rn((float)p[base + i], inc));
    } else {  // KF_CM_FLOAT
        const float *v = reinterpret_cast<const float *>(p);
        for (int i = threadIdx.x; i < nr * cols; i += 256)
            o[(long long)(i / cols) * ldo + i % cols] = (h16)v[base + i];
    }
}

}  // namespace

extern "C" int kf_cm_expand(const KfCmDesc *dev_desc, int nmat, int max_rows, int max_cols,
                            const void *dev_blob, void *dev_out, int ldo) {
    kf_take_pending(__func__);
    if (nmat <= 0) return 0;
    if (!dev_desc || !dev_blob || !dev_out || max_rows <= 0 || max_cols <= 0 ||
        max_cols > kMaxCols || ldo < max_cols) {
        kf_report_error("kf_cm_expand: bad arguments (nmat %d rows %d cols %d ldo %d; cols <= %d)",
                        nmat, max_rows, max_cols, ldo, kMaxCols);
        return -1;
    }
    const int slabs = (max_rows + kRows - 1) / kRows;
    const long long grid = (long long)slabs * nmat;
    if (grid > (1LL << 30)) {
        kf_report_error("kf_cm_expand: grid too large");
        return -1;
    }
    k_cm_expand<<<(unsigned)grid, 256, 0, kf_stream()>>>(dev_desc, (const uint8_t *)dev_blob,
                                                         (h16 *)dev_out, ldo, slabs);
    if (hipGetLastError() != hipSuccess) {
        kf_report_error("kf_cm_expand: launch failed");
        return -1;
    }
    return 0;
}

// Host-side packing: descriptors + payload blob go through one pinned staging buffer
// and one stream-ordered H2D copy into a device staging buffer, then one launch. The
// pinned buffer is reused only after the event recorded behind the previous copy has
// completed, so the caller may free its host arrays as soon as this returns.
namespace {
struct CmStaging {
    std::mutex mu;
    uint8_t *pinned = nullptr;
    void *dev = nullptr;
    size_t cap = 0;
    hipEvent_t done = nullptr;
    bool pending = false;
};
CmStaging g_cm;
}  // namespace

extern "C" int kf_cm_expand_host(const KfCmDesc *desc, int nmat, int max_rows, int max_cols,
                                 const void *blob, size_t blob_bytes, void *dev_out, int ldo) {
    if (nmat <= 0) return 0;
    if (!desc || (!blob && blob_bytes) || !dev_out) {
        kf_report_error("kf_cm_expand_host: null argument");
        return -1;
    }
    for (int i = 0; i < nmat; i++) {  // every access of the kernel stays inside the blob
        const KfCmDesc &d = desc[i];
        long long need = 0;
        if (d.rows <= 0 || d.cols <= 0 || d.cols > max_cols || d.rows > max_rows || d.out_row < 0 ||
            d.payload_off < 0) {
            kf_report_error("kf_cm_expand_host: bad descriptor %d (%dx%d, max %dx%d)", i, d.rows,
                            d.cols, max_rows, max_cols);
            return -1;
        }
        switch (d.format) {
        case KF_CM_ONEBYTE_COLHDR: need = 8LL * d.cols + (long long)d.rows * d.cols; break;
        case KF_CM_TWOBYTE: need = 2LL * d.rows * d.cols; break;
        case KF_CM_ONEBYTE: need = (long long)d.rows * d.cols; break;
        case KF_CM_FLOAT: need = 4LL * d.rows * d.cols; break;
        default: kf_report_error("kf_cm_expand_host: descriptor %d format %d", i, d.format); return -1;
        }
        const int align = d.format == KF_CM_FLOAT ? 4 : (d.format == KF_CM_ONEBYTE ? 1 : 2);
        if (d.payload_off % align || d.payload_off + need > (long long)blob_bytes) {
            kf_report_error("kf_cm_expand_host: descriptor %d payload [%lld, +%lld) outside blob %zu",
                            i, d.payload_off, need, blob_bytes);
            return -1;
        }
    }
    const size_t dbytes = ((size_t)nmat * sizeof(KfCmDesc) + 255) & ~(size_t)255;
    const size_t total = dbytes + blob_bytes;
    std::lock_guard<std::mutex> lock(g_cm.mu);
    if (g_cm.pending) {
        if (hipEventSynchronize(g_cm.done) != hipSuccess) {
            kf_report_error("kf_cm_expand_host: staging event failed");
            return -1;
        }
        g_cm.pending = false;
    }
    if (total > g_cm.cap) {
        if (g_cm.pinned) hipHostFree(g_cm.pinned);
        if (g_cm.dev) hipFree(g_cm.dev);
        g_cm.pinned = nullptr;
        g_cm.dev = nullptr;
        g_cm.cap = 0;
        const size_t cap = total + total / 4;
        if (hipHostMalloc((void **)&g_cm.pinned, cap, hipHostMallocDefault) != hipSuccess ||
            hipMalloc(&g_cm.dev, cap) != hipSuccess) {
            kf_report_error("kf_cm_expand_host: staging allocation of %zu bytes failed", cap);
            return -1;
        }
        g_cm.cap = cap;
        if (!g_cm.done && hipEventCreateWithFlags(&g_cm.done, hipEventDisableTiming) != hipSuccess) {
            kf_report_error("kf_cm_expand_host: event creation failed");
            return -1;
        }
    }
    memcpy(g_cm.pinned, desc, (size_t)nmat * sizeof(KfCmDesc));
    if (blob_bytes) memcpy(g_cm.pinned + dbytes, blob, blob_bytes);
    hipStream_t s = kf_stream();
    if (hipMemcpyAsync(g_cm.dev, g_cm.pinned, total, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipEventRecord(g_cm.done, s) != hipSuccess) {
        kf_report_error("kf_cm_expand_host: staging copy failed");
        return -1;
    }
    g_cm.pending = true;
    return kf_cm_expand((const KfCmDesc *)g_cm.dev, nmat, max_rows, max_cols,
                        (const uint8_t *)g_cm.dev + dbytes, dev_out, ldo);
}
