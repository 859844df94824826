// kf_common.h — shared device/host helpers for the MI355X kaldi-fp16 core.
// gfx950 only: wave64, _Float16 storage, v_cvt_f16_f32 (round-to-nearest-even).
#pragma once
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

typedef _Float16 h16;
typedef _Float16 half4 __attribute__((ext_vector_type(4)));
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef short short4v __attribute__((ext_vector_type(4)));
typedef float float4v __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------
// Per-module thread-local error text, mirroring the reference's
// `static __thread char g_ops_error[512]` pattern (ops.cu:12, bridge.cu:11,
// chain.cu:22, chain_den.cu:27, cgo_interface.cu:12). *_last_error() returns
// NULL when nothing is pending.
// ---------------------------------------------------------------------------
struct KfErr {
    char buf[512];
    void set(const char *fmt, va_list ap) { vsnprintf(buf, sizeof(buf), fmt, ap); }
    const char *get() const { return buf[0] ? buf : nullptr; }
    void clear() { buf[0] = 0; }
};

#define KF_DECLARE_ERR(prefix)                                                  \
    static __thread KfErr prefix##_err_;                                        \
    __attribute__((unused)) static void prefix##_set_error(const char *fmt, ...) { \
        va_list ap;                                                             \
        va_start(ap, fmt);                                                      \
        prefix##_err_.set(fmt, ap);                                             \
        va_end(ap);                                                             \
    }

// current stream (kf_ops.h: kf_set_stream)
hipStream_t kf_stream();

// consume and log an error an earlier HIP call left pending (kf_ops.h): called at the
// top of every entry that checks its own launches with hipGetLastError()
extern "C" int kf_take_pending(const char *where);

// sets the kf_last_error() text from another module (gemm.hip owns the slot)
void kf_report_error(const char *fmt, ...);

// kf_prof_* timing of a launch bracket on the current stream (gemm.hip);
// classes: 0 fused GEMM, 1 wgrad GEMM, 2 chain numerator, 3 chain denominator,
// 4 conv halo fwd / dX, 5 conv halo wgrad, 6 slab reduce (include/kf_ops.h)
enum { KF_PROF_CHAIN_NUM = 2, KF_PROF_CHAIN_DEN = 3 };
int kf_prof_start(int cls, double work);
void kf_prof_stop(int idx);

// persistent per-device scratch (never freed; grows monotonically)
void *kf_workspace(size_t bytes, int slot);
// scratch of the current stream (kf_stream()), never shared with another stream: the
// weight gradients' split-K slabs, which two streams fill at once (bridge.hip)
void *kf_workspace_stream(size_t bytes);

static inline int kf_blocks(long long n, int threads, int cap = 1 << 20) {
    long long b = (n + threads - 1) / threads;
    if (b < 1) b = 1;
    if (b > cap) b = cap;
    return (int)b;
}

__device__ __forceinline__ float h2f(h16 x) { return (float)x; }
__device__ __forceinline__ h16 f2h(float x) { return (h16)x; }  // RNE

__device__ __forceinline__ half8 load_h8(const void *p) {
    return *reinterpret_cast<const half8 *>(p);
}
__device__ __forceinline__ void store_h8(void *p, half8 v) { *reinterpret_cast<half8 *>(p) = v; }
