// dp.cpp — data-parallel gradient exchange over RCCL (include/kf_dp.h).
//
// The reference trains on one device (cpp/cuda/bridge.cu:38-47); SURVEY §8e asks
// for one process per GPU with the weight gradient averaged over ranks by an
// all-reduce over xGMI, issued bucket by bucket while the backward still runs.
// This module owns the communicator and a high-priority communication stream:
// every exchange is gated by an event recorded on the compute stream
// (kf_get_stream()) after the producing kernels were enqueued, so the host never
// blocks and the compute stream only waits once, at kf_dp_join.
// Host code only (no kernels). RCCL is bound at the first kf_dp call with dlopen:
// the copy already mapped into the process (torch's, soname librccl.so.1) when there
// is one, else ROCm's. Two RCCL copies in one process (a load-time dependency on
// ROCm's beside torch's) interpose each other's globals and corrupt the heap at exit.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <vector>

#include "../../include/kf_dp.h"

extern "C" int kf_take_pending(const char *where);  // bridge.hip (kf_ops.h)

hipStream_t kf_stream();
// ops.hip: buf[i] = (buf[i] + peer[i]) * 0.5f on `s` (the KF_DP_DEBUG_PEER_MEAN exchange)
int kf_dp_debug_mean_launch(float *buf, const float *peer, size_t n, hipStream_t s);

namespace {
__thread char g_err[512];
void set_err(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
}
bool hip_ok(hipError_t e, const char *what) {
    if (e == hipSuccess) return true;
    set_err("%s: %s", what, hipGetErrorString(e));
    return false;
}
const struct Rccl *rccl();
bool nccl_ok(ncclResult_t r, const char *what);
constexpr size_t kGates = 64;  // gate events in flight (buckets of one backward)

struct Rccl {
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) comm_init_rank = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclAllReduce) all_reduce = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
};
// nullptr (with the error set) when no RCCL can be loaded
const Rccl *rccl() {
    static Rccl r;
    static bool tried = false;
    if (tried) return r.all_reduce ? &r : nullptr;
    tried = true;
    void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
        set_err("RCCL not found (librccl.so.1): %s", dlerror());
        return nullptr;
    }
    r.get_unique_id = (decltype(r.get_unique_id))dlsym(h, "ncclGetUniqueId");
    r.comm_init_rank = (decltype(r.comm_init_rank))dlsym(h, "ncclCommInitRank");
    r.comm_destroy = (decltype(r.comm_destroy))dlsym(h, "ncclCommDestroy");
    r.error_string = (decltype(r.error_string))dlsym(h, "ncclGetErrorString");
    r.all_reduce = (decltype(r.all_reduce))dlsym(h, "ncclAllReduce");
    if (!r.get_unique_id || !r.comm_init_rank || !r.comm_destroy || !r.error_string || !r.all_reduce) {
        set_err("RCCL: missing symbols");
        r.all_reduce = nullptr;
        return nullptr;
    }
    return &r;
}
bool nccl_ok(ncclResult_t r, const char *what) {
    if (r == ncclSuccess) return true;
    set_err("%s: %s", what, rccl()->error_string(r));
    return false;
}
}  // namespace

struct KfDp {
    ncclComm_t comm = nullptr;
    hipStream_t comm_stream = nullptr;
    hipEvent_t gates[kGates] = {};  // recorded on the compute stream, one per bucket
    size_t next_gate = 0;
    hipEvent_t done = nullptr;      // recorded on the comm stream by kf_dp_join
    int rank = 0, world = 1, device = 0;
    long long launches = 0, values = 0;
    // kf_dp_debug: test hooks on the communication stream (0: off)
    int debug = 0;
    const float *dbg_base = nullptr;  // the gradient buffer the buckets lie in
    float *dbg_aux = nullptr;         // snapshot / peer buffer, same layout
    size_t dbg_n = 0;                 // values in both
};

extern "C" const char *kf_dp_last_error(void) { return g_err[0] ? g_err : nullptr; }

extern "C" int kf_dp_unique_id(unsigned char id[KF_DP_ID_BYTES]) {
    static_assert(sizeof(ncclUniqueId) == KF_DP_ID_BYTES, "ncclUniqueId size");
    ncclUniqueId u;
    if (!id) {
        set_err("kf_dp_unique_id: null");
        return -1;
    }
    const Rccl *R = rccl();
    if (!R || !nccl_ok(R->get_unique_id(&u), "ncclGetUniqueId")) return -1;
    memcpy(id, &u, sizeof u);
    return 0;
}

extern "C" KfDp *kf_dp_create(int rank, int world, const unsigned char id[KF_DP_ID_BYTES], int device) {
    g_err[0] = 0;
    if (!id || world < 1 || rank < 0 || rank >= world) {
        set_err("kf_dp_create: bad rank %d / world %d", rank, world);
        return nullptr;
    }
    if (!rccl()) return nullptr;
    KfDp *dp = new KfDp;
    dp->rank = rank;
    dp->world = world;
    dp->device = device;
    int least = 0, greatest = 0;
    ncclUniqueId u;
    memcpy(&u, id, sizeof u);
    bool ok = hip_ok(hipSetDevice(device), "hipSetDevice") &&
              hip_ok(hipDeviceGetStreamPriorityRange(&least, &greatest), "hipDeviceGetStreamPriorityRange") &&
              // greatest priority: the exchange kernels dispatch ahead of queued GEMM tiles
              hip_ok(hipStreamCreateWithPriority(&dp->comm_stream, hipStreamNonBlocking, greatest),
                     "comm stream") &&
              hip_ok(hipEventCreateWithFlags(&dp->done, hipEventDisableTiming), "event");
    for (size_t i = 0; ok && i < kGates; ++i)
        ok = hip_ok(hipEventCreateWithFlags(&dp->gates[i], hipEventDisableTiming), "event");
    if (!ok || !nccl_ok(rccl()->comm_init_rank(&dp->comm, world, u, rank), "ncclCommInitRank")) {
        kf_dp_free(dp);
        return nullptr;
    }
    return dp;
}

extern "C" void kf_dp_free(KfDp *dp) {
    if (!dp) return;
    if (dp->comm_stream) (void)hipStreamSynchronize(dp->comm_stream);
    if (dp->comm) (void)rccl()->comm_destroy(dp->comm);
    for (hipEvent_t e : dp->gates)
        if (e) (void)hipEventDestroy(e);
    if (dp->done) (void)hipEventDestroy(dp->done);
    if (dp->comm_stream) (void)hipStreamDestroy(dp->comm_stream);
    delete dp;
}

extern "C" int kf_dp_rank(const KfDp *dp) { return dp ? dp->rank : -1; }
extern "C" int kf_dp_world(const KfDp *dp) { return dp ? dp->world : -1; }

extern "C" int kf_dp_allreduce_mean_async(KfDp *dp, float *buf, size_t count) {
    kf_take_pending(__func__);
    if (!dp || (!buf && count)) {
        set_err("kf_dp_allreduce_mean_async: null");
        return -1;
    }
    if (!count) return 0;
    // reusing a gate event is safe: hipStreamWaitEvent captures its state at the call
    hipEvent_t gate = dp->gates[dp->next_gate];
    dp->next_gate = (dp->next_gate + 1) % kGates;
    if (!hip_ok(hipEventRecord(gate, kf_stream()), "hipEventRecord") ||
        !hip_ok(hipStreamWaitEvent(dp->comm_stream, gate, 0), "hipStreamWaitEvent"))
        return -1;
    // the hooks apply to buckets inside [grad_base, grad_base + n) only; any other
    // buffer would send the snapshot / peer mean past the end of aux
    const bool dbg = dp->debug != 0;
    if (dbg && (buf < dp->dbg_base || (size_t)(buf - dp->dbg_base) > dp->dbg_n ||
                count > dp->dbg_n - (size_t)(buf - dp->dbg_base))) {
        set_err("kf_dp_allreduce_mean_async: debug hooks on, bucket outside the registered gradient");
        return -1;
    }
    float *aux = dbg ? dp->dbg_aux + (buf - dp->dbg_base) : nullptr;
    // what the exchange would send, captured at the moment it starts
    if (dbg && (dp->debug & KF_DP_DEBUG_SNAPSHOT) &&
        !hip_ok(hipMemcpyAsync(aux, buf, count * 4, hipMemcpyDeviceToDevice, dp->comm_stream), "snapshot"))
        return -1;
    // also at world 1 (identity), so a one-GPU run exercises the same path
    if (!nccl_ok(rccl()->all_reduce(buf, buf, count, ncclFloat32, ncclAvg, dp->comm, dp->comm_stream),
                 "ncclAllReduce"))
        return -1;
    if (dbg && (dp->debug & KF_DP_DEBUG_PEER_MEAN) && kf_dp_debug_mean_launch(buf, aux, count, dp->comm_stream) != 0) {
        set_err("peer mean: %s", hipGetErrorString(hipGetLastError()));
        return -1;
    }
    dp->launches++;
    dp->values += (long long)count;
    return 0;
}

extern "C" int kf_dp_debug(KfDp *dp, int mode, const float *grad_base, float *aux_base, size_t count) {
    if (!dp || (mode & ~(KF_DP_DEBUG_SNAPSHOT | KF_DP_DEBUG_PEER_MEAN)) ||
        (mode && (!grad_base || !aux_base || !count)) ||
        ((mode & KF_DP_DEBUG_SNAPSHOT) && (mode & KF_DP_DEBUG_PEER_MEAN))) {
        set_err("kf_dp_debug: bad arguments");
        return -1;
    }
    dp->debug = mode;
    dp->dbg_base = mode ? grad_base : nullptr;
    dp->dbg_aux = mode ? aux_base : nullptr;
    dp->dbg_n = mode ? count : 0;
    return 0;
}

extern "C" int kf_dp_join(KfDp *dp) {
    if (!dp) {
        set_err("kf_dp_join: null");
        return -1;
    }
    if (!hip_ok(hipEventRecord(dp->done, dp->comm_stream), "hipEventRecord") ||
        !hip_ok(hipStreamWaitEvent(kf_stream(), dp->done, 0), "hipStreamWaitEvent"))
        return -1;
    return 0;
}

extern "C" int kf_dp_allreduce_mean(KfDp *dp, float *buf, size_t count) {
    return kf_dp_allreduce_mean_async(dp, buf, count) == 0 ? kf_dp_join(dp) : -1;
}

extern "C" int kf_dp_allreduce_sum_f64(KfDp *dp, double *buf, size_t count) {
    if (!dp || (!buf && count)) {
        set_err("kf_dp_allreduce_sum_f64: null");
        return -1;
    }
    if (!count || dp->world == 1) return 0;
    hipEvent_t gate = dp->gates[dp->next_gate];
    dp->next_gate = (dp->next_gate + 1) % kGates;
    if (!hip_ok(hipEventRecord(gate, kf_stream()), "hipEventRecord") ||
        !hip_ok(hipStreamWaitEvent(dp->comm_stream, gate, 0), "hipStreamWaitEvent") ||
        !nccl_ok(rccl()->all_reduce(buf, buf, count, ncclFloat64, ncclSum, dp->comm, dp->comm_stream),
                 "ncclAllReduce"))
        return -1;
    return kf_dp_join(dp);
}

extern "C" int kf_dp_stats(const KfDp *dp, long long *launches, long long *values) {
    if (!dp) return -1;
    if (launches) *launches = dp->launches;
    if (values) *values = dp->values;
    return 0;
}

extern "C" int kf_dp_plan(int nsteps, const long long *lo, const long long *hi, long long total,
                          long long bucket_elems, int max_buckets, int *after_step, long long *begin,
                          long long *end) {
    if (nsteps < 0 || total < 0 || max_buckets < 1 || (nsteps && (!lo || !hi)) || !after_step || !begin ||
        !end) {
        set_err("kf_dp_plan: bad arguments");
        return -1;
    }
    for (int i = 0; i < nsteps; ++i)
        if (lo[i] < 0 || hi[i] < lo[i] || hi[i] > total) {
            set_err("kf_dp_plan: group %d [%lld, %lld) outside [0, %lld]", i, lo[i], hi[i], total);
            return -1;
        }
    // [top, total) is covered by the buckets emitted so far; a group may only write
    // below top. A cut after group i exchanges [lo[i], top): every group visited so
    // far lies below top and is complete, and the buckets partition [0, total).
    int nb = 0;
    long long top = total;
    for (int i = 0; i < nsteps; ++i) {
        if (hi[i] == lo[i]) continue;
        if (hi[i] > top) {  // out of order: one bucket after the backward
            nb = 0;
            top = total;
            break;
        }
        if (lo[i] > 0 && top - lo[i] >= bucket_elems && nb + 1 < max_buckets) {
            after_step[nb] = i;
            begin[nb] = lo[i];
            end[nb] = top;
            ++nb;
            top = lo[i];
        }
    }
    if (top > 0 || nb == 0) {
        after_step[nb] = nsteps;
        begin[nb] = 0;
        end[nb] = top;
        ++nb;
    }
    return nb;
}
