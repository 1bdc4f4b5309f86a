// Multi-GPU helpers of the C ABI: device binding for host
// threads and the node-local all-gather of the 8-way cross-GPU match (C5) on
// RCCL over xGMI.  The reference has no multi-GPU path (it binds one Detector
// to the calling thread's current device, /root/reference/sift_cuda/interface/
// Detector.hh:26-29); these entry points let a C or C++ host run one Detector
// per device on its own thread and exchange descriptor sets between them
// (include/sift_cuda/MultiDetector.hh builds on them).
//
// RCCL is loaded with dlopen on the first sift_hip_comm_create, so
// libsift_hip.so has no link-time dependency on it: a host that never
// exchanges sets never loads librccl.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <mutex>
#include <string>
#include <vector>

#include "sift_hip.h"
#include "sift_kernels.h"

namespace {

struct Rccl {
    void* so = nullptr;
    ncclResult_t (*commInitAll)(ncclComm_t*, int, const int*) = nullptr;
    ncclResult_t (*commDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*allGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*groupStart)() = nullptr;
    ncclResult_t (*groupEnd)() = nullptr;
    const char* (*errorString)(ncclResult_t) = nullptr;
};

// dlopen once per process (the library stays loaded); std::call_once makes
// the lazy load safe from several host threads.
Rccl* rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
    for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
        r.so = dlopen(name, RTLD_NOW | RTLD_LOCAL);
        if (r.so) break;
    }
    if (!r.so) return;
    r.commInitAll = (decltype(r.commInitAll))dlsym(r.so, "ncclCommInitAll");
    r.commDestroy = (decltype(r.commDestroy))dlsym(r.so, "ncclCommDestroy");
    r.allGather = (decltype(r.allGather))dlsym(r.so, "ncclAllGather");
    r.groupStart = (decltype(r.groupStart))dlsym(r.so, "ncclGroupStart");
    r.groupEnd = (decltype(r.groupEnd))dlsym(r.so, "ncclGroupEnd");
    r.errorString = (decltype(r.errorString))dlsym(r.so, "ncclGetErrorString");
    if (!r.commInitAll || !r.commDestroy || !r.allGather || !r.groupStart || !r.groupEnd || !r.errorString) {
        dlclose(r.so);
        r.so = nullptr;
    }
    });
    return r.so ? &r : nullptr;
}

}  // namespace

struct sift_hip_comm {
    std::vector<int> devices;
    std::vector<ncclComm_t> comms;
    std::vector<hipStream_t> streams;  // one per rank, non-blocking
    ~sift_hip_comm() {
        Rccl* r = rccl();
        for (size_t k = 0; k < comms.size(); k++) {
            (void)hipSetDevice(devices[k]);
            if (streams[k]) (void)hipStreamDestroy(streams[k]);
            if (comms[k] && r) (void)r->commDestroy(comms[k]);
        }
    }
};

// Errors go through the ABI's thread-local message (sift_hip_last_error).
namespace {
int mfail(int code, const std::string& msg) {
    sift_amd::set_last_error(msg);
    return code;
}
}  // namespace

#define MHIPCHK(expr)                                                                                    \
    do {                                                                                                 \
        hipError_t e_ = (expr);                                                                          \
        if (e_ != hipSuccess) return mfail(SIFT_HIP_ERR_RUNTIME, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

extern "C" {

int sift_hip_set_device(int device) {
    MHIPCHK(hipSetDevice(device));
    return SIFT_HIP_OK;
}

int sift_hip_memcpy_d2d(void* dst, const void* src, size_t bytes, void* stream) {
    if (!dst || !src) return mfail(SIFT_HIP_ERR_INVALID, "null pointer");
    MHIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, (hipStream_t)stream));
    if (!stream) MHIPCHK(hipStreamSynchronize(nullptr));
    return SIFT_HIP_OK;
}

int sift_hip_comm_create(int ndev, const int* devices, sift_hip_comm_t* out) {
    if (!out || ndev < 1 || !devices) return mfail(SIFT_HIP_ERR_INVALID, "bad communicator arguments");
    *out = nullptr;
    for (int i = 0; i < ndev; i++)
        for (int j = 0; j < i; j++)
            if (devices[i] == devices[j])
                return mfail(SIFT_HIP_ERR_INVALID, "RCCL needs distinct devices (one rank per GPU)");
    Rccl* r = rccl();
    if (!r) return mfail(SIFT_HIP_ERR_RUNTIME, "librccl could not be loaded");
    auto* c = new sift_hip_comm();
    c->devices.assign(devices, devices + ndev);
    c->comms.assign(ndev, nullptr);
    c->streams.assign(ndev, nullptr);
    const ncclResult_t rc = r->commInitAll(c->comms.data(), ndev, devices);
    if (rc != ncclSuccess) {
        const std::string msg = std::string("ncclCommInitAll: ") + r->errorString(rc);
        c->comms.assign(ndev, nullptr);
        delete c;
        return mfail(SIFT_HIP_ERR_RUNTIME, msg);
    }
    for (int k = 0; k < ndev; k++) {
        if (hipSetDevice(devices[k]) != hipSuccess ||
            hipStreamCreateWithFlags(&c->streams[k], hipStreamNonBlocking) != hipSuccess) {
            delete c;
            return mfail(SIFT_HIP_ERR_RUNTIME, "stream creation failed");
        }
    }
    *out = c;
    return SIFT_HIP_OK;
}

int sift_hip_comm_destroy(sift_hip_comm_t c) {
    delete c;
    return SIFT_HIP_OK;
}

int sift_hip_comm_size(sift_hip_comm_t c, int* n) {
    if (!c || !n) return mfail(SIFT_HIP_ERR_INVALID, "null argument");
    *n = (int)c->devices.size();
    return SIFT_HIP_OK;
}

int sift_hip_comm_allgather(sift_hip_comm_t c, const void* const* send, void* const* recv, size_t bytes,
                            void* const* streams) {
    if (!c || !send || !recv) return mfail(SIFT_HIP_ERR_INVALID, "null argument");
    Rccl* r = rccl();
    const int n = (int)c->devices.size();
    if (r->groupStart() != ncclSuccess) return mfail(SIFT_HIP_ERR_RUNTIME, "ncclGroupStart failed");
    for (int k = 0; k < n; k++) {
        const hipError_t e = hipSetDevice(c->devices[k]);
        if (e != hipSuccess) {
            (void)r->groupEnd();  // never leave the thread's RCCL group open
            return mfail(SIFT_HIP_ERR_RUNTIME, std::string("hipSetDevice: ") + hipGetErrorString(e));
        }
        hipStream_t s = streams && streams[k] ? (hipStream_t)streams[k] : c->streams[k];
        const ncclResult_t rc = r->allGather(send[k], recv[k], bytes, ncclChar, c->comms[k], s);
        if (rc != ncclSuccess) {
            (void)r->groupEnd();
            return mfail(SIFT_HIP_ERR_RUNTIME, std::string("ncclAllGather: ") + r->errorString(rc));
        }
    }
    const ncclResult_t rc = r->groupEnd();
    if (rc != ncclSuccess) return mfail(SIFT_HIP_ERR_RUNTIME, std::string("ncclGroupEnd: ") + r->errorString(rc));
    if (!streams)
        for (int k = 0; k < n; k++) {
            MHIPCHK(hipSetDevice(c->devices[k]));
            MHIPCHK(hipStreamSynchronize(c->streams[k]));
        }
    return SIFT_HIP_OK;
}

}  // extern "C"
