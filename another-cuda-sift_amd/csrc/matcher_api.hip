// Matcher handle (sift_hip_matcher_*, sift_hip_match_*) and the descriptor
// sidecar registry of libsift_hip.so; the kernels are match.hip.  Replaces
// /root/reference/sift_cuda/sift_func/Match.cu:8-33 (matchBruteForce).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>

#include "detector_state.h"
#include "sift_match.h"

namespace sift_amd {
namespace det {

// Matcher sidecars of the descriptor buffers the detector handles hand out
// (one per results slot and frame of every lane): exact buffer base -> its
// int8 codes and key biases (sift_kernels.h Sidecar).  sift_hip_match_* look
// the query and train pointers up and, when both are detector buffers, match
// their codes directly (k_match_direct) instead of converting the fp16 rows.
// A caller that writes into a detector descriptor buffer declares it
// (sift_hip_descriptors_written, DeviceBuffer::mutable_data): the entry is
// then stale -- matches on the buffer convert its fp16 rows -- until the
// detector launches a frame into that buffer again (sidecar_refreshed).
struct SidecarReg {
    const uint16_t* desc;
    Sidecar side;
    int cap;
    const void* owner;
    bool stale;
};
std::mutex g_side_mu;
std::vector<SidecarReg> g_side;
std::atomic<int> g_side_stale{0};  // stale entries (the per-frame refresh is free while 0)

void register_sidecar(const void* owner, const uint16_t* desc, Sidecar side, int cap) {
    std::lock_guard<std::mutex> g(g_side_mu);
    g_side.push_back(SidecarReg{desc, side, cap, owner, false});
}
void unregister_sidecars(const void* owner) {
    std::lock_guard<std::mutex> g(g_side_mu);
    for (const SidecarReg& r : g_side)
        if (r.owner == owner && r.stale) g_side_stale--;
    g_side.erase(std::remove_if(g_side.begin(), g_side.end(), [&](const SidecarReg& r) { return r.owner == owner; }),
                 g_side.end());
}
bool find_sidecar(const uint16_t* desc, int n, Sidecar* out) {
    std::lock_guard<std::mutex> g(g_side_mu);
    for (const SidecarReg& r : g_side)
        if (r.desc == desc && n <= r.cap && !r.stale) {
            *out = r.side;
            return true;
        }
    return false;
}
bool sidecar_written(const uint16_t* desc) {
    std::lock_guard<std::mutex> g(g_side_mu);
    bool found = false;
    for (SidecarReg& r : g_side)
        if (r.desc == desc) {
            found = true;
            if (!r.stale) {
                r.stale = true;
                g_side_stale++;
            }
        }
    return found;
}
void sidecar_refreshed(const uint16_t* desc) {
    if (g_side_stale.load() == 0) return;
    std::lock_guard<std::mutex> g(g_side_mu);
    for (SidecarReg& r : g_side)
        if (r.desc == desc && r.stale) {
            r.stale = false;
            g_side_stale--;
        }
}

}  // namespace det
}  // namespace sift_amd

struct sift_hip_matcher {
    int device = 0;
    int maxQ = 0, maxT = 0, maxP = 0;
    unsigned long long* dKeys = nullptr;  // running top-2 keys per (pair, query), all ones between calls
    unsigned* dDone = nullptr;            // finished splits per (pair, 256-query block), zero between calls
    int* dMatch = nullptr;
    int8_t* dCodes = nullptr;             // int8 codes of a call's distinct sets (k_match_prep)
    int* dRowKeys = nullptr;              // key bias per code row; row codeRows: the zero/padding sentinel
    unsigned* dFlags = nullptr;           // per set slot: == epoch if the set is not all integers 0..255
    long codeRows = 0;
    unsigned epoch = 0;
    bool sidecars = true;  // single pairs of detector buffers: match their sidecar codes (k_match_direct)
    ~sift_hip_matcher() {
        (void)hipSetDevice(device);
        for (void* p : {(void*)dKeys, (void*)dDone, (void*)dMatch, (void*)dCodes, (void*)dRowKeys, (void*)dFlags})
            if (p) (void)hipFree(p);
    }
};

extern "C" {

int sift_hip_matcher_create(int device, int max_query, int max_train, int max_pairs, sift_hip_matcher_t* out) {
    if (!out || max_query <= 0 || max_train <= 0 || max_pairs <= 0 || max_pairs > kMaxMatchPairs)
        return fail(SIFT_HIP_ERR_INVALID, "bad matcher limits");
    *out = nullptr;
    auto* m = new sift_hip_matcher();
    if (device < 0) {
        if (hipGetDevice(&m->device) != hipSuccess) m->device = 0;
    } else {
        m->device = device;
    }
    m->maxQ = max_query;
    m->maxT = max_train;
    m->maxP = max_pairs;
    // Distinct sets of a call: at most 2 per pair, each at most max(maxQ, maxT) rows.
    m->codeRows = 2L * max_pairs * std::max(max_query, max_train);
    const size_t nkeys = 2 * (size_t)max_pairs * max_query;
    const size_t nblk = (size_t)max_pairs * ((max_query + kMatchQB - 1) / kMatchQB);
    if (hipSetDevice(m->device) != hipSuccess ||
        hipMalloc((void**)&m->dKeys, sizeof(unsigned long long) * nkeys) != hipSuccess ||
        hipMalloc((void**)&m->dDone, sizeof(unsigned) * nblk) != hipSuccess ||
        hipMalloc((void**)&m->dMatch, sizeof(int) * (size_t)max_pairs * max_query) != hipSuccess ||
        hipMalloc((void**)&m->dCodes, (size_t)(m->codeRows + 1) * 128) != hipSuccess ||
        hipMalloc((void**)&m->dRowKeys, sizeof(int) * (size_t)(m->codeRows + 1)) != hipSuccess ||
        hipMemset(m->dCodes + (size_t)m->codeRows * 128, 0, 128) != hipSuccess ||
        hipMemcpy(m->dRowKeys + m->codeRows, &kMatchPadKey, sizeof(int), hipMemcpyHostToDevice) != hipSuccess ||
        hipMalloc((void**)&m->dFlags, sizeof(unsigned) * 2 * kMaxMatchPairs) != hipSuccess ||
        hipMemset(m->dKeys, 0xff, sizeof(unsigned long long) * nkeys) != hipSuccess ||
        hipMemset(m->dDone, 0, sizeof(unsigned) * nblk) != hipSuccess ||
        hipMemset(m->dFlags, 0, sizeof(unsigned) * 2 * kMaxMatchPairs) != hipSuccess ||
        hipDeviceSynchronize() != hipSuccess) {
        delete m;
        return fail(SIFT_HIP_ERR_NOMEM, "matcher allocation failed");
    }
    *out = m;
    return SIFT_HIP_OK;
}

int sift_hip_matcher_set_sidecars(sift_hip_matcher_t m, int enable) {
    if (!m) return fail(SIFT_HIP_ERR_INVALID, "null matcher");
    m->sidecars = enable != 0;
    return SIFT_HIP_OK;
}

int sift_hip_matcher_destroy(sift_hip_matcher_t m) {
    delete m;
    return SIFT_HIP_OK;
}

int sift_hip_match_batched(sift_hip_matcher_t m, int P, const uint16_t* const* q, const int* nq,
                           const uint16_t* const* t, const int* nt, float ratio, int ratio_on_squared, int* idx2,
                           float* d2, int* match, void* stream) {
    if (!m || P <= 0 || P > m->maxP || !q || !nq || !t || !nt) return fail(SIFT_HIP_ERR_INVALID, "bad batch");
    Sidecar sq{}, st{};
    if (P == 1 && m->sidecars && nq[0] > 0 && nt[0] > 0 && nq[0] <= m->maxQ && nt[0] <= m->maxT &&
        find_sidecar(q[0], nq[0], &sq) && find_sidecar(t[0], nt[0], &st)) {
        // Both sets are detector buffers: their codes are ready (no conversion).
        HIPCHK(hipSetDevice(m->device));
        const MatchPair pr{q[0], t[0], nq[0], nt[0], 0, 0, 0, 0, 0, 0, 0};
        launch_match_direct(pr, sq.codes, sq.keys, st.codes, st.keys, m->dCodes + (size_t)m->codeRows * 128,
                            m->dRowKeys + m->codeRows, m->dKeys, m->dDone, ratio, ratio_on_squared, idx2, d2, match,
                            (hipStream_t)stream);
        HIPCHK(hipGetLastError());
        return SIFT_HIP_OK;
    }
    MatchBatch b{};
    MatchSets sets{};
    b.P = P;
    // Distinct sets by pointer (a set used by several pairs is prepared once).
    auto set_of = [&](const uint16_t* ptr, int n) {
        for (int k = 0; k < sets.nsets; k++)
            if (sets.set[k].src == ptr) {
                sets.set[k].n = std::max(sets.set[k].n, n);
                return k;
            }
        sets.set[sets.nsets] = MatchSet{ptr, n, 0};
        return sets.nsets++;
    };
    int off = 0, maxq = 1, maxt = 1;
    for (int p = 0; p < P; p++) {
        if (nq[p] < 0 || nt[p] < 0 || nq[p] > m->maxQ || nt[p] > m->maxT)
            return fail(SIFT_HIP_ERR_INVALID, "pair size exceeds matcher limits");
        if ((nq[p] && !q[p]) || (nt[p] && !t[p])) return fail(SIFT_HIP_ERR_INVALID, "null descriptor pointer");
        const int qs = set_of(q[p], nq[p]), ts = set_of(t[p], nt[p]);
        b.pair[p] = MatchPair{q[p], t[p], nq[p], nt[p], off, qs, ts, 0, 0, 0, 0};
        off += nq[p];
        maxq = std::max(maxq, nq[p]);
        maxt = std::max(maxt, nt[p]);
    }
    long row = 0;
    for (int k = 0; k < sets.nsets; k++) {
        sets.set[k].row0 = (int)row;
        row += sets.set[k].n;
        sets.maxn = std::max(sets.maxn, sets.set[k].n);
    }
    if (row > m->codeRows) return fail(SIFT_HIP_ERR_INVALID, "descriptor sets exceed the matcher's code buffer");
    for (int p = 0; p < P; p++) {
        b.pair[p].qrow0 = b.pair[p].qkrow0 = sets.set[b.pair[p].qset].row0;
        b.pair[p].trow0 = b.pair[p].tkrow0 = sets.set[b.pair[p].tset].row0;
    }
    m->epoch = m->epoch + 1 == 0 ? 1 : m->epoch + 1;  // flags from earlier calls never equal it
    HIPCHK(hipSetDevice(m->device));
    const MatchPlan plan = match_plan(maxq, maxt, P);
    launch_match(sets, b, plan, m->maxQ, m->dCodes, m->dRowKeys, (int)m->codeRows, m->dFlags, m->epoch, m->dKeys, m->dDone, ratio,
                 ratio_on_squared, idx2, d2, match, (hipStream_t)stream);
    HIPCHK(hipGetLastError());
    return SIFT_HIP_OK;
}

int sift_hip_match_codes_batched(sift_hip_matcher_t m, const int8_t* codes, const int* keys, int P, const int* qrow0,
                                 const int* qkey0, const int* nq, const int* trow0, const int* tkey0, const int* nt,
                                 float ratio, int ratio_on_squared, int* idx2, float* d2, int* match, void* stream) {
    if (!m || P <= 0 || P > m->maxP || !codes || !keys || !qrow0 || !qkey0 || !nq || !trow0 || !tkey0 || !nt)
        return fail(SIFT_HIP_ERR_INVALID, "bad code batch");
    MatchBatch b{};
    b.P = P;
    int off = 0, maxq = 1, maxt = 1;
    for (int p = 0; p < P; p++) {
        if (nq[p] < 0 || nt[p] < 0 || nq[p] > m->maxQ || nt[p] > m->maxT)
            return fail(SIFT_HIP_ERR_INVALID, "pair size exceeds matcher limits");
        if (qrow0[p] < 0 || trow0[p] < 0 || qkey0[p] < 0 || tkey0[p] < 0)
            return fail(SIFT_HIP_ERR_INVALID, "negative set row");
        b.pair[p] = MatchPair{nullptr, nullptr, nq[p], nt[p], off, 0, 0, qrow0[p], trow0[p], qkey0[p], tkey0[p]};
        off += nq[p];
        maxq = std::max(maxq, nq[p]);
        maxt = std::max(maxt, nt[p]);
    }
    HIPCHK(hipSetDevice(m->device));
    const MatchPlan plan = match_plan(maxq, maxt, std::max(P, 2));  // the batched kernel's plan, also for one pair
    launch_match_codes(b, plan, m->maxQ, codes, keys, m->dCodes + (size_t)m->codeRows * 128, m->dRowKeys + m->codeRows,
                       m->dKeys, m->dDone, ratio, ratio_on_squared, idx2, d2, match, (hipStream_t)stream);
    HIPCHK(hipGetLastError());
    return SIFT_HIP_OK;
}

int sift_hip_descriptors_written(const uint16_t* desc) {
    if (!desc) return fail(SIFT_HIP_ERR_INVALID, "null descriptor buffer");
    (void)sidecar_written(desc);  // a foreign buffer has no sidecar: nothing to drop
    return SIFT_HIP_OK;
}

int sift_hip_match_device(sift_hip_matcher_t m, const uint16_t* q, int nq, const uint16_t* t, int nt, float ratio,
                          int ratio_on_squared, int* idx2, float* d2, int* match, void* stream) {
    return sift_hip_match_batched(m, 1, &q, &nq, &t, &nt, ratio, ratio_on_squared, idx2, d2, match, stream);
}

int sift_hip_match_plan(int max_query, int max_train, int pairs, int* splits, int* waves) {
    if (max_query < 0 || max_train < 0 || pairs < 1 || !splits) return fail(SIFT_HIP_ERR_INVALID, "bad match shape");
    const MatchPlan pl = match_plan(max_query, max_train, pairs);
    *splits = pl.S;
    if (waves) *waves = pl.nw;
    return SIFT_HIP_OK;
}

int sift_hip_match_host(sift_hip_matcher_t m, const uint16_t* q, int nq, const uint16_t* t, int nt, float ratio,
                        int ratio_on_squared, int* out) {
    if (!m || !out) return fail(SIFT_HIP_ERR_INVALID, "null argument");
    if (nq <= 0) return SIFT_HIP_OK;
    int rc = sift_hip_match_device(m, q, nq, t, nt, ratio, ratio_on_squared, nullptr, nullptr, m->dMatch, nullptr);
    if (rc) return rc;
    HIPCHK(hipMemcpy(out, m->dMatch, sizeof(int) * nq, hipMemcpyDeviceToHost));
    return SIFT_HIP_OK;
}

int sift_hip_device_count(int* n) {
    if (!n) return fail(SIFT_HIP_ERR_INVALID, "null argument");
    if (hipGetDeviceCount(n) != hipSuccess) *n = 0;
    return SIFT_HIP_OK;
}
int sift_hip_malloc(void** p, size_t bytes) {
    HIPCHK(hipMalloc(p, bytes));
    return SIFT_HIP_OK;
}
int sift_hip_free(void* p) {
    HIPCHK(hipFree(p));
    return SIFT_HIP_OK;
}
int sift_hip_memcpy_h2d(void* dst, const void* src, size_t bytes) {
    HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
    return SIFT_HIP_OK;
}
int sift_hip_memcpy_d2h(void* dst, const void* src, size_t bytes) {
    HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
    return SIFT_HIP_OK;
}
int sift_hip_device_sync(void) {
    HIPCHK(hipDeviceSynchronize());
    return SIFT_HIP_OK;
}

}  // extern "C"