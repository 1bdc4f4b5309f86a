// Matcher launch interface (match.hip) used by detector.hip's C ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sift_amd {

constexpr int kMaxMatchPairs = 64;
constexpr int kMatchQB = 128;       // queries per workgroup, smallest plan (done counters are sized per kMatchQB block)
constexpr int kMatchTileRows = 32;  // train rows per MFMA tile
constexpr int kChunkTiles = 8;      // train tiles per LDS chunk (32 KiB of codes + 1 KiB of keys, double buffered)
constexpr int kMatchWgPerCu = 2;    // workgroups per CU the kernel is register-budgeted for
constexpr int kMatchPadKey = -2140000000;  // key bias of a padding row (below every valid key)

struct MatchPair {
    const uint16_t* q;  // nq x 128 half, row-major
    const uint16_t* t;  // nt x 128 half, row-major
    int nq, nt;
    int out_off;        // output row offset of this pair
    int qset, tset;     // this call's prepared sets (k_match_prep) holding q and t
    int qrow0, trow0;   // their first int8 code row
    int qkrow0, tkrow0; // their first key bias (prepared sets: = qrow0 / trow0; gathered code buffers may differ)
};
static_assert(sizeof(MatchPair) == 56, "kernarg layout");

// Passed by value: lives in the kernarg segment (64 x 56 B = 3.5 KiB).
struct MatchBatch {
    MatchPair pair[kMaxMatchPairs];
    int P;
};

// A distinct descriptor set of one call (sets are deduplicated by pointer: the
// 8-way match has 8 sets for 56 pairs): n rows at src -> codes row0 ...
struct MatchSet {
    const uint16_t* src;
    int n, row0;
};
struct MatchSets {
    MatchSet set[2 * kMaxMatchPairs];
    int nsets, maxn;
};

// Launch plan: waves per workgroup (64 queries per wave) and, for the fused
// single-pair kernel, train splits S (the train tiles are cut into S
// contiguous ranges, one workgroup per (query block, range), merged through
// the keys scratch); batched splits are whole key groups.
struct MatchPlan {
    int nw, S;
};
MatchPlan match_plan(int max_nq, int max_nt, int P);
// codes / rowkeys: int8 code rows (128 B) and per row the key bias
// -(256 |code|^2 + (row mod 256)); row `sentinel` of both is a zero code row with
// the padding key (written once at allocation, never by a call); capacity for the
// call's sets; flags: one word per set slot, == epoch when that set holds a
// value that is not an integer 0..255 (matched by the general f16 path).
// keys: 2 x u64 per (pair, query), all ones between calls; done: a counter per
// (pair, kMatchQB-query block), zero between calls (the merging workgroup resets both).
void launch_match(const MatchSets& sets, MatchBatch& batch, const MatchPlan& plan, int nq_stride, int8_t* codes,
                  int* rowkeys, int sentinel,
                  unsigned* flags, unsigned epoch, unsigned long long* keys, unsigned* done, float ratio,
                  int ratio_on_squared, int* idx2, float* d2, int* match, hipStream_t s);

// One pair of sets with matcher sidecars (detector-produced descriptor
// buffers, sift_kernels.h Sidecar): codes qc/tc (128 B rows) and key biases
// qk/tk; zc/zk the matcher's zero sentinel row and padding key.
void launch_match_direct(const MatchPair& pr, const int8_t* qc, const int* qk, const int8_t* tc, const int* tk,
                         const int8_t* zc, const int* zk, unsigned long long* keys, unsigned* done, float ratio,
                         int ratio_on_squared, int* idx2, float* d2, int* match, hipStream_t s);
int match_direct_splits(int nq, int nt);

// Pairs of ready code sets (e.g. the sidecars of every rank all-gathered: C5):
// k_match_batch on them with no prep launch and no flags (integers by
// construction); pair p reads code rows qrow0.. / trow0.. of `codes` and key
// biases qkrow0.. / tkrow0.. of `rowkeys`.  zc / zk: the zero code row and
// padding key.
void launch_match_codes(MatchBatch& batch, const MatchPlan& plan, int nq_stride, const int8_t* codes, const int* rowkeys,
                        const int8_t* zc, const int* zk, unsigned long long* keys, unsigned* done, float ratio,
                        int ratio_on_squared, int* idx2, float* d2, int* match, hipStream_t s);

}  // namespace sift_amd
