// Matcher launch interface (match.hip) used by detector.hip's C ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sift_amd {

constexpr int kMaxMatchPairs = 64;

struct MatchPair {
    const uint16_t* q;  // nq x 128 half, row-major
    const uint16_t* t;  // nt x 128 half, row-major
    int nq, nt;
    int out_off;        // output row offset of this pair
    int pad;
};

// Passed by value: lives in the kernarg segment (64 x 32 B = 2 KiB).
struct MatchBatch {
    MatchPair pair[kMaxMatchPairs];
    int P;
};

int match_splits(int max_nq, int max_nt, int P);
// keys: 2 x u64 per (pair, query), all ones between calls; done: a counter per
// (pair, 32-query block), zero between calls (the merging workgroup resets both).
void launch_match(const MatchBatch& batch, int S, int nq_stride, unsigned long long* keys, unsigned* done, float ratio,
                  int ratio_on_squared, int* idx2, float* d2, int* match, hipStream_t s);

}  // namespace sift_amd
