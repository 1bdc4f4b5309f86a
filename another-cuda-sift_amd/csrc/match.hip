// Brute-force L2 matcher on MFMA for gfx950.
//
// Replaces /root/reference/sift_cuda/sift_func/Match.cu:8-177 (32 lanes per
// query, half2 diff^2, an N x M fp32 score matrix written to and re-read from
// HBM, allocated per call).  Here the distance is a GEMM: for a tile of 32 train
// rows x 32 queries one wave issues 8 v_mfma_f32_32x32x16_f16 over K = 128 and
// gets dot(t, q) in fp32; d^2 = |t|^2 + |q|^2 - 2 dot is formed in registers and
// folded into a per-lane running top-2 in the epilogue, so the N x M matrix never
// leaves the register file.  Operand roles are chosen so that the accumulator's
// column (lane) is the query and its 16 registers are train rows: each lane
// scans train rows in increasing index order, giving OpenCV's batchDistance
// tie-break (lower train index first) with a strict '<' insert.
//
// Exactness: SIFT descriptors from this library are integers 0..255 stored in
// fp16; products are exact in fp32 and every partial sum is < 2^24, so d^2 is
// exact and the top-2 is identical to the oracle's (sift_oracle_knn2).
#include <float.h>

#include "sift_kernels.h"
#include "sift_match.h"

namespace sift_amd {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

struct Top2 {
    float d1, d2;
    int i1, i2;
};

__device__ __forceinline__ bool better(float da, int ia, float db, int ib) {
    return da < db || (da == db && ia < ib);
}

// Top-2 of the union of two disjoint sorted pairs, (distance, index) order.
// Written with value selects only (no struct-reference selects -> no scratch).
__device__ __forceinline__ Top2 merge_top2(const Top2 a, const Top2 b) {
    const bool bfirst = better(b.d1, b.i1, a.d1, a.i1);
    // winner w, loser-head l (first of the other list), runner-up of the winner's list wn.
    const float wd = bfirst ? b.d1 : a.d1, ld = bfirst ? a.d1 : b.d1, wnd = bfirst ? b.d2 : a.d2;
    const int wi = bfirst ? b.i1 : a.i1, li = bfirst ? a.i1 : b.i1, wni = bfirst ? b.i2 : a.i2;
    const bool lsecond = better(ld, li, wnd, wni);
    Top2 r;
    r.d1 = wd;
    r.i1 = wi;
    r.d2 = lsecond ? ld : wnd;
    r.i2 = lsecond ? li : wni;
    return r;
}

__device__ __forceinline__ Top2 shfl_top2(const Top2& t, int mask) {
    Top2 r;
    r.d1 = __shfl_xor(t.d1, mask);
    r.d2 = __shfl_xor(t.d2, mask);
    r.i1 = __shfl_xor(t.i1, mask);
    r.i2 = __shfl_xor(t.i2, mask);
    return r;
}

__device__ __forceinline__ half8 load_frag(const uint16_t* row, int koff) {
    return *reinterpret_cast<const half8*>(row + koff);
}

constexpr int kNone = 0x7fffffff;

// |v|^2 over a lane's eight 8-element fragments: v_dot2_f32_f16 in four
// independent chains (exact: integer products, partial sums < 2^24).
__device__ __forceinline__ float sumsq8(const half8 (&v)[8]) {
    typedef _Float16 half2v __attribute__((ext_vector_type(2)));
    float c[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 8; s++)
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const half2v x = {v[s][2 * j], v[s][2 * j + 1]};
            c[j] = __builtin_amdgcn_fdot2(x, x, c[j], false);
        }
    return (c[0] + c[1]) + (c[2] + c[3]);
}

// Global top-2 of a query across the S split workgroups, by 64-bit atomicMin
// on keys (d^2 bits << 32 | train index): d^2 >= 0 orders like its bits, and
// the index breaks ties to the lower train row (OpenCV's order).  A split
// min's its best into K1; whatever it displaced (or its best, if that lost)
// and its runner-up are candidates for K2, of which the smaller is min'ed in
// (the larger can never be second).  Every key except the final K1 reaches
// K2 this way, so K2 ends as the true second.  All exchange goes through
// device-scope atomics (coherent across XCDs, no cache write-back fences);
// the last split of a query block (a counter) decodes, writes the outputs
// and resets keys and counter for the next call.
__device__ __forceinline__ unsigned long long match_key(float d2, int idx) {
    return idx == kNone ? ~0ull : ((unsigned long long)__float_as_uint(d2) << 32) | (unsigned)idx;
}

// grid = (query blocks of 32, train splits, pairs); 4 waves per workgroup share
// the query block and stride over the split's 32-row train tiles.
__global__ __launch_bounds__(256) void k_match_partial(MatchBatch batch, int S, int nq_stride,
                                                       unsigned long long* __restrict__ keys,
                                                       unsigned* __restrict__ done, float ratio, int ratio_on_squared,
                                                       int* __restrict__ idx2, float* __restrict__ d2out,
                                                       int* __restrict__ match) {
    __shared__ Top2 wtop[4][32];
    __shared__ unsigned s_last;
    const int p = blockIdx.z;
    const MatchPair& pr = batch.pair[p];
    const int q0 = blockIdx.x * 32;
    if (q0 >= pr.nq) return;
    const int split = blockIdx.y;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int col = lane & 31, h = lane >> 5;

    const int qrow = q0 + col;
    const bool qvalid = qrow < pr.nq;
    half8 bq[8];
#pragma unroll
    for (int s = 0; s < 8; s++) bq[s] = qvalid ? load_frag(pr.q + (size_t)qrow * 128, 16 * s + 8 * h) : half8{};
    float qn = sumsq8(bq);
    qn += __shfl_xor(qn, 32);

    const int ntiles = (pr.nt + 31) / 32;
    const int tps = (ntiles + S - 1) / S;
    const int tbeg = split * tps, tend = min(ntiles, tbeg + tps);

    Top2 best{INFINITY, INFINITY, kNone, kNone};
    for (int tile = tbeg + w; tile < tend; tile += 4) {
        const int t0 = tile * 32;
        const int trow = t0 + col;
        const bool tvalid = trow < pr.nt;
        half8 a[8];
#pragma unroll
        for (int s = 0; s < 8; s++) a[s] = tvalid ? load_frag(pr.t + (size_t)trow * 128, 16 * s + 8 * h) : half8{};
        float tn = sumsq8(a);
        tn += __shfl_xor(tn, 32);
        // Two independent accumulation chains (even / odd K blocks), summed:
        // exact for integer descriptors (every partial sum < 2^24).
        f32x16 acc = {}, acc2 = {};
#pragma unroll
        for (int s = 0; s < 8; s += 2) {
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[s], bq[s], acc, 0, 0, 0);
            acc2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[s + 1], bq[s + 1], acc2, 0, 0, 0);
        }
        acc += acc2;
#pragma unroll
        for (int i = 0; i < 16; i++) {
            const int row = (i & 3) + 8 * (i >> 2) + 4 * h;
            const float tnr = __shfl(tn, row);
            const int tr = t0 + row;
            const float d = tnr - 2.f * acc[i];
            if (tr < pr.nt) {
                if (d < best.d2) {
                    if (d < best.d1) {
                        best.d2 = best.d1;
                        best.i2 = best.i1;
                        best.d1 = d;
                        best.i1 = tr;
                    } else {
                        best.d2 = d;
                        best.i2 = tr;
                    }
                }
            }
        }
    }
    best = merge_top2(best, shfl_top2(best, 32));
    if (h == 0) wtop[w][col] = best;
    __syncthreads();
    if (w == 0 && h == 0) {
        Top2 r = wtop[0][col];
        r = merge_top2(r, wtop[1][col]);
        r = merge_top2(r, wtop[2][col]);
        r = merge_top2(r, wtop[3][col]);
        if (qvalid) {
            unsigned long long* K = keys + 2 * ((size_t)p * nq_stride + qrow);
            const unsigned long long a1 = match_key(r.d1 + qn, r.i1), a2 = match_key(r.d2 + qn, r.i2);
            if (a1 != ~0ull) {
                const unsigned long long o1 = atomicMin(&K[0], a1);
                const unsigned long long c = a1 < o1 ? o1 : a1;
                const unsigned long long o2 = atomicMin(&K[1], c < a2 ? c : a2);
                __asm__ volatile("" ::"v"(o2));  // returned: the min is performed before the count below
            }
        }
    }
    __syncthreads();
    unsigned* cnt = done + (size_t)p * gridDim.x + blockIdx.x;
    if (threadIdx.x == 0) s_last = atomicAdd(cnt, 1u) == (unsigned)(S - 1);
    __syncthreads();
    if (!s_last || threadIdx.x >= 32 || q0 + (int)threadIdx.x >= pr.nq) return;
    const int q = q0 + threadIdx.x;
    unsigned long long* K = keys + 2 * ((size_t)p * nq_stride + q);
    const unsigned long long k1 = atomicExch(&K[0], ~0ull), k2 = atomicExch(&K[1], ~0ull);
    if (threadIdx.x == 0) atomicExch(cnt, 0u);
    const int i1 = k1 == ~0ull ? -1 : (int)(unsigned)k1, i2 = k2 == ~0ull ? -1 : (int)(unsigned)k2;
    const float e1 = i1 >= 0 ? __uint_as_float((unsigned)(k1 >> 32)) : FLT_MAX;
    const float e2 = i2 >= 0 ? __uint_as_float((unsigned)(k2 >> 32)) : FLT_MAX;
    const size_t o = (size_t)pr.out_off + q;
    if (idx2) {
        idx2[2 * o] = i1;
        idx2[2 * o + 1] = i2;
    }
    if (d2out) {
        d2out[2 * o] = e1;
        d2out[2 * o + 1] = e2;
    }
    if (match) {
        int m = -1;
        if (i1 >= 0) {
            if (i2 < 0)
                m = i1;
            else if (ratio_on_squared)
                m = e1 < ratio * e2 ? i1 : -1;
            else
                m = __builtin_sqrtf(e1) < ratio * __builtin_sqrtf(e2) ? i1 : -1;
        }
        match[o] = m;
    }
}

int match_splits(int max_nq, int max_nt, int P) {
    const int qblocks = (max_nq + 31) / 32;
    const int ntiles = (max_nt + 31) / 32;
    int S = (1024 + qblocks * P - 1) / (qblocks * P);
    S = S < 1 ? 1 : S;
    const int maxS = (ntiles + 3) / 4;  // keep >= 4 tiles (one per wave) per split
    if (S > maxS) S = maxS < 1 ? 1 : maxS;
    return S;
}

void launch_match(const MatchBatch& batch, int S, int nq_stride, unsigned long long* keys, unsigned* done, float ratio,
                  int ratio_on_squared, int* idx2, float* d2, int* match, hipStream_t s) {
    int max_nq = 1;
    for (int p = 0; p < batch.P; p++) max_nq = max(max_nq, batch.pair[p].nq);
    dim3 g1((max_nq + 31) / 32, S, batch.P);
    hipLaunchKernelGGL(k_match_partial, g1, dim3(256), 0, s, batch, S, nq_stride, keys, done, ratio, ratio_on_squared,
                       idx2, d2, match);
}

}  // namespace sift_amd
