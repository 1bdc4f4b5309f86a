// Brute-force L2 matcher on MFMA for gfx950.
//
// Replaces /root/reference/sift_cuda/sift_func/Match.cu:8-177 (32 lanes per
// query, half2 diff^2, an N x M fp32 score matrix written to and re-read from
// HBM and allocated per call).  Here the distance matrix never leaves the
// register file.  Two launches per batched call, one for a single pair:
//
//  k_match_prep    every distinct descriptor set of the call (fp16 rows)
//                  becomes int8 codes c = v - 128 (128 B per row) and a key
//                  bias -(256 |c|^2 + (row mod 256)) per row, once per set (the
//                  8-way match: 8 sets for 56 pairs).  A set holding a value
//                  that is not an integer 0..255 is flagged.
//  k_match_batch   the distance GEMM on v_mfma_i32_32x32x32_i8 for prepared
//                  sets: a workgroup owns 512 queries (8 waves x 64; a wave
//                  keeps its two 32-query B operands in registers) and one
//                  split of the train tiles, which it streams through two LDS
//                  chunk buffers of 8 tiles by LDS-DMA (the next chunk lands
//                  while this one computes: one barrier per 8 tiles instead
//                  of one per tile); per 32-row tile 8 MFMAs per wave.
//  k_match_single  one pair without the prep launch: each workgroup (256
//                  queries) converts its own query rows and train tiles.
//
// Exactness: d^2 = sum (t - q)^2 = |c_t|^2 + |c_q|^2 - 2 c_t.c_q for the
// shifted codes (translation invariant), so the int32 accumulator and every
// key below are exact.  A lane folds the 16 train rows of its accumulator
// into a running top-2 of keys key = 512 dot - (256 |c_t|^2 + r) (one
// v_lshl_add_u32 each), where r is the row's index inside its group of 8
// tiles; keys order (e = d^2 - |c_q|^2, train row) in reverse, and two new
// keys at a time enter the top-2 with v_med3 + v_max3 (3 VALU per 2 keys).
// Each staged chunk is one key group: its top-2 is decoded into (e, train
// index) and merged into the running pair.  Ties keep the lower train index
// -- OpenCV's batchDistance / knnMatch order and the oracle's
// (sift_oracle_knn2).
//
// A pair with a flagged set (non-integer or out-of-range fp16 values, e.g. the
// reference's own unrounded x512 descriptors) runs the general path in the
// same launch: v_mfma_f32_32x32x16_f16 dot products (exact products, fp32
// sums), fp32 norms, a float top-2 in train order.
//
// Splits of the train rows merge through 64-bit atomicMin keys (d^2 bits << 32 |
// train index) in the matcher's scratch; the last split of a query block (a
// counter) writes the outputs and restores the scratch.  With one split the
// workgroup writes the outputs itself.
#include <float.h>
#include <limits.h>

#include <type_traits>

#include "sift_kernels.h"
#include "sift_match.h"
#include "sift_math.h"

namespace sift_amd {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));

constexpr int kNone = 0x7fffffff;
// Row keys: key = 512 dot - (256 |c_t|^2 + r) orders (d^2, train row) in
// reverse for one query, where r < 256 is the row's index inside its group of
// kGroupTiles tiles: 256 (2 dot - |c_t|^2) = 256 (|c_q|^2 - d^2) lies in
// [-2^31 + 2^24, 2^29] for any codes (d^2 <= 128 * 255^2 < 2^23), so every key
// is an exact int32.  A padding row has zero codes and key kPadBias, below
// every valid key.
constexpr int kGroupTiles = 8;
constexpr int kPadBias = kMatchPadKey;
constexpr int kInvalidKey = kPadBias;  // keys <= this are padding rows (or none)

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

// 16 fp16 descriptor values -> int8 codes c = v - 128 (4 dwords), adding
// sum c^2 to nrm; bad is set by a value that is not an integer 0..255 (NaN,
// infinities and -0 included), whose code is then meaningless (the caller
// falls back to the fp16 path).  Packed: v + 1024 puts an integer 0..1023 in
// the mantissa bits exactly (0x6400 | v for v < 256), one v_perm gathers four
// such low bytes, and v ^ 0x80 is v - 128 as int8; v_dot4 adds the squares.
__device__ __forceinline__ i32x4 codes16(const uint4 a, const uint4 b, int& nrm, bool& bad) {
    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
    const unsigned w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    unsigned y[8];
#pragma unroll
    for (int e = 0; e < 8; e++) {
        const h2 yv = __builtin_bit_cast(h2, w[e]) + (h2){(_Float16)1024.f, (_Float16)1024.f};
        const h2 back = yv - (h2){(_Float16)1024.f, (_Float16)1024.f};
        y[e] = __builtin_bit_cast(unsigned, yv);
        bad |= (y[e] & 0xff00ff00u) != 0x64006400u || __builtin_bit_cast(unsigned, back) != w[e];
    }
    i32x4 pk;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        pk[k] = (int)(__builtin_amdgcn_perm(y[2 * k + 1], y[2 * k], 0x06040200u) ^ 0x80808080u);
        nrm = __builtin_amdgcn_sdot4(pk[k], pk[k], nrm, false);
    }
    return pk;
}

// ---------------------------------------------------------------------------
// Set preparation: 8 threads per row (16 halves each); per row the int8
// codes and the key bias -(256 |c|^2 + (row & 255)) (the norm is -bias >> 8).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_match_prep(MatchSets sets, int8_t* __restrict__ codes,
                                                    int* __restrict__ rowkeys, unsigned* __restrict__ flags,
                                                    unsigned epoch) {
    const MatchSet& st = sets.set[blockIdx.y];
    if ((int)blockIdx.x * 32 >= st.n) return;
    const int row = blockIdx.x * 32 + (threadIdx.x >> 3), part = threadIdx.x & 7;
    const bool in = row < st.n;
    const uint4* src = reinterpret_cast<const uint4*>(st.src + (size_t)min(row, st.n - 1) * 128 + part * 16);
    int nrm = 0;
    bool bad = false;
    const i32x4 pk = codes16(src[0], src[1], nrm, bad);  // codes of a flagged set are never used
    nrm += __shfl_xor(nrm, 1);
    nrm += __shfl_xor(nrm, 2);
    nrm += __shfl_xor(nrm, 4);
    if (in) {
        *reinterpret_cast<i32x4*>(codes + ((size_t)st.row0 + row) * 128 + part * 16) = pk;
        if (part == 0) rowkeys[st.row0 + row] = -(256 * nrm + (row & 255));  // the row's key bias (r = row mod 256)
        if (bad) flags[blockIdx.y] = epoch;  // every writer stores the same word
    }
}

// ---------------------------------------------------------------------------
// Integer path helpers.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int med3_i32(int a, int b, int c) {
    int r;
    __asm__("v_med3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

__device__ __forceinline__ int max3_i32(int a, int b, int c) {
    int r;
    __asm__("v_max3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

struct Best {
    int e1, i1, e2, i2;  // e = d^2 - |c_q|^2 (kNone: no entry), i = train index
};

// Merge a key group's top-2 (max-keys m1 >= m2 of the group starting at train
// row t0) into the running pair.  The running entries come from earlier groups
// (lower train indices), so they win ties.
__device__ __forceinline__ Best fold_group(const Best b, int m1, int m2, int t0) {
    const int be1 = b.e1, bi1 = b.i1, be2 = b.e2, bi2 = b.i2;  // values: no member-address selects (scratch)
    const bool v1 = m1 > kInvalidKey, v2 = m2 > kInvalidKey;
    const int s1 = v1 ? -m1 : 0, s2 = v2 ? -m2 : 0;  // 256 e + r
    const int te1 = v1 ? (s1 >> 8) : kNone, ti1 = t0 + (s1 & 255);
    const int te2 = v2 ? (s2 >> 8) : kNone, ti2 = t0 + (s2 & 255);
    const bool c1 = te1 < be1;
    const bool c2 = c1 ? te2 < be1 : te1 < be2;
    Best r;
    r.e2 = c1 ? (c2 ? te2 : be1) : (c2 ? te1 : be2);
    r.i2 = c1 ? (c2 ? ti2 : bi1) : (c2 ? ti1 : bi2);
    r.e1 = c1 ? te1 : be1;
    r.i1 = c1 ? ti1 : bi1;
    return r;
}

__device__ __forceinline__ bool lt_ei(int ea, int ia, int eb, int ib) { return ea < eb || (ea == eb && ia < ib); }

__device__ __forceinline__ Best merge_best(const Best a, const Best b) {
    const bool bf = lt_ei(b.e1, b.i1, a.e1, a.i1);
    const int we = bf ? b.e1 : a.e1, wi = bf ? b.i1 : a.i1;
    const int le = bf ? a.e1 : b.e1, li = bf ? a.i1 : b.i1;  // head of the other list
    const int ne = bf ? b.e2 : a.e2, ni = bf ? b.i2 : a.i2;  // runner-up of the winner's list
    const bool ls = lt_ei(le, li, ne, ni);
    return Best{we, wi, ls ? le : ne, ls ? li : ni};
}

// ---------------------------------------------------------------------------
// General (fp16) path helpers.
// ---------------------------------------------------------------------------
__device__ __forceinline__ half8 load_frag(const uint16_t* row, int koff) {
    return *reinterpret_cast<const half8*>(row + koff);
}

// |v|^2 over a lane's eight 8-element fragments: v_dot2_f32_f16 in four chains.
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

// One wave's 32 queries (rows q0 + col of the pair) against train tiles
// [tbeg, tend): f16 MFMA (train rows as A, queries as B, so the accumulator's
// lane is the query and its 16 registers are train rows in increasing order),
// float top-2 with a strict '<' insert.  Returns the full d^2.
__device__ Top2 match_f16_block(const MatchPair& pr, int q0, int tbeg, int tend, int col, int h) {
    const int qrow = q0 + col;
    const bool qvalid = qrow < pr.nq;
    half8 bq[8];
#pragma unroll
    for (int s = 0; s < 8; s++) bq[s] = qvalid ? load_frag(pr.q + (size_t)qrow * 128, 16 * s + 8 * h) : half8{};
    float qn = sumsq8(bq);
    qn += __shfl_xor(qn, 32);
    Top2 best{INFINITY, INFINITY, kNone, kNone};
    for (int tile = tbeg; tile < tend; tile++) {
        const int t0 = tile * kMatchTileRows, trow = t0 + col;
        const bool tvalid = trow < pr.nt;
        half8 a[8];
#pragma unroll
        for (int s = 0; s < 8; s++) a[s] = tvalid ? load_frag(pr.t + (size_t)trow * 128, 16 * s + 8 * h) : half8{};
        float tn = sumsq8(a);
        tn += __shfl_xor(tn, 32);
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
            const float d = __shfl(tn, row) - 2.f * acc[i];
            if (t0 + row < pr.nt && d < best.d2) {
                if (d < best.d1) {
                    best.d2 = best.d1;
                    best.i2 = best.i1;
                    best.d1 = d;
                    best.i1 = t0 + row;
                } else {
                    best.d2 = d;
                    best.i2 = t0 + row;
                }
            }
        }
    }
    best = merge_top2(best, shfl_top2(best, 32));
    best.d1 += qn;
    best.d2 += qn;
    return best;
}

__device__ __forceinline__ unsigned long long match_key(float d2, int idx) {
    return idx == kNone ? ~0ull : ((unsigned long long)__float_as_uint(d2) << 32) | (unsigned)idx;
}

__device__ __forceinline__ void write_match(int i1, float e1, int i2, float e2, size_t o, float ratio,
                                            int ratio_on_squared, int* idx2, float* d2out, int* match) {
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


// ---------------------------------------------------------------------------
// Integer-path building blocks shared by both kernels.
//
// Train tiles are staged in LDS a chunk (<= one key group of kGroupTiles
// tiles) at a time.  Code rows are stored unpadded (128 B) with their 16-byte
// pieces XOR-swizzled by (row >> 1) & 7, so a wave's ds_read_b128 of 32 rows x
// one piece covers the 64 banks once per 16-lane group; the swizzle also lets
// prepared codes go global -> LDS by LDS-DMA (a lane's source address is free,
// its LDS slot is lane x 16 B).
// ---------------------------------------------------------------------------
constexpr int kTileBytes = kMatchTileRows * 128;
// Waves per k_match_batch workgroup and 32-query blocks per wave (512 queries
// per workgroup).  (Measured alternative, round 3: 16 waves x 1 block, 42.1
// vs 39.1 us per C5 launch.)
constexpr int kMatchBatchNW = 8;
constexpr int kMatchBatchQBW = 2;
constexpr int kMatchBatchQB = 32 * kMatchBatchQBW * kMatchBatchNW;
constexpr int kMatchBatchWgPerCu = 2 * 8 / kMatchBatchNW > 0 ? 2 * 8 / kMatchBatchNW : 1;  // register budget: 16 waves per CU
constexpr int kChunkRows = kChunkTiles * kMatchTileRows;
static_assert(kChunkTiles == kGroupTiles, "a staged chunk is at most one key group");

__device__ __forceinline__ int piece_swz(int row, int piece) { return piece ^ ((row >> 1) & 7); }

// A wave's QBW 32-query B operands: lane (col, h) holds bytes [64h, 64h + 64)
// of query row q0w + 32 qb + col, one 16-byte fragment per MFMA; the A
// fragments take the same bytes of the train rows, so both sides pair the same
// descriptor dimensions in every K slot.  qn = |c_q|^2.
template <int QBW>
__device__ __forceinline__ void load_queries(const int8_t* __restrict__ qc, const int* __restrict__ qkeys, int nq,
                                             int q0w, int col, int h, i32x4 (&bq)[QBW][4], int (&qn)[QBW]) {
#pragma unroll
    for (int qb = 0; qb < QBW; qb++) {
        const int row = min(q0w + 32 * qb + col, nq - 1);
        const i32x4* src = reinterpret_cast<const i32x4*>(qc + (size_t)row * 128 + 64 * h);
#pragma unroll
        for (int kb = 0; kb < 4; kb++) bq[qb][kb] = src[kb];
        qn[qb] = (-qkeys[row]) >> 8;
    }
}

// Stage prepared train rows [row0, row0 + 32 nc) of a set (codes tc, key
// biases tk) into one LDS chunk by LDS-DMA; rows past nt read the zero
// sentinel row (zc, zk).  Codes: wave w fills 8-row blocks w, w + NW, ...
// (1 KiB each); lane l lands at slot (row 8b + l / 8, piece l & 7) and loads
// the global piece the swizzle puts there.  Keys: 64 rows per 4-byte-per-lane
// instruction.  Completion is this wave's vmcnt.
template <int NW>
__device__ __forceinline__ void stage_dma(const int8_t* __restrict__ tc, const int* __restrict__ tk, int nt, int row0,
                                          int nc, const int8_t* __restrict__ zc, const int* __restrict__ zk,
                                          int8_t* sc, int* sk, int w, int lane) {
    const int wv = __builtin_amdgcn_readfirstlane(w);
    for (int b = wv; b < nc * (kMatchTileRows / 8); b += NW) {
        const int r = 8 * b + (lane >> 3), gr = row0 + r;
        const int8_t* src = (gr < nt ? tc + (size_t)gr * 128 : zc) + 16 * piece_swz(r, lane & 7);
        __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)(sc + 1024 * b), 16,
                                         0, 0);
    }
    for (int b = wv; b < (nc * kMatchTileRows + 63) / 64; b += NW) {
        const int gr = row0 + 64 * b + lane;
        const int* src = gr < nt ? tk + gr : zk;
        __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)(sk + 64 * b), 4, 0,
                                         0);
    }
}

// One staged chunk of nc tiles (rows t0 ...) against a wave's two query
// blocks: per tile 8 MFMAs from LDS fragments, then each lane folds its 32
// keys into a per-block running key top-2 -- two at a time: for a pair (x, y)
// of new keys and the running m1 >= m2 the new second is max(med3(m1, x, y),
// m2) and the new first max3(m1, x, y), 3 VALU per 2 keys, in two chains per
// block (accumulator registers 0-7 / 8-15).  The chunk lies in one key group
// (r = row - t0 < 256), so its top-2 is decoded once into (e, train index) and
// merged into the running pair (earlier groups win ties).
template <int QBW>
__device__ __forceinline__ void chunk_top2(const int8_t* sc, const int* sk, int nc, int t0, int col, int h,
                                           const i32x4 (&bq)[QBW][4], Best (&best)[QBW]) {
    int m1e[QBW], m2e[QBW], m1o[QBW], m2o[QBW];  // registers 0-7 / 8-15
#pragma unroll
    for (int qb = 0; qb < QBW; qb++) m1e[qb] = m2e[qb] = m1o[qb] = m2o[qb] = INT_MIN;
    const int sw = (col >> 1) & 7;
    const int8_t* const ta0 = sc + col * 128;
    const int* const tk1 = sk + 4 * h;
#pragma unroll
    for (int j = 0; j < kChunkTiles; j++) {
        if (j < nc) {
            i32x4 a[4], tk[4];
#pragma unroll
            for (int kb = 0; kb < 4; kb++)
                a[kb] = *reinterpret_cast<const i32x4*>(ta0 + j * kTileBytes + 16 * ((4 * h + kb) ^ sw));
            // accumulator register i holds train row (i & 3) + 8 (i >> 2) + 4 h
#pragma unroll
            for (int g = 0; g < 4; g++) tk[g] = *reinterpret_cast<const i32x4*>(tk1 + j * kMatchTileRows + 8 * g);
            i32x16 acc[QBW] = {};
#pragma unroll
            for (int qb = 0; qb < QBW; qb++)
#pragma unroll
                for (int kb = 0; kb < 4; kb++)
                    acc[qb] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[kb], bq[qb][kb], acc[qb], 0, 0, 0);
#pragma unroll
            for (int qb = 0; qb < QBW; qb++)
#pragma unroll
                for (int i = 0; i < 8; i += 2) {
                    const int x0 = (acc[qb][i] << 9) + tk[i >> 2][i & 3];
                    const int y0 = (acc[qb][i + 1] << 9) + tk[i >> 2][(i & 3) + 1];
                    const int x1 = (acc[qb][i + 8] << 9) + tk[(i + 8) >> 2][i & 3];
                    const int y1 = (acc[qb][i + 9] << 9) + tk[(i + 8) >> 2][(i & 3) + 1];
                    m2e[qb] = max(med3_i32(m1e[qb], x0, y0), m2e[qb]);
                    m1e[qb] = max3_i32(m1e[qb], x0, y0);
                    m2o[qb] = max(med3_i32(m1o[qb], x1, y1), m2o[qb]);
                    m1o[qb] = max3_i32(m1o[qb], x1, y1);
                }
        }
    }
#pragma unroll
    for (int qb = 0; qb < QBW; qb++) {
        const int a1 = m1e[qb], a2 = m2e[qb], b1 = m1o[qb], b2 = m2o[qb];
        best[qb] = fold_group(best[qb], max(a1, b1), max(min(a1, b1), max(a2, b2)), t0);
    }
}

// A lane's two halves of the train rows (lane, lane ^ 32) -> the query's
// (d^2, index) top-2 (d^2 = e + |c_q|^2).
__device__ __forceinline__ Top2 finish_best(const Best b, int qn) {
    Best o;
    o.e1 = __shfl_xor(b.e1, 32);
    o.i1 = __shfl_xor(b.i1, 32);
    o.e2 = __shfl_xor(b.e2, 32);
    o.i2 = __shfl_xor(b.i2, 32);
    const Best r = merge_best(b, o);
    Top2 t;
    t.d1 = r.e1 == kNone ? INFINITY : (float)(r.e1 + qn);
    t.i1 = r.e1 == kNone ? kNone : r.i1;
    t.d2 = r.e2 == kNone ? INFINITY : (float)(r.e2 + qn);
    t.i2 = r.e2 == kNone ? kNone : r.i2;
    return t;
}

__device__ __forceinline__ void write_top2(const Top2 r, size_t o, float ratio, int ratio_on_squared, int* idx2,
                                           float* d2out, int* match) {
    const int i1 = r.i1 == kNone ? -1 : r.i1, i2 = r.i2 == kNone ? -1 : r.i2;
    write_match(i1, i1 >= 0 ? r.d1 : FLT_MAX, i2, i2 >= 0 ? r.d2 : FLT_MAX, o, ratio, ratio_on_squared, idx2, d2out,
                match);
}

// Global top-2 of a query over several contributions (train ranges):
// 64-bit atomicMin on keys (d^2 bits << 32 | train index).  A contribution
// min's its best into K1; whatever that displaced (or its best, if it lost)
// and its runner-up are candidates for K2, of which the smaller is min'ed in
// (the larger can never be second).  Every key except the final K1 reaches K2
// this way, so K2 ends as the true second.  Device-scope atomics only
// (coherent across XCDs, no cache write-back fences).  The contribution that
// completes the count (`units` of `total`, counted on *cnt) reads and
// restores the keys and the counter and writes the outputs.  Called by every
// thread of the workgroup, thread t for query q0 + t (s_res[t]).
__device__ __forceinline__ void merge_contribution(const Top2* s_res, unsigned* s_last, unsigned long long* K0,
                                                   unsigned* cnt, unsigned units, unsigned total, bool qv, size_t o,
                                                   float ratio, int ratio_on_squared, int* idx2, float* d2out,
                                                   int* match) {
    const int tid = threadIdx.x;
    unsigned long long* K = K0 + 2 * tid;
    if (qv) {
        const Top2 r = s_res[tid];
        const unsigned long long a1 = match_key(r.d1, r.i1), a2 = match_key(r.d2, r.i2);
        if (a1 != ~0ull) {
            const unsigned long long o1 = atomicMin(&K[0], a1);
            const unsigned long long c = a1 < o1 ? o1 : a1;
            const unsigned long long o2 = atomicMin(&K[1], c < a2 ? c : a2);
            __asm__ volatile("" ::"v"(o2));  // returned: the min is performed before the count below
        }
    }
    __syncthreads();
    if (tid == 0) *s_last = atomicAdd(cnt, units) + units == total;
    __syncthreads();
    if (!*s_last) return;
    if (qv) {
        const unsigned long long k1 = atomicExch(&K[0], ~0ull), k2 = atomicExch(&K[1], ~0ull);
        const int i1 = k1 == ~0ull ? -1 : (int)(unsigned)k1, i2 = k2 == ~0ull ? -1 : (int)(unsigned)k2;
        const float e1 = i1 >= 0 ? __uint_as_float((unsigned)(k1 >> 32)) : FLT_MAX;
        const float e2 = i2 >= 0 ? __uint_as_float((unsigned)(k2 >> 32)) : FLT_MAX;
        write_match(i1, e1, i2, e2, o, ratio, ratio_on_squared, idx2, d2out, match);
    }
    if (tid == 0) atomicExch(cnt, 0u);
}

// ---------------------------------------------------------------------------
// k_match_single: one pair, fp16 rows converted in the kernel (no prep
// launch).  grid = (query blocks of 64 NW, train splits S), 64 NW threads; a
// workgroup converts its query rows and its split's train rows as it stages
// them (8 threads per row: two 16-byte fp16 loads -> one swizzled 16-byte code
// piece; the row norm by three shuffles) and takes the fp16 path itself if
// any of them holds a non-integer value.  Mixing paths across workgroups is
// exact: on integer values 0..255 the fp16 path's dot products and norms are
// exact integers below 2^24, so both paths return the same (d^2, index) pairs
// with the same tie order.  Key groups start at the split's first tile.
// ---------------------------------------------------------------------------
template <int NW, int QBW>
__global__ __launch_bounds__(64 * NW, (kMatchWgPerCu * NW) / 4) void k_match_single(
    MatchPair pr, int S, unsigned long long* __restrict__ keys, unsigned* __restrict__ done, float ratio,
    int ratio_on_squared, int* __restrict__ idx2, float* __restrict__ d2out, int* __restrict__ match) {
    constexpr int NT = 64 * NW, QB = 32 * QBW * NW;  // threads, queries per workgroup (QBW 32-query blocks per wave)
    __shared__ __attribute__((aligned(16))) int8_t s_codes[2][kChunkTiles * kTileBytes];
    __shared__ __attribute__((aligned(16))) int s_key[2][kChunkRows];
    __shared__ unsigned s_last;
    static_assert(sizeof(Top2) * QB <= sizeof(s_codes), "results alias the code tiles");
    static_assert(QB <= NT, "the write-out gives each thread one query: at most 2 query blocks per wave");
    Top2* const s_res = reinterpret_cast<Top2*>(&s_codes[0][0]);
    const int q0 = blockIdx.x * QB;
    if (q0 >= pr.nq) return;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, col = lane & 31, h = lane >> 5;
    const int ntiles = (pr.nt + kMatchTileRows - 1) / kMatchTileRows, tps = (ntiles + S - 1) / S;
    const int tbeg = min(ntiles, (int)blockIdx.y * tps), tend = min(ntiles, tbeg + tps);
    const int q0w = q0 + 32 * QBW * w;
    Top2 res[QBW];
    bool bad = false;  // a non-integer value among this workgroup's rows
    {
        i32x4 bq[QBW][4];
        int qn[QBW];
#pragma unroll
        for (int qb = 0; qb < QBW; qb++) {
            const int row = min(q0w + 32 * qb + col, pr.nq - 1);
            const uint4* src = reinterpret_cast<const uint4*>(pr.q + (size_t)row * 128 + 64 * h);
            int nrm = 0;
#pragma unroll
            for (int kb = 0; kb < 4; kb++) bq[qb][kb] = codes16(src[2 * kb], src[2 * kb + 1], nrm, bad);
            qn[qb] = nrm + __shfl_xor(nrm, 32);
        }
        auto stage = [&](int c0, int buf) {
            const int nc = min(kChunkTiles, tend - c0);
            int8_t* const sc = s_codes[buf];
            int* const sk = s_key[buf];
            constexpr int U = 2;  // loads go out U pieces at a time
            const int npieces = nc * kMatchTileRows * 8;
            for (int base = 0; base < npieces; base += NT * U) {
                uint4 hv[U][2];
#pragma unroll
                for (int u = 0; u < U; u++) {
                    const int idx = min(base + tid + NT * u, npieces - 1), r = idx >> 3;
                    const uint4* src = reinterpret_cast<const uint4*>(
                        pr.t + (size_t)min(c0 * kMatchTileRows + r, pr.nt - 1) * 128 + 16 * (idx & 7));
                    hv[u][0] = src[0];
                    hv[u][1] = src[1];
                }
#pragma unroll
                for (int u = 0; u < U; u++) {
                    const int idx = base + tid + NT * u, r = idx >> 3, part = idx & 7;
                    const int gr = c0 * kMatchTileRows + r;
                    int nrm = 0;
                    const i32x4 pk = codes16(hv[u][0], hv[u][1], nrm, bad);
                    nrm += __shfl_xor(nrm, 1);
                    nrm += __shfl_xor(nrm, 2);
                    nrm += __shfl_xor(nrm, 4);
                    if (idx < npieces) {  // whole rows of 8 lanes: the shuffles above stay inside a row
                        *reinterpret_cast<i32x4*>(sc + r * 128 + 16 * piece_swz(r, part)) =
                            gr < pr.nt ? pk : (i32x4){0, 0, 0, 0};
                        if (part == 0)
                            sk[r] = gr < pr.nt ? -(256 * nrm + ((gr - tbeg * kMatchTileRows) & 255)) : kPadBias;
                    }
                }
            }
        };
        Best best[QBW];
#pragma unroll
        for (int qb = 0; qb < QBW; qb++) best[qb] = Best{kNone, kNone, kNone, kNone};
        if (tbeg < tend) stage(tbeg, 0);
        int buf = 0;
        for (int c0 = tbeg; c0 < tend; c0 += kChunkTiles, buf ^= 1) {
            __syncthreads();  // chunk c0 is staged; every wave is done with the other buffer
            if (c0 + kChunkTiles < tend) stage(c0 + kChunkTiles, buf ^ 1);
            chunk_top2(s_codes[buf], s_key[buf], min(kChunkTiles, tend - c0), c0 * kMatchTileRows, col, h, bq, best);
        }
#pragma unroll
        for (int qb = 0; qb < QBW; qb++) res[qb] = finish_best(best[qb], qn[qb]);
    }
    if (__syncthreads_or(bad)) {
        // ---- general path: fp16 values that are not integers 0..255 ----
#pragma unroll
        for (int qb = 0; qb < QBW; qb++) res[qb] = match_f16_block(pr, q0w + 32 * qb, tbeg, tend, col, h);
    }
    __syncthreads();  // s_res aliases the code tiles
    if (h == 0) {
#pragma unroll
        for (int qb = 0; qb < QBW; qb++) s_res[32 * QBW * w + 32 * qb + col] = res[qb];
    }
    __syncthreads();
    const int q = q0 + tid;
    const bool qv = tid < QB && q < pr.nq;
    const size_t o = (size_t)pr.out_off + q;
    if (S == 1) {
        if (qv) write_top2(s_res[tid], o, ratio, ratio_on_squared, idx2, d2out, match);
        return;
    }
    merge_contribution(s_res, &s_last, keys + 2 * (size_t)q0, done + blockIdx.x, 1u, (unsigned)S, qv, o, ratio,
                       ratio_on_squared, idx2, d2out, match);
}

// ---------------------------------------------------------------------------
// k_match_batch: prepared sets (k_match_prep), any number of pairs.
// grid = (query blocks of 64 NW, train splits S, pairs), 64 NW threads.  A
// split is whole key groups of the pair's train tiles; the workgroup loads
// each wave's query operands once and streams its split through two LDS chunk
// buffers (the next group by LDS-DMA while this one computes: one barrier per
// 8 tiles).  With S > 1 the splits merge through the keys scratch and the one
// that completes the query block's count writes the outputs.
// ---------------------------------------------------------------------------
template <int NW, int QBW>
__global__ __launch_bounds__(64 * NW, (kMatchBatchWgPerCu * NW) / 4) void k_match_batch(
    MatchBatch batch, int S, int nq_stride, const int8_t* __restrict__ codes, const int* __restrict__ rowkeys,
    const int8_t* __restrict__ zc, const int* __restrict__ zk, const unsigned* __restrict__ flags, unsigned epoch,
    unsigned long long* __restrict__ keys,
    unsigned* __restrict__ done, float ratio, int ratio_on_squared, int* __restrict__ idx2, float* __restrict__ d2out,
    int* __restrict__ match) {
    constexpr int QB = 32 * QBW * NW;  // queries per workgroup
    static_assert(QB <= 64 * NW, "the write-out gives each thread one query: at most 2 query blocks per wave");
    __shared__ __attribute__((aligned(16))) int8_t s_codes[2][kChunkTiles * kTileBytes];
    __shared__ __attribute__((aligned(16))) int s_key[2][kChunkRows];
    __shared__ unsigned s_last;
    static_assert(sizeof(Top2) * QB <= sizeof(s_codes), "results alias the code tiles");
    Top2* const s_res = reinterpret_cast<Top2*>(&s_codes[0][0]);
    const int p = blockIdx.z;
    const MatchPair& pr = batch.pair[p];
    const int q0 = blockIdx.x * QB;
    if (q0 >= pr.nq) return;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, col = lane & 31, h = lane >> 5;
    const int ntiles = (pr.nt + kMatchTileRows - 1) / kMatchTileRows;
    const int tps = ((ntiles + S - 1) / S + kGroupTiles - 1) / kGroupTiles * kGroupTiles;  // whole key groups
    const int tb = min(ntiles, (int)blockIdx.y * tps), te = min(ntiles, tb + tps);
    const int q0w = q0 + 32 * QBW * w;
    Top2 res[QBW];
    // flags == nullptr: code sets handed over ready (sift_hip_match_codes_batched), integers by construction.
    if (!flags || (flags[pr.qset] != epoch && flags[pr.tset] != epoch)) {
        // ---- integer path (zc / zk: the zero code row and padding key) ----
        const int8_t* __restrict__ tc = codes + (size_t)pr.trow0 * 128;
        const int* __restrict__ tk = rowkeys + pr.tkrow0;
        i32x4 bq[QBW][4];
        int qn[QBW];
        load_queries<QBW>(codes + (size_t)pr.qrow0 * 128, rowkeys + pr.qkrow0, pr.nq, q0w, col, h, bq, qn);
        Best best[QBW];
#pragma unroll
        for (int qb = 0; qb < QBW; qb++) best[qb] = Best{kNone, kNone, kNone, kNone};
        if (tb < te)
            stage_dma<NW>(tc, tk, pr.nt, tb * kMatchTileRows, min(kChunkTiles, te - tb), zc, zk, s_codes[0], s_key[0],
                          w, lane);
        int buf = 0;
        for (int c0 = tb; c0 < te; c0 += kChunkTiles, buf ^= 1) {
            // LDS-DMA writes are counted by vmcnt: this wave's copies of the
            // chunk have landed; the barrier publishes every wave's, and every
            // wave is done with the other buffer.
            __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            const int c1 = c0 + kChunkTiles;
            if (c1 < te)
                stage_dma<NW>(tc, tk, pr.nt, c1 * kMatchTileRows, min(kChunkTiles, te - c1), zc, zk, s_codes[buf ^ 1],
                              s_key[buf ^ 1], w, lane);
            chunk_top2(s_codes[buf], s_key[buf], min(kChunkTiles, te - c0), c0 * kMatchTileRows, col, h, bq, best);
        }
#pragma unroll
        for (int qb = 0; qb < QBW; qb++) res[qb] = finish_best(best[qb], qn[qb]);
    } else {
        // ---- general path: fp16 values that are not integers 0..255 ----
#pragma unroll
        for (int qb = 0; qb < QBW; qb++) res[qb] = match_f16_block(pr, q0w + 32 * qb, tb, te, col, h);
    }
    __syncthreads();  // s_res aliases the code tiles
    if (h == 0) {
#pragma unroll
        for (int qb = 0; qb < QBW; qb++) s_res[32 * QBW * w + 32 * qb + col] = res[qb];
    }
    __syncthreads();
    const int q = q0 + tid;
    const bool qv = tid < QB && q < pr.nq;  // (64 NW threads >= QB queries)
    const size_t o = (size_t)pr.out_off + q;
    if (S == 1) {
        if (qv) write_top2(s_res[tid], o, ratio, ratio_on_squared, idx2, d2out, match);
        return;
    }
    merge_contribution(s_res, &s_last, keys + 2 * ((size_t)p * nq_stride + q0), done + (size_t)p * gridDim.x + blockIdx.x,
                       1u, (unsigned)S, qv, o, ratio, ratio_on_squared, idx2, d2out, match);
}

// ---------------------------------------------------------------------------
// k_match_direct: one pair of detector-produced descriptor sets, read through
// their sidecars (int8 codes + key bias, written by the descriptor kernels:
// no conversion, no prep launch).  The integer path of k_match_batch with the
// codes and keys addressed directly: query operands from the query sidecar,
// the split's train key groups streamed through two LDS chunks by LDS-DMA.
// grid = (query blocks of 32 QBW NW, splits S of whole key groups).
// ---------------------------------------------------------------------------
template <int NW, int QBW>
__global__ __launch_bounds__(64 * NW) void k_match_direct(
    MatchPair pr, const int8_t* __restrict__ qc, const int* __restrict__ qk, const int8_t* __restrict__ tc,
    const int* __restrict__ tk, const int8_t* __restrict__ zc, const int* __restrict__ zk, int S,
    unsigned long long* __restrict__ keys, unsigned* __restrict__ done, float ratio, int ratio_on_squared,
    int* __restrict__ idx2, float* __restrict__ d2out, int* __restrict__ match) {
    constexpr int QB = 32 * QBW * NW;
    static_assert(QB <= 64 * NW, "the write-out gives each thread one query: at most 2 query blocks per wave");
    __shared__ __attribute__((aligned(16))) int8_t s_codes[2][kChunkTiles * kTileBytes];
    __shared__ __attribute__((aligned(16))) int s_key[2][kChunkRows];
    __shared__ unsigned s_last;
    static_assert(sizeof(Top2) * QB <= sizeof(s_codes), "results alias the code tiles");
    Top2* const s_res = reinterpret_cast<Top2*>(&s_codes[0][0]);
    const int q0 = blockIdx.x * QB;
    if (q0 >= pr.nq) return;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, col = lane & 31, h = lane >> 5;
    const int ntiles = (pr.nt + kMatchTileRows - 1) / kMatchTileRows;
    const int tps = ((ntiles + S - 1) / S + kGroupTiles - 1) / kGroupTiles * kGroupTiles;  // whole key groups
    const int tb = min(ntiles, (int)blockIdx.y * tps), te = min(ntiles, tb + tps);
    const int q0w = q0 + 32 * QBW * w;
    Top2 res[QBW];
    {
        if (tb < te)  // the first chunk's DMA before the query loads: both round trips overlap
            stage_dma<NW>(tc, tk, pr.nt, tb * kMatchTileRows, min(kChunkTiles, te - tb), zc, zk, s_codes[0], s_key[0],
                          w, lane);
        i32x4 bq[QBW][4];
        int qn[QBW];
        load_queries<QBW>(qc, qk, pr.nq, q0w, col, h, bq, qn);
        Best best[QBW];
#pragma unroll
        for (int qb = 0; qb < QBW; qb++) best[qb] = Best{kNone, kNone, kNone, kNone};
        int buf = 0;
        for (int c0 = tb; c0 < te; c0 += kChunkTiles, buf ^= 1) {
            __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            const int c1 = c0 + kChunkTiles;
            if (c1 < te)
                stage_dma<NW>(tc, tk, pr.nt, c1 * kMatchTileRows, min(kChunkTiles, te - c1), zc, zk, s_codes[buf ^ 1],
                              s_key[buf ^ 1], w, lane);
            chunk_top2(s_codes[buf], s_key[buf], min(kChunkTiles, te - c0), c0 * kMatchTileRows, col, h, bq, best);
        }
#pragma unroll
        for (int qb = 0; qb < QBW; qb++) res[qb] = finish_best(best[qb], qn[qb]);
    }
    __syncthreads();  // s_res aliases the code tiles
    if (h == 0) {
#pragma unroll
        for (int qb = 0; qb < QBW; qb++) s_res[32 * QBW * w + 32 * qb + col] = res[qb];
    }
    __syncthreads();
    const int q = q0 + tid;
    const bool qv = tid < QB && q < pr.nq;
    const size_t o = (size_t)pr.out_off + q;
    if (S == 1) {
        if (qv) write_top2(s_res[tid], o, ratio, ratio_on_squared, idx2, d2out, match);
        return;
    }
    merge_contribution(s_res, &s_last, keys + 2 * (size_t)q0, done + blockIdx.x, 1u, (unsigned)S, qv, o, ratio,
                       ratio_on_squared, idx2, d2out, match);
}

// Direct single pairs: 8 waves x 1 query block (256 queries per workgroup),
// one key group (256 train rows) per split up to kDirectWgTarget workgroups.
// 2000 x 2000 on detector buffers (tools/match_direct_time.py, two passes):
// 7.71 / 7.78 us; 4 waves 8.06 / 7.90; 4 waves x 2 blocks 8.97 / 8.98; two key
// groups per split (target 64) 9.65 / 9.72; the converting k_match_single
// on the same pair 11.2-11.4 (profiles/round5/match_direct_ab.jsonl).
constexpr int kDirectNW = 8, kDirectQBW = 1, kDirectQB = 32 * kDirectNW * kDirectQBW, kDirectWgTarget = 256;

int match_direct_splits(int nq, int nt) {
    const int ntiles = (nt + kMatchTileRows - 1) / kMatchTileRows, groups = (ntiles + kGroupTiles - 1) / kGroupTiles;
    const int qblocks = (max(nq, 1) + kDirectQB - 1) / kDirectQB;
    int S = max(1, min(groups, kDirectWgTarget / max(qblocks, 1)));
    const int tps = ((ntiles + S - 1) / S + kGroupTiles - 1) / kGroupTiles * kGroupTiles;
    return tps > 0 ? max(1, (ntiles + tps - 1) / tps) : 1;
}

void launch_match_direct(const MatchPair& pr, const int8_t* qc, const int* qk, const int8_t* tc, const int* tk,
                         const int8_t* zc, const int* zk, unsigned long long* keys, unsigned* done, float ratio,
                         int ratio_on_squared, int* idx2, float* d2, int* match, hipStream_t s) {
    const int S = match_direct_splits(pr.nq, pr.nt);
    dim3 g((max(pr.nq, 1) + kDirectQB - 1) / kDirectQB, S, 1);
    hipLaunchKernelGGL((k_match_direct<kDirectNW, kDirectQBW>), g, dim3(64 * kDirectNW), 0, s, pr, qc, qk, tc, tk, zc,
                       zk, S, keys, done, ratio, ratio_on_squared, idx2, d2, match);
}

// Single pairs of foreign buffers (k_match_single): workgroups a launch aims
// for when choosing train splits (64-1024 measured equal, round 2), waves per
// workgroup and 32-query blocks per wave (4 x 2: 256 queries per workgroup;
// 128-query workgroups measured equal, round 4), and no prep launch (the
// prep + batch kernel path: host-synchronous calls 32-42 vs 25-28 us, round 2).
constexpr int kMatchWgTargetSingle = 256;
constexpr int kMatchNWSingle = 4;
constexpr int kMatchQBWSingle = 2;
constexpr int kMatchSingleQB = 32 * kMatchQBWSingle * kMatchNWSingle;
// The matcher's done counters are sized per (pair, kMatchQB-query block)
// (sift_hip_matcher_create); a launch indexes them by its own block, which must
// therefore hold at least kMatchQB queries.
static_assert(kMatchSingleQB >= kMatchQB, "single-pair blocks smaller than the done-counter block");
static_assert(kMatchBatchQB >= kMatchQB, "batched blocks smaller than the done-counter block");
static_assert(kDirectQB >= kMatchQB, "direct blocks smaller than the done-counter block");

static int device_cus() {
    static int cus = [] {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
            n = 256;
        return n;
    }();
    return cus;
}

MatchPlan match_plan(int max_nq, int max_nt, int P) {
    MatchPlan pl;
    const int ntiles = (max_nt + kMatchTileRows - 1) / kMatchTileRows;
    if (P == 1) {
        pl.nw = kMatchNWSingle;
        const int qblocks = (max_nq + kMatchSingleQB - 1) / kMatchSingleQB;
        int S = (kMatchWgTargetSingle + qblocks - 1) / qblocks;
        // >= 4 tiles per split: every split converts its workgroup's query rows
        // again (C3, 2000 x 2000: 4 tiles 11.5 us per call, 3 tiles 11.9, 2 12.4,
        // 1 15.8, 6 12.3, 8 13.4; tools/r3_c3_dma.sh).
        constexpr int kMinTilesSingle = 4;
        const int maxS = (ntiles + kMinTilesSingle - 1) / kMinTilesSingle;
        S = S < maxS ? S : maxS;
        S = S < 1 ? 1 : S;
        // No empty splits (tps rounded up can leave trailing ones empty).
        const int tps = (ntiles + S - 1) / S;
        pl.S = tps > 0 ? (ntiles + tps - 1) / tps : 1;
    } else {
        // Splits (whole key groups each) that minimise the busiest CU's work
        // within one round of workgroups: a CU's tile rate is the same with
        // one workgroup (2 waves per SIMD) or two (4), so the time is
        // (workgroups on the busiest CU) x (tiles per split), plus the split
        // merge (~2.8 us, kMergeTiles tile-times) when S > 1.  C5 (224 query
        // blocks on 256 CUs): S = 1, 64 tiles and no merge, instead of S = 2
        // (two workgroups of 32 tiles on 192 CUs, then the merge).
        pl.nw = kMatchBatchNW;
        const int qblocks = (max_nq + kMatchBatchQB - 1) / kMatchBatchQB;
        const int groups = (ntiles + kGroupTiles - 1) / kGroupTiles;
        const int cus = device_cus(), units = qblocks * P;
        constexpr int kMergeTiles = 6;
        int best = 1;
        long best_cost = -1;
        for (int S = 1; S <= groups; S++) {
            const int tps = ((ntiles + S - 1) / S + kGroupTiles - 1) / kGroupTiles * kGroupTiles;
            const int s_eff = (ntiles + tps - 1) / tps;
            if (s_eff != S) continue;  // same split sizes as a smaller S
            const long wgs = (long)units * S;
            if (S > 1 && wgs > (long)kMatchBatchWgPerCu * cus) break;  // one round only
            const long cost = (wgs + cus - 1) / cus * tps + (S > 1 ? kMergeTiles : 0);
            if (best_cost < 0 || cost < best_cost) {
                best_cost = cost;
                best = S;
            }
        }
        pl.S = best;
    }
    return pl;
}

void launch_match(const MatchSets& sets, MatchBatch& batch, const MatchPlan& plan, int nq_stride, int8_t* codes,
                  int* rowkeys, int sentinel, unsigned* flags, unsigned epoch, unsigned long long* keys,
                  unsigned* done, float ratio, int ratio_on_squared, int* idx2, float* d2, int* match, hipStream_t s) {
    if (batch.P == 1) {
        const MatchPair& pr = batch.pair[0];
        dim3 g((max(pr.nq, 1) + kMatchSingleQB - 1) / kMatchSingleQB, plan.S, 1);
        hipLaunchKernelGGL((k_match_single<kMatchNWSingle, kMatchQBWSingle>), g, dim3(64 * kMatchNWSingle),
                           0, s, pr, plan.S, keys, done, ratio, ratio_on_squared, idx2, d2, match);
        return;
    }
    if (sets.maxn > 0)
        hipLaunchKernelGGL(k_match_prep, dim3((sets.maxn + 31) / 32, sets.nsets), dim3(256), 0, s, sets, codes, rowkeys,
                           flags, epoch);
    int max_nq = 1;
    for (int p = 0; p < batch.P; p++) max_nq = max(max_nq, batch.pair[p].nq);
    dim3 g((max_nq + kMatchBatchQB - 1) / kMatchBatchQB, plan.S, batch.P);
    hipLaunchKernelGGL((k_match_batch<kMatchBatchNW, kMatchBatchQBW>), g, dim3(64 * kMatchBatchNW), 0, s, batch, plan.S, nq_stride, codes,
                       rowkeys, codes + (size_t)sentinel * 128, rowkeys + sentinel, flags, epoch, keys, done, ratio,
                       ratio_on_squared, idx2, d2, match);
}

void launch_match_codes(MatchBatch& batch, const MatchPlan& plan, int nq_stride, const int8_t* codes, const int* rowkeys,
                        const int8_t* zc, const int* zk, unsigned long long* keys, unsigned* done, float ratio,
                        int ratio_on_squared, int* idx2, float* d2, int* match, hipStream_t s) {
    int max_nq = 1;
    for (int p = 0; p < batch.P; p++) max_nq = max(max_nq, batch.pair[p].nq);
    dim3 g((max_nq + kMatchBatchQB - 1) / kMatchBatchQB, plan.S, batch.P);
    hipLaunchKernelGGL((k_match_batch<kMatchBatchNW, kMatchBatchQBW>), g, dim3(64 * kMatchBatchNW), 0, s, batch, plan.S,
                       nq_stride, codes, rowkeys, zc, zk, (const unsigned*)nullptr, 0u, keys, done, ratio, ratio_on_squared,
                       idx2, d2, match);
}

}  // namespace sift_amd
