// Brute-force L2 matcher on MFMA for gfx950.
//
// Replaces /root/reference/sift_cuda/sift_func/Match.cu:8-177 (32 lanes per
// query, half2 diff^2, an N x M fp32 score matrix written to and re-read from
// HBM and allocated per call).  Here the distance matrix never leaves the
// register file.  Two launches per call (one for a single pair: k_match<true>
// converts its own rows, see there):
//
//  k_match_prep  every distinct descriptor set of the call (fp16 rows) becomes
//                int8 codes c = v - 128 (128 B per row) and |c|^2 per row, once
//                per set (the 8-way match: 8 sets for 56 pairs).  A set holding
//                a value that is not an integer 0..255 is flagged.
//  k_match       the distance GEMM on v_mfma_i32_32x32x32_i8.  A workgroup owns
//                256 queries (4 waves x 64; a wave keeps its two 32-query B
//                operands in registers for the whole launch) and streams its
//                split of the train rows through LDS in 32-row tiles, double
//                buffered (one 16-byte load per thread per tile, the next
//                tile in flight while this one computes): a tile is read from
//                L2 once per 256 queries and feeds 8 MFMAs per wave.
//
// Exactness: d^2 = sum (t - q)^2 = |c_t|^2 + |c_q|^2 - 2 c_t.c_q for the
// shifted codes (translation invariant); |c|^2 <= 2^21 and |c_t.c_q| <= 2^21, so
// the int32 accumulator and every key below are exact.  A lane folds the 16
// train rows of its accumulator into a running top-2 with three VALU per
// element: key = 256 dot - (128 |c_t|^2 + r) (v_lshl_add_u32), where r is the
// row's index inside a group of 4 tiles, orders (e = d^2 - |c_q|^2, train row)
// in reverse, and the top-2 of the keys is v_max_i32 + v_med3_i32.  Every 4
// tiles the group's top-2 is decoded into (e, train index) and merged into the
// running pair.  Ties keep the lower train index -- OpenCV's batchDistance /
// knnMatch order and the oracle's (sift_oracle_knn2).
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

#ifndef SIFT_MATCH_WG_TARGET
#define SIFT_MATCH_WG_TARGET 512  // workgroups a launch aims for (2 per CU) when choosing train splits
#endif

namespace sift_amd {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));

constexpr int kNone = 0x7fffffff;
constexpr int kRowPad = 144;  // LDS bytes per code row: rows 36 dwords apart -> conflict-free ds_read_b128
constexpr int kGroupTiles = 4;  // tiles per key group: local row r < 128 in the key's low 7 bits
constexpr int kInvalidKey = -(1 << 30);  // keys <= this are padding rows (or none)
constexpr int kPadBias = -(3 << 29);     // key bias of a padding row (codes 0: key = bias <= kInvalidKey)

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

// ---------------------------------------------------------------------------
// Set preparation: 8 threads per row (16 halves each).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_match_prep(MatchSets sets, int8_t* __restrict__ codes,
                                                    int* __restrict__ norms, unsigned* __restrict__ flags,
                                                    unsigned epoch) {
    const MatchSet& st = sets.set[blockIdx.y];
    if ((int)blockIdx.x * 32 >= st.n) return;
    const int row = blockIdx.x * 32 + (threadIdx.x >> 3), part = threadIdx.x & 7;
    const bool in = row < st.n;
    const uint4* src = reinterpret_cast<const uint4*>(st.src + (size_t)min(row, st.n - 1) * 128 + part * 16);
    const uint4 a = src[0], b = src[1];
    const unsigned w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    unsigned pk[4] = {0u, 0u, 0u, 0u};
    int nrm = 0;
    bool bad = false;
#pragma unroll
    for (int e = 0; e < 16; e++) {
        const float v = (float)__builtin_bit_cast(_Float16, (unsigned short)(w[e >> 1] >> (16 * (e & 1))));
        bad |= !(v >= 0.f && v <= 255.f && v == __builtin_rintf(v));  // NaN fails every test
        const int c = (int)fminf(fmaxf(v, 0.f), 255.f) - 128;
        nrm += c * c;
        pk[e >> 2] |= (unsigned)(c & 255) << (8 * (e & 3));
    }
    nrm += __shfl_xor(nrm, 1);
    nrm += __shfl_xor(nrm, 2);
    nrm += __shfl_xor(nrm, 4);
    if (in) {
        *reinterpret_cast<uint4*>(codes + ((size_t)st.row0 + row) * 128 + part * 16) =
            make_uint4(pk[0], pk[1], pk[2], pk[3]);
        if (part == 0) norms[st.row0 + row] = nrm;
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

struct Best {
    int e1, i1, e2, i2;  // e = d^2 - |c_q|^2 (kNone: no entry), i = train index
};

// Merge a key group's top-2 (max-keys m1 >= m2 of the group starting at train
// row t0) into the running pair.  The running entries come from earlier groups
// (lower train indices), so they win ties.
__device__ __forceinline__ Best fold_group(const Best b, int m1, int m2, int t0) {
    const int be1 = b.e1, bi1 = b.i1, be2 = b.e2, bi2 = b.i2;  // values: no member-address selects (scratch)
    const bool v1 = m1 > kInvalidKey, v2 = m2 > kInvalidKey;
    const int s1 = v1 ? -m1 : 0, s2 = v2 ? -m2 : 0;  // 128 e + r
    const int te1 = v1 ? (s1 >> 7) : kNone, ti1 = t0 + (s1 & 127);
    const int te2 = v2 ? (s2 >> 7) : kNone, ti2 = t0 + (s2 & 127);
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

// grid = (256-query blocks, train splits, pairs), 256 threads.
// kFused (single pairs): no k_match_prep launch -- the workgroup converts its
// own query rows and train tiles from fp16 as it loads them and takes the
// fp16 path itself if any of them holds a non-integer value.  Mixing paths
// across workgroups is exact: on integer values 0..255 the fp16 path's dot
// products and norms are exact integers below 2^24, so both paths return
// the same (d^2, index) pairs with the same tie order.
template <bool kFused>
__global__ __launch_bounds__(256, 2) void k_match(MatchBatch batch, int S, int nq_stride,
                                                  const int8_t* __restrict__ codes, const int* __restrict__ norms,
                                                  const unsigned* __restrict__ flags, unsigned epoch,
                                                  unsigned long long* __restrict__ keys, unsigned* __restrict__ done,
                                                  float ratio, int ratio_on_squared, int* __restrict__ idx2,
                                                  float* __restrict__ d2out, int* __restrict__ match) {
    __shared__ __attribute__((aligned(16))) int8_t s_tile[2][kMatchTileRows * kRowPad];
    __shared__ __attribute__((aligned(16))) int s_ntk[2][kMatchTileRows];
    __shared__ Top2 s_res[kMatchQB];
    __shared__ unsigned s_last;
    const int p = blockIdx.z;
    const MatchPair& pr = batch.pair[p];
    const int q0 = blockIdx.x * kMatchQB;
    if (q0 >= pr.nq) return;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, col = lane & 31, h = lane >> 5;
    const int ntiles = (pr.nt + kMatchTileRows - 1) / kMatchTileRows, tps = (ntiles + S - 1) / S;
    const int tbeg = min(ntiles, (int)blockIdx.y * tps), tend = min(ntiles, tbeg + tps);
    const int q0w = q0 + 64 * w;
    Top2 res[2];
    bool bad = false;  // kFused: a non-integer value among this workgroup's rows
    bool use_int = kFused || (flags[pr.qset] != epoch && flags[pr.tset] != epoch);
    if (use_int) {
        // ---- integer path ----
        const int8_t* __restrict__ qc = codes + (size_t)pr.qrow0 * 128;
        const int8_t* __restrict__ tc = codes + (size_t)pr.trow0 * 128;
        const int* __restrict__ tn = norms + pr.trow0;
        // B operands: lane (col, h) holds bytes [64h, 64h + 64) of query row
        // q0w + 32 qb + col, one 16-byte fragment per MFMA; the A fragments
        // take the same bytes of the train rows, so both sides pair the same
        // descriptor dimensions in every K slot.
        i32x4 bq[2][4];
        int qn[2];
#pragma unroll
        for (int qb = 0; qb < 2; qb++) {
            const int row = min(q0w + 32 * qb + col, pr.nq - 1);
            if constexpr (kFused) {
                const uint4* src = reinterpret_cast<const uint4*>(pr.q + (size_t)row * 128 + 64 * h);
                int nrm = 0;
#pragma unroll
                for (int kb = 0; kb < 4; kb++) bq[qb][kb] = codes16(src[2 * kb], src[2 * kb + 1], nrm, bad);
                qn[qb] = nrm + __shfl_xor(nrm, 32);
            } else {
                const i32x4* src = reinterpret_cast<const i32x4*>(qc + (size_t)row * 128 + 64 * h);
#pragma unroll
                for (int kb = 0; kb < 4; kb++) bq[qb][kb] = src[kb];
                qn[qb] = norms[pr.qrow0 + row];
            }
        }
        // Tile loader: thread -> 16 bytes (row tid >> 3, part tid & 7) of a
        // 4 KiB tile; thread r < 32 -> row r's negated key bias.  Loads run two
        // tiles ahead through a ring of two register slots (tile k in slot
        // k & 1), so a tile's global load has two iterations to land before
        // it is stored to its LDS buffer (k & 1) for iteration k.
        // The ring holds the RAW loaded words: the padding select and the key
        // are applied at stash time, so no instruction consumes a load right
        // after it is issued (a select on the loaded value made the compiler
        // wait for every prefetch at once -- vmcnt(0) before each tile's
        // MFMAs -- and the two-deep ring hid nothing).
        const int lrow = tid >> 3, lpart = tid & 7;
        i32x4 nv[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
        int nn[2] = {0, 0};
        uint4 hv[2][2] = {};  // kFused: the raw fp16 words (32 bytes per thread per tile)
        using I0 = std::integral_constant<int, 0>;
        using I1 = std::integral_constant<int, 1>;
        auto fetch = [&](int tile, auto slot) {
            constexpr int SL = decltype(slot)::value;
            const int r = tile * kMatchTileRows + lrow;
            if constexpr (kFused) {
                const uint4* src = reinterpret_cast<const uint4*>(pr.t + (size_t)min(r, pr.nt - 1) * 128 + 16 * lpart);
                hv[SL][0] = src[0];
                hv[SL][1] = src[1];
            } else {
                nv[SL] = *reinterpret_cast<const i32x4*>(tc + (size_t)min(r, pr.nt - 1) * 128 + 16 * lpart);
                nn[SL] = tn[min(tile * kMatchTileRows + (tid & 31), pr.nt - 1)];
            }
        };
        auto stash = [&](int tile, auto slot) {  // tile k, slot k & 1 -> LDS buffer k & 1
            constexpr int SL = decltype(slot)::value;
            const int r = tile * kMatchTileRows + lrow;
            if constexpr (kFused) {  // codes and the row's norm (8 threads per row, lanes 8k..8k+7)
                int nrm = 0;
                const i32x4 pk = codes16(hv[SL][0], hv[SL][1], nrm, bad);
                nrm += __shfl_xor(nrm, 1);
                nrm += __shfl_xor(nrm, 2);
                nrm += __shfl_xor(nrm, 4);
                *reinterpret_cast<i32x4*>(s_tile[SL] + lrow * kRowPad + 16 * lpart) = r < pr.nt ? pk : (i32x4){0, 0, 0, 0};
                if (lpart == 0) {
                    const int lr = ((tile - tbeg) & (kGroupTiles - 1)) * kMatchTileRows + lrow;
                    s_ntk[SL][lrow] = r < pr.nt ? -(128 * nrm + lr) : kPadBias;
                }
                return;
            }
            *reinterpret_cast<i32x4*>(s_tile[SL] + lrow * kRowPad + 16 * lpart) =
                r < pr.nt ? nv[SL] : (i32x4){0, 0, 0, 0};
            if (tid < kMatchTileRows) {
                const int rr = tile * kMatchTileRows + tid;
                const int lr = ((tile - tbeg) & (kGroupTiles - 1)) * kMatchTileRows + tid;  // row in the key group
                s_ntk[SL][tid] = rr < pr.nt ? -(128 * nn[SL] + lr) : kPadBias;
            }
        };
        Best best[2] = {{kNone, kNone, kNone, kNone}, {kNone, kNone, kNone, kNone}};
        // Running key top-2 per query block in two chains (even / odd
        // accumulator registers): half the dependent v_max / v_med3 chain.
        int m1e[2] = {INT_MIN, INT_MIN}, m2e[2] = {INT_MIN, INT_MIN};  // even registers
        int m1o[2] = {INT_MIN, INT_MIN}, m2o[2] = {INT_MIN, INT_MIN};  // odd registers
        if (tbeg < tend) {
            fetch(tbeg, I0{});
            stash(tbeg, I0{});
            if (tbeg + 1 < tend) fetch(tbeg + 1, I1{});
            if (tbeg + 2 < tend) fetch(tbeg + 2, I0{});
        }
        auto step = [&](int tile, auto par) {  // par = (tile - tbeg) & 1
            constexpr int PB = decltype(par)::value;
            lds_barrier();  // tile `tile` is in s_tile[PB]; every wave is done with s_tile[PB ^ 1]
            i32x4 a[4], tk[4];
            const int8_t* ta = s_tile[PB] + col * kRowPad + 64 * h;
#pragma unroll
            for (int kb = 0; kb < 4; kb++) a[kb] = *reinterpret_cast<const i32x4*>(ta + 16 * kb);
            // accumulator register i holds train row (i & 3) + 8 (i >> 2) + 4 h
#pragma unroll
            for (int g = 0; g < 4; g++) tk[g] = *reinterpret_cast<const i32x4*>(s_ntk[PB] + 8 * g + 4 * h);
            if (tile + 1 < tend) {
                stash(tile + 1, std::integral_constant<int, PB ^ 1>{});
                if (tile + 3 < tend) fetch(tile + 3, std::integral_constant<int, PB ^ 1>{});
            }
            i32x16 acc[2] = {{}, {}};
#pragma unroll
            for (int qb = 0; qb < 2; qb++)
#pragma unroll
                for (int kb = 0; kb < 4; kb++)
                    acc[qb] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[kb], bq[qb][kb], acc[qb], 0, 0, 0);
#pragma unroll
            for (int qb = 0; qb < 2; qb++)
#pragma unroll
                for (int i = 0; i < 16; i += 2) {
                    const int ke = (acc[qb][i] << 8) + tk[i >> 2][i & 3];
                    const int ko = (acc[qb][i + 1] << 8) + tk[i >> 2][(i & 3) + 1];
                    m2e[qb] = med3_i32(m1e[qb], ke, m2e[qb]);  // second largest of {m1 >= m2, key}
                    m1e[qb] = max(m1e[qb], ke);
                    m2o[qb] = med3_i32(m1o[qb], ko, m2o[qb]);
                    m1o[qb] = max(m1o[qb], ko);
                }
            const int gi = tile - tbeg;
            if ((gi & (kGroupTiles - 1)) == kGroupTiles - 1 || tile + 1 == tend) {
                const int t0 = (tile - (gi & (kGroupTiles - 1))) * kMatchTileRows;
#pragma unroll
                for (int qb = 0; qb < 2; qb++) {
                    const int a1 = m1e[qb], a2 = m2e[qb], b1 = m1o[qb], b2 = m2o[qb];
                    best[qb] = fold_group(best[qb], max(a1, b1), max(min(a1, b1), max(a2, b2)), t0);
                    m1e[qb] = m2e[qb] = m1o[qb] = m2o[qb] = INT_MIN;
                }
            }
        };
        for (int tile = tbeg; tile < tend; tile += 2) {
            step(tile, I0{});
            if (tile + 1 < tend) step(tile + 1, I1{});
        }
#pragma unroll
        for (int qb = 0; qb < 2; qb++) {
            Best o;  // the other half of the train rows (lane ^ 32)
            o.e1 = __shfl_xor(best[qb].e1, 32);
            o.i1 = __shfl_xor(best[qb].i1, 32);
            o.e2 = __shfl_xor(best[qb].e2, 32);
            o.i2 = __shfl_xor(best[qb].i2, 32);
            const Best r = merge_best(best[qb], o);
            res[qb].d1 = r.e1 == kNone ? INFINITY : (float)(r.e1 + qn[qb]);
            res[qb].i1 = r.e1 == kNone ? kNone : r.i1;
            res[qb].d2 = r.e2 == kNone ? INFINITY : (float)(r.e2 + qn[qb]);
            res[qb].i2 = r.e2 == kNone ? kNone : r.i2;
        }
    }
    if constexpr (kFused)
        if (__syncthreads_or(bad)) use_int = false;  // this workgroup's rows need the fp16 path
    if (!use_int) {
        // ---- general path: fp16 values that are not integers 0..255 ----
        res[0] = match_f16_block(pr, q0w, tbeg, tend, col, h);
        res[1] = match_f16_block(pr, q0w + 32, tbeg, tend, col, h);
    }
    if (h == 0) {
        s_res[64 * w + col] = res[0];
        s_res[64 * w + 32 + col] = res[1];
    }
    __syncthreads();
    const int q = q0 + tid;
    const bool qv = q < pr.nq;
    const size_t o = (size_t)pr.out_off + q;
    if (S == 1) {
        if (qv) {
            const Top2 r = s_res[tid];
            const int i1 = r.i1 == kNone ? -1 : r.i1, i2 = r.i2 == kNone ? -1 : r.i2;
            write_match(i1, i1 >= 0 ? r.d1 : FLT_MAX, i2, i2 >= 0 ? r.d2 : FLT_MAX, o, ratio, ratio_on_squared, idx2,
                        d2out, match);
        }
        return;
    }
    // Global top-2 of a query across the S splits: 64-bit atomicMin on keys.
    // A split min's its best into K1; whatever that displaced (or its best, if
    // it lost) and its runner-up are candidates for K2, of which the smaller is
    // min'ed in (the larger can never be second).  Every key except the final
    // K1 reaches K2 this way, so K2 ends as the true second.  Device-scope
    // atomics only (coherent across XCDs, no cache write-back fences).
    unsigned long long* K = keys + 2 * ((size_t)p * nq_stride + q);
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
    unsigned* cnt = done + (size_t)p * gridDim.x + blockIdx.x;
    if (tid == 0) s_last = atomicAdd(cnt, 1u) == (unsigned)(S - 1);
    __syncthreads();
    if (!s_last || !qv) return;
    const unsigned long long k1 = atomicExch(&K[0], ~0ull), k2 = atomicExch(&K[1], ~0ull);
    if (tid == 0) atomicExch(cnt, 0u);
    const int i1 = k1 == ~0ull ? -1 : (int)(unsigned)k1, i2 = k2 == ~0ull ? -1 : (int)(unsigned)k2;
    const float e1 = i1 >= 0 ? __uint_as_float((unsigned)(k1 >> 32)) : FLT_MAX;
    const float e2 = i2 >= 0 ? __uint_as_float((unsigned)(k2 >> 32)) : FLT_MAX;
    write_match(i1, e1, i2, e2, o, ratio, ratio_on_squared, idx2, d2out, match);
}

int match_splits(int max_nq, int max_nt, int P) {
    const int qblocks = (max_nq + kMatchQB - 1) / kMatchQB;
    const int ntiles = (max_nt + kMatchTileRows - 1) / kMatchTileRows;
#ifndef SIFT_MATCH_WG_TARGET_SINGLE
#define SIFT_MATCH_WG_TARGET_SINGLE SIFT_MATCH_WG_TARGET  // single pairs (fused conversion: fewer, longer splits)
#endif
    const int target = P == 1 ? SIFT_MATCH_WG_TARGET_SINGLE : SIFT_MATCH_WG_TARGET;
    int S = (target + qblocks * P - 1) / (qblocks * P);
    const int maxS = ntiles / 2 > 1 ? ntiles / 2 : 1;  // >= 2 tiles per split
    S = S < maxS ? S : maxS;
    return S < 1 ? 1 : S;
}

#ifndef SIFT_MATCH_FUSED_SINGLE
#define SIFT_MATCH_FUSED_SINGLE 1  // single pairs: no prep launch (tools A/B builds set 0)
#endif
void launch_match(const MatchSets& sets, const MatchBatch& batch, int S, int nq_stride, int8_t* codes, int* norms,
                  unsigned* flags, unsigned epoch, unsigned long long* keys, unsigned* done, float ratio,
                  int ratio_on_squared, int* idx2, float* d2, int* match, hipStream_t s) {
    if (batch.P == 1 && SIFT_MATCH_FUSED_SINGLE) {
        dim3 g((max(batch.pair[0].nq, 1) + kMatchQB - 1) / kMatchQB, S, 1);
        hipLaunchKernelGGL(k_match<true>, g, dim3(256), 0, s, batch, S, nq_stride, codes, norms, flags, epoch, keys,
                           done, ratio, ratio_on_squared, idx2, d2, match);
        return;
    }
    if (sets.maxn > 0)
        hipLaunchKernelGGL(k_match_prep, dim3((sets.maxn + 31) / 32, sets.nsets), dim3(256), 0, s, sets, codes, norms,
                           flags, epoch);
    int max_nq = 1;
    for (int p = 0; p < batch.P; p++) max_nq = max(max_nq, batch.pair[p].nq);
    dim3 g((max_nq + kMatchQB - 1) / kMatchQB, S, batch.P);
    hipLaunchKernelGGL(k_match<false>, g, dim3(256), 0, s, batch, S, nq_stride, codes, norms, flags, epoch, keys, done, ratio,
                       ratio_on_squared, idx2, d2, match);
}

}  // namespace sift_amd
