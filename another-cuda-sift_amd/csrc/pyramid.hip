// Gaussian pyramid and 3x3x3 scale-space extrema for gfx950.
//
// Replaces /root/reference/sift_cuda/image_func/{Filter,Resize,MatOps}.cu.
// Semantics follow OpenCV 4.x; the float
// operation order is the oracle's (oracle/sift_oracle.cpp gaussianBlur /
// upsample2x / isExtremum), so planes and candidate lists are bit-exact.
#include <array>
#include <cstring>
#include <utility>

#include "sift_kernels.h"
#include "sift_math.h"

namespace sift_amd {

// ---------------------------------------------------------------------------
// 2x bilinear upsample (OpenCV resize INTER_LINEAR on float; firstOctave = -1).
// Reference: Resize.cu:6-64 (half-pixel bilinear, target size ignored).
// ---------------------------------------------------------------------------
__device__ __forceinline__ void up_coeff(int d, int slen, int& s, float& a0, float& a1) {
    // (d + 0.5) * 0.5 - 0.5 = d / 2 - 0.25: exact in float for every d < 2^22,
    // so this is the oracle's double expression to the bit.
    float f = (float)d * 0.5f - 0.25f;
    int si = (int)floorf(f);
    f -= (float)si;
    if (si < 0) { f = 0.f; si = 0; }
    if (si >= slen - 1) { f = 0.f; si = slen - 1; }
    s = si;
    a0 = 1.f - f;
    a1 = f;
}

__device__ __forceinline__ float dpp_left_or(float own, float v) {  // lane i <- lane i-1, lane 0 <- own
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(own), __float_as_int(v), 0x138, 0xf, 0xf, false));
}
__device__ __forceinline__ float dpp_right_or(float own, float v) {  // lane i <- lane i+1, lane 63 <- own
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(own), __float_as_int(v), 0x130, 0xf, 0xf, false));
}

// One wave per 256 source columns and a run of source rows (rows per wave =
// H / (4 gridDim.y), rounded up): lane l holds columns c, c + 1 for c = base +
// 2l and c = base + 128 + 2l -- one 8-byte load per row and half, 512 B
// contiguous per wave -- and takes its neighbours c - 1, c + 2 from lanes l - 1
// / l + 1 by DPP (lanes 0 / 63 from the other half or one extra load per row).
// Each source row's horizontal interpolation is formed once and kept in a
// 3-row ring; rows 2m, 2m + 1 are then one 16-byte store per half whose 64
// lanes cover 1 KB contiguously.  Away from the left and right borders every
// horizontal output takes the fixed weights (0.25, 0.75) / (0.75, 0.25) --
// up_coeff's values there, in the same operation order; border lanes and every
// vertical step take up_coeff.  (Measured, round 6, per 16-frame 1920x1200
// launch: one output per thread 408 us (1.8 TB/s); 16 outputs per thread with
// two 16-byte stores 32 B apart 330; one wave per row with contiguous stores
// and three loads per window 242 -- 167 of it with the loads removed.)
template <typename T>
__global__ __launch_bounds__(256) void k_upsample2x(const T* __restrict__ src, int spitch, int W, int H,
                                                    float* __restrict__ dst, int dpitch, long sfs, long dfs) {
    src = fptr(src, blockIdx.z * sfs);  // frame blockIdx.z
    dst = fptr(dst, blockIdx.z * dfs);
    const int per = (H + 4 * (int)gridDim.y - 1) / (4 * (int)gridDim.y);  // source rows per wave
    const int m0 = (blockIdx.y * 4 + (threadIdx.x >> 6)) * per;
    if (m0 >= H) return;  // wave-uniform
    const int mEnd = min(m0 + per, H);
    const int lane = threadIdx.x & 63, base = blockIdx.x * 256;
    const int c[2] = {base + 2 * lane, base + 128 + 2 * lane};
    const int xe = lane == 0 ? max(base - 1, 0) : min(base + 256, W - 1);  // lanes 0 / 63: outer columns
    const bool vec = sizeof(T) == 4 && (reinterpret_cast<uintptr_t>(src) & 7) == 0 && (spitch & 1) == 0;
    struct Raw {
        float v[2][2], e;
    };
    // Source row y (clamped), columns clamped to the row: every lane's window
    // is src[clamp(c - 1 .. c + 2)].
    auto load = [&](int y, Raw& r) {
        const T* row = src + (size_t)min(max(y, 0), H - 1) * spitch;
#pragma unroll
        for (int h = 0; h < 2; h++) {
            if (vec && c[h] + 1 < W) {
                const float2 q = *reinterpret_cast<const float2*>(row + c[h]);
                r.v[h][0] = q.x;
                r.v[h][1] = q.y;
            } else {
                r.v[h][0] = (float)row[min(c[h], W - 1)];
                r.v[h][1] = (float)row[min(c[h] + 1, W - 1)];
            }
        }
        r.e = (float)row[xe];
    };
    auto horiz = [&](const Raw& r, float (&hh)[8]) {
        float w[2][4];
        const float a1_63 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(r.v[0][1]), 63));
        const float b0_0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(r.v[1][0]), 0));
        w[0][0] = dpp_left_or(r.e, r.v[0][1]);
        w[0][3] = dpp_right_or(b0_0, r.v[0][0]);
        w[1][0] = dpp_left_or(a1_63, r.v[1][1]);
        w[1][3] = dpp_right_or(r.e, r.v[1][0]);
#pragma unroll
        for (int h = 0; h < 2; h++) {
            w[h][1] = r.v[h][0];
            w[h][2] = r.v[h][1];
            if (c[h] >= 1 && c[h] + 2 < W) {
                hh[4 * h] = w[h][0] * 0.25f + w[h][1] * 0.75f;
                hh[4 * h + 1] = w[h][1] * 0.75f + w[h][2] * 0.25f;
                hh[4 * h + 2] = w[h][1] * 0.25f + w[h][2] * 0.75f;
                hh[4 * h + 3] = w[h][2] * 0.75f + w[h][3] * 0.25f;
            } else {
#pragma unroll
                for (int t = 0; t < 4; t++) {
                    int sx;
                    float ax0, ax1;
                    up_coeff(min(2 * c[h] + t, 2 * W - 1), W, sx, ax0, ax1);
                    const int k0 = min(max(sx - c[h] + 1, 0), 3), k1 = min(max(min(sx + 1, W - 1) - c[h] + 1, 0), 3);
                    const float s0 = k0 == 0 ? w[h][0] : (k0 == 1 ? w[h][1] : (k0 == 2 ? w[h][2] : w[h][3]));
                    const float s1 = k1 == 0 ? w[h][0] : (k1 == 1 ? w[h][1] : (k1 == 2 ? w[h][2] : w[h][3]));
                    hh[4 * h + t] = s0 * ax0 + s1 * ax1;
                }
            }
        }
    };
    Raw rr;
    float hp[8], hc[8], hn[8];
    load(m0 - 1, rr);
    horiz(rr, hp);
    load(m0, rr);
    horiz(rr, hc);
    load(m0 + 1, rr);
    for (int m = m0; m < mEnd; m++) {
        horiz(rr, hn);                  // source row m + 1
        if (m + 1 < mEnd) load(m + 2, rr);  // one row ahead of the stores
#pragma unroll
        for (int v = 0; v < 2; v++) {
            int sy;
            float ay0, ay1;
            up_coeff(2 * m + v, H, sy, ay0, ay1);  // sy in {m - 1, m}, its successor in {m, m + 1}
            const bool r0c = sy == m, r1c = min(sy + 1, H - 1) == m;
            float o[8];
#pragma unroll
            for (int i = 0; i < 8; i++) o[i] = (r0c ? hc[i] : hp[i]) * ay0 + (r1c ? hc[i] : hn[i]) * ay1;
            float* d = dst + (size_t)(2 * m + v) * dpitch;
#pragma unroll
            for (int h = 0; h < 2; h++) {
                if (c[h] + 2 <= W) {
                    *reinterpret_cast<float4*>(d + 2 * c[h]) = make_float4(o[4 * h], o[4 * h + 1], o[4 * h + 2], o[4 * h + 3]);
                } else if (c[h] < W) {  // W odd: the row's last two outputs
                    d[2 * c[h]] = o[4 * h];
                    d[2 * c[h] + 1] = o[4 * h + 1];
                }
            }
        }
#pragma unroll
        for (int i = 0; i < 8; i++) {
            hp[i] = hc[i];
            hc[i] = hn[i];
        }
    }
}

// Source rows per wave: 8 for frame batches (fewer, longer-lived waves), 2
// for a single frame (more waves in flight).
dim3 up_grid(int W, int H, int nf) {
    const int per = nf > 1 ? 8 : 2;
    return dim3((W + 255) / 256, (H + 4 * per - 1) / (4 * per), nf);
}

void launch_upsample2x(const float* src, int spitch, int W, int H, float* dst, int dpitch, const Frames& fr, long sfs,
                       hipStream_t s) {
    hipLaunchKernelGGL(k_upsample2x<float>, up_grid(W, H, fr.nf), dim3(256), 0, s, src, spitch, W, H, dst, dpitch, sfs,
                       fr.stride);
}

void launch_upsample2x_u8(const uint8_t* src, int spitch, int W, int H, float* dst, int dpitch, const Frames& fr,
                          long sfs, hipStream_t s) {
    hipLaunchKernelGGL(k_upsample2x<uint8_t>, up_grid(W, H, fr.nf), dim3(256), 0, s, src, spitch, W, H, dst, dpitch, sfs, fr.stride);
}

// ---------------------------------------------------------------------------
// Separable Gaussian blur, one 64 x BLUR_TH output tile per workgroup of
// BLUR_NW waves (each BLUR_TH / BLUR_NW rows of the column pass),
// instantiated per radius R (taps 2R+1) so every tap loop is fully unrolled.
// The (BLUR_TH+2R) x (64+2R) input tile (reflect-101 borders) is staged once
// in LDS; the blur of an octave's plane L also writes the next octave's base
// plane (its even rows and columns, OpenCV's INTER_NEAREST half-size resize).
// Row pass: 16 threads per row, each keeps a (2R+4)-float register window
// (ds_read_b128) and runs 4 independent fma chains (4 adjacent outputs).
// Column pass: one column per lane, 8 rows per thread, (2R+8)-float window.
// Row:    s = 0; s = fma(in[x-R+k], w[k], s), k = 0..2R          (2R+1 > 5)
//         s = in[x]*w[R]; s = fma(in[x-k]+in[x+k], w[R+k], s)      (2R+1 <= 5)
// Column: s = fma(mid[y], w[R], 0); s = fma(mid[y+k]+mid[y-k], w[R+k], s)
// Reference: Filter.cu:8-51 (no LDS, vertical first, modulo per tap).
// ---------------------------------------------------------------------------
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// (a.y, b.x) in one v_pk_mov_b32 (the compiler otherwise emits two v_mov).
__device__ __forceinline__ f32x2 pk_mov_hi_lo(f32x2 a, f32x2 b) {
    f32x2 r;
    __asm__("v_pk_mov_b32 %0, %1, %2 op_sel:[1,0]" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
constexpr int BLUR_TW = 64;
constexpr int BLUR_TH = 64;  // tile height: 64 (8 waves) beat 32 by 3-5 % of frame time (round 1)
// Waves per workgroup NW (a template parameter): 4 for launches of >= 2048
// tiles (octave-0 launches of frame batches: 2-8 % faster per launch, and a
// workgroup pair holds half of a CU's wave slots, so the other stream's
// keypoint kernels co-reside), 8 for the small launches (more waves per tile
// hide their latency better).
constexpr int kBlurBigTiles = 2048;
static_assert(BLUR_TH % 32 == 0, "blur tile height: 8-row column blocks for 4 or 8 waves");
static int blur_waves(int tiles) { return tiles >= kBlurBigTiles ? 4 : 8; }

// One blur launch's job: plane src -> dst, optionally the next octave's base
// plane (dec), the pixel range and the frame counters.
struct BlurJob {
    const void* src;  // float, or uint8_t for the frame's first blur of an 8-bit frame
    float* dst;
    DecOut dec;
    unsigned* range_keys;
    Counters* zero_ctr;
    int spitch, W, H, dpitch, tilesX, ntiles;
    int nf;         // frames; the launch has nf * ntiles tiles of this job
    long sfs, dfs;  // byte strides between frames: source; dst / dec / range_keys / zero_ctr
    Taps taps;
};

// LDS row pitch of a blur tile (floats).  The row pass stores each lane's 4
// outputs with ds_write_b128, whose 8-lane groups put blocks of one row
// beside the same blocks of the next row: conflict-free exactly when the pitch
// is 16 mod 32 dwords (the old pitch, 64 + 2R rounded up to 4, was only for
// R = 8: SQ_LDS_BANK_CONFLICT 16-21 % of the LDS cycles at R = 5, 6, 10, 13).
// A multiple-of-16 pitch also lets the column pass fetch (y, y + 4) pairs with
// one ds_read2st64_b32.
constexpr bool kBlurIW16 = true;
// Tiles with every input in the image read their staging rows as aligned
// 16-byte loads of columns x0 - ORG .. x0 + 63 + ORG, ORG = 8 for radius <= 8
// and R rounded up to a multiple of 4 above (12 at R = 10, 16 at R = 13): a
// quarter of the load instructions of the per-column dword staging.  The LDS
// tile starts at column x0 - ORG whichever staging ran.
// (Measured alternative, round 3: the per-column dword staging for R > 8 --
// the paired R = 13 launch 115.7 vs 113.0 us per 16 frames.)
constexpr bool kBlurX4Ld = true;
constexpr bool kBlurX4LdBig = true;  // the 16-byte staging for radii > 8 too
constexpr int kBlurX4LdMaxR = 24;
// Full tiles store their output rows as 16-byte stores (each wave's 8-row
// blocks transposed through the freed LDS tile) instead of one dword per
// lane and row: a quarter of the store instructions.
constexpr bool kBlurX4St = true;
// Interior-tile staging by LDS-DMA (global_load_lds_dwordx4) instead of
// 16-byte loads into VGPRs + ds_write_b128.
// (Measured alternative, round 2: VGPR staging -- the x4 launches 1-3 % slower.)
constexpr bool kBlurDma = true;
template <int R>
constexpr int blur_org() {  // tile column 0 = image column x0 - ORG
    return kBlurX4Ld && R <= 8 ? 8 : kBlurX4Ld && kBlurX4LdBig && R <= kBlurX4LdMaxR ? (R + 3) & ~3 : R;
}
// Radius 11..24 with the dword staging: pitch 112 (16 mod 32, conflict-free
// row-pass stores).  With the 16-byte staging (default) the rows stay unpadded
// (R = 13: 96 floats) so the interior tiles stage by LDS-DMA: the paired
// R = 13 launch 115.7 -> 113.0 us per 16 frames (tools/r3_blur_x4_ab.sh).
constexpr bool kBlurIW112 = false;
template <int R>
constexpr int blur_iw() {  // radius 9, 10: the next 16-mod-32 pitch (112) costs a workgroup per CU -- kept at 64 + 2R
    return kBlurIW16 && R <= 8 ? ((BLUR_TW + 2 * blur_org<R>() + 15) / 32) * 32 + 16
           : kBlurIW112 && R >= 11 && R <= 24 ? 112
                                                   : (BLUR_TW + 2 * blur_org<R>() + 3) & ~3;
}
template <int R>
constexpr int blur_lds_floats() {
    return blur_iw<R>() * (BLUR_TH + 2 * R) + 4;
}

// Tile `blk` of job J's nf * ntiles (64 x 32 outputs; frame-major, XCD order)
// with LDS `in`.  T = float, or uint8_t
// for a caller's 8-bit frame read by the frame's first blur (OpenCV converts
// CV_8U to float exactly, so the planes are those of the float frame with the
// same values).

template <int R, typename T, int NWAVES>
__device__ __forceinline__ void blur_tile(const BlurJob& J, int blk, float* __restrict__ in) {
    constexpr int BLUR_NW = NWAVES;                   // waves per workgroup
    constexpr int BLUR_CB = BLUR_TH / (8 * BLUR_NW);  // 8-row column-pass blocks per wave
    constexpr int IW = blur_iw<R>();                 // LDS row stride (floats)
    constexpr int IH = BLUR_TH + 2 * R;
    constexpr int ORG = blur_org<R>();               // LDS column 0 = image column x0 - ORG
    constexpr int SA = (ORG - R) & ~3, SS = (ORG - R) & 3;  // row window: aligned start, shift
    constexpr int NW = (SS + 2 * R + 4 + 3) / 4;     // float4 reads per row window
    static_assert(BLUR_TW - 4 + SA + 4 * NW <= IW, "row window inside the LDS row");
    const int t = xcd_tile(blk, J.ntiles * J.nf);
    const int f = t / J.ntiles, tile = t - f * J.ntiles;
    const T* __restrict__ src = fptr(static_cast<const T*>(J.src), f * J.sfs);
    float* __restrict__ dst = fptr(J.dst, f * J.dfs);
    float* __restrict__ dec_out = J.dec.p ? fptr(J.dec.p, f * J.dfs) : nullptr;
    unsigned* __restrict__ range_keys = J.range_keys ? fptr(J.range_keys, f * J.dfs) : nullptr;
    Counters* __restrict__ zero_ctr = J.zero_ctr ? fptr(J.zero_ctr, f * J.dfs) : nullptr;
    const int spitch = J.spitch, W = J.W, H = J.H, dpitch = J.dpitch;
    const Taps& taps = J.taps;
    // Row-pass results (`mid`, pitch IW) overwrite their own input row of
    // `in` in place: a row is read and written only by the same 16 lanes of
    // one wave, whose LDS reads complete before its writes (in-order LDS per
    // wave), so one tile of LDS serves both passes (more workgroups per CU).
    float* const mid = in;
    const int x0 = (tile % J.tilesX) * BLUR_TW, y0 = (tile / J.tilesX) * BLUR_TH;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // The frame's first blur also zeroes the frame counters (no memset node).
    // (Counters.pad[1] keeps its host-results request half: set by a host
    // frame's staging copy before this kernel, HostOut.)
    if (zero_ctr && tile == 0 && tid < (int)(sizeof(Counters) / 4))
        reinterpret_cast<unsigned*>(zero_ctr)[tid] =
            tid == offsetof(Counters, pad[1]) / 4 ? zero_ctr->pad[1] & ~((1u << kHostReqShift) - 1) : 0u;

    // Stage the input tile row by row: wave w takes rows w, w+4, ...; lane l
    // columns l and 64+l.  A row's source offset is wave-uniform (SGPR,
    // reflected in scalar code) and a lane's column offset is the same for
    // every row, so a staging load costs no vector address arithmetic.  All
    // loads are issued before the first LDS store.
    {
        constexpr int RW = BLUR_TW + 2 * R;  // <= 128: two column chunks
        constexpr int RPW = (IH + BLUR_NW - 1) / BLUR_NW;  // rows per wave
        const int wv = __builtin_amdgcn_readfirstlane(wave);
        const bool single = W > R + 1 && H > R + 1;  // one reflection suffices
        auto refl = [&](int p, int len) {
            if (single) {
                // One bounce is exact for every input of an in-image output
                // (|offset| <= R < len); tile positions past the image edge feed
                // only discarded outputs, so clamping them just keeps the read
                // in bounds.
                p = p < 0 ? -p : (p >= len ? 2 * len - 2 - p : p);
                return min(max(p, 0), len - 1);
            }
            return reflect101(p, len);
        };
        const int gx0 = refl(x0 - R + lane, W), gx1 = refl(x0 - R + 64 + min(lane, RW - 65), W);
        constexpr int ES = (int)sizeof(T);
        const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<T*>(src), 0, (int)min((long)spitch * H * ES, 0x7fffffffL), 0x00020000);
        const unsigned c0 = (unsigned)gx0 * ES, c1 = (unsigned)gx1 * ES;
        const int rowB = spitch * ES;  // bytes per source row
        float v0[RPW], v1[RPW];
        auto ld = [&](int i, int roff) {
            if constexpr (ES == 1) {
                v0[i] = (float)__builtin_amdgcn_raw_buffer_load_b8(rsrc, c0, roff, 0);
                v1[i] = (float)__builtin_amdgcn_raw_buffer_load_b8(rsrc, c1, roff, 0);
            } else {
                v0[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsrc, c0, roff, 0));
                v1[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsrc, c1, roff, 0));
            }
        };
        constexpr int QW = (BLUR_TW + 2 * ORG) / 4;  // float4s per staged row
        const bool x4 = ES == 4 && ORG % 4 == 0 && ORG >= R && x0 >= ORG &&
                        x0 + BLUR_TW + ORG <= W && y0 - R >= 0 && y0 - R + IH <= H;  // uniform
        if (x4) {
            // Interior tile: 16-byte loads of the QW-float4 rows, all in
            // flight before the first LDS store.
            static_assert(!(ES == 4 && ORG % 4 == 0) || 4 * QW <= IW, "x4 staging row inside the LDS row");
            constexpr int NQ = QW * IH, NT = 64 * BLUR_NW, QPT = (NQ + NT - 1) / NT;
            const int rb0 = (y0 - R) * spitch + x0 - ORG;
            if constexpr (kBlurDma && IW == 4 * QW) {
                // LDS-DMA (the LDS rows are unpadded: float4 q of the tile goes
                // to LDS float4 q; global_load_lds_dwordx4: a wave's 64 lanes
                // fill 1 KiB at M0), no VGPR round trip and no ds_write_b128.
                const float* fsrc = reinterpret_cast<const float*>(src);  // ES == 4 here
#pragma unroll
                for (int u = 0; u < QPT; u++) {
                    const int idx = tid + NT * u;
                    if (u < QPT - 1 || idx < NQ) {
                        const int row = idx / QW, qq = idx - row * QW;
                        __builtin_amdgcn_global_load_lds(
                            (const void*)(fsrc + rb0 + row * spitch + 4 * qq),
                            (__attribute__((address_space(3))) void*)(in + 4 * (NT * u + 64 * (tid >> 6))), 16, 0, 0);
                    }
                }
                // LDS-DMA writes are counted by vmcnt, not lgkmcnt: wait for this
                // wave's copies explicitly so the staging barrier below publishes
                // them whatever fence the compiler gives __syncthreads().
                __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
            } else {
                // Padded LDS rows (R = 13: 96 floats staged in a 112-float pitch):
                // 16-byte loads into VGPRs, then ds_write_b128 per float4.
                typedef unsigned u32x4s __attribute__((ext_vector_type(4)));
                u32x4s q4[QPT];
#pragma unroll
                for (int u = 0; u < QPT; u++) {
                    const int idx = min(tid + NT * u, NQ - 1), row = idx / QW, qq = idx - row * QW;
                    q4[u] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (unsigned)(rb0 + row * spitch + 4 * qq) * 4u, 0, 0);
                }
#pragma unroll
                for (int u = 0; u < QPT; u++) {
                    const int idx = tid + NT * u, row = idx / QW, qq = idx - row * QW;
                    if (u < QPT - 1 || idx < NQ) *reinterpret_cast<u32x4s*>(in + row * IW + 4 * qq) = q4[u];
                }
            }
        } else if (y0 - R >= 0 && y0 - R + IH <= H) {
            // Interior rows (most tiles): the row offset advances by a constant,
            // one s_add per row.  Rows past IH of the last step read in-range
            // data (or 0 past the buffer end) and are never stored.
            const int rb = __builtin_amdgcn_readfirstlane((y0 - R + wv) * rowB), rs = BLUR_NW * rowB;
#pragma unroll
            for (int i = 0; i < RPW; i++) ld(i, rb + i * rs);
        } else {
#pragma unroll
            for (int i = 0; i < RPW; i++) {
                const int ly = min(wv + BLUR_NW * i, IH - 1);
                ld(i, __builtin_amdgcn_readfirstlane(refl(y0 - R + ly, H) * rowB));
            }
        }
        // LDS row of step i: one base address + an immediate offset per row;
        // only the last step can fall past IH.
        float* const irow = in + wv * IW + lane + (ORG - R);
        if (!x4) {
#pragma unroll
            for (int i = 0; i < RPW; i++)
                if (i < RPW - 1 || wv + BLUR_NW * i < IH) irow[BLUR_NW * i * IW] = v0[i];
            if (lane < RW - 64) {
#pragma unroll
                for (int i = 0; i < RPW; i++)
                    if (i < RPW - 1 || wv + BLUR_NW * i < IH) irow[BLUR_NW * i * IW + 64] = v1[i];
            }
        }
    }
    __syncthreads();

    {
        // ds_read_b128 serves a wave in four 16-lane groups {0-3,12-15,20-27},
        // {4-11,16-19,28-31} (+32): give each group one row's 16 float4 blocks
        // so every group covers the 64 banks exactly once (conflict-free for
        // any row pitch).
        const int l = lane & 31;
        const bool grpB = (l >= 4 && l < 12) || (l >= 16 && l < 20) || l >= 28;
        const int blk = grpB ? (l < 12 ? l - 4 : (l < 20 ? l - 8 : l - 16)) : (l < 4 ? l : (l < 16 ? l - 8 : l - 12));
        const int xq = blk * 4;
        for (int ly = wave * 4 + (lane >> 5) * 2 + (grpB ? 1 : 0); ly < IH; ly += 4 * BLUR_NW) {
            float win[4 * NW];
            // The row's window starts at LDS column xq + ORG - R: read from the
            // aligned column xq + SA, the first SS values are skipped.
            const f32x4* p = reinterpret_cast<const f32x4*>(in + ly * IW + xq + SA);
#pragma unroll
            for (int v = 0; v < NW; v++) {
                f32x4 f = p[v];
                // Opaque use of all four lanes: otherwise the compiler narrows
                // the partly used last vector and splits the row into
                // misaligned ds_read2_b32/b64 pieces (bank conflicts).
                __asm__ volatile("" : "+v"(f));
                win[4 * v] = f[0];
                win[4 * v + 1] = f[1];
                win[4 * v + 2] = f[2];
                win[4 * v + 3] = f[3];
            }
            // Packed FP32: outputs (q, q+1) for q = 0, 2 share one v_pk_fma_f32
            // per tap (each lane an IEEE fma, so the chain is OpenCV's).  Their
            // operand (win[q+k], win[q+k+1]) is an even-aligned pair for even
            // q+k and an odd-aligned pair (built once per window) otherwise.
            f32x2 pe[2 * NW], po[2 * NW - 1];
#pragma unroll
            for (int j = 0; j < 2 * NW; j++) pe[j] = (f32x2){win[2 * j], win[2 * j + 1]};
#pragma unroll
            for (int j = 0; j < 2 * NW - 1; j++) po[j] = pk_mov_hi_lo(pe[j], pe[j + 1]);
            auto pr = [&](int i) -> f32x2 {  // (window[i], window[i+1]) = (win[SS+i], win[SS+i+1])
                i += SS;
                return (i & 1) ? po[i >> 1] : pe[i >> 1];
            };
            f32x2 s2[2];
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const int q = 2 * h;
                if constexpr (2 * R + 1 > 5) {
                    f32x2 a = {0.f, 0.f};
#pragma unroll
                    for (int k = 0; k <= 2 * R; k++) a = __builtin_elementwise_fma(pr(q + k), (f32x2)taps.w[k], a);
                    s2[h] = a;
                } else {
                    f32x2 a = pr(q + R) * (f32x2)taps.w[R];
#pragma unroll
                    for (int k = 1; k <= R; k++)
                        a = __builtin_elementwise_fma(pr(q + R - k) + pr(q + R + k), (f32x2)taps.w[R + k], a);
                    s2[h] = a;
                }
            }
            *reinterpret_cast<float4*>(mid + ly * IW + xq) = make_float4(s2[0][0], s2[0][1], s2[1][0], s2[1][1]);
        }
    }
    __syncthreads();

    float mx = -FLT_MAX, nmn = -FLT_MAX;  // pixel range (range_keys only)
    const int gx = x0 + lane;
    const bool full = y0 + BLUR_TH <= H && x0 + BLUR_TW <= W;  // uniform
    float outs[BLUR_CB][8];  // kBlurX4St: full-tile rows kept for the widened stores
#pragma unroll
    for (int cbk = 0; cbk < BLUR_CB; cbk++) {
        const int lx = lane, yb = (wave + cbk * BLUR_NW) * 8;
        // Column pairs (c[i], c[i+4]), one ds_read2st64_b32 each: output rows
        // (q, q+4) share every v_pk_add/v_pk_fma_f32 and no pair is assembled
        // from two loads.
        // (volatile: every element is loaded twice, into both pairs it belongs
        // to, instead of being loaded once and copied with v_mov.)
        const volatile __attribute__((address_space(3))) float* vmid =
            (const volatile __attribute__((address_space(3))) float*)(mid + yb * IW + lx);
        f32x2 cp[4 + 2 * R];
#pragma unroll
        for (int j = 0; j < 4 + 2 * R; j++) cp[j] = (f32x2){vmid[j * IW], vmid[(j + 4) * IW]};
        float out[8];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            f32x2 a = __builtin_elementwise_fma(cp[q + R], (f32x2)taps.w[R], (f32x2){0.f, 0.f});
#pragma unroll
            for (int k = 1; k <= R; k++) a = __builtin_elementwise_fma(cp[q + R + k] + cp[q + R - k], (f32x2)taps.w[R + k], a);
            out[q] = a[0];
            out[q + 4] = a[1];
        }
        if (kBlurX4St && full) {
#pragma unroll
            for (int q = 0; q < 8; q++) outs[cbk][q] = out[q];
        } else if (full) {
            // Full tile: unconditional buffer stores, the row step in the
            // scalar offset (no per-row address arithmetic or exec masking).
            const __amdgpu_buffer_rsrc_t drs = __builtin_amdgcn_make_buffer_rsrc(
                dst, 0, (int)min((long)dpitch * H * 4, 0x7fffffffL), 0x00020000);
            const unsigned voff = (unsigned)((y0 + yb) * dpitch + gx) * 4u;
#pragma unroll
            for (int q = 0; q < 8; q++)
                __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, out[q]), drs, voff, q * dpitch * 4, 0);
        } else {
#pragma unroll
            for (int q = 0; q < 8; q++) {
                const int gy = y0 + yb + q;
                if (gy < H && gx < W) dst[(size_t)gy * dpitch + gx] = out[q];
            }
        }
        if (dec_out && !(kBlurX4St && full)) {
            // The next octave's base plane (edge tiles; full tiles store it
            // from the LDS image below): even rows and columns of this plane
            // (y0, yb even), stored by the even lanes; other lanes get an
            // offset past the buffer, which the hardware drops (no branch).
            const __amdgpu_buffer_rsrc_t drs = __builtin_amdgcn_make_buffer_rsrc(
                dec_out, 0, (int)min((long)J.dec.pitch * J.dec.H * 4, 0x7fffffffL), 0x00020000);
            const bool cx = (gx & 1) == 0 && (gx >> 1) < J.dec.W;
#pragma unroll
            for (int q = 0; q < 8; q += 2) {
                const int dy = (y0 + yb + q) >> 1;
                const unsigned off = cx && dy < J.dec.H ? (unsigned)(dy * J.dec.pitch + (gx >> 1)) * 4u : 0x80000000u;
                __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, out[q]), drs, off, 0, 0);
            }
        }
        if (range_keys) {
#pragma unroll
            for (int q = 0; q < 8; q++) {
                if (y0 + yb + q < H && gx < W) {
                    mx = fmaxf(mx, out[q]);
                    nmn = fmaxf(nmn, -out[q]);
                }
            }
        }
    }
    if (kBlurX4St && full) {
        // Widened stores: every wave's column pass has read `mid` (barrier);
        // each wave writes its 8-row blocks into the free LDS tile as a plain
        // 64-float-pitch image and reads back its own rows as float4s (the
        // same wave, in-order LDS: no second barrier), one 16-byte store per
        // 4 columns.  ds_read_b128 groups then cover 64 distinct banks.
        __syncthreads();
#pragma unroll
        for (int cbk = 0; cbk < BLUR_CB; cbk++) {
            const int yb = (wave + cbk * BLUR_NW) * 8;
#pragma unroll
            for (int q = 0; q < 8; q++) in[(yb + q) * BLUR_TW + lane] = outs[cbk][q];
        }
        typedef unsigned u32x4t __attribute__((ext_vector_type(4)));
        const __amdgpu_buffer_rsrc_t drs =
            __builtin_amdgcn_make_buffer_rsrc(dst, 0, (int)min((long)dpitch * H * 4, 0x7fffffffL), 0x00020000);
#pragma unroll
        for (int cbk = 0; cbk < BLUR_CB; cbk++) {
            const int yb = (wave + cbk * BLUR_NW) * 8;
#pragma unroll
            for (int hh = 0; hh < 2; hh++) {
                const int row = yb + 4 * hh + (lane >> 4), c4 = 4 * (lane & 15);
                const u32x4t v = *reinterpret_cast<const u32x4t*>(in + row * BLUR_TW + c4);
                __builtin_amdgcn_raw_buffer_store_b128(v, drs, (unsigned)((y0 + row) * dpitch + x0 + c4) * 4u, 0, 0);
            }
        }
        if (dec_out) {
            // The next octave's base plane from the same LDS image: an 8-row
            // block gives 4 rows x 8 float4s of even rows and columns; lane l
            // takes block 2 it + l / 32, row (l % 32) / 8, float4 l % 8 (two
            // 16-byte LDS reads, the even elements, one 16-byte store).
            const __amdgpu_buffer_rsrc_t ers = __builtin_amdgcn_make_buffer_rsrc(
                dec_out, 0, (int)min((long)J.dec.pitch * J.dec.H * 4, 0x7fffffffL), 0x00020000);
            const int r4 = (lane & 31) >> 3, c8 = 8 * (lane & 7);
#pragma unroll
            for (int it = 0; it < (BLUR_CB + 1) / 2; it++) {
                const int cbk = 2 * it + (lane >> 5);
                const int yb = (wave + min(cbk, BLUR_CB - 1) * BLUR_NW) * 8;
                const f32x4* rp = reinterpret_cast<const f32x4*>(in + (yb + 2 * r4) * BLUR_TW + c8);
                const f32x4 a = rp[0], b = rp[1];
                const u32x4t v = __builtin_bit_cast(u32x4t, (f32x4){a[0], a[2], b[0], b[2]});
                const unsigned off =
                    cbk < BLUR_CB ? (unsigned)(((y0 + yb) / 2 + r4) * J.dec.pitch + x0 / 2 + c8 / 2) * 4u : 0x80000000u;
                __builtin_amdgcn_raw_buffer_store_b128(v, ers, off, 0, 0);
            }
        }
    }
    {
        // Pixel range of the plane (requested for octave 0 / plane 0 only: every
        // later plane is a convex combination of it).  The descriptor sizes its
        // fixed-point histogram scale from it.
        if (range_keys) {
            for (int off = 32; off > 0; off >>= 1) {
                mx = fmaxf(mx, __shfl_xor(mx, off));
                nmn = fmaxf(nmn, __shfl_xor(nmn, off));
            }
            __syncthreads();  // reuse `mid` for the per-wave partials
            if (lane == 0) {
                mid[wave] = mx;
                mid[BLUR_NW + wave] = nmn;
            }
            __syncthreads();
            if (tid == 0) {  // spread over kRangeSlots address pairs: no single hot atomic
                unsigned* slot = range_keys + 2 * (tile % kRangeSlots);
                float a = mid[0], b = mid[BLUR_NW];
                for (int w = 1; w < BLUR_NW; w++) {
                    a = fmaxf(a, mid[w]);
                    b = fmaxf(b, mid[BLUR_NW + w]);
                }
                atomicMax(slot, range_key(a));
                atomicMax(slot + 1, range_key(b));
            }
        }
    }
}

template <int R, typename T, int NW>
__global__ __launch_bounds__(64 * NW) void k_blur(BlurJob J) {
    __shared__ __attribute__((aligned(16))) float in[blur_lds_floats<R>()];
    blur_tile<R, T, NW>(J, blockIdx.x, in);
}

// Two independent blur jobs in one launch (blocks [0, A.ntiles) take A): the
// first blurs of octave o+1 run beside the last blurs of octave o, which they
// do not depend on, so a frame needs fewer launches (each costs ~0.7-1.5 us of
// dispatch) and small-octave tiles fill CUs the larger
// job leaves idle.
template <int RA, int RB, int NW>
__global__ __launch_bounds__(64 * NW) void k_blur2(BlurJob A, BlurJob B) {
    constexpr int NA = blur_lds_floats<RA>(), NB = blur_lds_floats<RB>();
    __shared__ __attribute__((aligned(16))) float in[NA > NB ? NA : NB];
    const int na = A.ntiles * A.nf;
    if ((int)blockIdx.x < na)
        blur_tile<RA, float, NW>(A, blockIdx.x, in);
    else
        blur_tile<RB, float, NW>(B, blockIdx.x - na, in);
}

static BlurJob make_job(const void* src, int spitch, int W, int H, float* dst, int dpitch, const DecOut& dec,
                        const Taps& taps, unsigned* range_keys, Counters* zero_ctr, const Frames& fr, long sfs) {
    BlurJob j;
    j.nf = fr.nf;
    j.sfs = sfs;
    j.dfs = fr.stride;
    j.src = src;
    j.dst = dst;
    j.dec = dec;
    j.range_keys = range_keys;
    j.zero_ctr = zero_ctr;
    j.spitch = spitch;
    j.W = W;
    j.H = H;
    j.dpitch = dpitch;
    j.tilesX = (W + BLUR_TW - 1) / BLUR_TW;
    j.ntiles = j.tilesX * ((H + BLUR_TH - 1) / BLUR_TH);
    j.taps = taps;
    return j;
}

using BlurLaunch = void (*)(const BlurJob&, hipStream_t);

template <int R>
void blur_launch_r(const BlurJob& j, hipStream_t s) {
    const int tiles = j.ntiles * j.nf;
    if (blur_waves(tiles) == 4)
        hipLaunchKernelGGL((k_blur<R, float, 4>), dim3(tiles), dim3(256), 0, s, j);
    else
        hipLaunchKernelGGL((k_blur<R, float, 8>), dim3(tiles), dim3(512), 0, s, j);
}

template <int... Rs>
constexpr std::array<BlurLaunch, sizeof...(Rs)> blur_table(std::integer_sequence<int, Rs...>) {
    return {&blur_launch_r<Rs + 1>...};
}
static const std::array<BlurLaunch, kMaxTaps / 2> kBlurTable = blur_table(std::make_integer_sequence<int, kMaxTaps / 2>{});

// Pair instantiations: the radii of the default pyramid (sigma 1.6, 3 layers:
// 5, 6, 8, 10, 13), larger radius first.  Other pairs launch separately.
template <int RA, int RB>
void blur2_launch(const BlurJob& a, const BlurJob& b, hipStream_t s) {
    const int tiles = a.ntiles * a.nf + b.ntiles * b.nf;
    if (blur_waves(tiles) == 4)
        hipLaunchKernelGGL((k_blur2<RA, RB, 4>), dim3(tiles), dim3(256), 0, s, a, b);
    else
        hipLaunchKernelGGL((k_blur2<RA, RB, 8>), dim3(tiles), dim3(512), 0, s, a, b);
}
bool launch_blur_pair_jobs(const BlurJob& a, const BlurJob& b, hipStream_t s) {
    const int ra = a.taps.n >> 1, rb = b.taps.n >> 1;
#define SIFT_PAIR(X, Y)                      \
    if (ra == X && rb == Y) {                \
        blur2_launch<X, Y>(a, b, s);         \
        return true;                         \
    }                                        \
    if (ra == Y && rb == X) {                \
        blur2_launch<X, Y>(b, a, s);         \
        return true;                         \
    }
    SIFT_PAIR(6, 5)
    SIFT_PAIR(8, 5)
    SIFT_PAIR(8, 6)
    SIFT_PAIR(10, 5)
    SIFT_PAIR(10, 6)
    SIFT_PAIR(10, 8)
    SIFT_PAIR(13, 5)
    SIFT_PAIR(13, 6)
    SIFT_PAIR(13, 8)
    SIFT_PAIR(13, 10)
#undef SIFT_PAIR
    return false;
}

bool launch_blur_pair(const BlurDesc& a, const BlurDesc& b, const Frames& fr, hipStream_t s) {
    return launch_blur_pair_jobs(make_job(a.src, a.spitch, a.W, a.H, a.dst, a.dpitch, a.dec, *a.taps,
                                          nullptr, nullptr, fr, fr.stride),
                                 make_job(b.src, b.spitch, b.W, b.H, b.dst, b.dpitch, b.dec, *b.taps,
                                          nullptr, nullptr, fr, fr.stride),
                                 s);
}

bool launch_blur_u8(const uint8_t* src, int spitch, int W, int H, float* dst, int dpitch, const Taps& taps,
                    const Frames& fr, long sfs, hipStream_t s, unsigned* range_keys, Counters* zero_ctr) {
    const BlurJob j = make_job(src, spitch, W, H, dst, dpitch, DecOut{}, taps, range_keys, zero_ctr, fr, sfs);
    const int tiles = j.ntiles * j.nf;
    const bool big = blur_waves(tiles) == 4;
    switch (taps.n >> 1) {
        case 5:
            if (big) hipLaunchKernelGGL((k_blur<5, uint8_t, 4>), dim3(tiles), dim3(256), 0, s, j);
            else hipLaunchKernelGGL((k_blur<5, uint8_t, 8>), dim3(tiles), dim3(512), 0, s, j);
            return true;
        case 6:
            if (big) hipLaunchKernelGGL((k_blur<6, uint8_t, 4>), dim3(tiles), dim3(256), 0, s, j);
            else hipLaunchKernelGGL((k_blur<6, uint8_t, 8>), dim3(tiles), dim3(512), 0, s, j);
            return true;
        default: return false;
    }
}

__global__ __launch_bounds__(256) void k_u8_to_f32(const uint8_t* __restrict__ src, int spitch, int W, int H,
                                                   float* __restrict__ dst, int dpitch, long sfs, long dfs) {
    src = fptr(src, blockIdx.z * sfs);
    dst = fptr(dst, blockIdx.z * dfs);
    const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y;
    if (x < W) dst[(size_t)y * dpitch + x] = (float)src[(size_t)y * spitch + x];
}

void launch_u8_to_f32(const uint8_t* src, int spitch, int W, int H, float* dst, int dpitch, const Frames& fr,
                      long sfs, hipStream_t s) {
    hipLaunchKernelGGL(k_u8_to_f32, dim3((W + 255) / 256, H, fr.nf), dim3(256), 0, s, src, spitch, W, H, dst, dpitch,
                       sfs, fr.stride);
}

// The kernel node launch_blur (without a decimated output) and
// launch_upsample2x would make, for a captured frame graph whose head node
// is re-pointed at each frame's input (hipGraphExecKernelNodeSetParams).
template <int R>
const void* blur_fn(int nw) {
    return nw == 4 ? reinterpret_cast<const void*>(&k_blur<R, float, 4>)
                   : reinterpret_cast<const void*>(&k_blur<R, float, 8>);
}
template <int... Rs>
constexpr std::array<const void* (*)(int), sizeof...(Rs)> blur_fn_table(std::integer_sequence<int, Rs...>) {
    return {&blur_fn<Rs + 1>...};
}
static const std::array<const void* (*)(int), kMaxTaps / 2> kBlurFnTable =
    blur_fn_table(std::make_integer_sequence<int, kMaxTaps / 2>{});
static_assert(sizeof(BlurJob) <= sizeof(HeadNode::args), "head node argument storage");

void head_blur_node(HeadNode& h, const float* src, int spitch, int W, int H, float* dst, int dpitch, const Taps& taps,
                    const Frames& fr, long sfs, unsigned* range_keys, Counters* zero_ctr) {
    const BlurJob j = make_job(src, spitch, W, H, dst, dpitch, DecOut{}, taps, range_keys, zero_ctr, fr, sfs);
    const int tiles = j.ntiles * j.nf, nw = blur_waves(tiles);
    std::memcpy(h.args, &j, sizeof j);
    h.argv[0] = h.args;
    h.p = hipKernelNodeParams{};
    h.p.func = const_cast<void*>(kBlurFnTable[(taps.n >> 1) - 1](nw));
    h.p.gridDim = dim3(tiles);
    h.p.blockDim = dim3(64 * nw);
    h.p.sharedMemBytes = 0;
    h.p.kernelParams = h.argv;
    h.p.extra = nullptr;
}

void head_upsample_node(HeadNode& h, const float* src, int spitch, int W, int H, float* dst, int dpitch,
                        const Frames& fr, long sfs) {
    // k_upsample2x<float>(src, spitch, W, H, dst, dpitch, sfs, dfs): each argument at its own slot.
    unsigned char* a = h.args;
    auto put = [&](int i, const void* v, size_t n) {
        std::memcpy(a + 16 * i, v, n);
        h.argv[i] = a + 16 * i;
    };
    put(0, &src, sizeof src);
    put(1, &spitch, sizeof spitch);
    put(2, &W, sizeof W);
    put(3, &H, sizeof H);
    put(4, &dst, sizeof dst);
    put(5, &dpitch, sizeof dpitch);
    put(6, &sfs, sizeof sfs);
    put(7, &fr.stride, sizeof fr.stride);
    h.p = hipKernelNodeParams{};
    h.p.func = reinterpret_cast<void*>(&k_upsample2x<float>);
    h.p.gridDim = up_grid(W, H, fr.nf);
    h.p.blockDim = dim3(256);
    h.p.sharedMemBytes = 0;
    h.p.kernelParams = h.argv;
    h.p.extra = nullptr;
}

void launch_blur(const float* src, int spitch, int W, int H, float* dst, int dpitch, const DecOut& dec,
                 const Taps& taps, const Frames& fr, long sfs, hipStream_t s, unsigned* range_keys,
                 Counters* zero_ctr) {
    const int r = taps.n >> 1;  // 1 .. kMaxTaps/2 (taps.n >= 3 by construction)
    kBlurTable[r - 1](make_job(src, spitch, W, H, dst, dpitch, dec, taps, range_keys, zero_ctr, fr, sfs), s);
}

// ---------------------------------------------------------------------------
// Pyramid tail: every blur of the small octaves o >= T of a frame in ONE
// workgroup (1024 threads, one per frame), planes held in LDS.  A single
// frame's small octaves were one launch per blur job (752x480, auto octaves:
// 14 launches of 1-2 tiles for octaves 3..6, ~5 us each: the launch and one
// tile's load -> LDS -> passes -> store chain, almost none of it work); here
// octave T's base plane is read once and every plane is blurred LDS -> LDS
// with the operations of blur_tile in the same order (OpenCV's sepFilter2D:
// the row filter, then the symmetric column filter; reflect-101 borders,
// looping for kernels wider than the octave), stored for the keypoint stages,
// and plane L's even rows and columns become the next octave's base (LDS and
// HBM).  Row pass A -> B, column pass B -> A; the LDS rows have an odd pitch:
// the row pass gives consecutive lanes consecutive rows, the column pass
// consecutive columns (conflict-free both ways).  The taps of the plane are
// staged in LDS (wave-uniform reads).  The octaves it takes are bounded by
// work, not LDS: one CU's VALU runs the whole tail (tail_first_octave).
// ---------------------------------------------------------------------------
constexpr int kTailThreads = 1024;
constexpr int kTailRun = 4;     // outputs per thread and run (along the pass)
constexpr int kTailRmax = 16;   // radius bound of the tail's unrolled windows
constexpr int kTailMaxDim = 512;  // octave width / height bound (reflection tables)

__host__ __device__ __forceinline__ int tail_pitch(int W) { return W | 1; }

// HBM stores as global_store (not flat: a flat store counts on lgkmcnt too,
// so the next run's LDS wait would also wait for it).  The tail's barriers
// fence LDS only (lds_barrier): __syncthreads() would wait for every plane
// store to be acknowledged before the next pass (56 us for 752x480's tail);
// the planes are read by later launches only.
__device__ __forceinline__ void gstore(float* p, size_t i, float v) {
    ((__attribute__((address_space(1))) float*)p)[i] = v;
}
__device__ __forceinline__ float gload(const float* p, size_t i) {
    return ((const __attribute__((address_space(1))) float*)p)[i];
}

// One instantiation per radius class RP (the largest radius of the tail's
// planes, rounded up to 4, 8, 13 or 16), every plane's taps zero-padded to
// 2 RP + 1: in these sums every term is >= 0 (non-negative pixels and taps),
// so a zero-weight fma adds a signed zero to a non-negative sum and leaves it
// bit-identical, and a leading one leaves s = +0 until the first real tap --
// the padded chain is OpenCV's chain.  (Per-radius instantiations dispatched
// per plane: 56 us for 752x480's tail, its code cold in the instruction cache
// at every plane.)  The window loads of a run are all issued before its
// first fma.
template <int RP>
__device__ __forceinline__ void tail_row_pass(const float* __restrict__ A, float* __restrict__ B, int W, int H, int P,
                                              bool small, const float* __restrict__ wp, const int* __restrict__ xo) {
    constexpr int NWIN = kTailRun + 2 * RP;
    const int nrx = (W + kTailRun - 1) / kTailRun, nruns = nrx * H;
    for (int r = threadIdx.x; r < nruns; r += kTailThreads) {
        const int y = r % H, xb = (r / H) * kTailRun;  // consecutive lanes: consecutive rows
        const float* row = A + y * P;
        // Source column of window slot k: xb - RP + k (runs at the borders
        // through the reflection table xo[j] = reflect101(j - RP), j = xb + k).
        float win[NWIN];
        if (xb - RP >= 0 && xb + kTailRun - 1 + RP < W) {
#pragma unroll
            for (int k = 0; k < NWIN; k++) win[k] = row[xb - RP + k];
        } else {
            int ix[NWIN];
#pragma unroll
            for (int k = 0; k < NWIN; k++) ix[k] = xo[xb + k];
#pragma unroll
            for (int k = 0; k < NWIN; k++) win[k] = row[ix[k]];
        }
        float s[kTailRun];
        if (!small) {  // RowFilter: s = 0; s = fma(x[k], w[k], s), k = 0..2R
#pragma unroll
            for (int q = 0; q < kTailRun; q++) s[q] = 0.f;
#pragma unroll
            for (int k = 0; k <= 2 * RP; k++) {
                const float wk = wp[k];
#pragma unroll
                for (int q = 0; q < kTailRun; q++) s[q] = __fmaf_rn(win[q + k], wk, s[q]);
            }
        } else {  // SymmRowSmall (2R + 1 <= 5): s = x0 w0; s = fma(x[-k] + x[+k], w_k, s)
            const float wc = wp[RP];
#pragma unroll
            for (int q = 0; q < kTailRun; q++) s[q] = win[q + RP] * wc;
#pragma unroll
            for (int k = 1; k <= 2 && k <= RP; k++) {
                const float wk = wp[RP + k];
#pragma unroll
                for (int q = 0; q < kTailRun; q++) s[q] = __fmaf_rn(win[q + RP - k] + win[q + RP + k], wk, s[q]);
            }
        }
#pragma unroll
        for (int q = 0; q < kTailRun; q++)
            if (xb + q < W) B[y * P + xb + q] = s[q];
    }
}

// Column pass (SymmColumnFilter: s = fma(c, w_R, 0); s = fma(down_k + up_k,
// w_{R+k}, s)) B -> A and the plane to HBM; with `dec`, the even rows and
// columns also go to the next octave's base (LDS N and HBM).
template <int RP>
__device__ __forceinline__ void tail_col_pass(const float* __restrict__ B, float* __restrict__ A, int W, int H, int P,
                                              const float* __restrict__ wp, const int* __restrict__ yo,
                                              float* __restrict__ gdst, int gpitch, bool dec, float* __restrict__ N,
                                              int NP, float* __restrict__ gnext, int gnpitch) {
    constexpr int NWIN = kTailRun + 2 * RP;
    const int nry = (H + kTailRun - 1) / kTailRun, nruns = nry * W;
    for (int r = threadIdx.x; r < nruns; r += kTailThreads) {
        const int x = r % W, yb = (r / W) * kTailRun;  // consecutive lanes: consecutive columns
        float win[NWIN];
        if (yb - RP >= 0 && yb + kTailRun - 1 + RP < H) {
#pragma unroll
            for (int k = 0; k < NWIN; k++) win[k] = B[(yb - RP + k) * P + x];
        } else {
            int iy[NWIN];
#pragma unroll
            for (int k = 0; k < NWIN; k++) iy[k] = yo[yb + k];
#pragma unroll
            for (int k = 0; k < NWIN; k++) win[k] = B[iy[k] * P + x];
        }
        float s[kTailRun];
        const float wc = wp[RP];
#pragma unroll
        for (int q = 0; q < kTailRun; q++) s[q] = __fmaf_rn(win[q + RP], wc, 0.f);
#pragma unroll
        for (int k = 1; k <= RP; k++) {
            const float wk = wp[RP + k];
#pragma unroll
            for (int q = 0; q < kTailRun; q++) s[q] = __fmaf_rn(win[q + RP + k] + win[q + RP - k], wk, s[q]);
        }
#pragma unroll
        for (int q = 0; q < kTailRun; q++) {
            const int y = yb + q;
            if (y < H) {
                A[y * P + x] = s[q];
#if !defined(SIFT_TAIL_DIAG) || SIFT_TAIL_DIAG != 4
                gstore(gdst, (size_t)y * gpitch + x, s[q]);
#endif
                if (dec && !((x | y) & 1) && (x >> 1) < (W >> 1) && (y >> 1) < (H >> 1)) {
                    N[(y >> 1) * NP + (x >> 1)] = s[q];
                    gstore(gnext, (size_t)(y >> 1) * gnpitch + (x >> 1), s[q]);
                }
            }
        }
    }
}

template <int RP>
__device__ __forceinline__ void tail_octaves(const TailDesc& T, float* lds, const float (*wall)[2 * kTailRmax + 1],
                                             int* xo, int* yo, long foff) {
    int aOff = 0, nOff = T.regionX;
    const int bOff = T.regionX + T.regionY;
    for (int o = T.o0; o < T.nOct; o++) {
        const OctGeom& g = T.oct[o];
        const OctGeom& gn = T.oct[o + 1 < T.nOct ? o + 1 : o];
        float* base = fptr(g.base, foff);
        const int P = tail_pitch(g.W);
        // Reflection tables for the padded radius (the same for every plane).
        lds_barrier();
        const int t = threadIdx.x;
        if (t < g.W + 2 * RP + kTailRun) xo[t] = reflect101(min(t - RP, g.W - 1 + RP), g.W);
        if (t < g.H + 2 * RP + kTailRun) yo[t] = reflect101(min(t - RP, g.H - 1 + RP), g.H);
        for (int i = 1; i < T.L + 3; i++) {
#if defined(SIFT_TAIL_DIAG) && SIFT_TAIL_DIAG == 5  // timing builds only: s_memtime per plane -> octave 0, plane 0
            if (threadIdx.x == 0) {
                const unsigned long long t0 = __builtin_amdgcn_s_memtime();
                unsigned* st = reinterpret_cast<unsigned*>(fptr(T.oct[0].base, foff));
                const int slot = (o - T.o0) * (T.L + 2) + (i - 1);
                st[2 * slot] = (unsigned)t0;
                st[2 * slot + 1] = (unsigned)(t0 >> 32);
            }
#endif
            const bool small = T.taps[i].n <= 5, dec = o + 1 < T.nOct && i == T.L;
            const float* wp = wall[i];
            lds_barrier();  // A written (load / previous column pass); tables set
#if !defined(SIFT_TAIL_DIAG) || SIFT_TAIL_DIAG != 1  // timing-variant builds only (tools/ab_variant.sh)
            tail_row_pass<RP>(lds + aOff, lds + bOff, g.W, g.H, P, small, wp, xo);
#endif
            lds_barrier();
#if !defined(SIFT_TAIL_DIAG) || SIFT_TAIL_DIAG != 2
            tail_col_pass<RP>(lds + bOff, lds + aOff, g.W, g.H, P, wp, yo, base + (size_t)i * g.planeStride, g.pitch,
                              dec, lds + nOff, tail_pitch(gn.W), dec ? fptr(gn.base, foff) : base, gn.pitch);
#endif
        }
        const int tt = aOff;  // the next octave works on its base; its own next base goes where this plane was
        aOff = nOff;
        nOff = tt;
    }
}

__global__ __launch_bounds__(kTailThreads) void k_blur_tail(TailDesc T, long fs) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    __shared__ float wall[kTailMaxPlanes][2 * kTailRmax + 1];  // every plane's taps, zero-padded to 2 RP + 1
    __shared__ int xo[kTailMaxDim + 2 * kTailRmax + kTailRun], yo[kTailMaxDim + 2 * kTailRmax + kTailRun];
    const long foff = (long)blockIdx.x * fs;
    const int RP = T.rpad;
    // LDS (float offsets into lds, not pointers, so every access stays a
    // ds_*): A = the plane (region X, then the next base's region,
    // alternating), B = the row pass's output, N = the next octave's base.
    {
        // Taps from the kernel arguments, padded: one round of loads here
        // instead of a dependent kernarg load before every plane.
        for (int t = threadIdx.x; t < kTailMaxPlanes * (2 * kTailRmax + 1); t += kTailThreads) {
            const int i = t / (2 * kTailRmax + 1), k = t - i * (2 * kTailRmax + 1);
            float v = 0.f;
            if (i < T.L + 3 && k <= 2 * RP) {
                const int R = T.taps[i].n >> 1, kk = k - RP + R;
                if (kk >= 0 && kk <= 2 * R) v = T.taps[i].w[kk];
            }
            wall[i][k] = v;
        }
        const OctGeom& g = T.oct[T.o0];
        const float* src = fptr(g.base, foff);
        const int P = tail_pitch(g.W);
        for (int i = threadIdx.x; i < g.W * g.H; i += kTailThreads) {
            const int y = i / g.W, x = i - y * g.W;
            lds[y * P + x] = gload(src, (size_t)y * g.pitch + x);
        }
    }
#if defined(SIFT_TAIL_DIAG) && SIFT_TAIL_DIAG == 3
    return;
#endif
    switch (RP) {
        case 4: tail_octaves<4>(T, lds, wall, xo, yo, foff); break;
        case 8: tail_octaves<8>(T, lds, wall, xo, yo, foff); break;
        case 13: tail_octaves<13>(T, lds, wall, xo, yo, foff); break;
        default: tail_octaves<16>(T, lds, wall, xo, yo, foff); break;
    }
}

constexpr long kTailMaxPx = 6000;  // largest octave the tail takes (one CU's VALU: 752x480 octave 3 = 94x60; 1920x1200 octave 4 (120x75) lost 10-20 us)
int tail_first_octave(const PyrDesc& pyr, const Taps* taps, int L) {
    for (int i = 1; i < L + 3; i++)
        if ((taps[i].n >> 1) > kTailRmax) return pyr.nOct;
    int T = pyr.nOct;
    for (int o = pyr.nOct - 1; o >= 0; o--) {
        const OctGeom& g = pyr.oct[o];
        const long px = (long)tail_pitch(g.W) * g.H;
        const long nxt = o + 1 < pyr.nOct ? (long)tail_pitch(pyr.oct[o + 1].W) * pyr.oct[o + 1].H : 0;
        if ((long)g.W * g.H > kTailMaxPx || 2 * px + nxt > kTailLdsFloats || g.W > kTailMaxDim ||
            g.H > kTailMaxDim)
            break;
        T = o;
    }
    return T;
}

hipError_t tail_init() {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&k_blur_tail),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)(sizeof(float) * kTailLdsFloats));
}

void launch_blur_tail(const PyrDesc& pyr, const Taps* taps, int L, int o0, const Frames& fr, hipStream_t s) {
    TailDesc T{};
    T.o0 = o0;
    T.nOct = pyr.nOct;
    T.L = L;
    for (int o = 0; o < pyr.nOct; o++) T.oct[o] = pyr.oct[o];
    for (int i = 0; i < L + 3 && i < kTailMaxPlanes; i++) T.taps[i] = taps[i];
    int rmax = 0;
    for (int i = 1; i < L + 3; i++) rmax = std::max(rmax, taps[i].n >> 1);
    T.rpad = rmax <= 4 ? 4 : rmax <= 8 ? 8 : rmax <= 13 ? 13 : 16;
    T.regionX = tail_pitch(pyr.oct[o0].W) * pyr.oct[o0].H;
    T.regionY = o0 + 1 < pyr.nOct ? tail_pitch(pyr.oct[o0 + 1].W) * pyr.oct[o0 + 1].H : 0;
    const size_t lds = sizeof(float) * (size_t)(2 * T.regionX + T.regionY);
    hipLaunchKernelGGL(k_blur_tail, dim3(fr.nf), dim3(kTailThreads), lds, s, T, fr.stride);
}

// ---------------------------------------------------------------------------
// DoG + 3x3x3 extremum scan for one octave.  DoG planes D_d = G_{d+1} - G_d are
// formed in LDS for a 64 x 16 tile plus a 1-pixel halo (never written to HBM);
// every (layer 1..L, r, c) with border 5 is tested exactly as OpenCV's
// findScaleSpaceExtremaComputer: |v| > threshold and v >= (<=) all 26
// neighbours.  Hits are compacted with a wave ballot and one atomic per wave.
// Reference: MatOps.cu:39-181 (mask + full-volume CUB scan + scatter).
// ---------------------------------------------------------------------------
constexpr int EX_TW = 64;
constexpr int EX_TH = 16;
constexpr int EX_SW = EX_TW + 2;
constexpr int EX_SH = EX_TH + 2;
constexpr int EX_LIST = 512;  // per-workgroup candidate list (LDS)

// LT = compile-time layer count (1..6), or 0 for the generic runtime-L path.
template <int LT>
__global__ __launch_bounds__(256) void k_extrema(OctGeom g, int Lrt, int o, float thr, uint2* __restrict__ cand,
                                                 Counters* __restrict__ ctr, unsigned cap, long fs) {
    extern __shared__ float dog[];  // (L+2) planes of EX_SH x EX_SW
    g.base = fptr(g.base, blockIdx.z * fs);  // frame blockIdx.z
    cand = fptr(cand, blockIdx.z * fs);
    ctr = fptr(ctr, blockIdx.z * fs);
    const int L = LT > 0 ? LT : Lrt;
    const int tid = threadIdx.x;
    const int tile = xcd_tile(blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * gridDim.y);
    const int x0 = (tile % gridDim.x) * EX_TW, y0 = (tile / gridDim.x) * EX_TH;
    const int W = g.W, H = g.H, pitch = g.pitch;
    constexpr int PS = EX_SH * EX_SW;
    constexpr int PER = (PS + 255) / 256;
    __shared__ unsigned s_cnt, s_base;
    __shared__ uint2 s_list[EX_LIST];
    if (tid == 0) s_cnt = 0;

    if constexpr (LT > 0) {
        // All (L+3) x PER loads of this thread in flight at once, then DoG -> LDS.
        float v[PER][LT + 3];
#pragma unroll
        for (int u = 0; u < PER; u++) {
            const int i = tid + 256 * u;
            const int ly = i / EX_SW, lx = i - ly * EX_SW;
            const int gy = y0 - 1 + ly, gx = x0 - 1 + lx;
            const bool in = i < PS && gy >= 0 && gy < H && gx >= 0 && gx < W;
            const float* p = g.base + (size_t)min(max(gy, 0), H - 1) * pitch + min(max(gx, 0), W - 1);
#pragma unroll
            for (int d = 0; d < LT + 3; d++) {
                const float x = p[(size_t)d * g.planeStride];  // unconditional (clamped) load
                v[u][d] = in ? x : 0.f;
            }
        }
#pragma unroll
        for (int u = 0; u < PER; u++) {
            const int i = tid + 256 * u;
            if (i < PS) {
#pragma unroll
                for (int d = 0; d < LT + 2; d++) dog[d * PS + i] = v[u][d + 1] - v[u][d];
            }
        }
    } else {
        for (int i = tid; i < PS; i += 256) {
            const int ly = i / EX_SW, lx = i - ly * EX_SW;
            const int gy = y0 - 1 + ly, gx = x0 - 1 + lx;
            if (gy >= 0 && gy < H && gx >= 0 && gx < W) {
                const float* p = g.base + (size_t)gy * pitch + gx;
                float prev = p[0];
                for (int d = 0; d < L + 2; d++) {
                    const float next = p[(size_t)(d + 1) * g.planeStride];
                    dog[d * PS + i] = next - prev;
                    prev = next;
                }
            } else {
                for (int d = 0; d < L + 2; d++) dog[d * PS + i] = 0.f;
            }
        }
    }
    __syncthreads();

    const int lane = tid & 63;
    const int total = EX_TH * EX_TW * L;
    for (int base = 0; base < total; base += 256) {
        const int i = base + tid;
        bool hit = false;
        int layer = 0, r = 0, c = 0;
        if (i < total) {
            layer = 1 + i / (EX_TH * EX_TW);
            const int rem = i - (layer - 1) * (EX_TH * EX_TW);
            const int ly = rem >> 6, lx = rem & 63;
            r = y0 + ly;
            c = x0 + lx;
            if (r >= 5 && r < H - 5 && c >= 5 && c < W - 5) {
                const float* cur = dog + layer * PS + (ly + 1) * EX_SW + (lx + 1);
                const float val = cur[0];
                if (fabsf(val) > thr) {
                    hit = true;
                    if (val > 0) {
#pragma unroll
                        for (int d = -1; d <= 1; d++)
#pragma unroll
                            for (int dy = -1; dy <= 1; dy++)
#pragma unroll
                                for (int dx = -1; dx <= 1; dx++) hit &= val >= cur[d * PS + dy * EX_SW + dx];
                    } else {
#pragma unroll
                        for (int d = -1; d <= 1; d++)
#pragma unroll
                            for (int dy = -1; dy <= 1; dy++)
#pragma unroll
                                for (int dx = -1; dx <= 1; dx++) hit &= val <= cur[d * PS + dy * EX_SW + dx];
                    }
                }
            }
        }
        // Hits go to a workgroup-local LDS list (wave ballot + one LDS atomic
        // per wave); the list is flushed with ONE global atomic per workgroup.
        const unsigned long long mask = __ballot(hit);
        if (mask) {
            unsigned basepos = 0;
            if (lane == 0) basepos = atomicAdd(&s_cnt, (unsigned)__popcll(mask));
            basepos = __shfl(basepos, 0);
            if (hit) {
                const unsigned pos = basepos + (unsigned)__popcll(mask & ((1ull << lane) - 1ull));
                const uint2 q = make_uint2((unsigned)(o << 8 | layer), (unsigned)(r << 16 | c));
                if (pos < EX_LIST) {
                    s_list[pos] = q;
                } else {  // plateau-heavy tile: spill straight to the global list
                    const unsigned gp = atomicAdd(&ctr->cand, 1u);
                    if (gp < cap)
                        cand[gp] = q;
                    else
                        atomicOr(&ctr->overflow, 1u);
                }
            }
        }
    }
    __syncthreads();
    const unsigned nl = min(s_cnt, (unsigned)EX_LIST);
    if (tid == 0) s_base = nl ? atomicAdd(&ctr->cand, nl) : 0u;
    __syncthreads();
    for (unsigned k = tid; k < nl; k += 256) {
        const unsigned pos = s_base + k;
        if (pos < cap)
            cand[pos] = s_list[k];
        else
            atomicOr(&ctr->overflow, 1u);
    }
}

// ---------------------------------------------------------------------------
// Register-streaming extrema for L = 1..6 (the common case; k_extrema above
// serves larger L).  Four columns per lane: one wave covers a 256-column x
// EX4_TR-row strip, rows streaming top to bottom with EX4_AHEAD rows' loads in
// flight, with
// 16-byte loads (one buffer_load_dwordx4 per row and plane), plus one dword
// per row and plane for the strip's outer neighbours (lane 0: column x0-1,
// lane 63: column x0+256).  Per row the 5 DoG planes are formed in registers
// and kept in a 3-row ring; a tested row takes the vertical max/min of its
// three rows per column, then the horizontal 3-max in-lane, with the columns
// across lane boundaries brought in by one DPP move each (lane 0 / 63 keep
// their own outer column as the DPP's old value).  "v >= all 26 neighbours"
// is exactly "v == max of the 3x3x3 block" (the block contains v), so the
// decision per pixel is OpenCV's and the oracle's: |v| > threshold and
// v >= (<=) all 26, with no LDS staging.
// ---------------------------------------------------------------------------
constexpr int EX4_LIST = 2048;  // per-workgroup candidate list (LDS): a 256 x 32 x L block can hold
                                // ~7 % extrema on textured frames; overflow spills to HBM
// Columns per lane of the extrema strips.  (Measured alternative, round 3: 2
// columns per lane, 137 VGPRs / 3 waves per SIMD: 266-268 vs 252 us per
// 16-frame launch.)
constexpr int kExCpl = 4;
constexpr int EX4_COLS = 64 * kExCpl;  // columns per wave

// One workgroup = 4 waves stacked vertically over a 256-column strip: block
// `tile` of the octave (strips across; the caller picks the XCD order).
// A wave tests NB * EX4_TR consecutive rows as one stream (the 3-row DoG ring
// and the loads ahead carry across its EX4_TR-row steps), so the two halo
// rows above and below are read once per NB * EX4_TR rows instead of once per
// EX4_TR: strips of 6 rows read 8 (1.20x algorithmic HBM bytes measured at
// 16 frames, round-3 verdict), 24-row streams read 26.
template <int LT, int EX4_TR, int EX4_AHEAD, int NB = 1, int CPL = kExCpl>
__device__ __forceinline__ void extrema_block(const OctGeom& g, int o, float thr, uint2* __restrict__ cand,
                                              Counters* __restrict__ ctr, unsigned cap, int tile, int strips,
                                              uint2* s_list, unsigned& s_cnt, unsigned& s_base) {
    constexpr int NG = LT + 3, ND = LT + 2;
    static_assert(CPL * LT <= 31 && (CPL == 2 || CPL == 4), "hit bits per row");
    static_assert(NB == 1 || (EX4_TR % 3 == 0 && EX4_TR % (EX4_AHEAD + 1) == 0),
                  "multi-step streams: the ring and the load sets repeat every EX4_TR rows");
    typedef float f4 __attribute__((ext_vector_type(CPL)));  // CPL columns of one lane
    constexpr int EX4_COLS = 64 * CPL;                          // columns per wave
    constexpr int TR = EX4_TR * NB;                             // rows per wave
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int x0 = (tile % strips) * EX4_COLS, y0 = ((tile / strips) * 4 + wave) * TR;
    const int W = g.W, H = g.H, pitch = g.pitch;
    const int xl = x0 + CPL * lane;
    const int xe = min(max(lane == 0 ? x0 - 1 : x0 + EX4_COLS, 0), W - 1);
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        g.base, 0, (int)min((long)NG * g.planeStride * 4, 0x7fffffffL), 0x00020000);
    if (tid == 0) s_cnt = 0;
    __syncthreads();

    bool colOK[CPL];
#pragma unroll
    for (int c = 0; c < CPL; c++) colOK[c] = xl + c >= 5 && xl + c < W - 5;

    // Ring slot: DoG of the lane's 4 columns and of its outer column, per plane.
    f4 rd[3][ND];
    float re[3][ND];
    // Raw rows in flight: EX4_AHEAD + 1 register sets, loads issued EX4_AHEAD
    // rows ahead of the row being formed.
    f4 rv[EX4_AHEAD + 1][NG];
    float rev[EX4_AHEAD + 1][NG];
    // Lanes whose columns start past the octave's width (the last strip of a
    // row overhangs it: 1920 = 7.5 strips) and the lanes that do not use the
    // outer column (all but lanes 0 and 63) load from an offset past the
    // buffer: the hardware returns 0 without a memory request.
#if defined(SIFT_EX_DIAG) && (SIFT_EX_DIAG == 1 || SIFT_EX_DIAG == 3)  // traffic variants (wrong results): no outer-column loads
    const bool l4 = xl < W, le = false;
#else
    const bool l4 = xl < W, le = lane == 0 || lane == 63;
#endif
    auto issue_row = [&](int y, f4 (&v)[NG], float (&e)[NG]) {
#if defined(SIFT_EX_DIAG) && (SIFT_EX_DIAG == 2 || SIFT_EX_DIAG == 3)  // traffic variants: halo rows -> the wave's own rows
        y = min(max(y, y0), y0 + TR - 1);
#endif
        const int yc = min(max(y, 0), H - 1);
        const unsigned off4 = l4 ? (unsigned)(yc * pitch + xl) * 4u : 0x80000000u;
        const unsigned offe = le ? (unsigned)(yc * pitch + xe) * 4u : 0x80000000u;
#pragma unroll
        for (int d = 0; d < NG; d++) {
            const int so = (int)((long)d * g.planeStride * 4);
            if constexpr (CPL == 4)
                v[d] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, off4, so, 0));
            else
                v[d] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b64(rsrc, off4, so, 0));
            e[d] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsrc, offe, so, 0));
        }
    };
    // Candidates of one tested row: one LDS reservation per row with hits;
    // each lane's slot offset is the exclusive prefix of the per-lane hit
    // counts, taken from ballots of the count's bits (count <= 4 * LT < 32).
    auto emit_row = [&](int r, unsigned hits) {
        if (!__ballot(hits != 0)) return;  // wave-uniform
        const unsigned cnt = (unsigned)__popc(hits);
        unsigned excl = 0, tot = 0;
#pragma unroll
        for (int b = 0; b < 5; b++) {
            const unsigned long long bm = __ballot((cnt >> b) & 1u);
            excl += __builtin_amdgcn_mbcnt_hi((unsigned)(bm >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bm, 0u)) << b;
            tot += (unsigned)__popcll(bm) << b;
        }
        unsigned base = 0;
        if (lane == 0) base = atomicAdd(&s_cnt, tot);
        unsigned pos = __builtin_amdgcn_readfirstlane(base) + excl;
        for (unsigned m = hits; m; m &= m - 1u, pos++) {
            const int f = __builtin_ctz(m), l = f / CPL + 1, c = f % CPL;
            const uint2 q = make_uint2((unsigned)(o << 8 | l), (unsigned)(r << 16 | (xl + c)));
            if (pos < EX4_LIST) {
                s_list[pos] = q;
            } else {  // plateau-heavy tile: spill straight to the global list
                const unsigned gp = atomicAdd(&ctr->cand, 1u);
                if (gp < cap)
                    cand[gp] = q;
                else
                    atomicOr(&ctr->overflow, 1u);
            }
        }
    };
    auto test_row = [&](int r, int A, int B, int C) -> unsigned {
        const bool rowOK = r >= 5 && r < H - 5;
        f4 hx[ND], hn[ND];
#pragma unroll
        for (int d = 0; d < ND; d++) {
            f4 vx, vn;
#pragma unroll
            for (int c = 0; c < CPL; c++) {
                vx[c] = fmaxf(fmaxf(rd[A][d][c], rd[B][d][c]), rd[C][d][c]);
                vn[c] = fminf(fminf(rd[A][d][c], rd[B][d][c]), rd[C][d][c]);
            }
            const float ex = fmaxf(fmaxf(re[A][d], re[B][d]), re[C][d]);
            const float en = fminf(fminf(re[A][d], re[B][d]), re[C][d]);
            const float lx = dpp_left_or(ex, vx[CPL - 1]), ln = dpp_left_or(en, vn[CPL - 1]);
            const float rx = dpp_right_or(ex, vx[0]), rn = dpp_right_or(en, vn[0]);
            // Column c's horizontal neighbours: c-1 and c+1 (across the lane
            // edges: the DPP values), max/min in the same operation order.
#pragma unroll
            for (int c = 0; c < CPL; c++) {
                const float xa = c == 0 ? lx : vx[c - 1], xb = c == CPL - 1 ? rx : vx[c + 1];
                const float na = c == 0 ? ln : vn[c - 1], nb = c == CPL - 1 ? rn : vn[c + 1];
                hx[d][c] = fmaxf(fmaxf(xa, vx[c]), xb);
                hn[d][c] = fminf(fminf(na, vn[c]), nb);
            }
        }
        unsigned hits = 0;  // bit (l - 1) * CPL + c
#pragma unroll
        for (int l = 1; l <= LT; l++)
#pragma unroll
            for (int c = 0; c < CPL; c++) {
                const float v = rd[B][l][c];
                const float M = fmaxf(fmaxf(hx[l - 1][c], hx[l][c]), hx[l + 1][c]);
                const float m = fminf(fminf(hn[l - 1][c], hn[l][c]), hn[l + 1][c]);
                // M >= v >= m always (v is one of the 27), so "v >= all" is v == M;
                // |v| > thr >= 0 excludes v == 0, and the sign picks the test.
                const bool h = rowOK && colOK[c] && fabsf(v) > thr && v == (v > 0 ? M : m);
                hits |= (unsigned)h << ((l - 1) * CPL + c);
            }
        return hits;
    };

    if (y0 < H) {
        // Strip row m = 0 .. TR + 1 (image row y0 - 1 + m) is loaded into raw
        // set m % NS; once formed, its set is reloaded with strip row m + NS
        // (rows past the image: clamped reads, never tested).
        constexpr int NS = EX4_AHEAD + 1;
        // Streams end at the image's last tested row (H - 6): no load or test
        // past it (uniform).
        const int nsteps = NB == 1 ? 1 : min(NB, (min(H - 5, y0 + TR) - y0 + EX4_TR - 1) / EX4_TR);
        const int nr = nsteps * EX4_TR + 2, yb = y0 + nsteps * EX4_TR;
        // Odd waves stream bottom to top.  Vertically adjacent waves share
        // two rows (each one's halo row is the other's edge row), and a row
        // a wave loads at the start of its stream was loaded by a same-way
        // neighbour at the end of its stream: by then the XCD's L2 (4 MiB
        // against ~20 MB streamed meanwhile) had dropped it, and the halo
        // rows came back over the fabric -- 1.19x the algorithmic bytes (the
        // Infinity Cache served them, FETCH_SIZE counted them).  With
        // alternating directions every shared row is loaded by both waves at
        // the same end of their streams.  The 3x3x3 test is symmetric in
        // the rows (exact max / min), so candidates are unchanged.
        const bool up = (wave & 1) != 0;
        auto strip_row = [&](int m) { return up ? yb - m : y0 - 1 + m; };   // image row of strip row m
        auto tested_row = [&](int k) { return up ? yb - 1 - k : y0 + k; };  // image row of tested row k
        auto form = [&](int m, int km, f4 (&d4)[ND], float (&de)[ND]) {  // km = m % NS (compile-time)
#pragma unroll
            for (int d = 0; d < ND; d++) {
                d4[d] = rv[km][d + 1] - rv[km][d];
                de[d] = rev[km][d + 1] - rev[km][d];
            }
            if (m + NS < nr) issue_row(strip_row(m + NS), rv[km], rev[km]);
        };
#pragma unroll
        for (int m = 0; m < NS; m++) issue_row(strip_row(m), rv[m], rev[m]);
        form(0, 0, rd[0], re[0]);
        form(1, 1 % NS, rd[1], re[1]);
        // Strip row k + 2 enters ring slot (k + 2) % 3, tested row k is tested.
#pragma unroll 1
        for (int kb = 0; kb < nsteps * EX4_TR; kb += EX4_TR) {
#pragma unroll
            for (int k6 = 0; k6 < EX4_TR; k6++) {
                const int k = kb + k6;
                const int A = k6 % 3, B = (k6 + 1) % 3, C = (k6 + 2) % 3;
                form(k + 2, (k6 + 2) % NS, rd[C], re[C]);
                const int r = tested_row(k);
                emit_row(r, test_row(r, A, B, C));
            }
        }
    }
    __syncthreads();
    const unsigned nl = min(s_cnt, (unsigned)EX4_LIST);
    if (tid == 0) s_base = nl ? atomicAdd(&ctr->cand, nl) : 0u;
    __syncthreads();
    for (unsigned k = tid; k < nl; k += 256) {
        const unsigned pos = s_base + k;
        if (pos < cap)
            cand[pos] = s_list[k];
        else
            atomicOr(&ctr->overflow, 1u);
    }
}

// All octaves of the frame in one launch (L = 1..6): blocks [start[o],
// start[o+1]) take octave o, with tall strips (6 rows per wave) where they
// still give >= 1024 waves, else 2 rows per wave (small octaves are
// latency-bound and want waves; tools/kernel_bench: 1920x1200 16.7 us at 6
// rows vs 19.8 at 2; 960x600 9.2 us at 2 rows vs 10.8 at 6).
constexpr int kExTallMin = 2048;  // single frames: 6-row wave strips from this many strips per launch, else 2-row (1920x1200: 1600 -> 2-row, 26.4 -> 25.5 us); batches: 1024
constexpr int kExStream = 2;  // 6-row steps per tall wave stream (12 rows: 247 vs 251 us per 16-frame launch; 18, 24 rows slower)
struct ExtremaPlan {
    int start[kMaxOctaves + 1];  // start[nOct] = blocks per frame
    int strips[kMaxOctaves];
    int tall[kMaxOctaves];
};

template <int LT>
__global__ __launch_bounds__(256) void k_extrema_all(PyrDesc pyr, ExtremaPlan plan, float thr,
                                                     uint2* __restrict__ cand, Counters* __restrict__ ctr,
                                                     unsigned cap, long fs) {
    __shared__ unsigned s_cnt, s_base;
    __shared__ uint2 s_list[EX4_LIST];
    // Frame-major block order over all frames, XCD-aware: each XCD takes a
    // contiguous run of (frame, octave, strip block), so vertically adjacent
    // blocks (shared halo rows) meet in the same L2.
    const int per = plan.start[pyr.nOct];
    const int t = xcd_tile(blockIdx.x, gridDim.x);
    const int f = t / per, b = t - f * per;
    int o = 0;
    while (o + 1 < pyr.nOct && b >= plan.start[o + 1]) o++;
    OctGeom g = pyr.oct[o];
    g.base = fptr(g.base, f * fs);
    cand = fptr(cand, f * fs);
    ctr = fptr(ctr, f * fs);
    const int blk = b - plan.start[o];
    if (plan.tall[o])
        extrema_block<LT, 6, 2, kExStream>(g, o, thr, cand, ctr, cap, blk, plan.strips[o], s_list, s_cnt, s_base);
    else
        extrema_block<LT, 2, 2>(g, o, thr, cand, ctr, cap, blk, plan.strips[o], s_list, s_cnt, s_base);
}

// Octave o alone, for L > 6 (LDS-staged k_extrema).
void launch_extrema(const PyrDesc& pyr, int o, float threshold, uint2* cand, Counters* ctr, unsigned cap,
                    const Frames& fr, hipStream_t s) {
    const OctGeom& g = pyr.oct[o];
    dim3 grid((g.W + EX_TW - 1) / EX_TW, (g.H + EX_TH - 1) / EX_TH, fr.nf);
    const size_t lds = sizeof(float) * (size_t)(pyr.L + 2) * EX_SH * EX_SW;
    hipLaunchKernelGGL(k_extrema<0>, grid, dim3(256), lds, s, g, pyr.L, o, threshold, cand, ctr, cap, fr.stride);
}

bool launch_extrema_all(const PyrDesc& pyr, float threshold, uint2* cand, Counters* ctr, unsigned cap,
                        const Frames& fr, hipStream_t s) {
    if (pyr.L < 1 || pyr.L > 6) return false;
    ExtremaPlan plan{};
    int total = 0;
    for (int o = 0; o < pyr.nOct; o++) {
        const OctGeom& g = pyr.oct[o];
        const int strips = (g.W + EX4_COLS - 1) / EX4_COLS;
        // Frames of a batch count too: each brings its own strips.
        // (8, 12 or 20 rows per wave for batches: 147, 149, 582 us vs 131 at 6.)
        const bool tall = strips * ((g.H + 5) / 6) * fr.nf >= (fr.nf > 1 ? 1024 : kExTallMin);
        const int tr = tall ? 6 * kExStream : 2;
        plan.start[o] = total;
        plan.strips[o] = strips;
        plan.tall[o] = tall;
        total += strips * ((g.H + 4 * tr - 1) / (4 * tr));
    }
    plan.start[pyr.nOct] = total;
    switch (pyr.L) {
#define SIFT_EX_CASE(LV) \
    case LV:                                                                                                    \
        hipLaunchKernelGGL(k_extrema_all<LV>, dim3(total * fr.nf), dim3(256), 0, s, pyr, plan, threshold, cand, ctr, \
                           cap, fr.stride);                                                                         \
        break;
        SIFT_EX_CASE(1)
        SIFT_EX_CASE(2)
        SIFT_EX_CASE(3)
        SIFT_EX_CASE(4)
        SIFT_EX_CASE(5)
        SIFT_EX_CASE(6)
#undef SIFT_EX_CASE
    }
    return true;
}

}  // namespace sift_amd
