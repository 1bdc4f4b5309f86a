// 4x4x8 SIFT descriptor for gfx950 (OpenCV 4.x sift.simd.hpp calcSIFTDescriptor).
//
// Replaces /root/reference/sift_cuda/sift_func/SiftOps.cu:454-623 (128 threads
// per keypoint, 8 shared-memory float atomics per sample, modff bins, serial
// lane-0 normalisation, half(x512) output).
//
// One 256-thread workgroup per keypoint.  Eight LDS float atomics per sample
// saturate the CU's LDS pipe on gfx950 (~30 cycles per ds_add_f32 wave
// instruction, measured: SQ_WAIT_INST_LDS ~40 % of wave cycles), so the
// trilinear histogram is built without per-sample atomics:
//   A  classify every sample of the (2R+1)^2 window, count it into its base
//      bucket (r0, c0, o0) -- 25 spatial base cells x 8 orientation bins; all
//      samples of a bucket feed the SAME 8 histogram bins;
//   B  exclusive scan of the 200 bucket counts;
//   C  recompute each sample (gradient, fastAtan2, magnitude, exp32f weight:
//      the oracle's operation order) and scatter a 12-byte record into its
//      bucket (counting sort in LDS);
//   E  every thread walks an equal slice of the bucket-ordered records, forms
//      the 8 trilinear contributions exactly as OpenCV does, accumulates them in
//      registers and flushes once per bucket run with 8 ds_add_u64.
// Sums are kept in 32.32 fixed point: integer addition is associative, so the
// histogram is bit-identical for any thread/record order (deterministic) and is
// the correctly rounded exact sum of the float contributions.  OpenCV sums the
// same float contributions sequentially, so descriptor bytes can differ from the
// oracle by +-1 where a float rounding lands on a .5 boundary (tests bound this).
// Then wrap, L2 norm (8 fma lanes + v_reduce_sum order), 0.2 clip, renorm and
// x512 rounding to 0..255 are the oracle's exact float operations.
#include <hip/hip_runtime.h>

#include "sift_kernels.h"
#include "sift_math.h"

namespace sift_amd {

__constant__ float c_exptab_d[64];

void upload_exp_table_desc(const float* tab64) {
    (void)hipMemcpyToSymbol(HIP_SYMBOL(c_exptab_d), tab64, 64 * sizeof(float));
}

constexpr int kD = 4, kN = 8;
constexpr int kHistLen = (kD + 2) * (kD + 2) * (kN + 2);  // 360
constexpr int kBuckets = 25 * 8;                           // base cell (r0+1, c0+1) x o0

struct DescGeom {
    float cos_t, sin_t, angle, bins_per_rad, exp_scale;
    int ptx, pty, radius, rows, cols;
};

struct DescRec {
    unsigned key;  // bucket << 16 | (i + R) << 8 | (j + R)
    float mag;     // |grad| * gaussian weight
    float obf;     // fractional orientation bin
};

// Rotated-grid coordinates of window sample (i, j) and its validity: the
// oracle's calcSIFTDescriptor loop body, operation for operation.
__device__ __forceinline__ bool desc_sample(const DescGeom& G, int i, int j, float& rbin, float& cbin, float& c_rot,
                                            float& r_rot) {
    c_rot = (float)j * G.cos_t - (float)i * G.sin_t;
    r_rot = (float)j * G.sin_t + (float)i * G.cos_t;
    rbin = r_rot + (float)(kD / 2) - 0.5f;
    cbin = c_rot + (float)(kD / 2) - 0.5f;
    const int r = G.pty + i, c = G.ptx + j;
    return rbin > -1 && rbin < kD && cbin > -1 && cbin < kD && r > 0 && r < G.rows - 1 && c > 0 && c < G.cols - 1;
}

// Exact 32.32 fixed-point image of a non-negative float < 2^31 (bits below
// 2^-32 are dropped).
__device__ __forceinline__ long long to_fx(float v) {
    const float hi = floorf(v);
    const unsigned lo = (unsigned)((v - hi) * 4294967296.0f);
    return ((long long)(int)hi << 32) | (long long)lo;
}

__device__ __forceinline__ float from_fx(long long x) { return (float)((double)x * 2.3283064365386962890625e-10); }

// The 8 contributions of one sample, OpenCV's order and names (v_rco[r][c][o]).
__device__ __forceinline__ void trilinear(float mag, float rbf, float cbf, float obf, float v[8]) {
    const float v_r1 = mag * rbf, v_r0 = mag - v_r1;
    const float v_rc11 = v_r1 * cbf, v_rc10 = v_r1 - v_rc11;
    const float v_rc01 = v_r0 * cbf, v_rc00 = v_r0 - v_rc01;
    v[7] = v_rc11 * obf;
    v[6] = v_rc11 - v[7];
    v[5] = v_rc10 * obf;
    v[4] = v_rc10 - v[5];
    v[3] = v_rc01 * obf;
    v[2] = v_rc01 - v[3];
    v[1] = v_rc00 * obf;
    v[0] = v_rc00 - v[1];
}

// Histogram offsets of v_rco000..111 from the base index ((r0+1)*6 + c0+1)*10 + o0.
__device__ __forceinline__ int tri_off(int q) {
    return (q & 4 ? (kD + 2) * (kN + 2) : 0) + (q & 2 ? (kN + 2) : 0) + (q & 1);
}

__device__ __forceinline__ int bucket_base_index(int b) {
    const int cell = b >> 3, o0 = b & 7;
    return ((cell / 5) * (kD + 2) + (cell % 5)) * (kN + 2) + o0;
}

__global__ __launch_bounds__(256) void k_descriptor(PyrDesc pyr, const OriKpt* __restrict__ kpts,
                                                    const int* __restrict__ final_order,
                                                    const Counters* __restrict__ ctr, float* __restrict__ kpts3,
                                                    float* __restrict__ feats4, uint16_t* __restrict__ desc,
                                                    KeypointParams kp) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
    long long* hist = reinterpret_cast<long long*>(lds_raw);  // kHistLen
    int* bcount = reinterpret_cast<int*>(hist + kHistLen);     // kBuckets
    int* bstart = bcount + kBuckets;                           // kBuckets + 8
    int* bcur = bstart + kBuckets + 8;                         // kBuckets
    float* raw = reinterpret_cast<float*>(bcur + kBuckets);    // 128
    float* nacc = raw + 128;                                   // 16
    DescRec* recs = reinterpret_cast<DescRec*>(nacc + 16);     // kp.descNrec

    const int tid = threadIdx.x, lane = tid & 63;
    const unsigned n = ctr->final_n;
    const int fo = pyr.firstOctave;
    for (unsigned p = blockIdx.x; p < n; p += gridDim.x) {
        const OriKpt kpt = kpts[final_order[p]];
        // unpackOctave + calcDescriptorsComputer (sift.dispatch.cpp).
        int octave = kpt.octave & 255;
        const int layer = (kpt.octave >> 8) & 255;
        octave = octave < 128 ? octave : (-128 | octave);
        const float scale = octave >= 0 ? 1.f / (float)(1 << octave) : (float)(1 << -octave);
        const float size = kpt.size * scale;
        const float ptfx = kpt.x * scale, ptfy = kpt.y * scale;
        const OctGeom& g = pyr.oct[octave - fo];
        const float* img = g.base + (size_t)layer * g.planeStride;
        const int pitch = g.pitch;
        float angle = 360.f - kpt.angle;
        if (fabsf(angle - 360.f) < FLT_EPSILON) angle = 0.f;
        const float scl = size * 0.5f;

        DescGeom G;
        G.rows = g.H;
        G.cols = g.W;
        G.ptx = cv_round(ptfx);
        G.pty = cv_round(ptfy);
        const float arg = angle * (float)(M_PI / 180);
        float cos_t = (float)cos((double)arg);
        float sin_t = (float)sin((double)arg);
        G.bins_per_rad = kN / 360.f;
        G.exp_scale = -1.f / (kD * kD * 0.5f);
        const float hist_width = 3.f * scl;
        int radius = cv_round(hist_width * 1.4142135623730951f * (float)(kD + 1) * 0.5f);
        radius = min(radius, (int)sqrt((double)G.cols * G.cols + (double)G.rows * G.rows));
        radius = min(radius, 120);  // record packing bound; unreachable for accepted keypoints
        G.cos_t = cos_t / hist_width;
        G.sin_t = sin_t / hist_width;
        G.angle = angle;
        G.radius = radius;
        const int side = 2 * radius + 1, total = side * side;

        for (int i = tid; i < kHistLen; i += 256) hist[i] = 0;
        for (int i = tid; i < kBuckets; i += 256) {
            bcount[i] = 0;
            bcur[i] = 0;
        }
        __syncthreads();

        // A: count samples per base bucket.
        for (int k = tid; k < total; k += 256) {
            const int i = k / side - radius, j = k - (k / side) * side - radius;
            float rbin, cbin, c_rot, r_rot;
            if (desc_sample(G, i, j, rbin, cbin, c_rot, r_rot)) {
                const float* pp = img + (size_t)(G.pty + i) * pitch + (G.ptx + j);
                const float dx = pp[1] - pp[-1], dy = pp[-pitch] - pp[pitch];
                const float obin = (cv_fast_atan2(dy, dx) - angle) * G.bins_per_rad;
                int o0 = cv_floor(obin);
                if (o0 < 0) o0 += kN;
                if (o0 >= kN) o0 -= kN;
                const int b = ((cv_floor(rbin) + 1) * 5 + (cv_floor(cbin) + 1)) * 8 + o0;
                atomicAdd(&bcount[b], 1);
            }
        }
        __syncthreads();

        // B: exclusive scan of the bucket counts (wave 0, 4 buckets per lane).
        if (tid < 64) {
            int c4[4], s = 0;
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int b = lane * 4 + u;
                c4[u] = b < kBuckets ? bcount[b] : 0;
                s += c4[u];
            }
            int x = s;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const int y = __shfl_up(x, off);
                if (lane >= off) x += y;
            }
            int run = x - s;
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int b = lane * 4 + u;
                if (b < kBuckets) bstart[b] = run;
                run += c4[u];
            }
            if (lane == 63) bstart[kBuckets] = x;
        }
        __syncthreads();
        const int nrec = bstart[kBuckets];
        const bool useRecs = nrec <= kp.descNrec;

        // C: full sample, scatter a record into its bucket (or, past the LDS
        // bound, add its 8 fixed-point contributions directly: same sums).
        for (int k = tid; k < total; k += 256) {
            const int i = k / side - radius, j = k - (k / side) * side - radius;
            float rbin, cbin, c_rot, r_rot;
            if (desc_sample(G, i, j, rbin, cbin, c_rot, r_rot)) {
                const float* pp = img + (size_t)(G.pty + i) * pitch + (G.ptx + j);
                const float dx = pp[1] - pp[-1], dy = pp[-pitch] - pp[pitch];
                const float wgt = cv_exp32f((c_rot * c_rot + r_rot * r_rot) * G.exp_scale, c_exptab_d);
                const float gori = cv_fast_atan2(dy, dx);
                const float gmag = cv_magnitude(dx, dy);
                float obin = (gori - angle) * G.bins_per_rad;
                const float mag = gmag * wgt;
                const int r0 = cv_floor(rbin), c0 = cv_floor(cbin);
                int o0 = cv_floor(obin);
                obin -= (float)o0;
                if (o0 < 0) o0 += kN;
                if (o0 >= kN) o0 -= kN;
                const int b = ((r0 + 1) * 5 + (c0 + 1)) * 8 + o0;
                if (useRecs) {
                    const int slot = bstart[b] + atomicAdd(&bcur[b], 1);
                    DescRec rec;
                    rec.key = (unsigned)b << 16 | (unsigned)(i + radius) << 8 | (unsigned)(j + radius);
                    rec.mag = mag;
                    rec.obf = obin;
                    recs[slot] = rec;
                } else {
                    float v[8];
                    trilinear(mag, rbin - (float)r0, cbin - (float)c0, obin, v);
                    const int base = bucket_base_index(b);
#pragma unroll
                    for (int q = 0; q < 8; q++) atomicAdd((unsigned long long*)&hist[base + tri_off(q)],
                                                          (unsigned long long)to_fx(v[q]));
                }
            }
        }
        __syncthreads();

        // E: balanced walk over the bucket-ordered records, register
        // accumulation, one 8-atomic flush per bucket run.
        if (useRecs) {
            const int chunk = (nrec + 255) / 256;
            const int e0 = min(nrec, tid * chunk), e1 = min(nrec, e0 + chunk);
            int curb = -1;
            long long acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
            for (int e = e0; e < e1; e++) {
                const DescRec rec = recs[e];
                const int b = (int)(rec.key >> 16);
                if (b != curb) {
                    if (curb >= 0) {
                        const int base = bucket_base_index(curb);
#pragma unroll
                        for (int q = 0; q < 8; q++) {
                            atomicAdd((unsigned long long*)&hist[base + tri_off(q)], (unsigned long long)acc[q]);
                            acc[q] = 0;
                        }
                    }
                    curb = b;
                }
                const int i = (int)((rec.key >> 8) & 255u) - radius, j = (int)(rec.key & 255u) - radius;
                float rbin, cbin, c_rot, r_rot;
                desc_sample(G, i, j, rbin, cbin, c_rot, r_rot);
                float v[8];
                trilinear(rec.mag, rbin - (float)cv_floor(rbin), cbin - (float)cv_floor(cbin), rec.obf, v);
#pragma unroll
                for (int q = 0; q < 8; q++) acc[q] += to_fx(v[q]);
            }
            if (curb >= 0) {
                const int base = bucket_base_index(curb);
#pragma unroll
                for (int q = 0; q < 8; q++)
                    atomicAdd((unsigned long long*)&hist[base + tri_off(q)], (unsigned long long)acc[q]);
            }
        }
        __syncthreads();

        // Wrap bins 8,9 into 0,1 (bin 9 never receives a contribution).
        if (tid < 128) {
            const int ii = tid >> 5, jj = (tid >> 3) & 3, kk = tid & 7;
            const int hidx = ((ii + 1) * (kD + 2) + (jj + 1)) * (kN + 2) + kk;
            float v = from_fx(hist[hidx]);
            if (kk < 2) v = v + from_fx(hist[hidx + kN]);
            raw[tid] = v;
        }
        __syncthreads();
        if (tid < 8) {
            float a = 0.f;
#pragma unroll
            for (int q = 0; q < 16; q++) a = __fmaf_rn(raw[tid + 8 * q], raw[tid + 8 * q], a);
            nacc[tid] = a;
        }
        __syncthreads();
        if (tid == 0) {
            const float t0 = nacc[0] + nacc[4], t1 = nacc[1] + nacc[5], t2 = nacc[2] + nacc[6], t3 = nacc[3] + nacc[7];
            float nrm2 = (t0 + t2) + (t1 + t3);
            const float thr = __builtin_sqrtf(nrm2) * 0.2f;
            nrm2 = 0.f;
#pragma unroll 1
            for (int q0 = 0; q0 < 128; q0 += 8) {
                float vals[8];
#pragma unroll
                for (int u = 0; u < 8; u++) vals[u] = raw[q0 + u];
#pragma unroll
                for (int u = 0; u < 8; u++) {
                    const float val = fminf(vals[u], thr);
                    raw[q0 + u] = val;
                    nrm2 = nrm2 + val * val;
                }
            }
            nacc[8] = 512.f / fmaxf(__builtin_sqrtf(nrm2), FLT_EPSILON);
            float* k3 = kpts3 + 3 * (size_t)p;
            k3[0] = kpt.x;
            k3[1] = kpt.y;
            k3[2] = (float)layer;
            reinterpret_cast<float4*>(feats4)[p] = make_float4((float)kpt.octave, kpt.size, kpt.response, kpt.angle);
        }
        __syncthreads();
        if (tid < 128) {
            int v = cv_round(raw[tid] * nacc[8]);
            v = v < 0 ? 0 : (v > 255 ? 255 : v);
            const _Float16 hv = (_Float16)(float)v;
            desc[(size_t)p * 128 + tid] = __builtin_bit_cast(uint16_t, hv);
        }
        __syncthreads();
    }
}

size_t descriptor_lds_bytes(const KeypointParams& kp) {
    return sizeof(long long) * kHistLen + sizeof(int) * (3 * kBuckets + 8) + sizeof(float) * (128 + 16) +
           sizeof(DescRec) * (size_t)kp.descNrec;
}

void launch_descriptor(const PyrDesc& pyr, const OriKpt* kpts, const int* final_order, const Counters* ctr,
                       float* kpts3, float* feats4, uint16_t* desc, const KeypointParams& kp, hipStream_t s) {
    hipLaunchKernelGGL(k_descriptor, dim3(2048), dim3(256), descriptor_lds_bytes(kp), s, pyr, kpts, final_order, ctr,
                       kpts3, feats4, desc, kp);
}

}  // namespace sift_amd
