// Host-side element types of the drop-in surface.  The reference exposes CUDA's
// float3 / float4 / half (Detector.hh:54-60); these PODs have the same layout
// and member names so caller code like `kpts[i].x` or `(float)desc[k]` compiles
// unchanged, without pulling HIP headers into the caller.
#pragma once
#include <cstddef>
#include <cstdint>
#include <cstring>

namespace sift_cuda {

struct Float3 {
    float x, y, z;
};
struct Float4 {
    float x, y, z, w;
};

// IEEE binary16 storage; SIFT descriptor values are integers 0..255, exact here.
struct Half {
    uint16_t bits{0};
    operator float() const {
        const uint32_t s = (bits & 0x8000u) << 16, e = (bits >> 10) & 0x1f, m = bits & 0x3ffu;
        uint32_t f;
        if (e == 0) {
            if (m == 0) {
                f = s;
            } else {  // subnormal
                int sh = 0;
                uint32_t mm = m;
                while (!(mm & 0x400u)) { mm <<= 1; sh++; }
                f = s | ((uint32_t)(113 - sh) << 23) | ((mm & 0x3ffu) << 13);
            }
        } else if (e == 31) {
            f = s | 0x7f800000u | (m << 13);
        } else {
            f = s | ((e + 112) << 23) | (m << 13);
        }
        float out;
        std::memcpy(&out, &f, 4);
        return out;
    }
};
static_assert(sizeof(Float3) == 12 && sizeof(Float4) == 16 && sizeof(Half) == 2, "layout");

// Non-owning view of a device array owned by a Detector (stands in for the
// reference's thrust::device_vector members, Detector.hh:54-57; data()/size()
// as there).  data() is read-only: the detector derives data from what it
// writes (the matcher's int8 sidecar of the descriptor rows), so a caller that
// writes takes mutable_data(), which tells the detector (for descriptor
// buffers, sift_hip_descriptors_written: matches then convert those rows).
template <class T>
class DeviceBuffer {
public:
    using WriteHook = void (*)(const void*);
    DeviceBuffer() = default;
    DeviceBuffer(T* p, size_t n, WriteHook on_write = nullptr) : ptr_(p), n_(n), on_write_(on_write) {}
    const T* data() const { return ptr_; }
    T* mutable_data() const {
        if (on_write_ && ptr_) on_write_(ptr_);
        return ptr_;
    }
    size_t size() const { return n_; }

private:
    T* ptr_{nullptr};
    size_t n_{0};
    WriteHook on_write_{nullptr};
};

}  // namespace sift_cuda
