// OpenCV interop for the drop-in surface.  Same
// namespace, function names and behaviour as the reference's
// /root/reference/cvUtils/Conversion.hh:12-70 (implementation
// Conversion.cc:21-58, ConversionImpl.hpp:8-83), over this build's host
// containers (std::vector<sift_cuda::Float3/Float4/Half> instead of
// thrust::host_vector<float3/float4/half>).  Header-only; usable only where
// OpenCV's headers are installed (they are not in this build's image, so the
// compile check is tests/test_abi.py::test_cvutils_header_gated).
#pragma once
#if !__has_include(<opencv2/core.hpp>)
#error "cvUtils/Conversion.hh needs OpenCV (opencv2/core.hpp); the rest of the surface does not"
#endif
#include <opencv2/core.hpp>

#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <type_traits>
#include <vector>

#include "sift_cuda/HostImage.hh"
#include "sift_cuda/Types.hh"

namespace OpencvUtils {

// ConversionImpl.hpp:8-31: single-channel CV_8U / CV_32F / CV_64F -> Image<T>.
template <typename DataType_T>
Image<DataType_T> cvMatToImage(const cv::Mat& mat) {
    if (mat.channels() > 1) throw std::runtime_error("More channels than expected");
    Image<DataType_T> img(mat.rows, mat.cols);
    auto& out = *img.m_data;
    for (int r = 0; r < mat.rows; r++) {
        DataType_T* row = out.data() + (size_t)r * mat.cols;
        switch (mat.depth()) {
            case CV_64F: std::transform(mat.ptr<double>(r), mat.ptr<double>(r) + mat.cols, row,
                                        [](double v) { return (DataType_T)v; }); break;
            case CV_32F: std::transform(mat.ptr<float>(r), mat.ptr<float>(r) + mat.cols, row,
                                        [](float v) { return (DataType_T)v; }); break;
            case CV_8U: std::transform(mat.ptr<uchar>(r), mat.ptr<uchar>(r) + mat.cols, row,
                                       [](uchar v) { return (DataType_T)v; }); break;
            default: throw std::runtime_error("cvMatToImage: unsupported cv::Mat depth");
        }
    }
    return img;
}

// ConversionImpl.hpp:33-46.
template <typename DataType_T>
cv::Mat imageToCvMat(const Image<DataType_T>& image) {
    static_assert(std::is_same_v<DataType_T, uint8_t> || std::is_same_v<DataType_T, float>, "u8 or float images");
    const int type = std::is_same_v<DataType_T, uint8_t> ? CV_8UC1 : CV_32FC1;
    cv::Mat m(image.rows(), image.cols(), type);
    std::memcpy(m.data, image.m_data->data(), image.m_data->size() * sizeof(DataType_T));
    return m;
}

// Conversion.cc:9-19.
inline bool areEqual(const cv::Mat& a, const cv::Mat& b) {
    if (a.channels() != b.channels() || a.rows != b.rows || a.cols != b.cols) return false;
    cv::Mat x;
    cv::bitwise_xor(a, b, x);
    return cv::countNonZero(x.reshape(1)) == 0;
}

// ConversionImpl.hpp:49-64: (v - min) * 255 / (max - min) truncated to u8.
template <typename DataType_T>
Image8U normalize(const Image<DataType_T>& image) {
    const auto [mn, mx] = std::minmax_element(image.m_data->begin(), image.m_data->end());
    Image8U out(image.rows(), image.cols());
    const DataType_T lo = *mn, scale = (DataType_T)255 / (*mx - lo);
    std::transform(image.m_data->begin(), image.m_data->end(), out.m_data->begin(),
                   [&](DataType_T v) { return (uint8_t)((v - lo) * scale); });
    return out;
}

// Conversion.cc:21-42: Detector::final_kpts / final_features -> cv::KeyPoint
// (x, y, packed octave, response, size, angle); size -1 = all.
inline std::vector<cv::KeyPoint> localKptToCvKpt(const std::vector<sift_cuda::Float3>& kpts,
                                                 const std::vector<sift_cuda::Float4>& features, int size = -1) {
    if (kpts.size() != features.size()) throw std::runtime_error("localKptToCvKpt: size mismatch");
    const size_t n = size < 0 ? kpts.size() : std::min((size_t)size, kpts.size());
    std::vector<cv::KeyPoint> out;
    out.reserve(n);
    for (size_t i = 0; i < n; i++) {
        cv::KeyPoint k;
        k.pt.x = kpts[i].x;
        k.pt.y = kpts[i].y;
        k.octave = (int)features[i].x;
        k.response = features[i].z;
        k.size = features[i].y;
        k.angle = features[i].w;
        out.push_back(k);
    }
    return out;
}

// ConversionImpl.hpp:66-82: row-major 128-wide descriptors -> CV_32F (n x 128).
template <typename Data_T>
cv::Mat descriptorToCvMat(const std::vector<Data_T>& descriptors, int num_pts) {
    num_pts = std::min(num_pts, (int)(descriptors.size() / 128));
    cv::Mat d(num_pts, 128, CV_32FC1);
    std::transform(descriptors.begin(), descriptors.begin() + (size_t)num_pts * 128, d.ptr<float>(),
                   [](const Data_T& v) { return (float)v; });
    return d;
}

// Conversion.cc:44-58: match index per query -> cv::DMatch (distance 0, -1 skipped).
inline std::vector<cv::DMatch> cvtMatchToDMatch(const std::vector<int>& match) {
    std::vector<cv::DMatch> out;
    out.reserve(match.size());
    for (int i = 0; i < (int)match.size(); i++)
        if (match[i] != -1) out.emplace_back(i, match[i], 0.f);
    return out;
}

}  // namespace OpencvUtils
