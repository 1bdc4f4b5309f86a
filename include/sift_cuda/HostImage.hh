// Host image container used by Detector::detectAndCompute.  Same public shape
// as /root/reference/sift_cuda/types/HostImage.hh:35-188 (row-major data in a
// shared std::vector, m_image_size {row, col}, at(row, col) / atXY(x, y)), so
// callers that fill an Imagef keep working.
#pragma once
#include <memory>
#include <stdexcept>
#include <vector>

struct Size {
    float row{0};
    float col{0};
    Size() = default;
    Size(float r, float c) : row(r), col(c) {}
    Size(int r, int c) : row((float)r), col((float)c) {}
};

template <typename T>
class Image {
public:
    Image() = default;
    Image(int rows, int cols)
        : m_data(std::make_shared<std::vector<T>>((size_t)rows * cols)), m_image_size(rows, cols) {}

    int rows() const { return (int)m_image_size.row; }
    int cols() const { return (int)m_image_size.col; }
    T& at(int row, int col) { return m_data->at(index(col, row)); }
    const T& at(int row, int col) const { return m_data->at(index(col, row)); }
    T& atXY(int x, int y) { return m_data->at(index(x, y)); }
    const T& atXY(int x, int y) const { return m_data->at(index(x, y)); }

    std::shared_ptr<std::vector<T>> m_data{};
    Size m_image_size{};

private:
    size_t index(int x, int y) const {
        if (!m_data) throw std::runtime_error("Image accessed before initialization");
        if (x < 0 || x >= cols() || y < 0 || y >= rows()) throw std::runtime_error("Image index out of range");
        return (size_t)y * cols() + x;
    }
};

typedef Image<unsigned char> Image8U;
typedef Image<float> Imagef;
