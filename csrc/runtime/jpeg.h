// Baseline (sequential Huffman) JPEG decoder -> RGB u8 HWC.
//
// Reference: the member decodes each query image with tch's
// `imagenet::load_image_and_resize` (src/services.rs:492), which uses
// libtorch-side image loading. This image has no libjpeg headers and no
// torchvision, so the node decodes with this self-contained decoder; every
// image of the reference's test_files/imagenet_1k set is baseline JPEG
// (981 YCbCr + 19 grayscale). Progressive / arithmetic-coded files are
// rejected with an error.
#pragma once
#include <cstdint>
#include <functional>
#include <string>
#include <vector>

namespace dmlc {

struct Image {
  int width = 0, height = 0;
  std::vector<uint8_t> rgb;  // HWC, 3 channels
};

// Throws std::runtime_error on malformed / unsupported input.
Image decode_jpeg(const uint8_t* data, size_t size);
Image decode_jpeg_file(const std::string& path);
// Decodes straight into a caller-provided buffer: out(width, height) returns
// width * height * 3 writable bytes (e.g. pinned staging memory for the H2D
// copy; saves the Image vector's zero-fill and a copy per query image).
void decode_jpeg_into(const uint8_t* data, size_t size, const std::function<uint8_t*(int, int)>& out);

}  // namespace dmlc
