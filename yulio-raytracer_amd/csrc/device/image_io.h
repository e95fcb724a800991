// image_io.h — image loading into the reference's Image4c representation.
#pragma once

#include <stdint.h>

#include <string>
#include <vector>

#include "objects.h"

namespace yrt {

// rtNewImage(type, w, h, data): "RGB8" (Image3c), "RGBA8" (Image4c), "RGB_FLOAT32",
// "RGBA_FLOAT32" (Image3f/4f).
void image_from_memory(const char* type, int width, int height, const void* data, ImageObj& out);

// loadImage (common/image/image.cpp:27-52): .ppm (loadPPM), .jpg/.jpeg (loadJPEG via
// TurboJPEG, flipped), everything else through FreeImage (PNG: bottom-up, 24/32 bpp only).
// Returns false when the file cannot be read (the device then substitutes 1x1 white).
bool image_load(const std::string& file, ImageObj& out);

// Decoders exposed for tests: 8-bit RGB(A) in file row order (top row first).
bool decode_jpeg(const std::vector<uint8_t>& file, int& w, int& h, std::vector<uint8_t>& rgb, std::string& err);
bool decode_png(const std::vector<uint8_t>& file, int& w, int& h, int& channels, std::vector<uint8_t>& px,
                std::string& err);

}  // namespace yrt
