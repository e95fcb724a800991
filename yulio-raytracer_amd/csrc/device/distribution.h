// distribution.h — piecewise-constant 1D/2D distributions
// (samplers/distribution1d.cpp:42-74, samplers/distribution2d.cpp:34-68), used by the
// pixel-filter importance table and the HDRI light.
#pragma once

#include <vector>

namespace yrt {

// f is row-major [h][w]. Outputs: ycdf (h+1), ypdf (h), xcdf (h*(w+1)), xpdf (h*w).
void dist2d_init(const float* f, int w, int h, std::vector<float>& ycdf, std::vector<float>& ypdf,
                 std::vector<float>& xcdf, std::vector<float>& xpdf);
// Distribution2D::sample -> (x, y) in [0,w)x[0,h) and pdf
void dist2d_sample(const std::vector<float>& ycdf, const std::vector<float>& ypdf, const std::vector<float>& xcdf,
                   const std::vector<float>& xpdf, int w, int h, float ux, float uy, float& sx, float& sy,
                   float& pdf);

}  // namespace yrt
