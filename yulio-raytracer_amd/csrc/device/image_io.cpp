// image_io.cpp — PPM / PNG / baseline-JPEG loading into Image4c texels.
//
// Pixel conversion follows the reference loaders, each of which pushes a float Color4 through
// Image4c::set, i.e. char(clamp(c)*255.0f) (common/math/color_scalar.h:60):
//   loadPPM        common/image/ppm.cpp:40-101     c = v * (1/maxColor), rows top-down
//   loadFreeImage  common/image/freeimage.cpp:98-180  c = byte/255.0f, DIB rows bottom-up,
//                  24/32 bpp only (other depths leave the image zero)
//   loadJPEG       common/image/jpeg.cpp:27-74     TurboJPEG RGB, ACCURATEDCT, c = byte*rcp(255),
//                  rows flipped
// The JPEG decoder is baseline sequential Huffman with the integer "islow" IDCT, fancy
// (triangle) chroma upsampling and fixed-point YCbCr->RGB — the libjpeg-turbo defaults that
// tjDecompress2(TJFLAG_ACCURATEDCT) uses; tests/ pin it against PIL (libjpeg) byte-exactly.
#include "image_io.h"

#include <math.h>
#include <stdio.h>
#include <string.h>
#include <strings.h>
#include <zlib.h>

#include <algorithm>
#include <fstream>
#include <stdexcept>

namespace yrt {

static inline uint8_t quantize(float c) {
  // Color4::set(Col4c): char(clamp(r)*255.0f) — truncation
  const float v = fmaxf(0.0f, fminf(c, 1.0f)) * 255.0f;
  return (uint8_t)(int)v;
}

void image_from_memory(const char* type, int width, int height, const void* data, ImageObj& out) {
  out.width = width;
  out.height = height;
  const size_t n = (size_t)width * height;
  std::string t = type ? type : "";
  if (!strcasecmp(t.c_str(), "RGB8") || !strcasecmp(t.c_str(), "RGBA8")) {
    const bool rgba = !strcasecmp(t.c_str(), "RGBA8");
    out.format = rgba ? IMG_RGBA8 : IMG_RGB8;
    out.data.resize(n * 4);
    const uint8_t* s = (const uint8_t*)data;
    for (size_t i = 0; i < n; ++i) {
      out.data[4 * i] = s[(rgba ? 4 : 3) * i];
      out.data[4 * i + 1] = s[(rgba ? 4 : 3) * i + 1];
      out.data[4 * i + 2] = s[(rgba ? 4 : 3) * i + 2];
      out.data[4 * i + 3] = rgba ? s[4 * i + 3] : 255;
    }
  } else if (!strcasecmp(t.c_str(), "RGB_FLOAT32") || !strcasecmp(t.c_str(), "RGBA_FLOAT32")) {
    const bool rgba = !strcasecmp(t.c_str(), "RGBA_FLOAT32");
    out.format = IMG_RGBAF32;
    out.data.resize(n * 16);
    const float* s = (const float*)data;
    float* d = (float*)out.data.data();
    for (size_t i = 0; i < n; ++i) {
      for (int k = 0; k < 3; ++k) d[4 * i + k] = s[(rgba ? 4 : 3) * i + k];
      d[4 * i + 3] = rgba ? s[4 * i + 3] : 1.0f;
    }
  } else {
    throw std::runtime_error("unknown image type: " + t);
  }
}

static bool read_file(const std::string& f, std::vector<uint8_t>& buf) {
  std::ifstream in(f, std::ios::binary);
  if (!in) return false;
  buf.assign(std::istreambuf_iterator<char>(in), std::istreambuf_iterator<char>());
  return true;
}

// ---------------------------------------------------------------- PPM
static bool load_ppm(const std::string& file, ImageObj& out) {
  FILE* f = fopen(file.c_str(), "rb");
  if (!f) return false;
  char type[8] = {0};
  if (fscanf(f, "%7s", type) != 1) { fclose(f); return false; }
  // skip comment lines (ppm.cpp readCommentLine)
  for (;;) {
    int c = fgetc(f);
    while (c == ' ' || c == '\t' || c == '\n' || c == '\r') c = fgetc(f);
    if (c == '#') {
      while (c != '\n' && c != EOF) c = fgetc(f);
      continue;
    }
    if (c != EOF) ungetc(c, f);
    break;
  }
  int width, height, maxColor;
  if (fscanf(f, "%i %i %i", &width, &height, &maxColor) != 3) { fclose(f); return false; }
  // the pixel array is allocated from these (a corrupt header must not ask for terabytes)
  if (width < 1 || height < 1 || (int64_t)width * height > (int64_t(1) << 28) || maxColor < 1 || maxColor > 65535) {
    fclose(f);
    return false;
  }
  const float rcpMaxColor = 1.0f / float(maxColor);
  fgetc(f);
  out.width = width;
  out.height = height;
  out.format = IMG_RGBA8;
  out.data.assign((size_t)width * height * 4, 0);
  auto put = [&](int x, int y, float r, float g, float b) {
    uint8_t* p = &out.data[((size_t)y * width + x) * 4];
    p[0] = quantize(r); p[1] = quantize(g); p[2] = quantize(b); p[3] = quantize(1.0f);
  };
  bool ok = true;
  if (!strcmp(type, "P3")) {
    for (int y = 0; y < height && ok; y++)
      for (int x = 0; x < width && ok; x++) {
        int r, g, b;
        if (fscanf(f, "%i %i %i", &r, &g, &b) != 3) { ok = false; break; }
        put(x, y, float(r) * rcpMaxColor, float(g) * rcpMaxColor, float(b) * rcpMaxColor);
      }
  } else if (!strcmp(type, "P6") && maxColor <= 255) {
    for (int y = 0; y < height && ok; y++)
      for (int x = 0; x < width && ok; x++) {
        unsigned char rgb[3];
        if (fread(rgb, 3, 1, f) != 1) { ok = false; break; }
        put(x, y, float(rgb[0]) * rcpMaxColor, float(rgb[1]) * rcpMaxColor, float(rgb[2]) * rcpMaxColor);
      }
  } else if (!strcmp(type, "P6")) {
    for (int y = 0; y < height && ok; y++)
      for (int x = 0; x < width && ok; x++) {
        unsigned short rgb[3];
        if (fread(rgb, 6, 1, f) != 1) { ok = false; break; }
        put(x, y, float(rgb[0]) * rcpMaxColor, float(rgb[1]) * rcpMaxColor, float(rgb[2]) * rcpMaxColor);
      }
  } else {
    ok = false;
  }
  fclose(f);
  return ok;
}

// ---------------------------------------------------------------- PNG
static uint32_t be32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

bool decode_png(const std::vector<uint8_t>& f, int& w, int& h, int& channels, std::vector<uint8_t>& px,
                std::string& err) {
  static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
  if (f.size() < 8 || memcmp(f.data(), sig, 8)) { err = "not a PNG"; return false; }
  size_t pos = 8;
  int depth = 0, ctype = -1, interlace = 0;
  std::vector<uint8_t> idat;
  while (pos + 8 <= f.size()) {
    const uint32_t len = be32(&f[pos]);
    const char* t = (const char*)&f[pos + 4];
    if (pos + 12 + len > f.size()) { err = "truncated chunk"; return false; }
    const uint8_t* d = &f[pos + 8];
    if (!memcmp(t, "IHDR", 4)) {
      if (len < 13) { err = "truncated IHDR"; return false; }
      w = (int)be32(d);
      h = (int)be32(d + 4);
      depth = d[8];
      ctype = d[9];
      interlace = d[12];
    } else if (!memcmp(t, "IDAT", 4)) {
      idat.insert(idat.end(), d, d + len);
    } else if (!memcmp(t, "IEND", 4)) {
      break;
    }
    pos += 12 + len;
  }
  if (depth != 8 || interlace != 0) { err = "only 8-bit non-interlaced PNG"; return false; }
  // the inflate buffer is allocated from these: refuse what no texture needs (256 Mpx)
  if (w < 1 || h < 1 || (int64_t)w * h > (int64_t(1) << 28)) { err = "bad PNG dimensions"; return false; }
  if (ctype == 2) channels = 3;
  else if (ctype == 6) channels = 4;
  else if (ctype == 4) channels = 2;
  else if (ctype == 0) channels = 1;
  else { err = "palette PNG not supported"; return false; }
  const size_t stride = (size_t)w * channels;
  std::vector<uint8_t> raw((stride + 1) * h);
  uLongf rawLen = raw.size();
  if (uncompress(raw.data(), &rawLen, idat.data(), idat.size()) != Z_OK || rawLen != raw.size()) {
    err = "inflate failed";
    return false;
  }
  px.assign(stride * h, 0);
  const int bpp = channels;
  for (int y = 0; y < h; ++y) {
    const uint8_t ft = raw[(size_t)y * (stride + 1)];
    const uint8_t* s = &raw[(size_t)y * (stride + 1) + 1];
    uint8_t* o = &px[(size_t)y * stride];
    const uint8_t* up = y ? &px[(size_t)(y - 1) * stride] : nullptr;
    for (size_t i = 0; i < stride; ++i) {
      const int a = i >= (size_t)bpp ? o[i - bpp] : 0;
      const int b = up ? up[i] : 0;
      const int c = (up && i >= (size_t)bpp) ? up[i - bpp] : 0;
      int v = s[i];
      switch (ft) {
        case 0: break;
        case 1: v += a; break;
        case 2: v += b; break;
        case 3: v += (a + b) >> 1; break;
        case 4: {
          const int p = a + b - c, pa = abs(p - a), pb = abs(p - b), pc = abs(p - c);
          v += (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c);
          break;
        }
        default: err = "bad PNG filter"; return false;
      }
      o[i] = (uint8_t)v;
    }
  }
  return true;
}

static bool load_freeimage_png(const std::string& file, ImageObj& out) {
  std::vector<uint8_t> buf;
  if (!read_file(file, buf)) return false;
  int w, h, ch;
  std::vector<uint8_t> px;
  std::string err;
  if (!decode_png(buf, w, h, ch, px, err)) return false;
  out.width = w;
  out.height = h;
  out.format = IMG_RGBA8;
  out.data.assign((size_t)w * h * 4, 0);
  // FreeImage: grey (8 bpp) is skipped by loadFreeImage's bpp switch; grey+alpha expands
  // to 32 bpp. DIB scanline 0 is the bottom row.
  if (ch == 1) return true;
  for (int y = 0; y < h; ++y) {
    const uint8_t* s = &px[(size_t)(h - 1 - y) * w * ch];
    for (int x = 0; x < w; ++x) {
      uint8_t* p = &out.data[((size_t)y * w + x) * 4];
      float r, g, b, a = 1.f;
      if (ch >= 3) {
        r = (float)s[x * ch] / 255.0f;
        g = (float)s[x * ch + 1] / 255.0f;
        b = (float)s[x * ch + 2] / 255.0f;
        if (ch == 4) a = (float)s[x * ch + 3] / 255.0f;
      } else {
        r = g = b = (float)s[x * ch] / 255.0f;
        a = (float)s[x * ch + 1] / 255.0f;
      }
      p[0] = quantize(r); p[1] = quantize(g); p[2] = quantize(b); p[3] = quantize(a);
    }
  }
  return true;
}

// ---------------------------------------------------------------- JPEG (baseline)
namespace {

const int kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
                         41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
                         30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

struct Huff {
  bool present = false;
  uint8_t bits[17] = {0};
  uint8_t vals[256] = {0};
  int mincode[17], maxcode[18], valptr[17];
  Huff() { build(); }  // an absent table decodes nothing instead of reading uninitialized bounds
  void build() {
    int code = 0, k = 0;
    for (int l = 1; l <= 16; ++l) {
      valptr[l] = k;
      mincode[l] = code;
      code += bits[l];
      k += bits[l];
      maxcode[l] = bits[l] ? code - 1 : -1;
      code <<= 1;
    }
    maxcode[17] = 0x7fffffff;
  }
};

struct Comp {
  int id, H, V, tq, td, ta;
  int bw, bh;          // blocks allocated (multiples of MCU)
  int dw, dh;          // downsampled_width/height
  std::vector<uint8_t> plane;  // bw*8 x bh*8
  int pred = 0;
};

struct BitReader {
  const uint8_t* p;
  const uint8_t* end;
  uint32_t acc = 0;
  int n = 0;
  bool marker = false;
  int getbit() {
    if (n == 0) {
      uint8_t b = 0;
      if (!marker && p < end) {
        b = *p++;
        if (b == 0xFF) {
          const uint8_t b2 = p < end ? *p : 0;
          if (b2 == 0x00) p++;
          else { marker = true; b = 0; p--; }  // stop at marker, feed zeros
        }
      }
      acc = b;
      n = 8;
    }
    n--;
    return (acc >> n) & 1;
  }
  int bits(int k) {
    // a corrupt table can ask for more than the 16 bits a baseline JPEG ever reads: take at
    // most 16 (unsigned, so no shift overflows; mutation fuzz finding)
    unsigned v = 0;
    for (int i = 0; i < k && i < 16; ++i) v = (v << 1) | (unsigned)getbit();
    return (int)v;
  }
  void reset() { n = 0; marker = false; }
};

int decode_huff(BitReader& br, const Huff& t) {
  int code = br.getbit();
  int l = 1;
  while (l <= 16 && code > t.maxcode[l]) {
    code = (code << 1) | br.getbit();
    l++;
  }
  if (l > 16) return 0;
  return t.vals[t.valptr[l] + code - t.mincode[l]];
}

inline int extend(int v, int t) { return v < (1 << (t - 1)) ? v - (1 << t) + 1 : v; }

// jpeg_idct_islow (integer LL&M IDCT, CONST_BITS 13, PASS1_BITS 2)
void idct_islow(const int* in /* natural order, dequantized */, uint8_t* out, int stride) {
  const int CB = 13, P1 = 2;
  auto D = [](long long x, int n) { return (int)((x + (1ll << (n - 1))) >> n); };
  const long F0298 = 2446, F0390 = 3196, F0541 = 4433, F0765 = 6270, F0899 = 7373, F1175 = 9633, F1501 = 12299,
             F1847 = 15137, F1961 = 16069, F2053 = 16819, F2562 = 20995, F3072 = 25172;
  int ws[64];
  for (int c = 0; c < 8; ++c) {
    const int* ip = in + c;
    if (!ip[8] && !ip[16] && !ip[24] && !ip[32] && !ip[40] && !ip[48] && !ip[56]) {
      const int dc = ip[0] * (1 << P1);  // a multiply: left shifts of negative values are UB (UBSan, r05)
      for (int r = 0; r < 8; ++r) ws[r * 8 + c] = dc;
      continue;
    }
    long long z2 = ip[16], z3 = ip[48];
    long long z1 = (z2 + z3) * F0541;
    long long tmp2 = z1 + z3 * (-F1847);
    long long tmp3 = z1 + z2 * F0765;
    z2 = ip[0];
    z3 = ip[32];
    long long tmp0 = (z2 + z3) * (1ll << CB);
    long long tmp1 = (z2 - z3) * (1ll << CB);
    const long long t10 = tmp0 + tmp3, t13 = tmp0 - tmp3, t11 = tmp1 + tmp2, t12 = tmp1 - tmp2;
    tmp0 = ip[56]; tmp1 = ip[40]; tmp2 = ip[24]; tmp3 = ip[8];
    z1 = tmp0 + tmp3; z2 = tmp1 + tmp2; z3 = tmp0 + tmp2; long long z4 = tmp1 + tmp3;
    const long long z5 = (z3 + z4) * F1175;
    tmp0 *= F0298; tmp1 *= F2053; tmp2 *= F3072; tmp3 *= F1501;
    z1 *= -F0899; z2 *= -F2562; z3 *= -F1961; z4 *= -F0390;
    z3 += z5; z4 += z5;
    tmp0 += z1 + z3; tmp1 += z2 + z4; tmp2 += z2 + z3; tmp3 += z1 + z4;
    ws[0 * 8 + c] = D(t10 + tmp3, CB - P1);
    ws[7 * 8 + c] = D(t10 - tmp3, CB - P1);
    ws[1 * 8 + c] = D(t11 + tmp2, CB - P1);
    ws[6 * 8 + c] = D(t11 - tmp2, CB - P1);
    ws[2 * 8 + c] = D(t12 + tmp1, CB - P1);
    ws[5 * 8 + c] = D(t12 - tmp1, CB - P1);
    ws[3 * 8 + c] = D(t13 + tmp0, CB - P1);
    ws[4 * 8 + c] = D(t13 - tmp0, CB - P1);
  }
  auto lim = [](int v) { v += 128; return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); };
  for (int r = 0; r < 8; ++r) {
    const int* w = ws + r * 8;
    uint8_t* o = out + r * stride;
    long long z2 = w[2], z3 = w[6];
    long long z1 = (z2 + z3) * F0541;
    long long tmp2 = z1 + z3 * (-F1847);
    long long tmp3 = z1 + z2 * F0765;
    long long tmp0 = ((long long)w[0] + w[4]) * (1ll << CB);
    long long tmp1 = ((long long)w[0] - w[4]) * (1ll << CB);
    const long long t10 = tmp0 + tmp3, t13 = tmp0 - tmp3, t11 = tmp1 + tmp2, t12 = tmp1 - tmp2;
    tmp0 = w[7]; tmp1 = w[5]; tmp2 = w[3]; tmp3 = w[1];
    z1 = tmp0 + tmp3; z2 = tmp1 + tmp2; z3 = tmp0 + tmp2; long long z4 = tmp1 + tmp3;
    const long long z5 = (z3 + z4) * F1175;
    tmp0 *= F0298; tmp1 *= F2053; tmp2 *= F3072; tmp3 *= F1501;
    z1 *= -F0899; z2 *= -F2562; z3 *= -F1961; z4 *= -F0390;
    z3 += z5; z4 += z5;
    tmp0 += z1 + z3; tmp1 += z2 + z4; tmp2 += z2 + z3; tmp3 += z1 + z4;
    const int S = CB + P1 + 3;
    o[0] = lim(D(t10 + tmp3, S)); o[7] = lim(D(t10 - tmp3, S));
    o[1] = lim(D(t11 + tmp2, S)); o[6] = lim(D(t11 - tmp2, S));
    o[2] = lim(D(t12 + tmp1, S)); o[5] = lim(D(t12 - tmp1, S));
    o[3] = lim(D(t13 + tmp0, S)); o[4] = lim(D(t13 - tmp0, S));
  }
}

}  // namespace

bool decode_jpeg(const std::vector<uint8_t>& f, int& W, int& Hh, std::vector<uint8_t>& rgb, std::string& err) {
  if (f.size() < 4 || f[0] != 0xFF || f[1] != 0xD8) { err = "not a JPEG"; return false; }
  uint16_t q[4][64] = {};
  Huff dc[4], ac[4];
  std::vector<Comp> comps;
  int restart = 0;
  size_t pos = 2;
  int Hmax = 1, Vmax = 1, mcux = 0, mcuy = 0;
  bool frame = false, done = false;
  while (pos + 4 <= f.size() && !done) {
    if (f[pos] != 0xFF) { pos++; continue; }
    const uint8_t m = f[pos + 1];
    pos += 2;
    if (m == 0xD8 || (m >= 0xD0 && m <= 0xD7) || m == 0x01 || m == 0xFF) continue;
    if (m == 0xD9) break;
    const size_t len = (size_t)f[pos] << 8 | f[pos + 1];
    // every marker segment must lie inside the file, and every table inside its segment
    // (the mutation fuzz of tools/run_sanitizers.sh found reads past both ends)
    if (len < 2 || pos + len > f.size()) { err = "truncated JPEG segment"; return false; }
    const uint8_t* d = &f[pos + 2];
    const size_t seg = pos + len;
    const size_t dl = len - 2;  // payload bytes of the segment
    if (m == 0xDB) {
      size_t i = 0;
      while (i + 1 < dl) {
        const int pq = d[i] >> 4, tq = d[i] & 15;
        i++;
        if (i + (pq ? 128 : 64) > dl) { err = "truncated quantization table"; return false; }
        for (int k = 0; k < 64; ++k) {
          const int v = pq ? (d[i] << 8 | d[i + 1]) : d[i];
          i += pq ? 2 : 1;
          q[tq & 3][kZigzag[k]] = (uint16_t)v;
        }
      }
    } else if (m == 0xC4) {
      size_t i = 0;
      while (i < dl) {
        if (i + 17 > dl) { err = "truncated Huffman table"; return false; }
        const int tc = d[i] >> 4, th = d[i] & 3;
        Huff& hh = tc ? ac[th] : dc[th];
        int total = 0;
        for (int l = 1; l <= 16; ++l) { hh.bits[l] = d[i + l]; total += d[i + l]; }
        if (total > 256 || i + 17 + (size_t)total > dl) { err = "bad Huffman table"; return false; }
        for (int k = 0; k < total; ++k) hh.vals[k] = d[i + 17 + k];
        hh.present = true;
        hh.build();
        i += 17 + total;
      }
    } else if (m == 0xC0 || m == 0xC1) {
      if (frame) { err = "second frame header"; return false; }
      if (dl < 6) { err = "truncated frame header"; return false; }
      if (d[0] != 8) { err = "12-bit JPEG"; return false; }
      Hh = d[1] << 8 | d[2];
      W = d[3] << 8 | d[4];
      const int nc = d[5];
      if (nc < 1 || nc > 4 || dl < 6 + 3 * (size_t)nc) { err = "bad frame header"; return false; }
      // decoded planes are allocated from these: refuse what no texture needs (256 Mpx)
      if (W < 1 || Hh < 1 || (int64_t)W * Hh > (int64_t(1) << 28)) { err = "bad JPEG dimensions"; return false; }
      comps.resize(nc);
      for (int c = 0; c < nc; ++c) {
        comps[c].id = d[6 + 3 * c];
        comps[c].H = d[7 + 3 * c] >> 4;
        comps[c].V = d[7 + 3 * c] & 15;
        comps[c].tq = d[8 + 3 * c];
        if (comps[c].H < 1 || comps[c].H > 4 || comps[c].V < 1 || comps[c].V > 4) {
          err = "bad sampling factors";
          return false;
        }
        Hmax = std::max(Hmax, comps[c].H);
        Vmax = std::max(Vmax, comps[c].V);
      }
      mcux = (W + 8 * Hmax - 1) / (8 * Hmax);
      mcuy = (Hh + 8 * Vmax - 1) / (8 * Vmax);
      for (auto& c : comps) {
        c.bw = mcux * c.H;
        c.bh = mcuy * c.V;
        c.dw = (W * c.H + Hmax - 1) / Hmax;
        c.dh = (Hh * c.V + Vmax - 1) / Vmax;
        c.plane.assign((size_t)c.bw * 8 * c.bh * 8, 0);
      }
      frame = true;
    } else if (m == 0xC2 || m == 0xC3 || (m >= 0xC5 && m <= 0xCF && m != 0xC8 && m != 0xCC)) {
      err = "progressive/lossless/arithmetic JPEG not supported";
      return false;
    } else if (m == 0xDD) {
      if (dl < 2) { err = "truncated restart interval"; return false; }
      restart = d[0] << 8 | d[1];
    } else if (m == 0xDA) {
      if (!frame) { err = "SOS before SOF"; return false; }
      if (dl < 1) { err = "truncated scan header"; return false; }
      const int ns = d[0];
      if (ns < 1 || dl < 1 + 2 * (size_t)ns) { err = "bad scan header"; return false; }
      std::vector<Comp*> sc;
      for (int i = 0; i < ns; ++i) {
        for (auto& c : comps)
          if (c.id == d[1 + 2 * i]) {
            c.td = d[2 + 2 * i] >> 4;
            c.ta = d[2 + 2 * i] & 15;
            sc.push_back(&c);
          }
      }
      if (sc.empty()) { err = "scan without a frame component"; return false; }
      BitReader br;
      br.p = f.data() + seg;
      br.end = f.data() + f.size();
      for (auto* c : sc) c->pred = 0;
      int coef[64], deq[64];
      auto block = [&](Comp& c, int bx, int by) {
        memset(coef, 0, sizeof(coef));
        const int t = std::min(decode_huff(br, dc[c.td & 3]), 16);  // categories beyond 16: corrupt data
        const int diff = t ? extend(br.bits(t), t) : 0;
        c.pred = (int)((unsigned)c.pred + (unsigned)diff);  // corrupt data: wrap, not overflow
        coef[0] = c.pred;
        for (int k = 1; k < 64;) {
          const int rs = decode_huff(br, ac[c.ta & 3]);
          const int r = rs >> 4, s = rs & 15;
          if (s == 0) {
            if (r == 15) { k += 16; continue; }
            break;
          }
          k += r;
          if (k > 63) break;
          coef[kZigzag[k]] = extend(br.bits(s), s);
          k++;
        }
        for (int k = 0; k < 64; ++k) {
          // valid data stays far inside int; corrupt coefficients are clamped, not overflowed
          const long long v = (long long)coef[k] * q[c.tq & 3][k];
          deq[k] = (int)std::max(-(1ll << 24), std::min(v, 1ll << 24));
        }
        const int stride = c.bw * 8;
        idct_islow(deq, &c.plane[(size_t)by * 8 * stride + bx * 8], stride);
      };
      int mcuCount = 0;
      auto handle_restart = [&]() {
        if (restart && mcuCount > 0 && mcuCount % restart == 0) {
          // skip to the RSTn marker
          while (br.p + 1 < br.end && !(br.p[0] == 0xFF && br.p[1] >= 0xD0 && br.p[1] <= 0xD7)) br.p++;
          if (br.p + 1 < br.end) br.p += 2;
          br.reset();
          for (auto* c : sc) c->pred = 0;
        }
      };
      if (ns == 1) {
        Comp& c = *sc[0];
        const int bw = (c.dw + 7) / 8, bh = (c.dh + 7) / 8;
        for (int by = 0; by < bh; ++by)
          for (int bx = 0; bx < bw; ++bx) {
            handle_restart();
            block(c, bx, by);
            mcuCount++;
          }
      } else {
        for (int my = 0; my < mcuy; ++my)
          for (int mx = 0; mx < mcux; ++mx) {
            handle_restart();
            for (auto* c : sc)
              for (int v = 0; v < c->V; ++v)
                for (int h = 0; h < c->H; ++h) block(*c, mx * c->H + h, my * c->V + v);
            mcuCount++;
          }
      }
      // continue after the entropy-coded segment
      pos = (size_t)(br.p - f.data());
      while (pos + 1 < f.size() && !(f[pos] == 0xFF && f[pos + 1] != 0x00 && !(f[pos + 1] >= 0xD0 && f[pos + 1] <= 0xD7)))
        pos++;
      continue;
    }
    pos = seg;
  }
  if (!frame) { err = "no frame"; return false; }
  for (const Comp& c : comps)
    if (Hmax % c.H || Vmax % c.V) { err = "non-integral sampling factors"; return false; }

  // upsample each component to full resolution (jdsample.c fancy h2v1 / h2v2, else replicate)
  const int nc = (int)comps.size();
  std::vector<std::vector<uint8_t>> full(nc, std::vector<uint8_t>((size_t)W * Hh));
  for (int ci = 0; ci < nc; ++ci) {
    Comp& c = comps[ci];
    const int st = c.bw * 8;
    auto in = [&](int x, int y) -> int { return c.plane[(size_t)y * st + x]; };
    const int hf = Hmax / c.H, vf = Vmax / c.V;
    std::vector<uint8_t>& o = full[ci];
    if (hf == 1 && vf == 1) {
      for (int y = 0; y < Hh; ++y)
        for (int x = 0; x < W; ++x) o[(size_t)y * W + x] = (uint8_t)in(x, y);
    } else if (hf == 2 && vf == 1) {
      std::vector<uint8_t> row(2 * c.dw + 2);
      for (int y = 0; y < Hh; ++y) {
        const int dw = c.dw;
        if (dw == 1) { row[0] = row[1] = (uint8_t)in(0, y); }
        else {
          int k = 0;
          int iv = in(0, y);
          row[k++] = (uint8_t)iv;
          row[k++] = (uint8_t)((iv * 3 + in(1, y) + 2) >> 2);
          for (int x = 1; x < dw - 1; ++x) {
            iv = in(x, y) * 3;
            row[k++] = (uint8_t)((iv + in(x - 1, y) + 1) >> 2);
            row[k++] = (uint8_t)((iv + in(x + 1, y) + 2) >> 2);
          }
          iv = in(dw - 1, y);
          row[k++] = (uint8_t)((iv * 3 + in(dw - 2, y) + 1) >> 2);
          row[k++] = (uint8_t)iv;
        }
        for (int x = 0; x < W; ++x) o[(size_t)y * W + x] = row[x];
      }
    } else if (hf == 2 && vf == 2) {
      std::vector<uint8_t> row(2 * c.dw + 2);
      for (int y = 0; y < Hh; ++y) {
        const int r = y >> 1;
        const int r1 = (y & 1) ? std::min(r + 1, c.dh - 1) : std::max(r - 1, 0);
        const int dw = c.dw;
        auto cs = [&](int x) { return in(x, r) * 3 + in(x, r1); };
        int k = 0;
        if (dw == 1) {
          const int t = cs(0);
          row[k++] = (uint8_t)((t * 4 + 8) >> 4);
          row[k++] = (uint8_t)((t * 4 + 7) >> 4);
        } else {
          int thiscs = cs(0), nextcs = cs(1), lastcs;
          row[k++] = (uint8_t)((thiscs * 4 + 8) >> 4);
          row[k++] = (uint8_t)((thiscs * 3 + nextcs + 7) >> 4);
          lastcs = thiscs;
          thiscs = nextcs;
          for (int x = 2; x < dw; ++x) {
            nextcs = cs(x);
            row[k++] = (uint8_t)((thiscs * 3 + lastcs + 8) >> 4);
            row[k++] = (uint8_t)((thiscs * 3 + nextcs + 7) >> 4);
            lastcs = thiscs;
            thiscs = nextcs;
          }
          row[k++] = (uint8_t)((thiscs * 3 + lastcs + 8) >> 4);
          row[k++] = (uint8_t)((thiscs * 4 + 7) >> 4);
        }
        for (int x = 0; x < W; ++x) o[(size_t)y * W + x] = row[x];
      }
    } else {
      for (int y = 0; y < Hh; ++y)
        for (int x = 0; x < W; ++x) o[(size_t)y * W + x] = (uint8_t)in(x / hf, y / vf);
    }
  }
  rgb.resize((size_t)W * Hh * 3);
  if (nc == 1) {
    for (size_t i = 0; i < (size_t)W * Hh; ++i) rgb[3 * i] = rgb[3 * i + 1] = rgb[3 * i + 2] = full[0][i];
    return true;
  }
  if (nc != 3) { err = "unsupported component count"; return false; }
  // jdcolor.c ycc_rgb_convert (SCALEBITS 16)
  auto FIX = [](double x) { return (long)(x * 65536.0 + 0.5); };
  auto clamp8 = [](int v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); };
  for (size_t i = 0; i < (size_t)W * Hh; ++i) {
    const int y = full[0][i], cb = full[1][i] - 128, cr = full[2][i] - 128;
    const int crr = (int)((FIX(1.40200) * cr + (1l << 15)) >> 16);
    const int cbb = (int)((FIX(1.77200) * cb + (1l << 15)) >> 16);
    const long crg = -FIX(0.71414) * cr;
    const long cbg = -FIX(0.34414) * cb + (1l << 15);
    rgb[3 * i] = clamp8(y + crr);
    rgb[3 * i + 1] = clamp8(y + (int)((cbg + crg) >> 16));
    rgb[3 * i + 2] = clamp8(y + cbb);
  }
  return true;
}

static bool load_jpeg(const std::string& file, ImageObj& out) {
  std::vector<uint8_t> buf;
  if (!read_file(file, buf)) return false;
  int w, h;
  std::vector<uint8_t> rgb;
  std::string err;
  if (!decode_jpeg(buf, w, h, rgb, err)) throw std::runtime_error("JPEG " + file + ": " + err);
  out.width = w;
  out.height = h;
  out.format = IMG_RGBA8;
  out.data.assign((size_t)w * h * 4, 0);
  const float rcp255 = rcpf_(255.f);
  for (int y = 0, yFlip = h - 1; y < h; y++, yFlip--)
    for (int x = 0; x < w; x++) {
      const uint8_t* s = &rgb[((size_t)y * w + x) * 3];
      uint8_t* p = &out.data[((size_t)yFlip * w + x) * 4];
      p[0] = quantize((float)s[0] * rcp255);
      p[1] = quantize((float)s[1] * rcp255);
      p[2] = quantize((float)s[2] * rcp255);
      p[3] = quantize(1.f);
    }
  return true;
}

bool image_load(const std::string& file, ImageObj& out) {
  std::string ext;
  const size_t dot = file.find_last_of('.');
  if (dot != std::string::npos) ext = file.substr(dot + 1);
  for (auto& ch : ext) ch = (char)tolower(ch);
  try {
    if (ext == "jpg" || ext == "jpeg") return load_jpeg(file, out);
    if (ext == "ppm") return load_ppm(file, out);
    return load_freeimage_png(file, out);
  } catch (const std::exception&) {
    return false;
  }
}

}  // namespace yrt
