// jpeg_encode.cpp — baseline JPEG writer for the cube-map outputs (.jpg, -jpegQuality).
//
// The reference stores its JPEGs through FreeImage (common/image/freeimage.cpp:191-232:
// 24-bit DIB, quality = -jpegQuality, libjpeg defaults: YCbCr 4:2:0, baseline Huffman
// tables). This writer follows the IJG libjpeg compression path step by step — fixed-point
// RGB->YCbCr (jccolor.c), 2x2 box downsampling with alternating rounding bias
// (jcsample.c h2v2_downsample), edge replication (jcprepct.c), the ISLOW integer FDCT
// (jfdctint.c), rounding quantization (jcdctmgr.c), dummy edge blocks (jccoefct.c) and the
// standard Huffman tables (jcparam.c / ITU T.81 K.3) — so its coefficients equal those of
// libjpeg-turbo (tests/test_frontend.py pins it through PIL). FreeImage 3.17 bundles IJG
// libjpeg 9a, whose default DCT-domain chroma downsampling differs from this 6b-style box
// filter in the last bits of the chroma planes (parity unpinned there: no FreeImage binary
// can run here).
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <stdexcept>
#include <string>
#include <vector>

namespace yrtfe {

namespace {

// ITU T.81 K.1 / K.2 (jcparam.c std_luminance_quant_tbl / std_chrominance_quant_tbl), natural order
const int kStdLum[64] = {16, 11, 10, 16, 24,  40,  51,  61,  12, 12, 14, 19, 26,  58,  60,  55,
                         14, 13, 16, 24, 40,  57,  69,  56,  14, 17, 22, 29, 51,  87,  80,  62,
                         18, 22, 37, 56, 68,  109, 103, 77,  24, 35, 55, 64, 81,  104, 113, 92,
                         49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99};
const int kStdChr[64] = {17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99, 24, 26, 56, 99, 99, 99,
                         99, 99, 47, 66, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99,
                         99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99};
const int kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
                         41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
                         30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

// K.3 standard Huffman tables (bits[1..16], values)
const uint8_t kDcLumBits[17] = {0, 0, 1, 5, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0};
const uint8_t kDcLumVal[12] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11};
const uint8_t kDcChrBits[17] = {0, 0, 3, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0};
const uint8_t kDcChrVal[12] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11};
const uint8_t kAcLumBits[17] = {0, 0, 2, 1, 3, 3, 2, 4, 3, 5, 5, 4, 4, 0, 0, 1, 0x7d};
const uint8_t kAcLumVal[162] = {
    0x01, 0x02, 0x03, 0x00, 0x04, 0x11, 0x05, 0x12, 0x21, 0x31, 0x41, 0x06, 0x13, 0x51, 0x61, 0x07, 0x22, 0x71,
    0x14, 0x32, 0x81, 0x91, 0xa1, 0x08, 0x23, 0x42, 0xb1, 0xc1, 0x15, 0x52, 0xd1, 0xf0, 0x24, 0x33, 0x62, 0x72,
    0x82, 0x09, 0x0a, 0x16, 0x17, 0x18, 0x19, 0x1a, 0x25, 0x26, 0x27, 0x28, 0x29, 0x2a, 0x34, 0x35, 0x36, 0x37,
    0x38, 0x39, 0x3a, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59,
    0x5a, 0x63, 0x64, 0x65, 0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a, 0x83,
    0x84, 0x85, 0x86, 0x87, 0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9a, 0xa2, 0xa3,
    0xa4, 0xa5, 0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3,
    0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca, 0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda, 0xe1, 0xe2,
    0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9, 0xea, 0xf1, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa};
const uint8_t kAcChrBits[17] = {0, 0, 2, 1, 2, 4, 4, 3, 4, 7, 5, 4, 4, 0, 1, 2, 0x77};
const uint8_t kAcChrVal[162] = {
    0x00, 0x01, 0x02, 0x03, 0x11, 0x04, 0x05, 0x21, 0x31, 0x06, 0x12, 0x41, 0x51, 0x07, 0x61, 0x71, 0x13, 0x22,
    0x32, 0x81, 0x08, 0x14, 0x42, 0x91, 0xa1, 0xb1, 0xc1, 0x09, 0x23, 0x33, 0x52, 0xf0, 0x15, 0x62, 0x72, 0xd1,
    0x0a, 0x16, 0x24, 0x34, 0xe1, 0x25, 0xf1, 0x17, 0x18, 0x19, 0x1a, 0x26, 0x27, 0x28, 0x29, 0x2a, 0x35, 0x36,
    0x37, 0x38, 0x39, 0x3a, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58,
    0x59, 0x5a, 0x63, 0x64, 0x65, 0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a,
    0x82, 0x83, 0x84, 0x85, 0x86, 0x87, 0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9a,
    0xa2, 0xa3, 0xa4, 0xa5, 0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba,
    0xc2, 0xc3, 0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca, 0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda,
    0xe2, 0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9, 0xea, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa};

struct Huff {
  uint16_t code[256];
  uint8_t size[256];
  void build(const uint8_t* bits, const uint8_t* val) {  // jchuff.c jpeg_make_c_derived_tbl
    memset(size, 0, sizeof(size));
    int k = 0, c = 0;
    for (int l = 1; l <= 16; ++l) {
      for (int i = 0; i < bits[l]; ++i, ++k) {
        code[val[k]] = (uint16_t)c++;
        size[val[k]] = (uint8_t)l;
      }
      c <<= 1;
    }
  }
};

struct BitWriter {
  std::vector<uint8_t>& out;
  uint32_t acc = 0;
  int n = 0;
  explicit BitWriter(std::vector<uint8_t>& o) : out(o) {}
  void put(uint32_t bits, int len) {
    while (len > 0) {
      const int take = len > 16 ? 16 : len;
      const uint32_t v = (bits >> (len - take)) & ((1u << take) - 1u);
      acc = (acc << take) | v;
      n += take;
      len -= take;
      while (n >= 8) {
        const uint8_t b = (uint8_t)(acc >> (n - 8));
        out.push_back(b);
        if (b == 0xFF) out.push_back(0);  // byte stuffing
        n -= 8;
      }
      acc &= (1u << n) - 1u;
    }
  }
};

// jfdctint.c (ISLOW), CONST_BITS 13, PASS1_BITS 2
inline int32_t descale(int64_t x, int n) { return (int32_t)((x + ((int64_t)1 << (n - 1))) >> n); }
void fdct_islow(int32_t d[64]) {
  const int CB = 13, P1 = 2;
  const int32_t F0298 = 2446, F0390 = 3196, F0541 = 4433, F0765 = 6270, F0899 = 7373, F1175 = 9633, F1501 = 12299,
                F1847 = 15137, F1961 = 16069, F2053 = 16819, F2562 = 20995, F3072 = 25172;
  for (int r = 0; r < 8; ++r) {
    int32_t* p = d + r * 8;
    int64_t t0 = p[0] + p[7], t7 = p[0] - p[7], t1 = p[1] + p[6], t6 = p[1] - p[6];
    int64_t t2 = p[2] + p[5], t5 = p[2] - p[5], t3 = p[3] + p[4], t4 = p[3] - p[4];
    int64_t t10 = t0 + t3, t13 = t0 - t3, t11 = t1 + t2, t12 = t1 - t2;
    p[0] = (int32_t)((t10 + t11) * (1 << P1));  // multiplies: left shifts of negative values are UB
    p[4] = (int32_t)((t10 - t11) * (1 << P1));
    int64_t z1 = (t12 + t13) * F0541;
    p[2] = descale(z1 + t13 * F0765, CB - P1);
    p[6] = descale(z1 + t12 * (-F1847), CB - P1);
    z1 = t4 + t7;
    int64_t z2 = t5 + t6, z3 = t4 + t6, z4 = t5 + t7;
    const int64_t z5 = (z3 + z4) * F1175;
    t4 *= F0298; t5 *= F2053; t6 *= F3072; t7 *= F1501;
    z1 *= -F0899; z2 *= -F2562; z3 *= -F1961; z4 *= -F0390;
    z3 += z5; z4 += z5;
    p[7] = descale(t4 + z1 + z3, CB - P1);
    p[5] = descale(t5 + z2 + z4, CB - P1);
    p[3] = descale(t6 + z2 + z3, CB - P1);
    p[1] = descale(t7 + z1 + z4, CB - P1);
  }
  for (int c = 0; c < 8; ++c) {
    int32_t* p = d + c;
    int64_t t0 = p[0] + p[56], t7 = p[0] - p[56], t1 = p[8] + p[48], t6 = p[8] - p[48];
    int64_t t2 = p[16] + p[40], t5 = p[16] - p[40], t3 = p[24] + p[32], t4 = p[24] - p[32];
    int64_t t10 = t0 + t3, t13 = t0 - t3, t11 = t1 + t2, t12 = t1 - t2;
    p[0] = descale(t10 + t11, P1);
    p[32] = descale(t10 - t11, P1);
    int64_t z1 = (t12 + t13) * F0541;
    p[16] = descale(z1 + t13 * F0765, CB + P1);
    p[48] = descale(z1 + t12 * (-F1847), CB + P1);
    z1 = t4 + t7;
    int64_t z2 = t5 + t6, z3 = t4 + t6, z4 = t5 + t7;
    const int64_t z5 = (z3 + z4) * F1175;
    t4 *= F0298; t5 *= F2053; t6 *= F3072; t7 *= F1501;
    z1 *= -F0899; z2 *= -F2562; z3 *= -F1961; z4 *= -F0390;
    z3 += z5; z4 += z5;
    p[56] = descale(t4 + z1 + z3, CB + P1);
    p[40] = descale(t5 + z2 + z4, CB + P1);
    p[24] = descale(t6 + z2 + z3, CB + P1);
    p[8] = descale(t7 + z1 + z4, CB + P1);
  }
}

// jcparam.c jpeg_quality_scaling + jpeg_add_quant_table(force_baseline)
void scale_table(const int* base, int quality, int out[64]) {
  if (quality <= 0) quality = 1;
  if (quality > 100) quality = 100;
  const int scale = quality < 50 ? 5000 / quality : 200 - quality * 2;
  for (int i = 0; i < 64; ++i) {
    long t = ((long)base[i] * scale + 50L) / 100L;
    if (t <= 0L) t = 1L;
    if (t > 255L) t = 255L;
    out[i] = (int)t;
  }
}

void put16(std::vector<uint8_t>& o, int v) {
  o.push_back((uint8_t)(v >> 8));
  o.push_back((uint8_t)(v & 255));
}

struct Plane {
  int w = 0, h = 0;  // padded to whole blocks
  std::vector<uint8_t> px;
  uint8_t at(int x, int y) const { return px[(size_t)y * w + x]; }
};

}  // namespace

// rgb: 8-bit RGB, top row first, `stride` bytes per row.
std::vector<uint8_t> encode_jpeg(const uint8_t* rgb, int width, int height, size_t stride, int quality) {
  if (width <= 0 || height <= 0 || width > 65535 || height > 65535) throw std::runtime_error("jpeg: bad size");
  // ---- color conversion (jccolor.c rgb_ycc_start/rgb_ycc_convert), SCALEBITS 16
  auto FIX = [](double x) { return (int32_t)(x * 65536.0 + 0.5); };
  int32_t tab[8][256];
  const int32_t ONE_HALF = 1 << 15, CBCR_OFFSET = 128 << 16;
  for (int i = 0; i < 256; ++i) {
    tab[0][i] = FIX(0.29900) * i;
    tab[1][i] = FIX(0.58700) * i;
    tab[2][i] = FIX(0.11400) * i + ONE_HALF;
    tab[3][i] = (-FIX(0.16874)) * i;
    tab[4][i] = (-FIX(0.33126)) * i;
    tab[5][i] = FIX(0.50000) * i + CBCR_OFFSET + ONE_HALF - 1;  // B=>Cb and R=>Cr share this table
    tab[6][i] = (-FIX(0.41869)) * i;
    tab[7][i] = (-FIX(0.08131)) * i;
  }
  // MCU 16x16; luma blocks cover ceil(W/8) x ceil(H/8), chroma ceil(ceil(W/2)/8) x ...
  const int mcuX = (width + 15) / 16, mcuY = (height + 15) / 16;
  const int cw = (width + 1) / 2, ch = (height + 1) / 2;
  const int lumBW = (width + 7) / 8, lumBH = (height + 7) / 8;
  const int chrBW = (cw + 7) / 8, chrBH = (ch + 7) / 8;
  // full-resolution component rows expanded (jcprepct/jcsample edge replication): width to
  // chrBW*16 (>= lumBW*8), height to a whole row group and then to whole blocks
  const int fullW = std::max(lumBW * 8, chrBW * 16), fullH = std::max(lumBH * 8, chrBH * 16);
  std::vector<uint8_t> Y((size_t)fullW * fullH), Cb((size_t)fullW * fullH), Cr((size_t)fullW * fullH);
  for (int y = 0; y < fullH; ++y) {
    const int sy = y < height ? y : height - 1;
    const uint8_t* row = rgb + (size_t)sy * stride;
    for (int x = 0; x < fullW; ++x) {
      const int sx = x < width ? x : width - 1;
      const int r = row[3 * sx], g = row[3 * sx + 1], b = row[3 * sx + 2];
      const size_t o = (size_t)y * fullW + x;
      Y[o] = (uint8_t)((tab[0][r] + tab[1][g] + tab[2][b]) >> 16);
      Cb[o] = (uint8_t)((tab[3][r] + tab[4][g] + tab[5][b]) >> 16);
      Cr[o] = (uint8_t)((tab[5][r] + tab[6][g] + tab[7][b]) >> 16);
    }
  }
  // libjpeg replicates the last real sample row/column of each *component* after
  // downsampling; rows/cols beyond the image were filled above from the last image
  // row/column, which the 2x2 box filter maps to the same values except where a box
  // straddles the edge — handled by computing the chroma plane from the real columns only.
  Plane lum;
  lum.w = lumBW * 8;
  lum.h = lumBH * 8;
  lum.px.resize((size_t)lum.w * lum.h);
  for (int y = 0; y < lum.h; ++y)
    for (int x = 0; x < lum.w; ++x) lum.px[(size_t)y * lum.w + x] = Y[(size_t)y * fullW + x];
  auto down = [&](const std::vector<uint8_t>& C, Plane& P) {
    // jcsample.c h2v2_downsample over rows expanded to output_cols*2; rows of the last row
    // group beyond the image are copies of the last image row (jcprepct expand_bottom_edge)
    P.w = chrBW * 8;
    P.h = chrBH * 8;
    P.px.resize((size_t)P.w * P.h);
    const int realRows = ch;  // downsampled rows that come from image rows
    for (int oy = 0; oy < P.h; ++oy) {
      if (oy >= realRows) {  // bottom padding: copy of the last real downsampled row
        memcpy(&P.px[(size_t)oy * P.w], &P.px[(size_t)(realRows - 1) * P.w], P.w);
        continue;
      }
      const uint8_t* r0 = &C[(size_t)(2 * oy) * fullW];
      const uint8_t* r1 = &C[(size_t)(2 * oy + 1) * fullW];
      int bias = 1;
      for (int ox = 0; ox < P.w; ++ox) {
        P.px[(size_t)oy * P.w + ox] = (uint8_t)((r0[2 * ox] + r0[2 * ox + 1] + r1[2 * ox] + r1[2 * ox + 1] + bias) >> 2);
        bias ^= 3;
      }
    }
  };
  Plane pcb, pcr;
  down(Cb, pcb);
  down(Cr, pcr);

  int qL[64], qC[64];
  scale_table(kStdLum, quality, qL);
  scale_table(kStdChr, quality, qC);
  Huff dcL, acL, dcC, acC;
  dcL.build(kDcLumBits, kDcLumVal);
  acL.build(kAcLumBits, kAcLumVal);
  dcC.build(kDcChrBits, kDcChrVal);
  acC.build(kAcChrBits, kAcChrVal);

  std::vector<uint8_t> o;
  o.reserve((size_t)width * height / 4 + 1024);
  // SOI, APP0 JFIF 1.01 (density 1:1, no units)
  const uint8_t head[] = {0xFF, 0xD8, 0xFF, 0xE0, 0x00, 0x10, 'J', 'F', 'I', 'F', 0x00, 0x01, 0x01, 0x00,
                          0x00, 0x01, 0x00, 0x01, 0x00, 0x00};
  o.insert(o.end(), head, head + sizeof(head));
  // DQT (zigzag order)
  for (int t = 0; t < 2; ++t) {
    o.push_back(0xFF); o.push_back(0xDB);
    put16(o, 67);
    o.push_back((uint8_t)t);
    const int* q = t ? qC : qL;
    for (int i = 0; i < 64; ++i) o.push_back((uint8_t)q[kZigzag[i]]);
  }
  // SOF0
  o.push_back(0xFF); o.push_back(0xC0);
  put16(o, 17);
  o.push_back(8);
  put16(o, height);
  put16(o, width);
  o.push_back(3);
  const uint8_t comps[9] = {1, 0x22, 0, 2, 0x11, 1, 3, 0x11, 1};
  o.insert(o.end(), comps, comps + 9);
  // DHT
  auto dht = [&](int cls, int id, const uint8_t* bits, const uint8_t* val) {
    int n = 0;
    for (int l = 1; l <= 16; ++l) n += bits[l];
    o.push_back(0xFF); o.push_back(0xC4);
    put16(o, 2 + 1 + 16 + n);
    o.push_back((uint8_t)((cls << 4) | id));
    for (int l = 1; l <= 16; ++l) o.push_back(bits[l]);
    o.insert(o.end(), val, val + n);
  };
  dht(0, 0, kDcLumBits, kDcLumVal);
  dht(1, 0, kAcLumBits, kAcLumVal);
  dht(0, 1, kDcChrBits, kDcChrVal);
  dht(1, 1, kAcChrBits, kAcChrVal);
  // SOS
  const uint8_t sos[] = {0xFF, 0xDA, 0x00, 0x0C, 0x03, 0x01, 0x00, 0x02, 0x11, 0x03, 0x11, 0x00, 0x3F, 0x00};
  o.insert(o.end(), sos, sos + sizeof(sos));

  BitWriter bw(o);
  int pred[3] = {0, 0, 0};
  auto nbits = [](int v) {
    int a = v < 0 ? -v : v, n = 0;
    while (a) { ++n; a >>= 1; }
    return n;
  };
  // encode one block (natural-order coefficients)
  auto enc = [&](const int32_t* coef, int comp, const Huff& dc, const Huff& ac) {
    int diff = coef[0] - pred[comp];
    pred[comp] = coef[0];
    int n = nbits(diff);
    bw.put(dc.code[n], dc.size[n]);
    if (n) bw.put((uint32_t)(diff < 0 ? diff - 1 : diff) & ((1u << n) - 1u), n);
    int run = 0;
    for (int k = 1; k < 64; ++k) {
      const int v = coef[kZigzag[k]];
      if (v == 0) {
        ++run;
        continue;
      }
      while (run > 15) {
        bw.put(ac.code[0xF0], ac.size[0xF0]);
        run -= 16;
      }
      n = nbits(v);
      const int sym = (run << 4) | n;
      bw.put(ac.code[sym], ac.size[sym]);
      bw.put((uint32_t)(v < 0 ? v - 1 : v) & ((1u << n) - 1u), n);
      run = 0;
    }
    if (run > 0) bw.put(ac.code[0], ac.size[0]);
  };
  // forward DCT + quantization of the block at (bx, by) of plane P (jcdctmgr.c forward_DCT)
  auto block = [&](const Plane& P, int bx, int by, const int* q, int32_t out[64]) {
    int32_t d[64];
    for (int y = 0; y < 8; ++y)
      for (int x = 0; x < 8; ++x) d[y * 8 + x] = (int32_t)P.at(bx * 8 + x, by * 8 + y) - 128;
    fdct_islow(d);
    for (int i = 0; i < 64; ++i) {
      const int32_t qv = q[i] << 3;
      int32_t t = d[i];
      if (t < 0) {
        t = -t + (qv >> 1);
        t = t >= qv ? t / qv : 0;
        t = -t;
      } else {
        t += qv >> 1;
        t = t >= qv ? t / qv : 0;
      }
      out[i] = t;
    }
  };
  int32_t coef[64], last[3][64];
  for (int my = 0; my < mcuY; ++my) {
    for (int mx = 0; mx < mcuX; ++mx) {
      // luma: 2x2 blocks; blocks beyond the component are dummy blocks (jccoefct.c): all AC
      // zero, DC copied from the previous block in the MCU row
      for (int v = 0; v < 2; ++v)
        for (int h = 0; h < 2; ++h) {
          const int bx = mx * 2 + h, by = my * 2 + v;
          if (bx < lumBW && by < lumBH) {
            block(lum, bx, by, qL, coef);
          } else {
            memset(coef, 0, sizeof(coef));
            coef[0] = last[0][0];
          }
          memcpy(last[0], coef, sizeof(coef));
          enc(coef, 0, dcL, acL);
        }
      for (int c = 0; c < 2; ++c) {
        const Plane& P = c ? pcr : pcb;
        if (mx < chrBW && my < chrBH) {
          block(P, mx, my, qC, coef);
        } else {
          memset(coef, 0, sizeof(coef));
          coef[0] = last[1 + c][0];
        }
        memcpy(last[1 + c], coef, sizeof(coef));
        enc(coef, 1 + c, dcC, acC);
      }
    }
  }
  // pad the last byte with 1 bits, EOI
  if (bw.n > 0) bw.put((1u << (8 - bw.n)) - 1u, 8 - bw.n);
  o.push_back(0xFF);
  o.push_back(0xD9);
  return o;
}

}  // namespace yrtfe
