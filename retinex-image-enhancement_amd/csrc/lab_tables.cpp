// Host construction of the 8-bit Lab tables (see lab_tables.h).
//
// OpenCV evaluates these with its softfloat/softdouble types; here float32 /
// float64 IEEE arithmetic is used in the same places (float32 where OpenCV
// uses softfloat, float64 where it uses softdouble), and cvRound is
// round-half-to-even.  Parity with cv2 itself is unpinned (cv2 is not
// installed in the build container); oracle/cv_u8.py restates the same
// construction independently in numpy and tests/test_cpu_lab.py compares them.
#include "lab_tables.h"

#include <cmath>
#include <mutex>

namespace upr {

static int cv_round(double v) { return (int)std::nearbyint(v); }  // default FE_TONEAREST: half-even

static double gamma_fwd(double x) {  // applyGamma, softdouble
  return x <= 809.0 / 20000.0 ? x / (323.0 / 25.0) : std::pow((x + 11.0 / 200.0) / (1.0 + 11.0 / 200.0), 12.0 / 5.0);
}
static double gamma_inv(double x) {  // applyInvGamma, softdouble
  return x <= 7827.0 / 2500000.0 ? x * (323.0 / 25.0)
                                 : std::pow(x, 1.0 / (12.0 / 5.0)) * (1.0 + 11.0 / 200.0) - 11.0 / 200.0;
}

static void build(LabTables& t) {
  const float f255 = 255.f;
  // sRGBGammaTab_b[i] = cvRound(intScale * applyGamma(i/255)), intScale = 255*8
  const float intScale = 255.f * 8.f;
  for (int i = 0; i < 256; ++i) {
    const float x = (float)i / f255;
    const float g = (float)gamma_fwd((double)x);
    t.gamma_b[i] = (uint16_t)cv_round((double)(intScale * g));
  }
  // LabCbrtTab_b[i] = cvRound(2^15 * (x < lthresh ? x*lscale + lbias : cbrt(x))), x = i / 2040
  const float lthresh = 216.f / 24389.f, lscale = 841.f / 108.f, lbias = 16.f / 116.f;
  const float cbScale = 1.f / (f255 * 8.f);
  const float lshift2 = 32768.f;
  for (int i = 0; i < 3072; ++i) {
    const float x = cbScale * (float)i;
    const float f = x < lthresh ? std::fmaf(x, lscale, lbias) : (float)std::cbrt((double)x);
    t.cbrt_b[i] = (uint16_t)cv_round((double)(lshift2 * f));
  }
  // sRGBInvGammaTab_b[i] = cvRound(255 * applyInvGamma(i/4096))
  for (int i = 0; i < 4096; ++i) {
    const float x = (1.f / 4096.f) * (float)i;
    const float g = (float)gamma_inv((double)x);
    t.invgamma_b[i] = (uint16_t)cv_round((double)(f255 * g));
  }
  // LabToYF_b
  const int BASE = 1 << 14;
  for (int i = 0; i < 256; ++i) {
    int y, ify;
    if (i <= 20) {
      y = cv_round((double)((float)(i * BASE * 20 * 9) / (float)(17 * 29 * 29 * 29)));
      ify = cv_round((double)((float)BASE * (16.f / 116.f + (float)(i * 5) / (float)(3 * 17 * 29))));
    } else {
      const float fy = (float)(i * 100 * BASE) / (float)(255 * 116) + (float)(16 * BASE) / 116.f;
      ify = cv_round((double)fy);
      y = cv_round((double)(fy * fy * fy / (float)(BASE * BASE)));
    }
    t.yf_b[2 * i] = (uint16_t)y;
    t.yf_b[2 * i + 1] = (uint16_t)ify;
  }
  // matrices (softdouble): sRGB2XYZ_D65, XYZ2sRGB_D65, D65 white point
  static const double rgb2xyz[9] = {0.412453, 0.357580, 0.180423, 0.212671, 0.715160,
                                    0.072169, 0.019334, 0.119193, 0.950227};
  static const double xyz2rgb[9] = {3.240479, -1.53715, -0.498535, -0.969256, 1.875991,
                                    0.041556, 0.055648, -0.204043, 1.057311};
  static const double wp[3] = {0.950456, 1.0, 1.088754};
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) {
      t.rgb2xyz[r * 3 + c] = cv_round(4096.0 * rgb2xyz[r * 3 + c] / wp[r]);
      t.xyz2rgb[r * 3 + c] = cv_round(4096.0 * xyz2rgb[r * 3 + c] * wp[c]);
    }
}

const LabTables& lab_tables() {
  static LabTables t;
  static std::once_flag once;
  std::call_once(once, [] { build(t); });
  return t;
}

}  // namespace upr
