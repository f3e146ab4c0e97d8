// Integer tables of OpenCV's bit-exact 8-bit sRGB <-> CIE Lab conversion
// (third-party dependency of enhancers/adaptive_params.py:145,158: cv2.cvtColor
// COLOR_BGR2LAB / COLOR_LAB2BGR; OpenCV 4.x imgproc/src/color_lab.cpp,
// RGB2Lab_b + Lab2RGBinteger).  Built on the host, uploaded once per device.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define UPR_HD __host__ __device__
#else
#define UPR_HD
#endif

namespace upr {

struct LabTables {
  // RGB -> Lab
  uint16_t gamma_b[256];      // sRGBGammaTab_b: round(2040 * gamma(i/255))
  uint16_t cbrt_b[3072];      // LabCbrtTab_b: round(2^15 * f(i/2040))
  int32_t rgb2xyz[9];         // rows X,Y,Z; columns R,G,B; scaled by 2^12 / whitepoint
  // Lab -> RGB
  uint16_t yf_b[512];         // LabToYF_b: (y, ify) pairs, BASE = 2^14
  uint16_t invgamma_b[4096];  // sRGBInvGammaTab_b: round(255 * invgamma(i/4096))
  int32_t xyz2rgb[9];         // rows R,G,B; columns X,Y,Z; scaled by 2^12 * whitepoint
};

const LabTables& lab_tables();

// abTozXZ_b entry for index v (OpenCV computes it by this integer formula).
UPR_HD inline int ab_to_xz(int v) {
  const int BASE = 1 << 14;
  if (v <= 3390) return v * 108 / 841 - BASE * 16 / 116 * 108 / 841;
  return v * v / BASE * v / BASE;
}

}  // namespace upr
