// Shared definitions for the UP-Retinex gfx950 kernel library (libupr.so).
//
// Activations live in HBM as NHWC (channels innermost) in the model's storage
// type T (float or _Float16); accumulation is always fp32.  The C ABI itself
// (include/upr.h) exposes only plain pointers, sizes and a stream handle.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

#define UPR_CHECK_HIP(expr)                                  \
  do {                                                       \
    hipError_t _e = (expr);                                  \
    if (_e != hipSuccess) return (int)_e;                    \
  } while (0)

namespace upr {

typedef _Float16 half_t;

// Status codes (mirrored in include/upr.h).
enum : int {
  kOk = 0,
  kErrArg = -1,
  kErrShape = -2,
  kErrMissingParam = -3,
  kErrWorkspace = -4,
  kErrUnsupported = -5,
};

enum DType : int { kF32 = 0, kF16 = 1 };

// ---------------------------------------------------------------------------
// Implicit-GEMM convolution descriptor.
//
// GEMM view: M = B*Ho*Wo output pixels, N = output channels, K = sum over
// segments of (kh*kw*C_seg).  A segment is one operand of a "virtual concat":
// it reads C channels of an NHWC source at channel offset coff (pixel stride
// cs), through a kh x kw window with its own stride / padding / dilation.  The
// packed weight matrix is [N][Kpad] (k contiguous), K ordered (segment, tap,
// channel).
// ---------------------------------------------------------------------------
enum SegPre : int {
  kPreNone = 0,
  kPreAffineRelu = 1,  // v = max(v*pre_scale[c] + pre_shift[c], 0), in-bounds taps only
  kPreMaxPool3 = 2,    // 3x3/s1/p1 max-pool of the source (padding ignored), then the tap
};

struct ConvSeg {
  const void* src;
  int C, cs, coff;      // channels read, source pixel stride, channel offset
  int Hin, Win;
  int kh, kw, stride, pad, dil;
  int pre;
  const float* pre_scale;
  const float* pre_shift;
  int kbase;            // first k row of this segment in the packed weights
};

enum StoreMode : int {
  kStoreNHWC = 0,       // out[m*out_cs + out_coff + n]
  kStoreConvT2x2 = 1,   // ConvTranspose2d k2 s2 pixel shuffle: n = (dy*2+dx)*Cout + co
  kStoreHeadIllu = 2,   // residual head: illu = sigmoid(mean_c(x) + relu(v).w2 + b2) (N == 32)
};

struct ConvOp {
  int nseg;
  ConvSeg seg[4];
  int B, Ho, Wo, N;
  int Kpad;
  const void* W;          // packed weights [N][Kpad], type T
  const float* scale;     // per output channel (nullable => 1)
  const float* bias;      // per output channel (nullable => 0)
  const float* img_bias;  // per (image, channel) [B][N] (nullable)
  const void* res1; int res1_cs;  // added before ReLU (nullable)
  int relu;
  const void* res2; int res2_cs;  // added after ReLU (nullable)
  void* out; int out_cs, out_coff;
  int store;
  float* pool;            // per (image, channel) sum of the stored value (nullable)
  // kStoreConvT2x2: Cout = N/4, out is [B, 2Ho, 2Wo, out_cs]
  // kStoreHeadIllu:
  const float* head_w;    // [32] 1x1 weights
  float head_b;
  const float* x_nchw;    // network input (fp32 or T per x_f16), [B,3,Ho,Wo]
  int x_f16;
  float* illu;            // [B,1,Ho,Wo] fp32 output (or T when illu_f16)
  int illu_f16;
  // second output (fp16, kStoreNHWC only; nullable): out2[m*out2_cs + n] =
  // relu(fma(o, pre2_scale[n], pre2_shift[n])) of the fp16-rounded stored value
  // o -- the next PreActResBlock's relu(bn1(x)) (models/model.py:164-166)
  // written by the producer's epilogue instead of a separate pass
  void* out2; int out2_cs;
  const float* pre2_scale;
  const float* pre2_shift;
  // fp32 output of an fp16 conv (the training step's autocast convs, nullable;
  // launch_conv_out32 only): out32[pix * out32_cs + out32_coff + n] =
  // (float)(fp16-rounded result) + res32[pix * res32_cs + n] (res32 nullable,
  // may alias out32); `out` is not written
  float* out32; int out32_cs, out32_coff;
  const float* res32; int res32_cs;
  // with out32 (nullable): a compact fp16 copy of the same outputs,
  // out32_h16[pix * out32_h16_cs + n] = (half)(the fp32 value stored) -- the
  // next autocast conv's operand, so it needs no cast pass of its own
  void* out32_h16; int out32_h16_cs;
  // with out32 (nullable): both outputs zeroed where mask16[pix * mask16_cs +
  // n] <= 0 -- the ReLU backward of the activation this input gradient flows
  // into, fused (mask16 = that activation's fp16 copy); skip32: out32 is not
  // written, only out32_h16 (a gradient whose one reader takes the fp16 copy)
  const void* mask16; int mask16_cs; int skip32;
  // with out32, a 1x1 stride-1 op over an H x W input (launch_conv_pw only):
  // input pixel (b, i, j) lands at output pixel (b, 2i, 2j) of a 2H x 2W map,
  // the others are not written (the 1x1 stride-2 conv's input gradient)
  int out_s2;
  // hwide4 pointwise form (set by its dispatcher, 0 elsewhere): each tile walks
  // its K chunks starting at chunk mtile % NCH instead of 0
  int krot;
};

// fp16 convs with an fp32 output (ConvOp::out32): the wide-tile and row-ring
// kernels; kErrUnsupported when neither takes the op
int launch_conv_out32(const ConvOp& op, hipStream_t stream);
// the input gradient of a 3x3 stride-2 pad-1 conv straight from dy (conv_pw.hip;
// op = the stride-1 dgrad op over dy with the flipped filter, output 2H x 2W)
int launch_conv_s2dg(const ConvOp& op, hipStream_t stream, bool probe = false);
// fp16 1x1 streaming convs (conv_pw.hip); probe: only answer kOk / kErrUnsupported
int launch_conv_pw(const ConvOp& op, hipStream_t stream, bool probe = false);

int launch_conv(const ConvOp& op, int dtype, hipStream_t stream);

inline int cdiv(int a, int b) { return (a + b - 1) / b; }

// Per-(image, channel) pool sums (ConvOp::pool: EnhancedFAM channel attention,
// ASPP global branch) are accumulated as 64-bit fixed point (2^-24 units) with
// integer atomics: the sum no longer depends on the order in which tiles /
// units finish, so a forward is bit-for-bit reproducible.  A pool entry is 16
// bytes (the float* is only the carrier type): the int64 sum, then a uint32 of
// non-finite flags (bit 0 a +inf, bit 1 a -inf, bit 2 a NaN contribution),
// set with an atomic OR instead of converting the value, so pool_get returns
// what torch's mean would (+inf, -inf, or NaN for NaN / +inf with -inf).
constexpr float kPoolScale = 16777216.f;  // 2^24
constexpr int kPoolEntryFloats = 4;       // 16-byte entries
#ifdef __HIPCC__
__device__ __forceinline__ void pool_add(float* pool, size_t idx, float v) {
  if (__builtin_isfinite(v)) {
    atomicAdd((unsigned long long*)pool + 2 * idx, (unsigned long long)__float2ll_rn(v * kPoolScale));
  } else {
    const unsigned f = __builtin_isnan(v) ? 4u : (v > 0.f ? 1u : 2u);
    atomicOr((unsigned*)pool + 4 * idx + 2, f);
  }
}
__device__ __forceinline__ float pool_get(const float* pool, size_t idx) {
  const unsigned f = ((const unsigned*)pool)[4 * idx + 2];
  if (f) return (f & 4u) || (f & 3u) == 3u ? __builtin_nanf("") : ((f & 1u) ? __builtin_inff() : -__builtin_inff());
  return (float)((double)(long long)((const unsigned long long*)pool)[2 * idx] * (1.0 / 16777216.0));
}
#endif
inline size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

// Per-(device, stream) scratch of the training kernels (split-K slabs,
// argmax codes, bilinear row sums, partial sums): one growable buffer per
// slot, reused by every later call on that stream -- the calls are
// stream-ordered, so a buffer is never live in two of them at once; buffers
// that ARE live together (a nested call) take different slots.  Replaces
// hipMallocAsync / hipFreeAsync, which cost 0.1-0.5 ms of host time per
// call on this stack (13 of 36 ms per training step went to them) and
// stalled the launch queue.  Growth (warm-up only) synchronises the stream
// before freeing the smaller buffer.  Returns nullptr when out of memory.
// At most kScratchStreams (device, stream) pairs hold buffers; a new pair past
// that reclaims the least recently used entry that only the calling thread
// ever used (after a device synchronise: that thread's earlier calls have all
// enqueued their launches), and gets nullptr (the caller's entry point returns
// an error) only when every entry is another thread's or shared, or while its
// stream is being captured.
constexpr int kScratchStreams = 64;
enum ScratchSlot { kSlotSlab = 0, kSlotCast, kSlotTmp, kSlotCode, kSlotRows, kSlotPart, kSlotMs, kSlotCount };
// fresh (optional): set true when the returned buffer was (re)allocated by this call
void* scratch(int slot, size_t bytes, hipStream_t st, bool* fresh = nullptr);

}  // namespace upr
