// UP-Retinex forward executor: weight packing (host) + launch sequence (device).
//
// The layer graph follows models/model.py of the reference; every fold below
// is exact algebra on the eval-mode network (only fp rounding changes):
//  * BatchNorm2d(eval) after a conv folds into the conv's weights and bias.
//  * ResBlock/PreActResBlock projecting shortcut (conv1x1 s2 + BN) becomes a
//    second K-segment of conv2 (same GEMM, same output).
//  * PreAct's relu(bn1(x)) is a per-channel prologue of the segments reading x.
//  * EnhancedFAM: branch1, branch2 (after its max-pool) and the two cascaded
//    second convs are linear, so fusion(cat[b1,b2,b3,b4]) is ONE GEMM over the
//    virtual concat [h3 (3x3), h4 (3x3 d2), x (1x1), maxpool(x) (1x1)] with the
//    fusion 1x1 composed into each branch's weights.
//  * The head fusion(96->32) and output_layer(32->3) have no activation between
//    them and bilinear upsampling is linear per channel, so each scale's FAM
//    output is projected to 3 channels at its own resolution and only the
//    3-channel maps are upsampled (models/model.py:430-439).
//  * Spatial attention is a per-pixel scalar and commutes with that projection.
//  * ASPP's global branch is a per-(image, channel) bias of the ASPP fusion GEMM.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "upr_common.h"
#include "../../include/upr.h"

namespace upr {

int launch_prep(const void* x, void* x2p, void* x3p, int B, int H, int W, int dtype, hipStream_t st);
int launch_preact_f16(const void* x, const float* sc, const float* sh, void* o, size_t npix, int C, hipStream_t st);
int launch_conv3(const void* x, const float* w, const float* bias, void* out0, void* out1, int B, int h, int wd,
                 int dtype, hipStream_t st, void* out2 = nullptr, const float* ps = nullptr,
                 const float* ph = nullptr);
int launch_fam_ca(const float* pool, const float* w1, const float* b1, const float* w2, const float* b2, float* ca,
                  int B, int HW, hipStream_t st);
int launch_fam_mix(const void* y, const float* ca, const float* P, float* mm, float* p, int B, int HW, int dtype,
                   hipStream_t st);
int launch_fam_sa(const float* mm, const float* p, const float* w, float bias, float* q, int B, int h, int wd,
                  hipStream_t st);
int launch_tail(const void* x, const float* illu_f32, const void* illu_t, const float* q1, const float* q2,
                const float* q3, const float* cst, void* enh, void* refl, int B, int H, int W, int h2, int w2, int h3,
                int w3, int dtype, hipStream_t st, int refl_in);

// ---------------------------------------------------------------------------
// ASPP global-pool branch -> per-image bias of the ASPP fusion GEMM
//   g[b]  = relu(Wg (pool[b] / HW) + bg)          (models/model.py:215-220)
//   ib[b] = Wfg g[b]                              (fusion cols 1024..1279)
// One 256-thread block per image; C = 256.
// ---------------------------------------------------------------------------
__global__ void aspp_global_kernel(const float* __restrict__ pool, const float* __restrict__ Wg,
                                   const float* __restrict__ bg, const float* __restrict__ Wfg,
                                   float* __restrict__ ib, int C, float inv_hw) {
  extern __shared__ float sm[];
  float* mean = sm;
  float* g = sm + C;
  const int b = blockIdx.x;
  for (int c = threadIdx.x; c < C; c += blockDim.x) mean[c] = pool_get(pool, (size_t)b * C + c) * inv_hw;
  __syncthreads();
  for (int o = threadIdx.x; o < C; o += blockDim.x) {
    float s = bg[o];
    for (int c = 0; c < C; ++c) s += Wg[o * C + c] * mean[c];
    g[o] = fmaxf(s, 0.f);
  }
  __syncthreads();
  for (int o = threadIdx.x; o < C; o += blockDim.x) {
    float s = 0.f;
    for (int c = 0; c < C; ++c) s += Wfg[o * C + c] * g[c];
    ib[b * C + o] = s;
  }
}

// ---------------------------------------------------------------------------
// host-side parameter access
// ---------------------------------------------------------------------------
struct HostTensor {
  std::vector<int64_t> shape;
  std::vector<double> v;
  int64_t numel() const { return (int64_t)v.size(); }
};

struct ParamSet {
  std::map<std::string, HostTensor> t;
  std::string missing;
  const HostTensor* get(const std::string& k) {
    auto it = t.find(k);
    if (it == t.end()) {
      if (missing.empty()) missing = k;
      return nullptr;
    }
    return &it->second;
  }
  bool has(const std::string& k) const { return t.count(k) != 0; }
};

// Folded BatchNorm: y*s + sh
struct BNFold {
  std::vector<double> s, sh;
};
static bool bn_fold(ParamSet& P, const std::string& p, int C, BNFold& out) {
  const HostTensor* w = P.get(p + ".weight");
  const HostTensor* b = P.get(p + ".bias");
  const HostTensor* rm = P.get(p + ".running_mean");
  const HostTensor* rv = P.get(p + ".running_var");
  if (!w || !b || !rm || !rv) return false;
  if (w->numel() != C) return false;
  out.s.resize(C);
  out.sh.resize(C);
  for (int c = 0; c < C; ++c) {
    const double s = w->v[c] / std::sqrt(rv->v[c] + 1e-5);
    out.s[c] = s;
    out.sh[c] = b->v[c] - rm->v[c] * s;
  }
  return true;
}

// ---------------------------------------------------------------------------
// packed layers
// ---------------------------------------------------------------------------
struct SegSpec {
  int src;       // buffer id
  int C, coff, cs;
  int kh, kw, stride, pad, dil;
  int pre;
  size_t pre_scale = 0, pre_shift = 0;  // float offsets (bytes) in blob
  int kbase;
};

struct GemmLayer {
  int N = 0, Kpad = 0;
  size_t w = 0;                 // bytes offset of [N][Kpad] T
  size_t bias = SIZE_MAX;       // float [N]
  std::vector<SegSpec> segs;
};

// Blob builder: accumulates host bytes, later uploaded as one allocation.
struct Blob {
  std::vector<uint8_t> bytes;
  size_t add(const void* p, size_t n) {
    size_t off = align_up(bytes.size(), 256);
    bytes.resize(off + n);
    memcpy(bytes.data() + off, p, n);
    return off;
  }
  size_t add_f32(const std::vector<double>& v) {
    std::vector<float> f(v.begin(), v.end());
    return add(f.data(), f.size() * 4);
  }
  size_t add_t(const std::vector<double>& v, int dtype) {
    if (dtype == kF16) {
      std::vector<_Float16> h(v.size());
      for (size_t i = 0; i < v.size(); ++i) h[i] = (_Float16)(float)v[i];
      return add(h.data(), h.size() * 2);
    }
    return add_f32(v);
  }
};

// A K-segment's weights before packing: w[n][c][r][s] (row-major), already
// multiplied by any per-output-channel fold.
struct SegWeights {
  SegSpec spec;
  std::vector<double> w;  // N * C * kh * kw
};

static GemmLayer pack_gemm(Blob& blob, int dtype, int N, std::vector<SegWeights>& segs,
                           const std::vector<double>& bias) {
  GemmLayer L;
  L.N = N;
  int K = 0;
  for (auto& s : segs) {
    s.spec.kbase = K;
    K += s.spec.kh * s.spec.kw * s.spec.C;
  }
  L.Kpad = (int)align_up(K, 32);
  std::vector<double> W((size_t)N * L.Kpad, 0.0);
  for (auto& s : segs) {
    const int C = s.spec.C, kh = s.spec.kh, kw = s.spec.kw;
    for (int n = 0; n < N; ++n)
      for (int c = 0; c < C; ++c)
        for (int r = 0; r < kh; ++r)
          for (int q = 0; q < kw; ++q)
            W[(size_t)n * L.Kpad + s.spec.kbase + (r * kw + q) * C + c] =
                s.w[(((size_t)n * C + c) * kh + r) * kw + q];
    L.segs.push_back(s.spec);
  }
  L.w = blob.add_t(W, dtype);
  if (!bias.empty()) L.bias = blob.add_f32(bias);
  return L;
}

// Conv weight [N][C][kh][kw] from a HostTensor, rows scaled by mul (optional).
static std::vector<double> conv_w(const HostTensor& t, const std::vector<double>* mul) {
  std::vector<double> w = t.v;
  if (mul) {
    const size_t per = w.size() / mul->size();
    for (size_t n = 0; n < mul->size(); ++n)
      for (size_t i = 0; i < per; ++i) w[n * per + i] *= (*mul)[n];
  }
  return w;
}

// Compose a 1x1 map A [O][M] after a conv W [M][C][kh][kw]: (A W)[O][C][kh][kw]
static std::vector<double> compose(const std::vector<double>& A, int O, int Mdim, const std::vector<double>& W,
                                   int C, int khw) {
  std::vector<double> out((size_t)O * C * khw, 0.0);
  for (int o = 0; o < O; ++o)
    for (int m = 0; m < Mdim; ++m) {
      const double a = A[(size_t)o * Mdim + m];
      if (a == 0.0) continue;
      for (int i = 0; i < C * khw; ++i) out[(size_t)o * C * khw + i] += a * W[(size_t)m * C * khw + i];
    }
  return out;
}

// Columns [c0, c0+n) of a [rows][cols] matrix
static std::vector<double> cols(const std::vector<double>& A, int rows, int ncols, int c0, int n) {
  std::vector<double> out((size_t)rows * n);
  for (int r = 0; r < rows; ++r)
    for (int c = 0; c < n; ++c) out[(size_t)r * n + c] = A[(size_t)r * ncols + c0 + c];
  return out;
}

static SegSpec seg(int src, int C, int cs, int coff, int k, int stride, int pad, int dil, int pre = kPreNone) {
  SegSpec s;
  s.src = src; s.C = C; s.cs = cs; s.coff = coff;
  s.kh = k; s.kw = k; s.stride = stride; s.pad = pad; s.dil = dil;
  s.pre = pre; s.kbase = 0;
  return s;
}

// ---------------------------------------------------------------------------
// graph ops
// ---------------------------------------------------------------------------
enum BufId : int {
  BX = 0,  // network input (NCHW), not in workspace
  B_X2P, B_X3P,
  B_X1, B_S1IN, B_S2IN, B_S3IN,
  B_E1T, B_X2, B_E2T, B_X3, B_E3T, B_X4,
  B_B0T, B_B0, B_ASPP, B_AP, B_B1T, B_X5,
  B_U3, B_V3, B_D3, B_U2, B_V2, B_D2, B_U1, B_V1, B_D1,
  B_H1, B_Y1, B_H2, B_Y2, B_H3, B_Y3,
  B_MM1, B_P1, B_Q1, B_MM2, B_P2, B_Q2, B_MM3, B_P3, B_Q3,
  B_POOL,   // pool sums (FAM x3 + ASPP; 64-bit fixed point, upr_common.h pool_add), zeroed each forward
  B_CA,     // float ca [3][B][32]
  B_IB,     // float ASPP per-image bias [B][256]
  B_ILLU32, // float illu when the model dtype is fp16 (head writes fp32 then tail reads)
  B_PA1, B_PA2, B_PA3, B_PA4,  // fp16 PreAct: materialised relu(bn1(x)) of the blocks at levels 0..3
  B_FT,     // fp32 FAM fusion split: the partial sum between its parts (32 ch, level 0 size)
  B_COUNT
};

// [nout][3*3*3] (c, ky, kx) conv weights -> k-major [27][nout]: the direct 3->32
// kernel reads channel pairs of one tap as adjacent scalars (packed FMAs)
static std::vector<double> conv3_kmajor(const std::vector<double>& w) {
  const size_t nout = w.size() / 27;
  std::vector<double> t(w.size());
  for (size_t o = 0; o < nout; ++o)
    for (size_t k = 0; k < 27; ++k) t[k * nout + o] = w[o * 27 + k];
  return t;
}

enum OpKind { OP_GEMM, OP_CONV3, OP_PREP, OP_FAM_CA, OP_FAM_MIX, OP_FAM_SA, OP_ASPP_G, OP_TAIL, OP_PREACT };

struct Op {
  OpKind kind;
  std::string name;
  // GEMM
  int layer = -1;
  int level = 0;  // resolution level of the output pixels: H >> level (ConvT: input level)
  int out = -1, out_cs = 0, out_coff = 0;
  int res1 = -1, res1_cs = 0, res2 = -1, res2_cs = 0;
  int relu = 0, store = kStoreNHWC;
  int pool_slot = -1;   // index into pool buffer (units of B*256 16-byte entries)
  int img_bias = 0;
  size_t head_w = 0; float head_b = 0.f;
  // conv3 / fam
  int in = -1, out1 = -1, out2 = -1;  // conv3: out2 = fused enc1 PreAct output (scale b2/sh2)
  size_t ps = 0, ph = 0;
  size_t w = 0, b = 0;
  int fam = 0;       // which scale (0..2)
  size_t ca_w1 = 0, ca_b1 = 0, ca_w2 = 0, ca_b2 = 0, P = 0, sa_w = 0;
  float sa_b = 0.f;
  int lvl_shift = 0;  // FAM/conv3 resolution: 0 (H), 2 (H/4), 4 (H/16) in floor-halvings
  size_t cst = 0;
};

}  // namespace upr

struct UprModel {
  int dtype = 0;
  int use_preact = 0, use_aspp = 0, flags = 0;
  void* dev_blob = nullptr;
  size_t blob_bytes = 0;
  std::vector<upr::GemmLayer> layers;
  std::vector<upr::Op> ops;
  // profiling (upr_model_profile): per-op event pairs of every profiled forward
  bool prof = false;
  std::vector<std::vector<hipEvent_t>> ev_pending;  // [forward][2*op]
  std::vector<hipEvent_t> ev_free;
  std::vector<double> st_ms, st_flops, st_bytes;
  std::vector<int> st_calls;
  std::vector<double> cur_flops, cur_bytes;  // geometry of the latest forward, per op
  // multi-scale branch ops [side_begin, side_end) (scale pyramid, scale2/3 first
  // convs, the three EnhancedFAM blocks) depend only on the input and on op 0's
  // scale1 output, and the IENet ops [1, side_begin) never read theirs: they run
  // on a side stream forked after op 0 and joined before the tail (-1: no fork)
  int side_begin = -1, side_end = -1;
  struct Side {
    hipStream_t s = nullptr;
    hipEvent_t fork = nullptr, join = nullptr;
    unsigned long long last_use = 0;
    ~Side() {
      if (s) (void)hipStreamSynchronize(s);
      if (join) (void)hipEventDestroy(join);
      if (fork) (void)hipEventDestroy(fork);
      if (s) (void)hipStreamDestroy(s);
    }
  };
  // per (device, caller stream), least recently used evicted beyond kMaxSides
  // (a forward holds its entry's reference until it has enqueued everything)
  static constexpr size_t kMaxSides = 16;
  std::map<std::pair<int, hipStream_t>, std::shared_ptr<Side>> sides;
  unsigned long long side_clock = 0;
  std::mutex sides_mu;
  std::atomic<long long> forks{0};  // forwards that ran the two-stream schedule (upr_model_forks)
};

namespace upr {

// buffer geometry: channels and resolution level (floor-halving count) and elt
struct BufGeom {
  int C;          // channels per pixel
  int shift;      // resolution = dim >> shift  (for pyramid buffers: special)
  int is_f32;     // stored as fp32 regardless of model dtype
  int pyramid;    // 1: x2p (H4), 2: x3p (H16)
};

static BufGeom buf_geom(int id, int use_aspp) {
  switch (id) {
    case B_X2P: return {3, 2, 0, 1};
    case B_X3P: return {3, 4, 0, 2};
    case B_X1: case B_S1IN: return {32, 0, 0, 0};
    case B_S2IN: return {32, 2, 0, 1};
    case B_S3IN: return {32, 4, 0, 2};
    case B_E1T: case B_X2: return {64, 1, 0, 0};
    case B_E2T: case B_X3: return {128, 2, 0, 0};
    case B_E3T: case B_X4: case B_B0T: case B_B0: case B_AP: case B_B1T: case B_X5: return {256, 3, 0, 0};
    case B_ASPP: return {use_aspp ? 1024 : 0, 3, 0, 0};
    case B_U3: case B_V3: case B_D3: return {128, 2, 0, 0};
    case B_U2: case B_V2: case B_D2: return {64, 1, 0, 0};
    case B_U1: case B_V1: case B_D1: return {32, 0, 0, 0};
    case B_H1: return {64, 0, 0, 0};
    case B_Y1: return {32, 0, 0, 0};
    case B_H2: return {64, 2, 0, 1};
    case B_Y2: return {32, 2, 0, 1};
    case B_H3: return {64, 4, 0, 2};
    case B_Y3: return {32, 4, 0, 2};
    case B_MM1: return {2, 0, 1, 0};
    case B_P1: case B_Q1: return {3, 0, 1, 0};
    case B_MM2: return {2, 2, 1, 1};
    case B_P2: case B_Q2: return {3, 2, 1, 1};
    case B_MM3: return {2, 4, 1, 2};
    case B_P3: case B_Q3: return {3, 4, 1, 2};
    case B_ILLU32: return {1, 0, 1, 0};
    case B_PA1: return {32, 0, 0, 0};
    case B_PA2: return {64, 1, 0, 0};
    case B_PA3: return {128, 2, 0, 0};
    case B_PA4: return {256, 3, 0, 0};
    case B_FT: return {32, 0, 0, 0};
    default: return {0, 0, 1, 0};
  }
}

// spatial dims of a buffer for input H x W
static void buf_dims(const BufGeom& g, int H, int W, int& h, int& w) {
  if (g.pyramid == 1) { h = (H / 2) / 2; w = (W / 2) / 2; return; }
  if (g.pyramid == 2) { h = (H / 4) / 4; w = (W / 4) / 4; return; }
  h = H >> g.shift; w = W >> g.shift;
}

// fp16 PreAct blocks materialise o = relu(bn1(x)) once (OP_PREACT) so that
// conv1 and the projecting shortcut read plain segments: >= 64 channels run on
// the wide-tile LDS-DMA kernel (conv_wide.hip), 32 channels on the halo kernel
// without its per-tap prologue (measured: enc1 0.84 + 0.49 ms -> 0.40 + 0.38
// ms against ~0.15 ms for the extra pass).  fp32 keeps the per-tap prologue
// (MFMA-bound there: the prologue is hidden).
static bool preact_materialised(const UprModel* m) { return m->use_preact && m->dtype == kF16; }

// fp32 EnhancedFAM fusion (K = 640, N = 32) as two launches instead of one
// halo-kernel GEMM: y = relu(conv_d2(h4) + (conv(h3) + x-part + bias)), both on
// the fp32 row ring with their filters in registers (the fused K = 640 filter
// does not fit registers, and one ring with both halos and x does not fit
// LDS); the x / maxpool3(x) 1x1 slices ride with the h3 part (second ring).
// Same sum in a different association (fp32 rounding only).
static bool fam32_split(const UprModel* m) { return m->dtype != kF16 && !(m->flags & UPR_MODEL_IENET_ONLY); }

static size_t ws_layout(const UprModel* m, int B, int H, int W, size_t* offs) {
  size_t off = 0;
  const size_t elt = m->dtype == kF16 ? 2 : 4;
  for (int id = 1; id < B_COUNT; ++id) {
    size_t bytes = 0;
    if (id == B_POOL) bytes = (size_t)4 * B * 256 * 4 * kPoolEntryFloats;
    else if (id == B_CA) bytes = (size_t)3 * B * 32 * 4;
    else if (id == B_IB) bytes = (size_t)B * 256 * 4;
    else {
      BufGeom g = buf_geom(id, m->use_aspp);
      int h, w;
      buf_dims(g, H, W, h, w);
      bytes = (size_t)B * h * w * g.C * (g.is_f32 ? 4 : elt);
    }
    if (id >= B_PA1 && id <= B_PA4 && !preact_materialised(m)) bytes = 0;
    if (id == B_FT && !fam32_split(m)) bytes = 0;
    const bool scale_buf = id == B_X2P || id == B_X3P || id == B_S1IN || id == B_S2IN || id == B_S3IN ||
                           (id >= B_H1 && id <= B_Q3) || id == B_FT;
    if ((m->flags & UPR_MODEL_IENET_ONLY) && scale_buf) bytes = 0;
    if ((m->flags & UPR_MODEL_HEAD_ONLY) && !scale_buf && id != B_POOL && id != B_CA) bytes = 0;
    off = align_up(off, 256);
    if (offs) offs[id] = off;
    off += bytes;
  }
  return align_up(off, 256);
}

// ---------------------------------------------------------------------------
// model construction
// ---------------------------------------------------------------------------
struct Builder {
  ParamSet& P;
  Blob& blob;
  UprModel* m;
  int dt;
  bool ok = true;

  const HostTensor* T(const std::string& k) {
    const HostTensor* t = P.get(k);
    if (!t) ok = false;
    return t;
  }
  std::vector<double> V(const std::string& k) {
    const HostTensor* t = T(k);
    return t ? t->v : std::vector<double>();
  }
  int add_layer(int N, std::vector<SegWeights>& segs, const std::vector<double>& bias) {
    m->layers.push_back(pack_gemm(blob, dt, N, segs, bias));
    return (int)m->layers.size() - 1;
  }
  void gemm(const std::string& name, int layer, int level, int out, int out_cs, int relu, int res1 = -1,
            int res1_cs = 0, int res2 = -1, int res2_cs = 0, int store = kStoreNHWC, int out_coff = 0,
            int pool_slot = -1, int img_bias = 0) {
    Op o;
    o.kind = OP_GEMM; o.name = name; o.layer = layer; o.level = level; o.out = out; o.out_cs = out_cs; o.out_coff = out_coff;
    o.relu = relu; o.res1 = res1; o.res1_cs = res1_cs; o.res2 = res2; o.res2_cs = res2_cs; o.store = store;
    o.pool_slot = pool_slot; o.img_bias = img_bias;
    m->ops.push_back(o);
  }

  // ResBlock (models/model.py:100-135) or PreActResBlock (:138-178)
  void block(const std::string& p, int in, int tmp, int out, int cin, int cout, int stride, int in_level,
             int pool_slot = -1) {
    const int lvl = in_level + (stride == 2 ? 1 : 0);
    const bool proj = stride != 1 || cin != cout;
    const HostTensor* w1 = T(p + ".conv1.weight");
    const HostTensor* w2 = T(p + ".conv2.weight");
    if (!ok) return;
    if (!m->use_preact) {
      BNFold bn1, bn2, bns;
      if (!bn_fold(P, p + ".bn1", cout, bn1) || !bn_fold(P, p + ".bn2", cout, bn2)) { ok = false; return; }
      std::vector<SegWeights> s1(1);
      s1[0].spec = seg(in, cin, cin, 0, 3, stride, 1, 1);
      s1[0].w = conv_w(*w1, &bn1.s);
      int l1 = add_layer(cout, s1, bn1.sh);
      gemm(p + ".conv1", l1, lvl, tmp, cout, 1);
      std::vector<SegWeights> s2(1);
      s2[0].spec = seg(tmp, cout, cout, 0, 3, 1, 1, 1);
      s2[0].w = conv_w(*w2, &bn2.s);
      std::vector<double> bias = bn2.sh;
      if (proj) {
        const HostTensor* ws = T(p + ".shortcut.0.weight");
        if (!ws || !bn_fold(P, p + ".shortcut.1", cout, bns)) { ok = false; return; }
        SegWeights sc;
        sc.spec = seg(in, cin, cin, 0, 1, stride, 0, 1);
        sc.w = conv_w(*ws, &bns.s);
        s2.push_back(sc);
        for (int c = 0; c < cout; ++c) bias[c] += bns.sh[c];
      }
      int l2 = add_layer(cout, s2, bias);
      gemm(p + ".conv2", l2, lvl, out, cout, 1, proj ? -1 : in, proj ? 0 : cin, -1, 0, kStoreNHWC, 0, pool_slot);
    } else {
      BNFold bn1, bn2, bns;
      if (!bn_fold(P, p + ".bn1", cin, bn1) || !bn_fold(P, p + ".bn2", cout, bn2)) { ok = false; return; }
      const size_t pre_s = blob.add_f32(bn1.s), pre_h = blob.add_f32(bn1.sh);
      int osrc = in, opre = kPreAffineRelu;
      Op* conv3_producer = nullptr;
      for (auto& o : m->ops)
        if (o.kind == OP_CONV3 && o.out == in) conv3_producer = &o;
      // the GEMM that produced `in` as a whole NHWC tensor (the previous block's conv2, the ASPP fusion)
      Op* gemm_producer = nullptr;
      for (auto& o : m->ops)
        if (o.kind == OP_GEMM && o.out == in && o.store == kStoreNHWC && o.out_coff == 0 && o.out_cs == cin &&
            m->layers[o.layer].N == cin)
          gemm_producer = &o;
      const int pa = in_level == 0 ? B_PA1 : (in_level == 1 ? B_PA2 : (in_level == 2 ? B_PA3 : B_PA4));
      if (preact_materialised(m) && conv3_producer) {
        // enc1: the 3->32 input conv writes relu(bn1(x1)) beside x1 (one pass)
        conv3_producer->out2 = B_PA1; conv3_producer->ps = pre_s; conv3_producer->ph = pre_h;
        osrc = B_PA1; opre = kPreNone;
      } else if (preact_materialised(m) && gemm_producer) {
        // enc2 / enc3 / bottleneck: the producing conv's epilogue writes
        // relu(bn1(x)) beside x (ConvOp::out2) -- no separate read of x
        gemm_producer->out2 = pa; gemm_producer->ps = pre_s; gemm_producer->ph = pre_h;
        osrc = pa; opre = kPreNone;
      } else if (preact_materialised(m)) {
        Op po;
        po.kind = OP_PREACT; po.name = p + ".bn1_relu"; po.in = in; po.level = in_level; po.w = pre_s; po.b = pre_h;
        po.out = pa;
        m->ops.push_back(po);
        osrc = po.out; opre = kPreNone;
      }
      std::vector<SegWeights> s1(1);
      s1[0].spec = seg(osrc, cin, cin, 0, 3, stride, 1, 1, opre);
      s1[0].spec.pre_scale = pre_s; s1[0].spec.pre_shift = pre_h;
      s1[0].w = conv_w(*w1, &bn2.s);
      int l1 = add_layer(cout, s1, bn2.sh);
      gemm(p + ".conv1", l1, lvl, tmp, cout, 1);
      std::vector<SegWeights> s2(1);
      s2[0].spec = seg(tmp, cout, cout, 0, 3, 1, 1, 1);
      s2[0].w = conv_w(*w2, nullptr);
      std::vector<double> bias(cout, 0.0);
      if (proj) {
        const HostTensor* ws = T(p + ".shortcut.0.weight");
        if (!ws || !bn_fold(P, p + ".shortcut.1", cout, bns)) { ok = false; return; }
        SegWeights sc;
        sc.spec = seg(osrc, cin, cin, 0, 1, stride, 0, 1, opre);
        sc.spec.pre_scale = pre_s; sc.spec.pre_shift = pre_h;
        sc.w = conv_w(*ws, &bns.s);
        s2.push_back(sc);
        bias = bns.sh;
      }
      int l2 = add_layer(cout, s2, bias);
      gemm(p + ".conv2", l2, lvl, out, cout, 0, proj ? -1 : in, proj ? 0 : cin, -1, 0, kStoreNHWC, 0, pool_slot);
    }
  }

  // ASPPModule (models/model.py:181-251) on a 256-channel level-3 tensor
  void aspp(const std::string& p, int in, int out) {
    const int C = 256, lvl = 3;
    BNFold bn;
    // 1x1 branch
    {
      const HostTensor* w = T(p + ".conv1x1.0.weight");
      if (!ok || !bn_fold(P, p + ".conv1x1.1", C, bn)) { ok = false; return; }
      std::vector<SegWeights> s(1);
      s[0].spec = seg(in, C, C, 0, 1, 1, 0, 1);
      s[0].w = conv_w(*w, &bn.s);
      gemm(p + ".conv1x1", add_layer(C, s, bn.sh), lvl, B_ASPP, 4 * C, 1, -1, 0, -1, 0, kStoreNHWC, 0);
    }
    const int dil[3] = {6, 12, 18};
    for (int i = 0; i < 3; ++i) {
      const std::string q = p + ".aspp_branches." + std::to_string(i);
      const HostTensor* w = T(q + ".0.weight");
      if (!ok || !bn_fold(P, q + ".1", C, bn)) { ok = false; return; }
      std::vector<SegWeights> s(1);
      s[0].spec = seg(in, C, C, 0, 3, 1, dil[i], dil[i]);
      s[0].w = conv_w(*w, &bn.s);
      gemm(q, add_layer(C, s, bn.sh), lvl, B_ASPP, 4 * C, 1, -1, 0, -1, 0, kStoreNHWC, (i + 1) * C);
    }
    // global branch -> per-image bias (computed by OP_ASPP_G from pool slot 3)
    BNFold bng, bnf;
    const HostTensor* wg = T(p + ".global_pool.1.weight");
    const HostTensor* wf = T(p + ".fusion.0.weight");
    if (!ok || !bn_fold(P, p + ".global_pool.2", C, bng) || !bn_fold(P, p + ".fusion.1", C, bnf)) { ok = false; return; }
    std::vector<double> Wf = conv_w(*wf, &bnf.s);  // [256][1280]
    Op g;
    g.kind = OP_ASPP_G; g.name = p + ".global_pool";
    g.w = blob.add_f32(conv_w(*wg, &bng.s));
    g.b = blob.add_f32(bng.sh);
    g.P = blob.add_f32(cols(Wf, C, 5 * C, 4 * C, C));
    m->ops.push_back(g);
    std::vector<SegWeights> s(1);
    s[0].spec = seg(B_ASPP, 4 * C, 4 * C, 0, 1, 1, 0, 1);
    s[0].w = cols(Wf, C, 5 * C, 0, 4 * C);
    gemm(p + ".fusion", add_layer(C, s, bnf.sh), lvl, out, C, 1, -1, 0, -1, 0, kStoreNHWC, 0, -1, 1);
  }

  // UpBlock (models/model.py:254-274) + skip add (:346-348)
  void upblock(const std::string& p, int in, int u, int v, int out, int cin, int cout, int in_level, int skip) {
    const HostTensor* wt = T(p + ".up.weight");  // [cin][cout][2][2]
    const HostTensor* bt = T(p + ".up.bias");
    const HostTensor* w0 = T(p + ".conv.0.weight");
    const HostTensor* b0 = T(p + ".conv.0.bias");
    const HostTensor* w3 = T(p + ".conv.3.weight");
    const HostTensor* b3 = T(p + ".conv.3.bias");
    BNFold bn1, bn2;
    if (!ok || !bn_fold(P, p + ".conv.1", cout, bn1) || !bn_fold(P, p + ".conv.4", cout, bn2)) { ok = false; return; }
    // ConvT as GEMM: N = 4*cout, n = (dy*2+dx)*cout + co, K = cin
    std::vector<SegWeights> st(1);
    st[0].spec = seg(in, cin, cin, 0, 1, 1, 0, 1);
    st[0].w.assign((size_t)4 * cout * cin, 0.0);
    std::vector<double> bias(4 * cout);
    for (int q = 0; q < 4; ++q)
      for (int co = 0; co < cout; ++co) {
        const int n = q * cout + co;
        bias[n] = bt->v[co];
        for (int ci = 0; ci < cin; ++ci)
          st[0].w[(size_t)n * cin + ci] = wt->v[(((size_t)ci * cout + co) * 2 + (q >> 1)) * 2 + (q & 1)];
      }
    gemm(p + ".up", add_layer(4 * cout, st, bias), in_level, u, cout, 0, -1, 0, -1, 0, kStoreConvT2x2);
    const int lvl = in_level - 1;
    std::vector<SegWeights> s0(1);
    s0[0].spec = seg(u, cout, cout, 0, 3, 1, 1, 1);
    s0[0].w = conv_w(*w0, &bn1.s);
    std::vector<double> bb0(cout);
    for (int c = 0; c < cout; ++c) bb0[c] = b0->v[c] * bn1.s[c] + bn1.sh[c];
    gemm(p + ".conv.0", add_layer(cout, s0, bb0), lvl, v, cout, 1);
    std::vector<SegWeights> s3(1);
    s3[0].spec = seg(v, cout, cout, 0, 3, 1, 1, 1);
    s3[0].w = conv_w(*w3, &bn2.s);
    std::vector<double> bb3(cout);
    for (int c = 0; c < cout; ++c) bb3[c] = b3->v[c] * bn2.s[c] + bn2.sh[c];
    gemm(p + ".conv.3", add_layer(cout, s3, bb3), lvl, out, cout, 1, -1, 0, skip, cout);
  }

  // EnhancedFAM (models/model.py:11-97) + its slice of the head projection
  void fam(const std::string& p, int k, int in, int hbuf, int ybuf, int mm, int pbuf, int qbuf, int lshift,
           const std::vector<double>& Whead /* [3][96] = Wo * Wfus */) {
    const int C = 32;
    const HostTensor* w1 = T(p + ".branch1.weight");
    const HostTensor* bb1 = T(p + ".branch1.bias");
    const HostTensor* w2 = T(p + ".branch2_conv.weight");
    const HostTensor* bb2 = T(p + ".branch2_conv.bias");
    const HostTensor* w3a = T(p + ".branch3_conv1.weight");
    const HostTensor* b3a = T(p + ".branch3_conv1.bias");
    const HostTensor* w3b = T(p + ".branch3_conv2.weight");
    const HostTensor* b3b = T(p + ".branch3_conv2.bias");
    const HostTensor* w4a = T(p + ".branch4_conv1.weight");
    const HostTensor* b4a = T(p + ".branch4_conv1.bias");
    const HostTensor* w4b = T(p + ".branch4_conv2.weight");
    const HostTensor* b4b = T(p + ".branch4_conv2.bias");
    const HostTensor* wf = T(p + ".fusion.weight");  // [32][128]
    const HostTensor* bf = T(p + ".fusion.bias");
    const HostTensor* ca1w = T(p + ".channel_attention.1.weight");
    const HostTensor* ca1b = T(p + ".channel_attention.1.bias");
    const HostTensor* ca3w = T(p + ".channel_attention.3.weight");
    const HostTensor* ca3b = T(p + ".channel_attention.3.bias");
    const HostTensor* saw = T(p + ".spatial_attention.0.weight");
    const HostTensor* sab = T(p + ".spatial_attention.0.bias");
    if (!ok) return;
    // (1) h = relu([branch3_conv1; branch4_conv1](x))  -> 64 channels
    std::vector<SegWeights> sh(1);
    sh[0].spec = seg(in, C, C, 0, 3, 1, 1, 1);
    sh[0].w = w3a->v;
    sh[0].w.insert(sh[0].w.end(), w4a->v.begin(), w4a->v.end());
    std::vector<double> hb = b3a->v;
    hb.insert(hb.end(), b4a->v.begin(), b4a->v.end());
    gemm(p + ".branch34_conv1", add_layer(2 * C, sh, hb), lshift, hbuf, 2 * C, 1);
    // (2) y = relu(fusion(cat[b1,b2,b3,b4])) as one GEMM over the virtual concat
    const std::vector<double>& F = wf->v;
    std::vector<double> F1 = cols(F, C, 4 * C, 0, C), F2 = cols(F, C, 4 * C, C, C);
    std::vector<double> F3 = cols(F, C, 4 * C, 2 * C, C), F4 = cols(F, C, 4 * C, 3 * C, C);
    std::vector<SegWeights> sf(4);
    sf[0].spec = seg(hbuf, C, 2 * C, 0, 3, 1, 1, 1);
    sf[0].w = compose(F3, C, C, w3b->v, C, 9);
    sf[1].spec = seg(hbuf, C, 2 * C, C, 3, 1, 2, 2);
    sf[1].w = compose(F4, C, C, w4b->v, C, 9);
    sf[2].spec = seg(in, C, C, 0, 1, 1, 0, 1);
    sf[2].w = compose(F1, C, C, w1->v, C, 1);
    sf[3].spec = seg(in, C, C, 0, 1, 1, 0, 1, kPreMaxPool3);
    sf[3].w = compose(F2, C, C, w2->v, C, 1);
    std::vector<double> fb = bf->v;
    for (int o = 0; o < C; ++o)
      for (int mm_ = 0; mm_ < C; ++mm_)
        fb[o] += F1[o * C + mm_] * bb1->v[mm_] + F2[o * C + mm_] * bb2->v[mm_] + F3[o * C + mm_] * b3b->v[mm_] +
                 F4[o * C + mm_] * b4b->v[mm_];
    if (fam32_split(m)) {
      std::vector<SegWeights> s3x{sf[0], sf[2], sf[3]}, s4(1, sf[1]);
      const std::vector<double> nob;
      gemm(p + ".fusion.h3x", add_layer(C, s3x, fb), lshift, B_FT, C, 0);
      gemm(p + ".fusion.h4", add_layer(C, s4, nob), lshift, ybuf, C, 1, B_FT, C, -1, 0, kStoreNHWC, 0, k);
    } else {
      gemm(p + ".fusion", add_layer(C, sf, fb), lshift, ybuf, C, 1, -1, 0, -1, 0, kStoreNHWC, 0, k);
    }
    // (3) channel attention, (4) mix + projection, (5) spatial attention
    Op oc;
    oc.kind = OP_FAM_CA; oc.name = p + ".channel_attention"; oc.fam = k; oc.lvl_shift = lshift;
    oc.ca_w1 = blob.add_f32(ca1w->v); oc.ca_b1 = blob.add_f32(ca1b->v);
    oc.ca_w2 = blob.add_f32(ca3w->v); oc.ca_b2 = blob.add_f32(ca3b->v);
    m->ops.push_back(oc);
    Op om;
    om.kind = OP_FAM_MIX; om.name = p + ".mix_project"; om.fam = k; om.lvl_shift = lshift; om.in = ybuf; om.out = mm; om.out1 = pbuf;
    om.P = blob.add_f32(cols(Whead, 3, 96, 32 * k, 32));
    m->ops.push_back(om);
    Op os;
    os.kind = OP_FAM_SA; os.name = p + ".spatial_attention"; os.fam = k; os.lvl_shift = lshift; os.in = mm; os.out1 = pbuf; os.out = qbuf;
    os.sa_w = blob.add_f32(saw->v); os.sa_b = (float)sab->v[0];
    m->ops.push_back(os);
  }
};

static int build_model(UprModel* m, ParamSet& P) {
  Blob blob;
  Builder bd{P, blob, m, m->dtype};
  const int pre = m->use_preact;
  const std::string ie = "ie_net";
  const bool head_only = (m->flags & UPR_MODEL_HEAD_ONLY) != 0;
  if (head_only) {
    // multi_scale_enhance alone (models/model.py:415-443): scale1's first conv
    // on its own, no IENet ops; the tail reads the caller's reflectance
    const HostTensor* ws = bd.T("scale1.0.weight");
    const HostTensor* bs = bd.T("scale1.0.bias");
    if (!bd.ok) return kErrMissingParam;
    Op o;
    o.kind = OP_CONV3; o.name = "scale1.0"; o.in = BX; o.out = B_S1IN; o.lvl_shift = 0;
    o.w = blob.add_f32(conv3_kmajor(ws->v)); o.b = blob.add_f32(bs->v);
    m->ops.push_back(o);
  }
  // input layer (+ scale1's first conv, same input, one launch)
  if (!head_only) {
    const HostTensor* wi = bd.T(ie + ".input_layer.weight");
    const HostTensor* bi = bd.T(ie + ".input_layer.bias");
    if (!bd.ok) return kErrMissingParam;
    std::vector<double> w = wi->v, b = bi->v;
    Op o;
    o.kind = OP_CONV3; o.name = "ie_net.input_layer+scale1.0"; o.in = BX; o.out = B_X1; o.lvl_shift = 0;
    if (!(m->flags & UPR_MODEL_IENET_ONLY)) {
      const HostTensor* ws = bd.T("scale1.0.weight");
      const HostTensor* bs = bd.T("scale1.0.bias");
      if (!bd.ok) return kErrMissingParam;
      w.insert(w.end(), ws->v.begin(), ws->v.end());
      b.insert(b.end(), bs->v.begin(), bs->v.end());
      o.out1 = B_S1IN;
    }
    o.w = blob.add_f32(conv3_kmajor(w)); o.b = blob.add_f32(b);
    m->ops.push_back(o);
  }
  (void)pre;
  if (!head_only) {
  bd.block(ie + ".enc1", B_X1, B_E1T, B_X2, 32, 64, 2, 0);
  bd.block(ie + ".enc2", B_X2, B_E2T, B_X3, 64, 128, 2, 1);
  bd.block(ie + ".enc3", B_X3, B_E3T, B_X4, 128, 256, 2, 2);
  if (m->use_aspp) {
    bd.block(ie + ".bottleneck.0", B_X4, B_B0T, B_B0, 256, 256, 1, 3, /*pool_slot=*/3);
    bd.aspp(ie + ".bottleneck.1", B_B0, B_AP);
    bd.block(ie + ".bottleneck.2", B_AP, B_B1T, B_X5, 256, 256, 1, 3);
  } else {
    bd.block(ie + ".bottleneck.0", B_X4, B_B0T, B_B0, 256, 256, 1, 3);
    bd.block(ie + ".bottleneck.1", B_B0, B_B1T, B_X5, 256, 256, 1, 3);
  }
  if (!bd.ok) return P.missing.empty() ? kErrShape : kErrMissingParam;
  bd.upblock(ie + ".dec3", B_X5, B_U3, B_V3, B_D3, 256, 128, 3, B_X3);
  bd.upblock(ie + ".dec2", B_D3, B_U2, B_V2, B_D2, 128, 64, 2, B_X2);
  bd.upblock(ie + ".dec1", B_D2, B_U1, B_V1, B_D1, 64, 32, 1, B_X1);
  // residual head + illumination (models/model.py:324-328, :351-358)
  {
    const HostTensor* w0 = bd.T(ie + ".residual_head.0.weight");
    const HostTensor* b0 = bd.T(ie + ".residual_head.0.bias");
    const HostTensor* w2 = bd.T(ie + ".residual_head.2.weight");
    const HostTensor* b2 = bd.T(ie + ".residual_head.2.bias");
    if (!bd.ok) return kErrMissingParam;
    std::vector<SegWeights> s(1);
    s[0].spec = seg(B_D1, 32, 32, 0, 3, 1, 1, 1);
    s[0].w = w0->v;
    int l = bd.add_layer(32, s, b0->v);
    Op o;
    o.kind = OP_GEMM; o.name = ie + ".residual_head"; o.layer = l; o.level = 0; o.store = kStoreHeadIllu;
    o.head_w = blob.add_f32(w2->v); o.head_b = (float)b2->v[0];
    m->ops.push_back(o);
  }
  }  // !head_only
  if (!(m->flags & UPR_MODEL_IENET_ONLY)) {
    const HostTensor* wfu = bd.T("fusion.weight");   // [32][96]
    const HostTensor* bfu = bd.T("fusion.bias");
    const HostTensor* wo = bd.T("output_layer.weight");  // [3][32]
    const HostTensor* bo = bd.T("output_layer.bias");
    if (!bd.ok) return kErrMissingParam;
    std::vector<double> Whead = compose(wo->v, 3, 32, wfu->v, 96, 1);  // [3][96]
    std::vector<double> cst(3);
    for (int o = 0; o < 3; ++o) {
      double s = bo->v[o];
      for (int c = 0; c < 32; ++c) s += wo->v[o * 32 + c] * bfu->v[c];
      cst[o] = s;
    }
    // pyramid inputs of scale2/scale3 and their first convs
    Op op;
    op.kind = OP_PREP; op.name = "scale_pyramid";
    if (!head_only) m->side_begin = (int)m->ops.size();
    m->ops.push_back(op);
    for (int k = 1; k <= 2; ++k) {
      const std::string p = "scale" + std::to_string(k + 1) + ".1";
      const HostTensor* w = bd.T(p + ".weight");
      const HostTensor* b = bd.T(p + ".bias");
      if (!bd.ok) return kErrMissingParam;
      Op o;
      o.kind = OP_CONV3; o.name = p; o.in = k == 1 ? B_X2P : B_X3P; o.out = k == 1 ? B_S2IN : B_S3IN;
      o.lvl_shift = k == 1 ? 2 : 4;
      o.w = blob.add_f32(conv3_kmajor(w->v)); o.b = blob.add_f32(b->v);
      m->ops.push_back(o);
    }
    bd.fam("scale1.2", 0, B_S1IN, B_H1, B_Y1, B_MM1, B_P1, B_Q1, 0, Whead);
    bd.fam("scale2.3", 1, B_S2IN, B_H2, B_Y2, B_MM2, B_P2, B_Q2, 2, Whead);
    bd.fam("scale3.3", 2, B_S3IN, B_H3, B_Y3, B_MM3, B_P3, B_Q3, 4, Whead);
    if (!bd.ok) return kErrMissingParam;
    Op t;
    t.kind = OP_TAIL; t.name = "retinex_tail";
    t.cst = blob.add_f32(cst);
    if (m->side_begin >= 0) m->side_end = (int)m->ops.size();
    m->ops.push_back(t);
  }
  if (!bd.ok) return kErrMissingParam;
  m->blob_bytes = blob.bytes.size();
  UPR_CHECK_HIP(hipMalloc(&m->dev_blob, std::max<size_t>(m->blob_bytes, 256)));
  UPR_CHECK_HIP(hipMemcpy(m->dev_blob, blob.bytes.data(), m->blob_bytes, hipMemcpyHostToDevice));
  return kOk;
}

// ---------------------------------------------------------------------------
// forward
// ---------------------------------------------------------------------------
// The multi-scale side stream of (current device, caller stream), created on
// first use: non-blocking, joined through events every forward.  nullptr keeps
// the whole forward on the caller's stream: UPR_MS_STREAMS=0 (A/B timing and
// the rocprofv3 kernel summaries).
// The side stream forks before the bottleneck (run_forward; round 3 measured
// no gain from a later fork, round 5's kernels 1.5-1.8%: profiles/r5_ms_fork_ab.txt);
// a capped CU budget for the side stream's ring convs (r3_side_cus_ab.txt), a
// low-priority side stream (r3_ms_streams_ab.txt) and CU-partitioned streams
// (r5_cu_mask_streams_ab.txt) measured no better.

using Side = UprModel::Side;
static std::shared_ptr<Side> side_of(UprModel* m, hipStream_t st) {
  static const int en = [] {
    const char* e = getenv("UPR_MS_STREAMS");
    return e ? (atoi(e) != 0 ? 1 : 0) : -1;
  }();
  // default: every model forks (fp32 too since round 5: +1.1% with the fork
  // before the bottleneck, profiles/r5_ms_fork_ab.txt).  Per-kernel durations
  // for the roofline come from the serialised profiled step, and the rocprofv3
  // kernel summaries are taken with UPR_MS_STREAMS=0 (tools/gpu/r5_final.sh)
  if (en == 0) return nullptr;
  // hipStreamPerThread names a different real stream per calling thread: a
  // Side keyed by it would be shared by threads whose fork / join events then
  // interleave, so those forwards stay on the one stream (upr.h).  The null
  // stream is ONE real stream here (libupr is built without per-thread default
  // streams), and torch's default stream passes it: it forks like any other.
  if (st == hipStreamPerThread) return nullptr;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lk(m->sides_mu);
  auto it = m->sides.find({dev, st});
  if (it != m->sides.end()) {
    it->second->last_use = ++m->side_clock;
    return it->second;
  }
  auto sd = std::make_shared<Side>();
  if (hipStreamCreateWithFlags(&sd->s, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&sd->fork, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&sd->join, hipEventDisableTiming) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;  // ~Side releases what was created
  }
  if (m->sides.size() >= UprModel::kMaxSides) {
    auto old = m->sides.begin();
    for (auto i = m->sides.begin(); i != m->sides.end(); ++i)
      if (i->second->last_use < old->second->last_use) old = i;
    m->sides.erase(old);
  }
  sd->last_use = ++m->side_clock;
  m->sides[{dev, st}] = sd;
  return sd;
}

static int run_forward(UprModel* m, const void* x, int B, int H, int W, void* enh, void* refl, void* illu,
                       uint8_t* ws, hipStream_t st) {
  size_t offs[B_COUNT] = {0};
  ws_layout(m, B, H, W, offs);
  const uint8_t* blob = (const uint8_t*)m->dev_blob;
  auto fptr = [&](size_t off) { return (const float*)(blob + off); };
  auto buf = [&](int id) -> void* {
    if (id == BX) return const_cast<void*>(x);
    return ws + offs[id];
  };
  const int dt = m->dtype;
  float* pool = (float*)buf(B_POOL);
  float* ca = (float*)buf(B_CA);
  float* ib = (float*)buf(B_IB);
  UPR_CHECK_HIP(hipMemsetAsync(pool, 0, (size_t)4 * B * 256 * 4 * kPoolEntryFloats, st));
  const int H4 = (H / 2) / 2, W4 = (W / 2) / 2, H16 = (H / 4) / 4, W16 = (W / 4) / 4;
  auto lvl_dims = [&](int lshift, int& h, int& w) {
    if (lshift == 2) { h = H4; w = W4; }
    else if (lshift == 4) { h = H16; w = W16; }
    else { h = H >> lshift; w = W >> lshift; }
  };
  float* illu32 = dt == kF16 ? (float*)buf(B_ILLU32) : (float*)illu;
  const size_t nops = m->ops.size();
  std::vector<hipEvent_t> evs;
  if (m->prof) {
    evs.resize(2 * nops);
    for (auto& e : evs) {
      if (!m->ev_free.empty()) { e = m->ev_free.back(); m->ev_free.pop_back(); }
      else UPR_CHECK_HIP(hipEventCreate(&e));
    }
    m->cur_flops.assign(nops, 0.0);
    m->cur_bytes.assign(nops, 0.0);
  }
  const double elt = dt == kF16 ? 2.0 : 4.0;
  // launch op oi on stream st (the caller's stream or the multi-scale side stream)
  auto run_op = [&](size_t oi, hipStream_t st) -> int {
    const Op& o = m->ops[oi];
    int rc = kOk;
    if (m->prof) UPR_CHECK_HIP(hipEventRecord(evs[2 * oi], st));
    switch (o.kind) {
      case OP_PREP:
        rc = launch_prep(x, buf(B_X2P), buf(B_X3P), B, H, W, dt, st);
        break;
      case OP_CONV3: {
        int h, w;
        lvl_dims(o.lvl_shift, h, w);
        rc = launch_conv3(buf(o.in), fptr(o.w), fptr(o.b), buf(o.out), o.out1 >= 0 ? buf(o.out1) : nullptr, B, h, w,
                          dt, st, o.out2 >= 0 ? buf(o.out2) : nullptr, o.out2 >= 0 ? fptr(o.ps) : nullptr,
                          o.out2 >= 0 ? fptr(o.ph) : nullptr);
        break;
      }
      case OP_GEMM: {
        const GemmLayer& L = m->layers[o.layer];
        ConvOp c;
        memset(&c, 0, sizeof(c));
        c.nseg = (int)L.segs.size();
        int ho, wo;
        lvl_dims(o.level, ho, wo);
        for (int i = 0; i < c.nseg; ++i) {
          const SegSpec& s = L.segs[i];
          ConvSeg& cs = c.seg[i];
          cs.src = buf(s.src);
          cs.C = s.C; cs.cs = s.cs; cs.coff = s.coff;
          // source resolution: stride-2 segments read the level above
          int hi = ho * s.stride, wi = wo * s.stride;
          cs.Hin = hi; cs.Win = wi;
          cs.kh = s.kh; cs.kw = s.kw; cs.stride = s.stride; cs.pad = s.pad; cs.dil = s.dil;
          cs.pre = s.pre;
          cs.pre_scale = s.pre == kPreAffineRelu ? fptr(s.pre_scale) : nullptr;
          cs.pre_shift = s.pre == kPreAffineRelu ? fptr(s.pre_shift) : nullptr;
          cs.kbase = s.kbase;
        }
        c.B = B; c.Ho = ho; c.Wo = wo; c.N = L.N; c.Kpad = L.Kpad;
        c.W = blob + L.w;
        c.scale = nullptr;
        c.bias = L.bias != SIZE_MAX ? fptr(L.bias) : nullptr;
        c.img_bias = o.img_bias ? ib : nullptr;
        c.res1 = o.res1 >= 0 ? buf(o.res1) : nullptr; c.res1_cs = o.res1_cs;
        c.relu = o.relu;
        c.res2 = o.res2 >= 0 ? buf(o.res2) : nullptr; c.res2_cs = o.res2_cs;
        c.store = o.store;
        if (o.store == kStoreHeadIllu) {
          c.head_w = fptr(o.head_w); c.head_b = o.head_b;
          c.x_nchw = (const float*)x; c.x_f16 = dt == kF16;
          c.illu = illu32; c.illu_f16 = 0;
          c.out = nullptr;
        } else {
          c.out = buf(o.out); c.out_cs = o.out_cs; c.out_coff = o.out_coff;
        }
        c.pool = o.pool_slot >= 0 ? pool + (size_t)o.pool_slot * B * 256 * kPoolEntryFloats : nullptr;
        if (o.out2 >= 0) {
          c.out2 = buf(o.out2); c.out2_cs = L.N;
          c.pre2_scale = fptr(o.ps); c.pre2_shift = fptr(o.ph);
        }
        rc = launch_conv(c, dt, st);
        if (m->prof) {
          // GEMM work of this launch: 2*M*N*K; algorithmic bytes: every source read once,
          // weights once, residuals once, output written once
          const double Mpx = (double)B * ho * wo;
          double K = 0, bytes = (double)L.N * L.Kpad * elt;
          for (int i = 0; i < c.nseg; ++i) {
            K += (double)c.seg[i].kh * c.seg[i].kw * c.seg[i].C;
            bytes += (double)B * c.seg[i].Hin * c.seg[i].Win * c.seg[i].C * elt;
          }
          const double nout = o.store == kStoreHeadIllu ? 1.0 : (double)L.N;
          bytes += Mpx * nout * (o.store == kStoreHeadIllu ? 4.0 : elt);
          if (c.res1) bytes += Mpx * L.N * elt;
          if (c.res2) bytes += Mpx * L.N * elt;
          if (c.out2) bytes += Mpx * L.N * elt;
          m->cur_flops[oi] = 2.0 * Mpx * L.N * K;
          m->cur_bytes[oi] = bytes;
        }
        break;
      }
      case OP_PREACT: {
        int h, w;
        lvl_dims(o.level, h, w);
        const int C = buf_geom(o.out, m->use_aspp).C;
        rc = launch_preact_f16(buf(o.in), fptr(o.w), fptr(o.b), buf(o.out), (size_t)B * h * w, C, st);
        if (m->prof) m->cur_bytes[oi] = 2.0 * B * h * w * C * elt;
        break;
      }
      case OP_ASPP_G: {
        const int h = H >> 3, w = W >> 3;
        hipLaunchKernelGGL(aspp_global_kernel, dim3(B), dim3(256), 2 * 256 * sizeof(float), st,
                           pool + (size_t)3 * B * 256 * kPoolEntryFloats, fptr(o.w), fptr(o.b), fptr(o.P), ib, 256,
                           1.f / (float)(h * w));
        rc = (int)hipGetLastError();
        break;
      }
      case OP_FAM_CA: {
        int h, w;
        lvl_dims(o.lvl_shift, h, w);
        rc = launch_fam_ca(pool + (size_t)o.fam * B * 256 * kPoolEntryFloats, fptr(o.ca_w1), fptr(o.ca_b1), fptr(o.ca_w2),
                           fptr(o.ca_b2), ca + (size_t)o.fam * B * 32, B, h * w, st);
        break;
      }
      case OP_FAM_MIX: {
        int h, w;
        lvl_dims(o.lvl_shift, h, w);
        rc = launch_fam_mix(buf(o.in), ca + (size_t)o.fam * B * 32, fptr(o.P), (float*)buf(o.out),
                            (float*)buf(o.out1), B, h * w, dt, st);
        break;
      }
      case OP_FAM_SA: {
        int h, w;
        lvl_dims(o.lvl_shift, h, w);
        rc = launch_fam_sa((const float*)buf(o.in), (const float*)buf(o.out1), fptr(o.sa_w), o.sa_b,
                           (float*)buf(o.out), B, h, w, st);
        break;
      }
      case OP_TAIL:
        rc = launch_tail(x, illu32, nullptr, (const float*)buf(B_Q1), (const float*)buf(B_Q2),
                         (const float*)buf(B_Q3), fptr(o.cst), enh, refl, B, H, W, H4, W4, H16, W16, dt, st,
                         (m->flags & UPR_MODEL_HEAD_ONLY) ? 1 : 0);
        break;
    }
    if (m->prof) UPR_CHECK_HIP(hipEventRecord(evs[2 * oi + 1], st));
    return rc;
  };
  // profiled forwards stay on one stream (per-op events time one kernel each)
  const std::shared_ptr<Side> sd =
      (!m->prof && m->side_begin > 0 && m->side_end > m->side_begin) ? side_of(m, st) : nullptr;
  if (!sd) {
    for (size_t oi = 0; oi < nops; ++oi) {
      const int rc = run_op(oi, st);
      if (rc != kOk) return rc;
    }
  } else {
    // IENet ops [0, fork) -> fork -> side: the multi-scale ops, main: the rest
    // of the IENet -> join -> tail
    // fork before the bottleneck: the side ops (HBM-bound FAM convs) then run
    // beside the MFMA-bound bottleneck / ASPP convs instead of competing with the
    // HBM-bound encoder for bandwidth (fp16 preact+ASPP bs 32: 5.47 ms forking
    // after op 0, 5.37-5.41 before the bottleneck, 5.40-5.43 before enc3, 5.45
    // before enc2, 5.50 before dec3; profiles/r5_ms_fork_ab.txt).  The side ops
    // need only op 0's outputs, so any fork point is exact.  UPR_MS_FORK=<op
    // name prefix> overrides ("-": right after op 0)
    static const std::string fork_at = [] {
      const char* e = getenv("UPR_MS_FORK");
      return std::string(e ? e : "ie_net.bottleneck");
    }();
    int fk = 1;
    if (fork_at != "-")
      for (int oi = 1; oi < m->side_begin; ++oi)
        if (m->ops[oi].name.compare(0, fork_at.size(), fork_at) == 0) { fk = oi; break; }
    int rc = kOk;
    m->forks.fetch_add(1, std::memory_order_relaxed);
    for (int oi = 0; oi < fk; ++oi)
      if ((rc = run_op(oi, st)) != kOk) return rc;
    UPR_CHECK_HIP(hipEventRecord(sd->fork, st));
    UPR_CHECK_HIP(hipStreamWaitEvent(sd->s, sd->fork, 0));
    for (int oi = m->side_begin; oi < m->side_end; ++oi)
      if ((rc = run_op(oi, sd->s)) != kOk) break;
    // joined on every path once forked: after an error return too, completion
    // of the caller's stream still covers whatever the side stream enqueued
    UPR_CHECK_HIP(hipEventRecord(sd->join, sd->s));
    if (rc == kOk)
      for (int oi = fk; oi < m->side_begin; ++oi)
        if ((rc = run_op(oi, st)) != kOk) break;
    UPR_CHECK_HIP(hipStreamWaitEvent(st, sd->join, 0));
    if (rc != kOk) return rc;
    for (size_t oi = m->side_end; oi < nops; ++oi)
      if ((rc = run_op(oi, st)) != kOk) return rc;
  }
  if (m->prof) {
    m->ev_pending.push_back(evs);
    if (m->st_ms.size() != nops) {
      m->st_ms.assign(nops, 0.0); m->st_flops.assign(nops, 0.0); m->st_bytes.assign(nops, 0.0);
      m->st_calls.assign(nops, 0);
    }
    for (size_t i = 0; i < nops; ++i) { m->st_flops[i] += m->cur_flops[i]; m->st_bytes[i] += m->cur_bytes[i]; }
  }
  if (dt == kF16 && !(m->flags & UPR_MODEL_HEAD_ONLY)) {
    // illumination in the model dtype
    extern int launch_cast_f32_to_f16(const float*, void*, size_t, hipStream_t);
    int rc = launch_cast_f32_to_f16(illu32, illu, (size_t)B * H * W, st);
    if (rc != kOk) return rc;
  }
  return kOk;
}

__global__ void cast_f32_f16_kernel(const float* __restrict__ a, half_t* __restrict__ b, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) b[i] = (half_t)a[i];
}
int launch_cast_f32_to_f16(const float* a, void* b, size_t n, hipStream_t st) {
  hipLaunchKernelGGL(cast_f32_f16_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, a, (half_t*)b, n);
  return (int)hipGetLastError();
}

}  // namespace upr

// ===========================================================================
// C ABI
// ===========================================================================
using namespace upr;

extern "C" {

int upr_model_create(const UprTensorDesc* params, int n_params, int use_preact, int use_aspp, int dtype, int flags,
                     UprModel** out) {
  if (!out || (n_params > 0 && !params) || (dtype != UPR_F32 && dtype != UPR_F16)) return UPR_ERR_ARG;
  *out = nullptr;
  // one of the two partial graphs at most, and no unknown bits (IENET_ONLY |
  // HEAD_ONLY would build neither the IENet nor the head and write nothing)
  constexpr int kKnownFlags = UPR_MODEL_IENET_ONLY | UPR_MODEL_HEAD_ONLY;
  if ((flags & ~kKnownFlags) || (flags & kKnownFlags) == kKnownFlags) return UPR_ERR_ARG;
  ParamSet P;
  for (int i = 0; i < n_params; ++i) {
    const UprTensorDesc& d = params[i];
    if (!d.name || d.ndim < 0 || d.ndim > 4) return UPR_ERR_ARG;
    HostTensor t;
    int64_t n = 1;
    for (int k = 0; k < d.ndim; ++k) { t.shape.push_back(d.shape[k]); n *= d.shape[k]; }
    if (n > 0 && !d.data) return UPR_ERR_ARG;
    t.v.assign(d.data, d.data + n);
    P.t[d.name] = std::move(t);
  }
  std::unique_ptr<UprModel> m(new UprModel());
  m->dtype = dtype; m->use_preact = use_preact ? 1 : 0; m->use_aspp = use_aspp ? 1 : 0; m->flags = flags;
  int rc = build_model(m.get(), P);
  if (rc != kOk) {
    if (m->dev_blob) (void)hipFree(m->dev_blob);
    return rc;
  }
  *out = m.release();
  return UPR_OK;
}

size_t upr_model_workspace(const UprModel* model, int B, int H, int W) {
  if (!model || B <= 0 || H <= 0 || W <= 0) return 0;
  return ws_layout(model, B, H, W, nullptr);
}

int upr_model_forward(UprModel* model, const void* x, int B, int H, int W, void* enh, void* refl, void* illu,
                      void* workspace, size_t workspace_bytes, void* stream) {
  const bool head_only = (model && (model->flags & UPR_MODEL_HEAD_ONLY));
  if (!model || !x || (!illu && !head_only) || B <= 0) return UPR_ERR_ARG;
  if (!(model->flags & UPR_MODEL_IENET_ONLY) && (!enh || !refl)) return UPR_ERR_ARG;
  if (H % 8 || W % 8 || H < 16 || W < 16) return UPR_ERR_SHAPE;
  if ((long long)B * H * W > (1LL << 31) / 32) return UPR_ERR_SHAPE;  // 32-bit pixel indexing in kernels
  const size_t need = ws_layout(model, B, H, W, nullptr);
  if (!workspace || workspace_bytes < need) return UPR_ERR_WORKSPACE;
  return run_forward(model, x, B, H, W, enh, refl, illu, (uint8_t*)workspace, (hipStream_t)stream);
}

int upr_model_profile(UprModel* model, int enable) {
  if (!model) return UPR_ERR_ARG;
  for (auto& v : model->ev_pending)
    for (auto e : v) model->ev_free.push_back(e);
  model->ev_pending.clear();
  model->st_ms.clear(); model->st_flops.clear(); model->st_bytes.clear(); model->st_calls.clear();
  model->prof = enable != 0;
  return UPR_OK;
}

int upr_model_profile_read(UprModel* model, UprOpStat* out, int max_ops, int* n_ops) {
  if (!model || !n_ops) return UPR_ERR_ARG;
  const size_t nops = model->ops.size();
  for (auto& v : model->ev_pending) {
    UPR_CHECK_HIP(hipEventSynchronize(v.back()));
    for (size_t i = 0; i < nops && 2 * i + 1 < v.size(); ++i) {
      float ms = 0.f;
      UPR_CHECK_HIP(hipEventElapsedTime(&ms, v[2 * i], v[2 * i + 1]));
      model->st_ms[i] += ms;
      model->st_calls[i] += 1;
    }
    for (auto e : v) model->ev_free.push_back(e);
  }
  model->ev_pending.clear();
  *n_ops = (int)nops;
  if (out) {
    for (size_t i = 0; i < nops && (int)i < max_ops; ++i) {
      UprOpStat& s = out[i];
      memset(&s, 0, sizeof(s));
      strncpy(s.name, model->ops[i].name.c_str(), sizeof(s.name) - 1);
      s.kind = model->ops[i].kind == OP_GEMM ? UPR_OP_CONV_IGEMM : UPR_OP_OTHER;
      if (i < model->st_ms.size()) {
        s.calls = model->st_calls[i];
        s.ms = model->st_ms[i];
        s.flops = model->st_flops[i];
        s.bytes = model->st_bytes[i];
      }
    }
  }
  return UPR_OK;
}

long long upr_model_forks(const UprModel* model) { return model ? model->forks.load() : -1; }

void upr_model_destroy(UprModel* model) {
  if (!model) return;
  upr_model_profile(model, 0);
  for (auto e : model->ev_free) (void)hipEventDestroy(e);
  model->sides.clear();  // ~Side: synchronise, destroy
  if (model->dev_blob) (void)hipFree(model->dev_blob);
  delete model;
}

const char* upr_status_string(int status) {
  switch (status) {
    case UPR_OK: return "ok";
    case UPR_ERR_ARG: return "invalid argument";
    case UPR_ERR_SHAPE: return "unsupported or inconsistent shape";
    case UPR_ERR_MISSING_PARAM: return "state_dict is missing a parameter the model needs";
    case UPR_ERR_WORKSPACE: return "workspace missing or too small";
    case UPR_ERR_UNSUPPORTED: return "unsupported configuration";
    default: return status > 0 ? hipGetErrorString((hipError_t)status) : "unknown error";
  }
}

int upr_conv2d_nhwc(const void* x, int B, int H, int W, int Cin, const void* w, const float* bias, int Cout, int kh,
                    int kw, int stride, int pad, int dil, const void* residual, int relu, void* y, int dtype,
                    void* stream) {
  if (!x || !w || !y || B <= 0 || H <= 0 || W <= 0 || Cin % 32 || Cout % 32 || Cin <= 0 || Cout <= 0) return UPR_ERR_ARG;
  if (kh <= 0 || kw <= 0 || stride <= 0 || dil <= 0 || pad < 0) return UPR_ERR_ARG;
  if (dtype != UPR_F32 && dtype != UPR_F16) return UPR_ERR_ARG;
  const int Ho = (H + 2 * pad - dil * (kh - 1) - 1) / stride + 1;
  const int Wo = (W + 2 * pad - dil * (kw - 1) - 1) / stride + 1;
  if (Ho <= 0 || Wo <= 0) return UPR_ERR_SHAPE;
  ConvOp c;
  memset(&c, 0, sizeof(c));
  c.nseg = 1;
  ConvSeg& s = c.seg[0];
  s.src = x; s.C = Cin; s.cs = Cin; s.coff = 0; s.Hin = H; s.Win = W;
  s.kh = kh; s.kw = kw; s.stride = stride; s.pad = pad; s.dil = dil; s.pre = kPreNone; s.kbase = 0;
  c.B = B; c.Ho = Ho; c.Wo = Wo; c.N = Cout; c.Kpad = kh * kw * Cin;
  c.W = w; c.bias = bias; c.relu = relu;
  // without ReLU, "added before" and "added after" coincide: use the post-ReLU
  // slot, which every kernel family takes
  if (relu) { c.res1 = residual; c.res1_cs = Cout; }
  else { c.res2 = residual; c.res2_cs = Cout; }
  c.out = y; c.out_cs = Cout; c.out_coff = 0; c.store = kStoreNHWC;
  return launch_conv(c, dtype, (hipStream_t)stream);
}

}  // extern "C"
