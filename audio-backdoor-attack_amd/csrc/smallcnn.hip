// smallcnn training/eval step for gfx950: forward, backward, loss, Adam, metrics.
//
// Replaces utils/models.py:17-65 (smallcnn), utils/training_tools.py:52-85 (train
// inner step: CrossEntropyLoss on log-probs, backward, optim.Adam.step, loss/acc/ASR
// bookkeeping) and :87-134 (test).
//
// Layout (DESIGN.md "smallcnn"): activations are NHWC (channels innermost) so every
// implicit-GEMM operand row is a contiguous 128/256-byte channel vector; the flatten
// before fc1 is written in the reference's NCHW (c,h,w) order so fc1.weight is used
// exactly as torch stores it.  The 2x2 convolutions, their data/weight gradients and
// fc1 run as fp32-in/fp32-accumulate MFMA (v_mfma_f32_32x32x2_f32: exact f32 FMA
// chains, the only MFMA that meets the 1e-4 fp32 parity target).  conv1 (K=4) is
// VALU work and is recomputed in every pass instead of materialising its
// (B,64,H0-1,W0-1) output.  BatchNorm uses batch statistics reduced through
// per-block partials summed in double (deterministic order), max-pool argmax is
// recomputed (first maximum in scan order, like ATen's CPU kernel), and dropout masks
// come from a counter-based hash (or are supplied, for parity tests).
#include "abd_common.h"
#include "prof.h"

#include <algorithm>
#include <type_traits>
#include <cmath>
#include <vector>
#include <map>
#include <array>
#include <mutex>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// Activations kept as exact bf16 planes (plane-major): np = 3 splits x = x0 + x1 + x2 exactly
// (x0 = rne(x), x1 = rne(x - x0), x2 = x - x0 - x1), np = 1 stores rne(x).  The conv2 GEMMs read
// them as MFMA operands directly -- the split is done once, by the producer, instead of at every
// use (4 taps x every tile) inside the GEMMs.  4 consecutive channels of element e -> one 8-B
// store per plane.
__device__ __forceinline__ void store_planes4(uint16_t* base, int64_t plane, int64_t e, float4 x, int np) {
  f32x2 v[2] = {f32x2{x.x, x.y}, f32x2{x.z, x.w}};
#pragma unroll
  for (int pl = 0; pl < 3; ++pl) {
    if (pl >= np) break;
    uint32_t u[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      u[h] = __builtin_bit_cast(uint32_t, __builtin_convertvector(v[h], bf16x2));
      const f32x2 back = {__builtin_bit_cast(float, u[h] << 16), __builtin_bit_cast(float, u[h] & 0xffff0000u)};
      v[h] -= back;  // exact: x - rne(x) fits in fp32
    }
    *reinterpret_cast<uint2*>(base + pl * plane + e) = make_uint2(u[0], u[1]);
  }
}

namespace {

constexpr int kT = 256;
using abd::kWave;
constexpr float kEps = 1e-5f;
constexpr float kMomentum = 0.1f;
constexpr float kP1 = 0.4f, kP2 = 0.5f;
constexpr int kR1 = 8;  // max conv1 rows per chunk (LDS staging size); C1Args::rows is the actual

struct Geo {
  int H0, W0, K, H1, W1, W1p, H2, W2, H2p, W2p, H3, W3, H3p, W3p, flat;
};

Geo make_geo(int H0, int W0, int K) {
  Geo g;
  g.H0 = H0;
  g.W0 = W0;
  g.K = K;
  g.H1 = H0 - 1;
  g.W1 = W0 - 1;
  g.W1p = g.W1 / 3;
  g.H2 = g.H1 - 1;
  g.W2 = g.W1p - 1;
  g.H2p = g.H2 / 2 + 1;
  g.W2p = g.W2 / 2 + 1;
  g.H3 = g.H2p - 1;
  g.W3 = g.W2p - 1;
  g.H3p = (g.H3 - 2) / 2 + 1;
  g.W3p = g.W3 / 2 + 1;
  g.flat = 32 * g.H3p * g.W3p;
  return g;
}

// ------------------------------------------------------------------ parameter layout
enum {
  P_C1W, P_C1B, P_BN1W, P_BN1B, P_C2W, P_C2B, P_BN2W, P_BN2B,
  P_C3W, P_C3B, P_BN3W, P_BN3B, P_F1W, P_F1B, P_F2W, P_F2B, P_COUNT
};

void param_sizes(const Geo& g, int64_t* sz) {
  const int64_t s[P_COUNT] = {256, 64, 64, 64, 16384, 64, 64, 64, 8192, 32, 32, 32,
                              128LL * g.flat, 128, (int64_t)g.K * 128, g.K};
  for (int i = 0; i < P_COUNT; ++i) sz[i] = s[i];
}

// ------------------------------------------------------------------ dropout hash
__device__ __forceinline__ bool keep_hash(uint64_t seed, uint64_t stream, uint64_t idx, float p) {
  uint64_t z = seed ^ (stream * 0x9E3779B97F4A7C15ull) ^ (idx * 0xD1B54A32D192ED03ull);
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  const float u = (float)(uint32_t)(z >> 40) * (1.0f / 16777216.0f);
  return u >= p;  // keep with probability 1-p (torch: bernoulli_(1-p))
}

struct DropArgs {
  const uint8_t* mask_in;
  uint8_t* mask_out;
  uint64_t seed, stream;
  uint64_t base;  // global element index of this launch's element 0 (DP: row_offset * columns)
  float p, scale;
  int enabled;
};

__device__ __forceinline__ float drop_apply(const DropArgs& d, int64_t idx, float v) {
  if (!d.enabled) return v;
  bool k = d.mask_in ? (d.mask_in[idx] != 0) : keep_hash(d.seed, d.stream, d.base + (uint64_t)idx, d.p);
  if (d.mask_out) d.mask_out[idx] = k ? 1 : 0;
  return v * (k ? d.scale : 0.0f);
}

// ------------------------------------------------------------------ block helpers
// Reduce `nvals` per-thread values over the threads sharing a channel (channel = tid % C)
// and write them as partials part[(j*C + c)*nblk + blk].
template <int NV>
__device__ __forceinline__ void channel_partials(float (&v)[NV], int C, float* part, int nblk, int blk) {
  __shared__ float red[NV * kT];
  const int t = threadIdx.x;
#pragma unroll
  for (int j = 0; j < NV; ++j) red[j * kT + t] = v[j];
  __syncthreads();
  if (t < C) {
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      float s = 0.0f;
      for (int q = t; q < kT; q += C) s += red[j * kT + q];
      part[((int64_t)j * C + t) * nblk + blk] = s;
    }
  }
}

// per-channel partial sums of NV values over the threads sharing a channel group
// (thread t holds channels CPT*(t % CG) .. +CPT-1, CG = C/CPT); part[(j*C + c)*nblk + blk]
template <int NV, int CPT = 4>
__device__ __forceinline__ void cgroup_partials(float (&v)[NV][CPT], int C, float* part, int nblk, int blk) {
  __shared__ float red[NV * CPT][kT];
  const int t = threadIdx.x, CG = C / CPT;
#pragma unroll
  for (int j = 0; j < NV; ++j)
#pragma unroll
    for (int q = 0; q < CPT; ++q) red[j * CPT + q][t] = v[j][q];
  __syncthreads();
  for (int o = t; o < NV * C; o += kT) {
    const int j = o / C, c = o - j * C;
    const int cg = c / CPT, q = c % CPT;
    float sacc = 0.0f;
    for (int u = cg; u < kT; u += CG) sacc += red[j * CPT + q][u];
    part[((int64_t)j * C + c) * nblk + blk] = sacc;
  }
}

// ------------------------------------------------------------------ conv1 (VALU, recomputed)
// BatchNorm backward per-channel coefficients kept in double: dx = g * (dy - mdy - xhat * mdyx).
// The batch means are subtracted from every element and the later weight-gradient sums
// cancel 200-5000x, so rounding mdy / mdyx to fp32 would bias every element the same way.
// With g = gamma*invstd, mdy = mean(dy), mdyx = mean(dy*xhat), xhat = (r - mean)*invstd:
//   dx = g*(dy - mdy - xhat*mdyx) = g*dy + A + B*r,  A = g*(mdyx*invstd*mean - mdy),  B = -g*mdyx*invstd
// evaluated as two double fmas.
struct BCoef {
  double g, A, B, pad;
};

#ifndef ABD_C1_DD
#define ABD_C1_DD 0
#endif
#ifndef ABD_C1W_U
#define ABD_C1W_U 4  // pool windows per thread whose gradient loads conv1_wgrad_kernel batches
#endif
__device__ __forceinline__ float bn_dx(float dy, float r, float4 /*cf*/, const BCoef& bc) {
  return (float)fma(bc.B, (double)r, fma(bc.g, (double)dy, bc.A));
}

// bn_dx in float-float arithmetic: each double coefficient carried as hi + lo fp32 parts (the
// parts' sum is the double to ~2^-48), dx = (B_hi r + g_hi dy + A_hi) + (B_lo r + g_lo dy + A_lo).
// The batch-mean terms keep their double precision (no systematic bias for the cancelling
// weight-gradient sums); what remains is the per-element fp32 rounding the double path also has
// at its final store.  Channel pairs as float2 vector FMAs (conv1_wgrad_kernel; the library is built
// without packed FP32, Makefile PKFLAGS, so each is two v_fma_f32); ABD_C1_DD=1 builds the
// double-precision evaluation instead.
struct BCoefF {
  float gh, gl, Ah, Al, Bh, Bl;
};
__device__ __forceinline__ BCoefF bcoef_ff(const BCoef& c) {
  BCoefF f;
  f.gh = (float)c.g;
  f.gl = (float)(c.g - (double)f.gh);
  f.Ah = (float)c.A;
  f.Al = (float)(c.A - (double)f.Ah);
  f.Bh = (float)c.B;
  f.Bl = (float)(c.B - (double)f.Bh);
  return f;
}

// weight repacks: fwd W'[co][t][ci] and dgrad Wd[ci][t][co] (taps flipped via offsets), fc1^T
constexpr int kGuardTickets = 4;  // BN1, BN2, BN3 guard tickets (+ a spare)
struct PrepArgs {
  const float *c2w, *c3w, *f1w;
  int flat;
  float *w2f, *w2d, *w3f, *w3d, *f1t;
  unsigned* tickets;  // the step's guard arrival tickets, zeroed here every step
  int ntickets;
};

__device__ __forceinline__ void prep_weights_body(const PrepArgs& a, int bx, int nb) {
  const int64_t n2 = 64 * 64 * 4, n3 = 32 * 64 * 4, nf = 128LL * a.flat;
  const int64_t total = n2 + n3 + nf;
  if (bx == 0 && a.tickets != nullptr)
    for (int i = threadIdx.x; i < a.ntickets; i += kT) a.tickets[i] = 0u;
  for (int64_t e = bx * (int64_t)kT + threadIdx.x; e < total; e += (int64_t)nb * kT) {
    if (e < n2) {
      const int co = (int)(e / 256), ci = (int)(e / 4 % 64), t = (int)(e % 4);
      const float v = a.c2w[e];
      a.w2f[(co * 4 + t) * 64 + ci] = v;
      a.w2d[(ci * 4 + t) * 64 + co] = v;
    } else if (e < n2 + n3) {
      const int64_t f = e - n2;
      const int co = (int)(f / 256), ci = (int)(f / 4 % 64), t = (int)(f % 4);
      const float v = a.c3w[f];
      a.w3f[(co * 4 + t) * 64 + ci] = v;
      a.w3d[(ci * 4 + t) * 32 + co] = v;
    } else {
      const int64_t f = e - n2 - n3;
      const int j = (int)(f / a.flat), k = (int)(f % a.flat);
      a.f1t[(int64_t)k * 128 + j] = a.f1w[f];
    }
  }
}
__global__ void __launch_bounds__(kT) prep_weights_kernel(PrepArgs a) { prep_weights_body(a, blockIdx.x, gridDim.x); }

struct C1Args {
  const float* x;   // (B, H0, W0)
  const float* w;   // conv1.weight (64,1,2,2)
  const float* b;   // conv1.bias
  const float4* coef;  // BN1 (mean, invstd, alpha, beta')
  const float* dp1;    // (B,H1,W1p,64) grad of pool1 output
  const BCoef* bcoef;  // BN1 backward
  float* p1;
  float* part;
  int nblk;
  Geo g;
  int B;
  int rows;  // conv1 rows per chunk (<= kR1)
  int coef_bstride;  // 0: one BN1 coefficient set; 64: per utterance (coef + b*64)
  PrepArgs prep;     // conv1_stats_kernel: blocks [0, nprep) repack the weights
  int nprep;
  const float* gamma;  // conv1_stats_fold_kernel: BN1 weight (the sign picks max or min per window)
  // conv1_stats_fold_kernel: p1s != nullptr stores m as np exact bf16 planes (plane-major, plane
  // stride `plane` elements; split once here instead of at every use in conv2's GEMMs) instead of p1
  uint16_t* p1s;
  int64_t plane;
  int np;
};

// Stage x rows [h0, h0+kR1] of utterance b into LDS.
__device__ __forceinline__ void stage_x(const C1Args& a, int b, int h0, float* xs) {
  const int rows = min(a.rows + 1, a.g.H0 - h0);
  const float* src = a.x + ((int64_t)b * a.g.H0 + h0) * a.g.W0;
  if ((a.g.W0 & 3) == 0) {  // rows start 16-byte aligned: one float4 per thread (W0 = 40: 90 loads)
    const int n4 = rows * a.g.W0 / 4;
    for (int i = threadIdx.x; i < n4; i += kT)
      reinterpret_cast<float4*>(xs)[i] = reinterpret_cast<const float4*>(src)[i];
  } else {
    for (int i = threadIdx.x; i < rows * a.g.W0; i += kT) xs[i] = src[i];
  }
  __syncthreads();
}

// conv1 kernels: one block per (utterance, kR1 rows); thread t owns channels 4*(t%16)..+3
// (float4 weights / BN coefficients / NHWC stores) and walks positions or pool windows
// t/16, t/16 + 16, ...  The x patch is read from LDS (broadcast across the 16 channel
// groups).
struct C1W {
  float4 w00, w01, w10, w11, b;  // per-channel taps (kh,kw) and bias, 4 channels
};

__device__ __forceinline__ C1W c1_weights(const C1Args& a, int c0) {
  C1W r;
  float t[4][5];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
#pragma unroll
    for (int k = 0; k < 4; ++k) t[q][k] = a.w[(c0 + q) * 4 + k];
    t[q][4] = a.b[c0 + q];
  }
  r.w00 = make_float4(t[0][0], t[1][0], t[2][0], t[3][0]);
  r.w01 = make_float4(t[0][1], t[1][1], t[2][1], t[3][1]);
  r.w10 = make_float4(t[0][2], t[1][2], t[2][2], t[3][2]);
  r.w11 = make_float4(t[0][3], t[1][3], t[2][3], t[3][3]);
  r.b = make_float4(t[0][4], t[1][4], t[2][4], t[3][4]);
  return r;
}

// relu(conv1) for 4 channels at one position: channel pairs as float2 vector FMAs (two v_fma_f32 each:
// no packed FP32 in this library, Makefile PKFLAGS), the same fma chain per channel as the oracle
// replay (b, w00, w01, w10, w11)
typedef float c1f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ c1f2 c1_lo(const float4& v) { return c1f2{v.x, v.y}; }
__device__ __forceinline__ c1f2 c1_hi(const float4& v) { return c1f2{v.z, v.w}; }
__device__ __forceinline__ float4 c1_at_ptr(const float* r0, int W0, const C1W& k) {
  const float x00 = r0[0], x01 = r0[1], x10 = r0[W0], x11 = r0[W0 + 1];
  c1f2 lo = __builtin_elementwise_fma(c1_lo(k.w00), c1f2{x00, x00}, c1_lo(k.b));
  c1f2 hi = __builtin_elementwise_fma(c1_hi(k.w00), c1f2{x00, x00}, c1_hi(k.b));
  lo = __builtin_elementwise_fma(c1_lo(k.w01), c1f2{x01, x01}, lo);
  hi = __builtin_elementwise_fma(c1_hi(k.w01), c1f2{x01, x01}, hi);
  lo = __builtin_elementwise_fma(c1_lo(k.w10), c1f2{x10, x10}, lo);
  hi = __builtin_elementwise_fma(c1_hi(k.w10), c1f2{x10, x10}, hi);
  lo = __builtin_elementwise_fma(c1_lo(k.w11), c1f2{x11, x11}, lo);
  hi = __builtin_elementwise_fma(c1_hi(k.w11), c1f2{x11, x11}, hi);
  return make_float4(fmaxf(lo.x, 0.0f), fmaxf(lo.y, 0.0f), fmaxf(hi.x, 0.0f), fmaxf(hi.y, 0.0f));
}
__device__ __forceinline__ float4 c1_at(const float* xs, int W0, int hl, int w, const C1W& k) {
  return c1_at_ptr(xs + hl * W0 + w, W0, k);
}

__device__ __forceinline__ float4 c1_coef_col(const float4* coef, int c0, int comp) {
  float v[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float4 cf = coef[c0 + q];
    v[q] = comp == 0 ? cf.x : comp == 1 ? cf.y : comp == 2 ? cf.z : cf.w;
  }
  return make_float4(v[0], v[1], v[2], v[3]);
}

// forward stats: sum / sumsq of relu(conv1) per channel
__global__ void __launch_bounds__(kT) conv1_stats_kernel(C1Args a) {
  __shared__ __attribute__((aligned(16))) float xs[(kR1 + 1) * 128];
  if ((int)blockIdx.x < a.nprep) {
    prep_weights_body(a.prep, blockIdx.x, a.nprep);
    return;
  }
  const int bid = (int)blockIdx.x - a.nprep;
  const int nbh = (a.g.H1 + a.rows - 1) / a.rows;
  const int nchunks = a.B * nbh;
  const int c0 = (threadIdx.x & 15) * 4, pl = threadIdx.x >> 4;
  const C1W k = c1_weights(a, c0);
  float v[2][4] = {};
  for (int chunk = bid; chunk < nchunks; chunk += a.nblk) {
    const int b = chunk / nbh, h0 = (chunk % nbh) * a.rows;
    stage_x(a, b, h0, xs);
    const int rows = min(a.rows, a.g.H1 - h0);
    // positions pl, pl + 16, ... in row-major (hl, w) order, stepped without dividing by W1
    int hl = pl / a.g.W1, w = pl - hl * a.g.W1;
    for (int idx = pl; idx < rows * a.g.W1; idx += 16) {
      const float4 r = c1_at(xs, a.g.W0, hl, w, k);
      w += 16;
      while (w >= a.g.W1) {
        w -= a.g.W1;
        ++hl;
      }
      v[0][0] += r.x;
      v[0][1] += r.y;
      v[0][2] += r.z;
      v[0][3] += r.w;
      v[1][0] = fmaf(r.x, r.x, v[1][0]);
      v[1][1] = fmaf(r.y, r.y, v[1][1]);
      v[1][2] = fmaf(r.z, r.z, v[1][2]);
      v[1][3] = fmaf(r.w, r.w, v[1][3]);
    }
    __syncthreads();  // xs is restaged by the next chunk
  }
  cgroup_partials<2>(v, 64, a.part, a.nblk, bid);
}

// first maximum of bn(r) over a (1,3) window, per channel: returns the slot index 0..2
__device__ __forceinline__ int c1_argmax(float r0, float r1, float r2, float al, float be, float& best) {
  const float y0 = fmaf(al, r0, be), y1 = fmaf(al, r1, be), y2 = fmaf(al, r2, be);
  int j = 0;
  best = y0;
  if (y1 > best) {
    best = y1;
    j = 1;
  }
  if (y2 > best) {
    best = y2;
    j = 2;
  }
  return j;
}

// forward: relu(conv1) -> BN1 -> maxpool(1,3) -> p1 (NHWC)
__global__ void __launch_bounds__(kT) conv1_bn_pool_kernel(C1Args a) {
  __shared__ __attribute__((aligned(16))) float xs[(kR1 + 1) * 128];
  const int nbh = (a.g.H1 + a.rows - 1) / a.rows;
  const int nchunks = a.B * nbh;
  const int c0 = (threadIdx.x & 15) * 4, pl = threadIdx.x >> 4;
  const C1W k = c1_weights(a, c0);
  float4 al = c1_coef_col(a.coef, c0, 2), be = c1_coef_col(a.coef, c0, 3);
  const int NW = a.g.W1p;
  for (int chunk = blockIdx.x; chunk < nchunks; chunk += gridDim.x) {
    const int b = chunk / nbh, h0 = (chunk % nbh) * a.rows;
    if (a.coef_bstride) {  // per-utterance BatchNorm (abd_smallcnn_forward_per_utterance)
      al = c1_coef_col(a.coef + (int64_t)b * a.coef_bstride, c0, 2);
      be = c1_coef_col(a.coef + (int64_t)b * a.coef_bstride, c0, 3);
    }
    stage_x(a, b, h0, xs);
    const int rows = min(a.rows, a.g.H1 - h0);
    int hl = pl / NW, wo = pl - hl * NW;  // (hl, wo) of idx, stepped without dividing by NW
    for (int idx = pl; idx < rows * NW; idx += 16, wo += 16) {
      while (wo >= NW) {
        wo -= NW;
        ++hl;
      }
      const int w = 3 * wo;
      const float4 r0 = c1_at(xs, a.g.W0, hl, w, k), r1 = c1_at(xs, a.g.W0, hl, w + 1, k),
                   r2 = c1_at(xs, a.g.W0, hl, w + 2, k);
      float4 o;
      c1_argmax(r0.x, r1.x, r2.x, al.x, be.x, o.x);
      c1_argmax(r0.y, r1.y, r2.y, al.y, be.y, o.y);
      c1_argmax(r0.z, r1.z, r2.z, al.z, be.z, o.z);
      c1_argmax(r0.w, r1.w, r2.w, al.w, be.w, o.w);
      *reinterpret_cast<float4*>(a.p1 + (((int64_t)b * a.g.H1 + h0 + hl) * NW + wo) * 64 + c0) = o;
    }
    __syncthreads();  // xs is restaged by the next chunk
  }
}

// Training forward of layer 1 with BN1 folded into conv2 (train step, f32split weight-stationary
// conv2): ONE pass computes relu(conv1) everywhere, BN1's batch statistics, and per pool1 window
// the element the pool will select, m = max r (gamma >= 0) or min r (gamma < 0).  For either sign of
// alpha = gamma * invstd, max_j fl(alpha r_j + beta') = fl(alpha m + beta') (fl is monotone), so
// p1 = alpha m + beta' once the statistics are known; conv2 consumes m with alpha folded into its
// weights and beta' into its bias (NTArgs::fold), its weight gradient is corrected the same way
// (slab_reduce_kernel fold), and conv1_bn_pool_kernel's second conv1 pass disappears.  p1's buffer
// holds m.  Blocks [0, nprep) repack the weights (prep_weights_body) as in conv1_stats_kernel.
// forward() caps the chunk grid at the kernel's residency (73 VGPRs: 6 blocks per CU), so the chunks
// run in one round (a 64-VGPR build for 8 blocks per CU spills and measured the same)
#ifndef ABD_C1S_OCC  // waves per SIMD conv1_stats_fold_kernel is register-budgeted for (measurement builds)
#define ABD_C1S_OCC 1
#endif
__global__ void __launch_bounds__(kT, ABD_C1S_OCC) conv1_stats_fold_kernel(C1Args a) {
  __shared__ __attribute__((aligned(16))) float xs[(kR1 + 1) * 128];
  if ((int)blockIdx.x < a.nprep) {
    prep_weights_body(a.prep, blockIdx.x, a.nprep);
    return;
  }
  const int bid = (int)blockIdx.x - a.nprep;
  const int nbh = (a.g.H1 + a.rows - 1) / a.rows;
  const int nchunks = a.B * nbh;
  const int c0 = (threadIdx.x & 15) * 4, pl = threadIdx.x >> 4;
  const C1W k = c1_weights(a, c0);
  bool neg[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) neg[q] = a.gamma[c0 + q] < 0.0f;
  const int NW = (a.g.W1 + 2) / 3;  // windows incl. a partial trailing one (statistics only)
  const int NWp = a.g.W1p;
  float v[2][4] = {};
  for (int chunk = bid; chunk < nchunks; chunk += a.nblk) {
    const int b = chunk / nbh, h0 = (chunk % nbh) * a.rows;
    stage_x(a, b, h0, xs);
    const int rows = min(a.rows, a.g.H1 - h0);
    int hl = pl / NW, wo = pl - hl * NW;  // (hl, wo) of idx, stepped without dividing by NW
    for (int idx = pl; idx < rows * NW; idx += 16, wo += 16) {
      while (wo >= NW) {
        wo -= NW;
        ++hl;
      }
      const int w = 3 * wo;
      const int nw = min(3, a.g.W1 - w);
      float rr[3][4];
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const float4 r = c1_at(xs, a.g.W0, hl, w + j, k);
        const bool in = j < nw;  // positions past W1 (trailing partial window) contribute nothing
        rr[j][0] = in ? r.x : 0.0f;
        rr[j][1] = in ? r.y : 0.0f;
        rr[j][2] = in ? r.z : 0.0f;
        rr[j][3] = in ? r.w : 0.0f;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          v[0][q] += rr[j][q];
          v[1][q] = fmaf(rr[j][q], rr[j][q], v[1][q]);
        }
      }
      if (wo < NWp) {  // a real pool1 window (nw == 3)
        float o[4];
#pragma unroll
        for (int q = 0; q < 4; ++q)
          o[q] = neg[q] ? fminf(fminf(rr[0][q], rr[1][q]), rr[2][q]) : fmaxf(fmaxf(rr[0][q], rr[1][q]), rr[2][q]);
        const int64_t e = (((int64_t)b * a.g.H1 + h0 + hl) * NWp + wo) * 64 + c0;
        if (a.p1s != nullptr) store_planes4(a.p1s, a.plane, e, make_float4(o[0], o[1], o[2], o[3]), a.np);
        else *reinterpret_cast<float4*>(a.p1 + e) = make_float4(o[0], o[1], o[2], o[3]);
      }
    }
    __syncthreads();  // xs is restaged by the next chunk
  }
  cgroup_partials<2>(v, 64, a.part, a.nblk, bid);
}

// backward stats: s1 = sum dy, s2 = sum dy * xhat over pool1 argmax positions
// The derived BatchNorm backward statistics (bn_bwd_derived_kernel, slab_reduce_derive_kernel, the fc1
// data-gradient epilogue for BN3) read xhat back from the stored BN output as (p - beta) / gamma: the
// fp32 rounding of p is amplified by |beta| / |gamma|, and at gamma = 0 p holds no xhat at all
// (ADVICE r2).  A channel is "tiny" when |gamma| <= 1e-2 |beta| + 1e-5 (amplification <= 100x:
// <= ~6e-6 relative); the guarded kernels below then recompute the whole layer's statistics from the
// activations (the passes the derivation replaced) and exit at once otherwise.  Wave-uniform, C <= 64.
__device__ __forceinline__ bool bn_any_tiny(const float* __restrict__ gamma, const float* __restrict__ beta, int C) {
  const int lane = threadIdx.x & 63;
  bool t = false;
  if (lane < C) t = fabsf(gamma[lane]) <= 1e-2f * fabsf(beta[lane]) + 1e-5f;
  return __ballot(t) != 0ull;
}

__device__ __forceinline__ void conv1_bwd_stats_body(const C1Args& a);
__global__ void __launch_bounds__(kT) conv1_bwd_stats_kernel(C1Args a) { conv1_bwd_stats_body(a); }
// The guarded fallbacks' finalize, in the same launch: every block publishes its partials, the last
// block to arrive (agent-scope release -> ticket -> acquire, MI355X_MICROARCH.md inter-workgroup
// visibility) reduces them per channel exactly as bn_bwd_finalize_kernel does and overwrites the
// derived dgamma / dbeta / backward coefficients.  The ticket is zeroed by the step's prep blocks.
struct GuardOut {
  double count;
  const float4* coef;
  float* dgamma;
  float* dbeta;
  BCoef* bcoef;
  unsigned* ticket;
};
// the last of n arrivals (n = gridDim.x)
__device__ __forceinline__ bool last_arrival(unsigned* ticket, unsigned n) {
  __shared__ unsigned last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = (t == n - 1) ? 1u : 0u;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      // every block has taken its ticket: re-arm it, so a launch that finds no prep block before it
      // (a second abd_smallcnn_backward after one forward) still sees a zeroed ticket
      __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  return last != 0u;
}
__device__ __forceinline__ bool guard_last_block(unsigned* ticket) { return last_arrival(ticket, gridDim.x); }
__device__ __forceinline__ void guard_finalize(const float* part, int nblk, int C, const float* gamma, const GuardOut& g) {
  __shared__ double red[2][kT / kWave];
  for (int c = 0; c < C; ++c) {
    double s1 = 0.0, s2 = 0.0;
    for (int i = threadIdx.x; i < nblk; i += kT) {
      s1 += part[(int64_t)c * nblk + i];
      s2 += part[((int64_t)C + c) * nblk + i];
    }
    s1 = abd::wave_sum_d(s1);
    s2 = abd::wave_sum_d(s2);
    if ((threadIdx.x & 63) == 0) {
      red[0][threadIdx.x >> 6] = s1;
      red[1][threadIdx.x >> 6] = s2;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      s1 = red[0][0] + red[0][1] + red[0][2] + red[0][3];
      s2 = red[1][0] + red[1][1] + red[1][2] + red[1][3];
      g.dgamma[c] = (float)s2;
      g.dbeta[c] = (float)s1;
      const double gg = (double)gamma[c] * (double)g.coef[c].y, mdy = s1 / g.count, mdyx = s2 / g.count;
      const double mean = (double)g.coef[c].x, invstd = (double)g.coef[c].y;
      g.bcoef[c] = BCoef{gg, gg * (mdyx * invstd * mean - mdy), -gg * mdyx * invstd, 0.0};
    }
    __syncthreads();
  }
}

// guarded fallback: BN1's statistics from the activations when a gamma is tiny (bn_any_tiny); runs
// inside slab_reduce_derive_kernel's launch (a.nblk = that grid)
struct C1Guard {
  C1Args a;
  const float* gamma;
  const float* beta;
  GuardOut go;
  __device__ void operator()() const {
    if (!bn_any_tiny(gamma, beta, 64)) return;
    conv1_bwd_stats_body(a);
    if (guard_last_block(go.ticket)) guard_finalize(a.part, a.nblk, 64, gamma, go);
  }
};
__device__ __forceinline__ void conv1_bwd_stats_body(const C1Args& a) {
  __shared__ __attribute__((aligned(16))) float xs[(kR1 + 1) * 128];
  const int nbh = (a.g.H1 + a.rows - 1) / a.rows;
  const int nchunks = a.B * nbh;
  const int c0 = (threadIdx.x & 15) * 4, pl = threadIdx.x >> 4;
  const C1W k = c1_weights(a, c0);
  const float4 mu = c1_coef_col(a.coef, c0, 0), is = c1_coef_col(a.coef, c0, 1);
  const float4 al = c1_coef_col(a.coef, c0, 2), be = c1_coef_col(a.coef, c0, 3);
  const int NW = a.g.W1p;
  float v[2][4] = {};
  for (int chunk = blockIdx.x; chunk < nchunks; chunk += gridDim.x) {
    const int b = chunk / nbh, h0 = (chunk % nbh) * a.rows;
    stage_x(a, b, h0, xs);
    const int rows = min(a.rows, a.g.H1 - h0);
    int hl = pl / NW, wo = pl - hl * NW;  // (hl, wo) of idx, stepped without dividing by NW
    for (int idx = pl; idx < rows * NW; idx += 16, wo += 16) {
      while (wo >= NW) {
        wo -= NW;
        ++hl;
      }
      const int w = 3 * wo;
      const float4 r0 = c1_at(xs, a.g.W0, hl, w, k), r1 = c1_at(xs, a.g.W0, hl, w + 1, k),
                   r2 = c1_at(xs, a.g.W0, hl, w + 2, k);
      const float4 dy = *reinterpret_cast<const float4*>(a.dp1 + (((int64_t)b * a.g.H1 + h0 + hl) * NW + wo) * 64 + c0);
      const float rr0[4] = {r0.x, r0.y, r0.z, r0.w}, rr1[4] = {r1.x, r1.y, r1.z, r1.w}, rr2[4] = {r2.x, r2.y, r2.z, r2.w};
      const float aa[4] = {al.x, al.y, al.z, al.w}, bb[4] = {be.x, be.y, be.z, be.w};
      const float mm[4] = {mu.x, mu.y, mu.z, mu.w}, ii[4] = {is.x, is.y, is.z, is.w};
      const float dd[4] = {dy.x, dy.y, dy.z, dy.w};
  #pragma unroll
      for (int q = 0; q < 4; ++q) {
        float best;
        const int j = c1_argmax(rr0[q], rr1[q], rr2[q], aa[q], bb[q], best);
        const float rs = j == 0 ? rr0[q] : (j == 1 ? rr1[q] : rr2[q]);
        v[0][q] += dd[q];
        v[1][q] = fmaf(dd[q], (rs - mm[q]) * ii[q], v[1][q]);
      }
    }
    __syncthreads();  // xs is restaged by the next chunk
  }
  cgroup_partials<2>(v, 64, a.part, a.nblk, blockIdx.x);
}

// backward: BN1 dx -> relu mask -> conv1 weight / bias gradient partials (5 per channel).
// 2 channels per thread (the double-precision BN coefficients would otherwise cap occupancy).
// FULL (W1 % 3 == 0, every BASELINE geometry): no partial trailing window, branch-free body.
#ifndef ABD_C1W_OCC  // waves per SIMD conv1_wgrad_kernel is register-budgeted for (measurement builds)
#define ABD_C1W_OCC 1
#endif
template <bool FULL>
__global__ void __launch_bounds__(kT, ABD_C1W_OCC) conv1_wgrad_kernel(C1Args a) {
  __shared__ __attribute__((aligned(16))) float xs[(kR1 + 1) * 128];
  const int nbh = (a.g.H1 + a.rows - 1) / a.rows;
  const int nchunks = a.B * nbh;
  constexpr int CPT = 2;
  const int c0 = (threadIdx.x & 31) * CPT, pl = threadIdx.x >> 5;
  float kw[CPT][5], aa[CPT], bb[CPT];
  BCoef bc[CPT];
#pragma unroll
  for (int q = 0; q < CPT; ++q) {
#pragma unroll
    for (int t = 0; t < 4; ++t) kw[q][t] = a.w[(c0 + q) * 4 + t];
    kw[q][4] = a.b[c0 + q];
    const float4 cf = a.coef[c0 + q];
    aa[q] = cf.z;
    bb[q] = cf.w;
    bc[q] = a.bcoef[c0 + q];
  }
#if !ABD_C1_DD
  c1f2 fgh, fgl, fAh, fAl, fBh, fBl;  // float-float coefficients of the channel pair
  {
    const BCoefF f0 = bcoef_ff(bc[0]), f1 = bcoef_ff(bc[1]);
    fgh = c1f2{f0.gh, f1.gh};
    fgl = c1f2{f0.gl, f1.gl};
    fAh = c1f2{f0.Ah, f1.Ah};
    fAl = c1f2{f0.Al, f1.Al};
    fBh = c1f2{f0.Bh, f1.Bh};
    fBl = c1f2{f0.Bl, f1.Bl};
  }
#endif
  const int NW = (a.g.W1 + 2) / 3;  // windows incl. a partial trailing one (dy = 0 there)
  static_assert(CPT == 2, "one packed channel pair per thread");
  c1f2 kp[5], vp[5];
#pragma unroll
  for (int t = 0; t < 5; ++t) {
    kp[t] = c1f2{kw[0][t], kw[1][t]};
    vp[t] = c1f2{0.0f, 0.0f};
  }
  for (int chunk = blockIdx.x; chunk < nchunks; chunk += gridDim.x) {
    const int b = chunk / nbh, h0 = (chunk % nbh) * a.rows;
    stage_x(a, b, h0, xs);
    const int rows = min(a.rows, a.g.H1 - h0);
    const int nwin = rows * NW;
    constexpr int WS = kT / 32;  // windows in flight per block
    int hl = pl / NW, wo = pl - hl * NW;  // (hl, wo) of idx, stepped without dividing by NW
    // ABD_C1W_U windows per thread per batch: their pooled-gradient loads are all issued before
    // the first window's arithmetic (one exposed load latency per batch instead of per window);
    // windows are still accumulated in idx order, so the sums are those of the one-window loop
    for (int base = pl; base < nwin; base += ABD_C1W_U * WS) {
      int hls[ABD_C1W_U], wos[ABD_C1W_U];
      float2 dvs[ABD_C1W_U];
  #pragma unroll
      for (int u = 0; u < ABD_C1W_U; ++u) {
        hls[u] = hl;
        wos[u] = wo;
        const bool ld = base + u * WS < nwin && (FULL || wo < a.g.W1p);
        dvs[u] = ld ? *reinterpret_cast<const float2*>(a.dp1 + (((int64_t)b * a.g.H1 + h0 + hl) * a.g.W1p + wo) * 64 + c0)
                    : float2{0.0f, 0.0f};
        wo += WS;
        while (wo >= NW) {
          wo -= NW;
          ++hl;
        }
      }
  #pragma unroll
      for (int u = 0; u < ABD_C1W_U; ++u) {
      if (base + u * WS >= nwin) break;
      const int hl = hls[u], wo = wos[u];
      const int w = 3 * wo;
      const int nw = FULL ? 3 : min(3, a.g.W1 - w);
      const bool real = FULL || wo < a.g.W1p;
      const float* x0 = xs + hl * a.g.W0 + w;
      float xv[2][4];
  #pragma unroll
      for (int j = 0; j < 4; ++j) {
        xv[0][j] = (j <= nw) ? x0[j] : 0.0f;
        xv[1][j] = (j <= nw) ? x0[a.g.W0 + j] : 0.0f;
      }
      const float dd[CPT] = {dvs[u].x, dvs[u].y};
      // the channel pair as float2 vector FMAs: per channel the same fma chain as the oracle replay
      // (b, w00, w01, w10, w11) and the same accumulation order
      float r[CPT][3];
  #pragma unroll
      for (int j = 0; j < 3; ++j) {
        c1f2 acc = __builtin_elementwise_fma(kp[0], c1f2{xv[0][j], xv[0][j]}, kp[4]);
        acc = __builtin_elementwise_fma(kp[1], c1f2{xv[0][j + 1], xv[0][j + 1]}, acc);
        acc = __builtin_elementwise_fma(kp[2], c1f2{xv[1][j], xv[1][j]}, acc);
        acc = __builtin_elementwise_fma(kp[3], c1f2{xv[1][j + 1], xv[1][j + 1]}, acc);
        r[0][j] = (j < nw) ? fmaxf(acc.x, 0.0f) : 0.0f;
        r[1][j] = (j < nw) ? fmaxf(acc.y, 0.0f) : 0.0f;
      }
      int jm[CPT];
  #pragma unroll
      for (int q = 0; q < CPT; ++q) {
        float best;
        jm[q] = real ? c1_argmax(r[q][0], r[q][1], r[q][2], aa[q], bb[q], best) : -1;
      }
  #pragma unroll
      for (int j = 0; j < 3; ++j) {
        if (j >= nw) continue;
        c1f2 dz;
#if ABD_C1_DD
        dz.x = r[0][j] > 0.0f ? bn_dx(j == jm[0] ? dd[0] : 0.0f, r[0][j], float4{}, bc[0]) : 0.0f;
        dz.y = r[1][j] > 0.0f ? bn_dx(j == jm[1] ? dd[1] : 0.0f, r[1][j], float4{}, bc[1]) : 0.0f;
#else
        {
          const c1f2 dy = c1f2{j == jm[0] ? dd[0] : 0.0f, j == jm[1] ? dd[1] : 0.0f};
          const c1f2 rr = c1f2{r[0][j], r[1][j]};
          const c1f2 hi = __builtin_elementwise_fma(fBh, rr, __builtin_elementwise_fma(fgh, dy, fAh));
          const c1f2 lo = __builtin_elementwise_fma(fBl, rr, __builtin_elementwise_fma(fgl, dy, fAl));
          const c1f2 v = hi + lo;
          dz.x = rr.x > 0.0f ? v.x : 0.0f;
          dz.y = rr.y > 0.0f ? v.y : 0.0f;
        }
#endif
        vp[0] = __builtin_elementwise_fma(dz, c1f2{xv[0][j], xv[0][j]}, vp[0]);
        vp[1] = __builtin_elementwise_fma(dz, c1f2{xv[0][j + 1], xv[0][j + 1]}, vp[1]);
        vp[2] = __builtin_elementwise_fma(dz, c1f2{xv[1][j], xv[1][j]}, vp[2]);
        vp[3] = __builtin_elementwise_fma(dz, c1f2{xv[1][j + 1], xv[1][j + 1]}, vp[3]);
        vp[4] += dz;
      }
      }
    }
    __syncthreads();  // xs is restaged by the next chunk
  }
  float v[5][CPT];
#pragma unroll
  for (int t = 0; t < 5; ++t) {
    v[t][0] = vp[t].x;
    v[t][1] = vp[t].y;
  }
  cgroup_partials<5, CPT>(v, 64, a.part, a.nblk, blockIdx.x);
}

// ------------------------------------------------------------------ input gradient (eval mode)
// FlowMur's frozen benign model (utils/flowmur_generate_trigger.py:98-103) is differentiated
// w.r.t. its input only.  Eval BatchNorm is affine, so its backward is dz = relu'(r) * alpha * dy.
// conv1_dz_eval_kernel: thread = (utterance, conv1 row, pool1 window, 4 channels): relu(conv1)
// recomputed, pool1 argmax, dz1 for the window's positions (NHWC).  A trailing partial window
// (W1 % 3 != 0) gets zero.
__global__ void __launch_bounds__(kT) conv1_dz_eval_kernel(C1Args a, float* __restrict__ dz1) {
  const int NWx = (a.g.W1 + 2) / 3;
  const int total = a.B * a.g.H1 * NWx * 16;
  const int c0 = (threadIdx.x & 15) * 4;  // fixed per thread: the grid stride is a multiple of 16
  const C1W k = c1_weights(a, c0);
  const float4 al = c1_coef_col(a.coef, c0, 2), be = c1_coef_col(a.coef, c0, 3);
  const float aa[4] = {al.x, al.y, al.z, al.w}, bb[4] = {be.x, be.y, be.z, be.w};
  for (int o = blockIdx.x * kT + threadIdx.x; o < total; o += gridDim.x * kT) {
    int q = o >> 4;
    const int wo = q % NWx;
    q /= NWx;
    const int h = q % a.g.H1, b = q / a.g.H1;
    const float* xr = a.x + ((int64_t)b * a.g.H0 + h) * a.g.W0;
    const int w = 3 * wo;
    const int nw = min(3, a.g.W1 - w);
    const bool real = wo < a.g.W1p;
    float r[3][4];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const float4 v = (j < nw) ? c1_at(xr, a.g.W0, 0, w + j, k) : make_float4(0.f, 0.f, 0.f, 0.f);
      r[j][0] = v.x;
      r[j][1] = v.y;
      r[j][2] = v.z;
      r[j][3] = v.w;
    }
    const float4 dy = real ? *reinterpret_cast<const float4*>(a.dp1 + (((int64_t)b * a.g.H1 + h) * a.g.W1p + wo) * 64 + c0)
                           : make_float4(0.f, 0.f, 0.f, 0.f);
    const float dd[4] = {dy.x, dy.y, dy.z, dy.w};
    float dz[3][4];
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {
      float best;
      const int jm = real ? c1_argmax(r[0][qq], r[1][qq], r[2][qq], aa[qq], bb[qq], best) : -1;
#pragma unroll
      for (int j = 0; j < 3; ++j) dz[j][qq] = (j == jm && r[j][qq] > 0.0f) ? aa[qq] * dd[qq] : 0.0f;
    }
    for (int j = 0; j < nw; ++j)
      *reinterpret_cast<float4*>(dz1 + (((int64_t)b * a.g.H1 + h) * a.g.W1 + w + j) * 64 + c0) =
          make_float4(dz[j][0], dz[j][1], dz[j][2], dz[j][3]);
  }
}

// dx[b][i][j] = sum_{kh,kw} sum_c conv1.w[c][kh][kw] * dz1[b][i-kh][j-kw][c]
__global__ void __launch_bounds__(kT) conv1_dx_kernel(const float* __restrict__ w1, const float* __restrict__ dz1,
                                                      int B, Geo g, float* __restrict__ dx) {
  __shared__ float4 wsh[4][16];  // [tap][channel group]: 4 channels' weights
  if (threadIdx.x < 64) {
    const int t = threadIdx.x >> 4, cg = threadIdx.x & 15;
    wsh[t][cg] = make_float4(w1[(4 * cg + 0) * 4 + t], w1[(4 * cg + 1) * 4 + t], w1[(4 * cg + 2) * 4 + t],
                             w1[(4 * cg + 3) * 4 + t]);
  }
  __syncthreads();
  const int total = B * g.H0 * g.W0;
  for (int o = blockIdx.x * kT + threadIdx.x; o < total; o += gridDim.x * kT) {
    const int b = o / (g.H0 * g.W0), rem = o - b * g.H0 * g.W0;
    const int i = rem / g.W0, j = rem - i * g.W0;
    float acc = 0.0f;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int hi = i - (t >> 1), wj = j - (t & 1);
      if (hi < 0 || hi >= g.H1 || wj < 0 || wj >= g.W1) continue;
      const float4* z = reinterpret_cast<const float4*>(dz1 + (((int64_t)b * g.H1 + hi) * g.W1 + wj) * 64);
#pragma unroll 4
      for (int cg = 0; cg < 16; ++cg) {
        const float4 zv = z[cg], wv = wsh[t][cg];
        acc = fmaf(zv.x, wv.x, acc);
        acc = fmaf(zv.y, wv.y, acc);
        acc = fmaf(zv.z, wv.z, acc);
        acc = fmaf(zv.w, wv.w, acc);
      }
    }
    dx[o] = acc;
  }
}

// ------------------------------------------------------------------ BN statistics
// part layout: [(j*C + c) * nblk + blk], j = 0 sum, 1 sumsq
// nbt (optional): BatchNorm num_batches_tracked of all three layers, incremented once
// fw != nullptr (BN1 folded into conv2, conv1_stats_fold_kernel): block c also writes conv2's folded
// weights fwo = fw * alpha_c for input channel c (fw: the [co][tap][ci] repack, 64 output channels)
// and ft[c][n] = sum_tap fw[n][tap][c] * beta'_c (double) for the folded bias
__global__ void __launch_bounds__(kT) bn_finalize_kernel(const float* part, int nblk, int C, double count,
                                                         const float* gamma, const float* beta, float* rm, float* rv,
                                                         float4* coef, int64_t* nbt = nullptr,
                                                         const float* fw = nullptr, float* fwo = nullptr,
                                                         double* ft = nullptr) {
  const int c = blockIdx.x;
  __shared__ float fab[2];
  if (nbt != nullptr && c == 0 && threadIdx.x < 3) nbt[threadIdx.x] += 1;
  double s = 0.0, ss = 0.0;
  for (int i = threadIdx.x; i < nblk; i += kT) {
    s += part[(int64_t)c * nblk + i];
    ss += part[((int64_t)C + c) * nblk + i];
  }
  __shared__ double red[2][kT / kWave];
  s = abd::wave_sum_d(s);
  ss = abd::wave_sum_d(ss);
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = s;
    red[1][threadIdx.x >> 6] = ss;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    s = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    ss = red[1][0] + red[1][1] + red[1][2] + red[1][3];
    const double mean = s / count;
    double var = ss / count - mean * mean;
    if (var < 0.0) var = 0.0;
    const float invstd = (float)(1.0 / sqrt(var + (double)kEps));
    const float alpha = gamma[c] * invstd;
    const float meanf = (float)mean;
    coef[c] = make_float4(meanf, invstd, alpha, beta[c] - meanf * alpha);
    fab[0] = alpha;
    fab[1] = beta[c] - meanf * alpha;
    if (rm) {
      const double mo = (double)kMomentum;
      rm[c] = (float)(mo * mean + (1.0 - mo) * (double)rm[c]);
      rv[c] = (float)(mo * (var * count / (count - 1.0)) + (1.0 - mo) * (double)rv[c]);
    }
  }
  if (fw == nullptr) return;
  __syncthreads();
  const float al = fab[0], bp = fab[1];
  for (int q = threadIdx.x; q < 64 * 4; q += kT) {  // q = co * 4 + tap
    const int64_t e = (int64_t)q * C + c;
    fwo[e] = fw[e] * al;
  }
  if (threadIdx.x < 64) {
    const int n = threadIdx.x;
    double acc = 0.0;
#pragma unroll
    for (int t = 0; t < 4; ++t) acc = fma((double)fw[(int64_t)(n * 4 + t) * C + c], (double)bp, acc);
    ft[(int64_t)c * 64 + n] = acc;
  }
}

// ------------------------------------------------------------------ per-utterance BatchNorm
// A train-mode forward at batch 1 (utils/daba_selection_tools.py:68-87 runs the untrained
// model that way, once per clip) normalises every utterance by its own statistics.  These
// kernels give a whole batch of such forwards at once: one block per utterance reduces
// sum / sumsq per channel (float per thread, double across threads) into coefficients
// coef[b * C + c] laid out like bn_finalize_kernel's (biased variance, eps 1e-5).
__device__ __forceinline__ float4 bn_coef_from_sums(double s, double ss, double count, float gamma, float beta) {
  const double mean = s / count;
  double var = ss / count - mean * mean;
  if (var < 0.0) var = 0.0;
  const float invstd = (float)(1.0 / sqrt(var + (double)kEps));
  const float alpha = gamma * invstd;
  const float meanf = (float)mean;
  return make_float4(meanf, invstd, alpha, beta - meanf * alpha);
}

// relu(conv1) statistics of utterance blockIdx.x (recomputed from x like conv1_stats_kernel)
__global__ void __launch_bounds__(kT) inst_conv1_coef_kernel(C1Args a, const float* gamma, const float* beta,
                                                             float4* coef) {
  __shared__ __attribute__((aligned(16))) float xs[(kR1 + 1) * 128];
  __shared__ double red[2][16][64];
  const int b = blockIdx.x;
  const int nbh = (a.g.H1 + a.rows - 1) / a.rows;
  const int c0 = (threadIdx.x & 15) * 4, pl = threadIdx.x >> 4;
  const C1W k = c1_weights(a, c0);
  float v[2][4] = {};
  for (int hb = 0; hb < nbh; ++hb) {
    const int h0 = hb * a.rows;
    stage_x(a, b, h0, xs);
    const int rows = min(a.rows, a.g.H1 - h0);
    for (int idx = pl; idx < rows * a.g.W1; idx += 16) {
      const int hl = idx / a.g.W1, w = idx - hl * a.g.W1;
      const float4 r = c1_at(xs, a.g.W0, hl, w, k);
      const float rr[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        v[0][q] += rr[q];
        v[1][q] = fmaf(rr[q], rr[q], v[1][q]);
      }
    }
    __syncthreads();  // xs is restaged by the next row chunk
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    red[0][pl][c0 + q] = (double)v[0][q];
    red[1][pl][c0 + q] = (double)v[1][q];
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    const int c = threadIdx.x;
    double s = 0.0, ss = 0.0;
    for (int l = 0; l < 16; ++l) {
      s += red[0][l][c];
      ss += red[1][l][c];
    }
    coef[(int64_t)b * 64 + c] = bn_coef_from_sums(s, ss, (double)a.g.H1 * a.g.W1, gamma[c], beta[c]);
  }
}

// statistics of an NHWC relu(conv) map (HW positions x C channels, C = 32 or 64) per utterance
__global__ void __launch_bounds__(kT) inst_coef_kernel(const float* __restrict__ r, int HW, int C,
                                                       const float* gamma, const float* beta, float4* coef) {
  __shared__ double red[2][1024];
  const int b = blockIdx.x;
  const int CG = C / 4, lanes = kT / CG;
  const int cg = threadIdx.x % CG, lane = threadIdx.x / CG;
  const float* src = r + (int64_t)b * HW * C + cg * 4;
  float v[2][4] = {};
  for (int pos = lane; pos < HW; pos += lanes) {
    const float4 x = *reinterpret_cast<const float4*>(src + (int64_t)pos * C);
    const float xx[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      v[0][q] += xx[q];
      v[1][q] = fmaf(xx[q], xx[q], v[1][q]);
    }
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    red[0][lane * C + cg * 4 + q] = (double)v[0][q];
    red[1][lane * C + cg * 4 + q] = (double)v[1][q];
  }
  __syncthreads();
  if (threadIdx.x < C) {
    const int c = threadIdx.x;
    double s = 0.0, ss = 0.0;
    for (int l = 0; l < lanes; ++l) {
      s += red[0][l * C + c];
      ss += red[1][l * C + c];
    }
    coef[(int64_t)b * C + c] = bn_coef_from_sums(s, ss, (double)HW, gamma[c], beta[c]);
  }
}

__global__ void bn_eval_coef_kernel(const float* gamma, const float* beta, const float* rm, const float* rv, int C,
                                    float4* coef) {
  const int c = threadIdx.x;
  if (c >= C) return;
  const float invstd = 1.0f / sqrtf(rv[c] + kEps);
  const float alpha = gamma[c] * invstd;
  coef[c] = make_float4(rm[c], invstd, alpha, beta[c] - rm[c] * alpha);
}

// eval BatchNorm backward as bn_dx coefficients: dx = alpha * dy (A = B = 0; the double
// product of two floats is exact, so the result is the correctly rounded float alpha * dy)
__global__ void bn_eval_bcoef_kernel(const float4* coef, int C, BCoef* bcoef) {
  const int c = threadIdx.x;
  if (c < C) bcoef[c] = BCoef{(double)coef[c].z, 0.0, 0.0, 0.0};
}

// backward finalize: s1 = sum dy (-> dbeta), s2 = sum dy*xhat (-> dgamma); coefficients for dx
__global__ void __launch_bounds__(kT) bn_bwd_finalize_kernel(const float* part, int nblk, int C, double count,
                                                             const float* gamma, const float4* coef, float* dgamma,
                                                             float* dbeta, BCoef* bcoef,
                                                             const float* guard_beta = nullptr) {
  // guard_beta != nullptr: the guarded fallback's finalize (runs only when a gamma is tiny)
  if (guard_beta != nullptr && !bn_any_tiny(gamma, guard_beta, C)) return;
  const int c = blockIdx.x;
  double s1 = 0.0, s2 = 0.0;
  for (int i = threadIdx.x; i < nblk; i += kT) {
    s1 += part[(int64_t)c * nblk + i];
    s2 += part[((int64_t)C + c) * nblk + i];
  }
  __shared__ double red[2][kT / kWave];
  s1 = abd::wave_sum_d(s1);
  s2 = abd::wave_sum_d(s2);
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = s1;
    red[1][threadIdx.x >> 6] = s2;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    s1 = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    s2 = red[1][0] + red[1][1] + red[1][2] + red[1][3];
    dgamma[c] = (float)s2;
    dbeta[c] = (float)s1;
    const double g = (double)gamma[c] * (double)coef[c].y, mdy = s1 / count, mdyx = s2 / count;
    const double mean = (double)coef[c].x, invstd = (double)coef[c].y;
    bcoef[c] = BCoef{g, g * (mdyx * invstd * mean - mdy), -g * mdyx * invstd, 0.0};
  }
}

// ------------------------------------------------------------------ synchronised BatchNorm
// The SyncBN path splits each finalize in two around the caller's all-reduce: this rank's
// double sums (the same fixed-tree reduction as the kernels above) -> SUM over ranks ->
// coefficients from the global sums and count.  On one rank the result is bit-identical to
// bn_finalize_kernel / bn_bwd_finalize_kernel.
__device__ __forceinline__ void block_pair_sum(const float* part, int nblk, int C, int c, double& s, double& ss) {
  s = 0.0;
  ss = 0.0;
  for (int i = threadIdx.x; i < nblk; i += kT) {
    s += part[(int64_t)c * nblk + i];
    ss += part[((int64_t)C + c) * nblk + i];
  }
  __shared__ double red[2][kT / kWave];
  s = abd::wave_sum_d(s);
  ss = abd::wave_sum_d(ss);
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = s;
    red[1][threadIdx.x >> 6] = ss;
  }
  __syncthreads();
  s = red[0][0] + red[0][1] + red[0][2] + red[0][3];
  ss = red[1][0] + red[1][1] + red[1][2] + red[1][3];
}

// out[c] = sum_c, out[C + c] = sum2_c, out[2C] = count; backward (dgamma != nullptr) also writes
// this rank's BN weight / bias gradient shares
__global__ void __launch_bounds__(kT) bn_local_sums_kernel(const float* part, int nblk, int C, double count,
                                                           double* out, float* dgamma, float* dbeta) {
  const int c = blockIdx.x;
  double s, ss;
  block_pair_sum(part, nblk, C, c, s, ss);
  if (threadIdx.x == 0) {
    out[c] = s;
    out[C + c] = ss;
    if (c == 0) out[2 * C] = count;
    if (dgamma) {
      dgamma[c] = (float)ss;
      dbeta[c] = (float)s;
    }
  }
}

__global__ void bn_sync_finalize_kernel(const double* sums, int C, const float* gamma, const float* beta, float* rm,
                                        float* rv, float4* coef, int64_t* nbt) {
  const int c = threadIdx.x;
  if (nbt != nullptr && c < 3) nbt[c] += 1;
  if (c >= C) return;
  const double count = sums[2 * C];
  const double mean = sums[c] / count;
  double var = sums[C + c] / count - mean * mean;
  if (var < 0.0) var = 0.0;
  const float invstd = (float)(1.0 / sqrt(var + (double)kEps));
  const float alpha = gamma[c] * invstd;
  const float meanf = (float)mean;
  coef[c] = make_float4(meanf, invstd, alpha, beta[c] - meanf * alpha);
  if (rm) {
    const double mo = (double)kMomentum;
    rm[c] = (float)(mo * mean + (1.0 - mo) * (double)rm[c]);
    rv[c] = (float)(mo * (var * count / (count - 1.0)) + (1.0 - mo) * (double)rv[c]);
  }
}

__global__ void bn_sync_bwd_finalize_kernel(const double* sums, int C, const float* gamma, const float4* coef,
                                            BCoef* bcoef) {
  const int c = threadIdx.x;
  if (c >= C) return;
  const double count = sums[2 * C], s1 = sums[c], s2 = sums[C + c];
  const double g = (double)gamma[c] * (double)coef[c].y, mdy = s1 / count, mdyx = s2 / count;
  const double mean = (double)coef[c].x, invstd = (double)coef[c].y;
  bcoef[c] = BCoef{g, g * (mdyx * invstd * mean - mdy), -g * mdyx * invstd, 0.0};
}

// BatchNorm backward statistics of the layer that feeds a 2x2 convolution without padding (BN1 ->
// pool1 -> conv2, BN2 -> pool2 -> conv3), from that convolution's weight / bias gradients instead
// of a pass over the activations.  Max-pool routes each pooled gradient dp to one element, whose
// normalised value is (p - beta) / gamma with p the stored BN+pool output (the conv's input), so
//   sum dy         = sum_pos dp(pos, c)
//   sum dy * xhat  = sum_pos dp(pos, c) * (p(pos, c) - beta_c) / gamma_c,
// and with dp = conv^T(dz) (every output o feeds input o + tap):
//   sum_pos dp(pos, c)             = sum_{n,t} W[n,c,t] * db[n]      (db = sum_o dz: the bias gradient)
//   sum_pos dp(pos, c) * p(pos, c) = sum_{n,t} W[n,c,t] * G[n,c,t]   (G: the conv weight gradient)
// -- a 4 * Cout-term contraction per channel, evaluated in double.  sums != nullptr (SyncBN): this
// rank's sums go to sums[c], sums[C + c], sums[2C] = count for the all-reduce; otherwise the backward
// coefficients are written as bn_bwd_finalize_kernel does.
// sum_{i < n} p[i * stride] in index order (the same rounding as a serial loop), loads issued
// 8 at a time so a thread keeps 8 HBM reads in flight
__device__ __forceinline__ float ordered_sum(const float* __restrict__ p, int64_t stride, int n) {
  float v = 0.0f;
  int i = 0;
  for (; i + 8 <= n; i += 8) {
    float t[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) t[j] = p[(int64_t)(i + j) * stride];
#pragma unroll
    for (int j = 0; j < 8; ++j) v += t[j];
  }
  for (; i < n; ++i) v += p[(int64_t)i * stride];
  return v;
}
// fold != nullptr (conv weight gradient over the folded source m, conv1_stats_fold_kernel): the gradient
// w.r.t. the conv's true input alpha m + beta' is alpha_ci G_m + beta'_ci db[n] (db: the bias gradient)
__device__ __forceinline__ float unfold_wgrad(float gm, const float4* fold, const float* db, int n, int ci) {
  return fold ? (float)fma((double)fold[ci].z, (double)gm, (double)fold[ci].w * (double)db[n]) : gm;
}

// block-reduce this thread's (s1, s2) share of channel c and write its BN backward outputs;
// folded: s2 is sum W (G_m - mean db), scaled by invstd instead of divided by gamma
__device__ __forceinline__ void bn_bwd_derived_finish(int c, double s1, double s2, int Cin, const float* gamma,
                                                      const float4* coef, double count, float* dgamma, float* dbeta,
                                                      BCoef* bcoef, double* sums, bool folded = false) {
  __shared__ double red[2][kT / kWave];
  s1 = abd::wave_sum_d(s1);
  s2 = abd::wave_sum_d(s2);
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = s1;
    red[1][threadIdx.x >> 6] = s2;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    s1 = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    s2 = red[1][0] + red[1][1] + red[1][2] + red[1][3];
    s2 = folded ? s2 * (double)coef[c].y : s2 / (double)gamma[c];
    dgamma[c] = (float)s2;
    dbeta[c] = (float)s1;
    if (sums) {
      sums[c] = s1;
      sums[Cin + c] = s2;
      if (c == 0) sums[2 * Cin] = count;
      return;
    }
    const double g = (double)gamma[c] * (double)coef[c].y, mdy = s1 / count, mdyx = s2 / count;
    const double mean = (double)coef[c].x, invstd = (double)coef[c].y;
    bcoef[c] = BCoef{g, g * (mdyx * invstd * mean - mdy), -g * mdyx * invstd, 0.0};
  }
}

// The next BatchNorm's derivation fused into the conv weight gradient's last slab reduction
// (slab_reduce_kernel with conv_cin = Cin): block c reduces the Cout * 4 entries of input channel c
// (the same ordered_sum, so the gradient is bit-identical), stores them, and contracts them with the
// conv weights: sum_(n,t) W[n,c,t] db[n] and sum W[n,c,t] (G[n,c,t] - beta_c db[n]).
// db (the conv bias gradient) is final before this launch.
struct DeriveArgs {
  const float4* fold;  // the weight gradient's source is folded (unfold_wgrad)
  const float* W;
  const float* db;
  const float* gamma;
  const float* beta;
  const float4* coef;
  double count;
  float* dgamma;
  float* dbeta;
  BCoef* bcoef;
};
__device__ __forceinline__ void slab_reduce_derive_body(const float* slab, int nslab, int Cout, int Ktot, int Cin,
                                                        float* out, const DeriveArgs& d) {
  const int c = blockIdx.x;
  const int64_t total = (int64_t)Cout * Ktot;
  // folded source m (BN1 fold): xhat of the pool-selected element is (m - mean) invstd, so
  //   sum dy xhat = invstd sum_{n,t} W (G_m - mean db)  -- no division by gamma
  // otherwise xhat = (p - beta) / gamma from the stored BN output p
  const double b = d.fold ? (double)d.coef[c].x : (double)d.beta[c];
  double s1 = 0.0, s2 = 0.0;
  for (int i = threadIdx.x; i < Cout * 4; i += kT) {
    const int n = i >> 2, t = i & 3;
    const float gm = ordered_sum(slab + (int64_t)n * Ktot + t * Cin + c, total, nslab);
    const float gv = unfold_wgrad(gm, d.fold, d.db, n, c);
    const int64_t o = ((int64_t)n * Cin + c) * 4 + t;
    out[o] = gv;
    const double w = (double)d.W[o], dbn = (double)d.db[n];
    s1 = fma(w, dbn, s1);
    s2 = fma(w, fma(-b, dbn, (double)(d.fold ? gm : gv)), s2);
  }
  bn_bwd_derived_finish(c, s1, s2, Cin, d.gamma, d.coef, d.count, d.dgamma, d.dbeta, d.bcoef, nullptr,
                        d.fold != nullptr);
}


// sum of nv partial columns: out[j][c] = sum_i part[(j*C + c)*nblk + i]
// conv1 mode (gw != nullptr): columns j*64 + c, j < 4 -> conv1.weight (c,1,kh,kw) = gw[c*4 + j], j = 4 -> gb[c]
__device__ __forceinline__ void partial_sum_body(const float* part, int nblk, float* out, float* gw, float* gb,
                                                 int col) {
  double s = 0.0;
  for (int i = threadIdx.x; i < nblk; i += kT) s += part[(int64_t)col * nblk + i];
  __shared__ double red[kT / kWave];
  s = abd::wave_sum_d(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float v = (float)(red[0] + red[1] + red[2] + red[3]);
    if (gw == nullptr) out[col] = v;
    else if (col < 4 * 64) gw[(col % 64) * 4 + col / 64] = v;
    else gb[col - 4 * 64] = v;
  }
}
__global__ void __launch_bounds__(kT) partial_sum_kernel(const float* part, int nblk, int ncols, float* out,
                                                         float* gw = nullptr, float* gb = nullptr) {
  partial_sum_body(part, nblk, out, gw, gb, blockIdx.x);
}

// a conv bias gradient (column sums of BN-backward partials) carried by another launch
struct BiasSum {
  const float* part = nullptr;
  int nblk = 0, ncols = 0;
  float* out = nullptr;
};

// ------------------------------------------------------------------ BN + max-pool (layers 2, 3)
struct PoolArgs {
  const float* r;  // NHWC (B,H,W,C) relu(conv) output
  int B, H, W, C, Ho, Wo, kh, kw, sh, sw, ph, pw;
  const float4* coef;
  int coef_bstride;  // 0: shared coefficients; C: per utterance (coef + b*C)
  float* out;      // NHWC pooled, or NCHW-flat (flat_n > 0)
  int flat_n;
  DropArgs drop;
  const float* dp;     // grad wrt pooled output (same layout as out)
  const BCoef* bcoef;
  float* dz;           // NHWC
  float* part;
  int nblk;
  // bn_bwd_apply_kernel: dzs != nullptr stores dz as dznp exact bf16 planes (plane stride dzplane)
  uint16_t* dzs;
  int64_t dzplane;
  int dznp;
};

// Pool windows tile the grid (kernel == stride for both pools), so the pool kernels run one
// thread per (window, 4 channels): the argmax is found once per window with int32 index
// math and float4 channel vectors, and the backward kernel writes every element of its
// window.  Windows are enumerated over the extended grid Hx x Wx that also covers rows /
// columns no real window reaches (pool3 drops the last conv3 row): those get dy = 0.
struct WinIdx {
  int b, ho, wo, cg;
};

__device__ __forceinline__ WinIdx win_index(int o, int CG, int Wx, int Hx) {
  WinIdx r;
  r.cg = o % CG;
  int q = o / CG;
  r.wo = q % Wx;
  q /= Wx;
  r.ho = q % Hx;
  r.b = q / Hx;
  return r;
}

__device__ __forceinline__ float f4get(const float4& v, int i) { return i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w; }
__device__ __forceinline__ void f4set(float4& v, int i, float x) {
  if (i == 0) v.x = x;
  else if (i == 1) v.y = x;
  else if (i == 2) v.z = x;
  else v.w = x;
}

// a window's (up to 2x2) elements for 4 channels: in[slot] = inside the window and the source grid
__device__ __forceinline__ void win_load(const PoolArgs& a, int b, int ho, int wo, int c0, bool valid, float4 (&rv)[4],
                                         bool (&in)[4]) {
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int slot = i * 2 + j;
      const int h = ho * a.sh - a.ph + i, w = wo * a.sw - a.pw + j;
      in[slot] = valid && (i < a.kh) && (j < a.kw) && h >= 0 && h < a.H && w >= 0 && w < a.W;
      rv[slot] = in[slot] ? *reinterpret_cast<const float4*>(a.r + ((b * a.H + h) * a.W + w) * a.C + c0)
                          : make_float4(0.f, 0.f, 0.f, 0.f);
    }
}
// argmax (first maximum in scan order, strict '>') of bn(r) over the loaded window, per channel;
// arg = window slot i*kw + j, -1 if empty
__device__ __forceinline__ void win_pick(const float4* cf, const float4 (&rv)[4], const bool (&in)[4],
                                         float (&best)[4], int (&arg)[4]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    best[q] = -INFINITY;
    arg[q] = -1;
  }
#pragma unroll
  for (int slot = 0; slot < 4; ++slot) {
    if (!in[slot]) continue;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float y = fmaf(cf[q].z, f4get(rv[slot], q), cf[q].w);
      if (y > best[q]) {
        best[q] = y;
        arg[q] = slot;
      }
    }
  }
}
__device__ __forceinline__ void win_argmax(const PoolArgs& a, int b, int ho, int wo, int c0, const float4* cf,
                                           float4 (&rv)[4], bool (&in)[4], float (&best)[4], int (&arg)[4]) {
  win_load(a, b, ho, wo, c0, true, rv, in);
  win_pick(cf, rv, in, best, arg);
}

__device__ __forceinline__ int pooled_index(const PoolArgs& a, int b, int ho, int wo, int c) {
  if (a.flat_n > 0) return b * a.flat_n + (c * a.Ho + ho) * a.Wo + wo;
  return ((b * a.Ho + ho) * a.Wo + wo) * a.C + c;
}

// the 4 channels' pooled gradients of one window: one float4 load in the NHWC layout (pool2),
// 4 strided loads in the NCHW-flat layout feeding fc1 (pool3)
__device__ __forceinline__ void load_dy4(const PoolArgs& a, int b, int ho, int wo, int c0, bool real, float (&dy)[4]) {
  if (!real) {
#pragma unroll
    for (int q = 0; q < 4; ++q) dy[q] = 0.0f;
  } else if (a.flat_n == 0) {
    const float4 d = *reinterpret_cast<const float4*>(a.dp + pooled_index(a, b, ho, wo, c0));
    dy[0] = d.x;
    dy[1] = d.y;
    dy[2] = d.z;
    dy[3] = d.w;
  } else {
#pragma unroll
    for (int q = 0; q < 4; ++q) dy[q] = a.dp[pooled_index(a, b, ho, wo, c0 + q)];
  }
}

__global__ void __launch_bounds__(kT) bn_pool_fwd_kernel(PoolArgs a) {
  const int CG = a.C / 4;
  const int total = a.B * a.Ho * a.Wo * CG;
  for (int o = blockIdx.x * kT + threadIdx.x; o < total; o += gridDim.x * kT) {
    const WinIdx wi = win_index(o, CG, a.Wo, a.Ho);
    const int c0 = wi.cg * 4;
    float4 cf[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) cf[q] = a.coef[wi.b * a.coef_bstride + c0 + q];
    float4 rv[4];
    bool in[4];
    float best[4];
    int arg[4];
    win_argmax(a, wi.b, wi.ho, wi.wo, c0, cf, rv, in, best, arg);
    if (a.flat_n > 0) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int oi = pooled_index(a, wi.b, wi.ho, wi.wo, c0 + q);
        a.out[oi] = drop_apply(a.drop, oi, best[q]);
      }
    } else {
      const int oi = pooled_index(a, wi.b, wi.ho, wi.wo, c0);
      float4 r;
#pragma unroll
      for (int q = 0; q < 4; ++q) f4set(r, q, drop_apply(a.drop, oi + q, best[q]));
      *reinterpret_cast<float4*>(a.out + oi) = r;
    }
  }
}

// BN backward sums over pooled outputs: sum dy, sum dy * xhat(r at the argmax)
__device__ __forceinline__ void bn_pool_bwd_stats_body(const PoolArgs& a);
__global__ void __launch_bounds__(kT) bn_pool_bwd_stats_kernel(PoolArgs a) { bn_pool_bwd_stats_body(a); }
// guarded fallback: BN2 / BN3 statistics from the activations when a gamma is tiny (bn_any_tiny)
struct PoolGuard {
  PoolArgs a;
  const float* gamma;
  const float* beta;
  GuardOut go;
  __device__ void operator()() const {
    if (!bn_any_tiny(gamma, beta, a.C)) return;
    bn_pool_bwd_stats_body(a);
    if (guard_last_block(go.ticket)) guard_finalize(a.part, a.nblk, a.C, gamma, go);
  }
};
struct NoGuard {
  __device__ void operator()() const {}
};
// BN3's guard in its own launch (the separate-backward path's fc1 data-gradient epilogue sums)
__global__ void __launch_bounds__(kT) bn_pool_bwd_stats_guard_kernel(PoolGuard gd) { gd(); }
// The derivation's launch carries the guard of the BatchNorm it derives (PoolGuard for BN2, C1Guard
// for BN1): one block per input channel in both, the guard's partials take gridDim.x slots, and its
// last block to arrive -- after every block's derived outputs are stored -- overwrites them.  Two
// launches fewer per step (r4_v1: 4.8 us each, all blocks exiting at the tininess test).
template <class Guard>
__global__ void __launch_bounds__(kT) slab_reduce_derive_kernel(const float* slab, int nslab, int Cout, int Ktot,
                                                                int Cin, float* out, DeriveArgs d, Guard gd) {
  slab_reduce_derive_body(slab, nslab, Cout, Ktot, Cin, out, d);
  gd();
}
__device__ __forceinline__ void bn_pool_bwd_stats_body(const PoolArgs& a) {
  const int CG = a.C / 4;
  const int total = a.B * a.Ho * a.Wo * CG;
  const int c0 = (threadIdx.x % CG) * 4;  // fixed per thread: grid stride is a multiple of CG
  float4 cf[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) cf[q] = a.coef[c0 + q];
  float v[2][4] = {};
  for (int o = blockIdx.x * kT + threadIdx.x; o < total; o += gridDim.x * kT) {
    const WinIdx wi = win_index(o, CG, a.Wo, a.Ho);
    float4 rv[4];
    bool in[4];
    float best[4];
    int arg[4];
    win_argmax(a, wi.b, wi.ho, wi.wo, c0, cf, rv, in, best, arg);
    float dyv[4];
    load_dy4(a, wi.b, wi.ho, wi.wo, c0, true, dyv);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float dy = dyv[q];
      float r = 0.0f;
#pragma unroll
      for (int slot = 0; slot < 4; ++slot) r = (arg[q] == slot) ? f4get(rv[slot], q) : r;
      v[0][q] += dy;
      v[1][q] = fmaf(dy, (r - cf[q].x) * cf[q].y, v[1][q]);
    }
  }
  cgroup_partials<2>(v, a.C, a.part, a.nblk, blockIdx.x);
}

// dz = relu'(r) * BN backward(dy scattered to the argmax) over every element of each
// (extended) window; bias-grad partials.  kApplyIT windows per thread per grid-stride round, all
// their loads (4 window rows + the pooled gradient each) issued before the first window's
// arithmetic: round 3's one-window body kept ~5 loads in flight per thread (0.069 ms, 5.3 TB/s).
#ifndef ABD_APPLY_IT  // measurement builds: windows per thread and round
#define ABD_APPLY_IT 2
#endif
constexpr int kApplyIT = ABD_APPLY_IT;
#ifndef ABD_BNA_OCC  // waves per SIMD bn_bwd_apply_kernel is register-budgeted for (measurement builds)
#define ABD_BNA_OCC 1
#endif
__global__ void __launch_bounds__(kT, ABD_BNA_OCC) bn_bwd_apply_kernel(PoolArgs a, int Hx, int Wx) {
  const int CG = a.C / 4;
  const int total = a.B * Hx * Wx * CG;
  const int c0 = (threadIdx.x % CG) * 4;  // fixed per thread: kT and the grid stride are multiples of CG
  float4 cf[4];
  BCoef bc[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    cf[q] = a.coef[c0 + q];
    bc[q] = a.bcoef[c0 + q];
  }
  float v[1][4] = {};
  for (int o0 = blockIdx.x * (kT * kApplyIT) + threadIdx.x; o0 < total; o0 += gridDim.x * (kT * kApplyIT)) {
    float4 rv[kApplyIT][4];
    bool in[kApplyIT][4];
    float dy[kApplyIT][4];
    WinIdx wi[kApplyIT];
    bool val[kApplyIT];
#pragma unroll
    for (int it = 0; it < kApplyIT; ++it) {
      const int o = o0 + it * kT;
      val[it] = o < total;
      wi[it] = win_index(val[it] ? o : 0, CG, Wx, Hx);
      const bool real = val[it] && wi[it].ho < a.Ho && wi[it].wo < a.Wo;
      win_load(a, wi[it].b, wi[it].ho, wi[it].wo, c0, val[it], rv[it], in[it]);
      load_dy4(a, wi[it].b, wi[it].ho, wi[it].wo, c0, real, dy[it]);
    }
#pragma unroll
    for (int it = 0; it < kApplyIT; ++it) {
      if (!val[it]) continue;
      const bool real = wi[it].ho < a.Ho && wi[it].wo < a.Wo;
      float best[4];
      int arg[4];
      win_pick(cf, rv[it], in[it], best, arg);
#pragma unroll
      for (int slot = 0; slot < 4; ++slot) {
        if (!in[it][slot]) continue;
        const int h = wi[it].ho * a.sh - a.ph + slot / 2, w = wi[it].wo * a.sw - a.pw + slot % 2;
        float4 dz;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float r = f4get(rv[it][slot], q);
          const float d = (real && arg[q] == slot) ? dy[it][q] : 0.0f;
          const float z = r > 0.0f ? bn_dx(d, r, cf[q], bc[q]) : 0.0f;
          f4set(dz, q, z);
          v[0][q] += z;
        }
        const int64_t e = ((int64_t)(wi[it].b * a.H + h) * a.W + w) * a.C + c0;
        if (a.dzs != nullptr) store_planes4(a.dzs, a.dzplane, e, dz, a.dznp);
        else *reinterpret_cast<float4*>(a.dz + e) = dz;
      }
    }
  }
  cgroup_partials<1>(v, a.C, a.part, a.nblk, blockIdx.x);
}

// ------------------------------------------------------------------ fp32 MFMA GEMMs
// NT: C[m][n] = sum_t sum_c A_t(m)[c] * Bw[n][t*Cs + c]; A_t(m) is the NHWC channel row
// of src at output position m shifted by tap t (zero outside the source grid).
enum { EPI_STORE = 0, EPI_CONV = 1, EPI_FC1 = 2, EPI_DROPGRAD = 3, EPI_PARTIAL = 4 };

struct NTArgs {
  const float* src;
  int Hs, Ws, Cs;
  int Ho, Wo, M;
  int taps;
  int dh[4], dw[4];
  const float* Bw;
  int ldb, N;
  const float* bias;
  float* out;
  int ldc;
  float* part;   // EPI_CONV stats partials [(j*N + n)*nblk + blk]
  int nblk;
  DropArgs drop;  // EPI_FC1 (dropout2 on relu(fc1)), EPI_DROPGRAD (dropout1 mask)
  int ksplit;     // EPI_PARTIAL: K chunks split over blockIdx.z, raw sums to out[z][M][ldc]
  // conv_ws_split_kernel, EPI_CONV: the source holds m with src = alpha_ci m + beta'_ci
  // (conv1_stats_fold_kernel); Bw holds the weights times alpha and fold_t[ci][n] the beta' terms of
  // the bias (bn_finalize_kernel), summed into it in the prologue
  const double* fold_t;
  // gemm_nt_kernel, EPI_DROPGRAD (fc1 data gradient): part != nullptr also forms BN3's backward sums
  // sum dy and sum dy * xhat, xhat = (p3d / scale - beta) / gamma over the stored dropout output p3d
  // (dropped elements have dy = 0), one partial pair per block; bias = beta, bn_period = columns per
  // channel (a multiple of NB)
  const float* bnp;
  const float* bn_gamma;
  int bn_period;
  // conv_ws_split_kernel<..., PA = true>: the A source as NP exact bf16 planes (plane-major, plane
  // stride splane elements, same NHWC indexing as src)
  const uint16_t* srcs;
  int64_t splane;
};

constexpr int kBM = 128, kKC = 32;

// MI = 32-row m-tiles per wave (block rows = 128 * MI): MI = 2 gives each wave a 2 x NJ
// accumulator grid, one LDS read per MFMA instead of 1.5 for NB = 64.
#ifndef ABD_NT_MINW
#define ABD_NT_MINW 1
#endif
#ifndef ABD_NT_DEBUG
#define ABD_NT_DEBUG 0
#endif
template <int NB, int EPI, int MI = 1, int KC = kKC>
__global__ void __launch_bounds__(kT, ABD_NT_MINW) gemm_nt_kernel(NTArgs a) {
  // KC-deep K chunks: QPR float4 per staged row, RP rows per pass of the block
  constexpr int LDA = KC + 1, QPR = KC / 4, RP = kT / QPR;
  constexpr int BM = kBM * MI, RPT = BM / RP;
  __shared__ float As[BM * LDA];
  __shared__ float Bs[NB * LDA];
  constexpr int NJ = NB / 32, NBL = NB * QPR / kT;
  static_assert(NBL >= 1 && (NB * QPR) % kT == 0, "B tile / thread mismatch");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n0 = blockIdx.y * NB;
  const int q4 = tid % QPR;
  const int mtiles = (a.M + BM - 1) / BM;
  float st[NJ][2];  // EPI_CONV: BN statistics over every tile this block handles
#pragma unroll
  for (int j = 0; j < NJ; ++j) st[j][0] = st[j][1] = 0.0f;
  // persistent when gridDim.x < mtiles (no tail wave of partially filled CUs)
  for (int tile = blockIdx.x; tile < mtiles; tile += gridDim.x) {
  const int m0 = tile * BM;
  int rb[RPT], rh[RPT], rw[RPT];
  bool rok[RPT];
#pragma unroll
  for (int i = 0; i < RPT; ++i) {
    const int m = m0 + tid / QPR + RP * i;
    rok[i] = m < a.M;
    const int mm = rok[i] ? m : 0;
    rb[i] = mm / (a.Ho * a.Wo);
    const int rem = mm - rb[i] * a.Ho * a.Wo;
    rh[i] = rem / a.Wo;
    rw[i] = rem - rh[i] * a.Wo;
  }
  const int cpt = a.Cs / KC;
  const int nch_all = a.taps * cpt;
  const int ks = a.ksplit > 1 ? a.ksplit : 1;
  const int ch_begin = (int)((int64_t)nch_all * blockIdx.z / ks);
  const int nch = (int)((int64_t)nch_all * (blockIdx.z + 1) / ks);
  float4 ra[RPT], rbv[NBL];
  auto load = [&](int ch) {
    const int t = ch / cpt;
    const int c0 = (ch - t * cpt) * KC;
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
      const int hs = rh[i] + a.dh[t], ws = rw[i] + a.dw[t];
      const bool ok = rok[i] && hs >= 0 && hs < a.Hs && ws >= 0 && ws < a.Ws;
      ra[i] = ok ? *reinterpret_cast<const float4*>(a.src + (((int64_t)rb[i] * a.Hs + hs) * a.Ws + ws) * a.Cs + c0 +
                                                    4 * q4)
                 : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int j = 0; j < NBL; ++j) {
      const int idx = tid + kT * j;
      const int n = idx / QPR, q = idx % QPR;
      rbv[j] = (n0 + n < a.N) ? *reinterpret_cast<const float4*>(a.Bw + (int64_t)(n0 + n) * a.ldb + t * a.Cs + c0 + 4 * q)
                              : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  f32x16 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

  load(ch_begin);
  for (int ch = ch_begin; ch < nch; ++ch) {
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
      float* d = As + (tid / QPR + RP * i) * LDA + 4 * q4;
      d[0] = ra[i].x;
      d[1] = ra[i].y;
      d[2] = ra[i].z;
      d[3] = ra[i].w;
    }
#pragma unroll
    for (int j = 0; j < NBL; ++j) {
      const int idx = tid + kT * j;
      float* d = Bs + (idx / QPR) * LDA + 4 * (idx % QPR);
      d[0] = rbv[j].x;
      d[1] = rbv[j].y;
      d[2] = rbv[j].z;
      d[3] = rbv[j].w;
    }
    __syncthreads();
#if ABD_NT_DEBUG == 1  // experiment: operands loaded once per tile (measures MFMA + LDS)
    if (ch == ch_begin && ch + 1 < nch) load(ch + 1);
#else
    if (ch + 1 < nch) load(ch + 1);
#endif
    const float* ap = As + (wave * 32 * MI + (lane & 31)) * LDA + (lane >> 5);
    const float* bp = Bs + (lane & 31) * LDA + (lane >> 5);
#pragma unroll
    for (int kk = 0; kk < KC; kk += 2) {
      float av[MI];
#pragma unroll
      for (int i = 0; i < MI; ++i) av[i] = ap[i * 32 * LDA + kk];
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const float bv = bp[j * 32 * LDA + kk];
#pragma unroll
        for (int i = 0; i < MI; ++i) {
#if ABD_NT_DEBUG == 2  // experiment: no MFMA (measures the load / LDS / barrier skeleton)
          acc[i][j][0] += av[i] * bv;
#else
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i], bv, acc[i][j], 0, 0, 0);
#endif
        }
      }
    }
    __syncthreads();
  }

  // epilogue: acc[i][j][r] -> row i*32 + (r&3) + 8(r>>2) + 4(lane>>5) of the wave's 32*MI, col lane&31 of tile j
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int col = n0 + j * 32 + (lane & 31);
    const bool cok = col < a.N;
    float bias = 0.0f;
    if constexpr (EPI == EPI_CONV || EPI == EPI_FC1) bias = cok ? a.bias[col] : 0.0f;
    float bnb = 0.0f, bngi = 0.0f, inv_scale = 0.0f;  // EPI_DROPGRAD + BN3 sums
    if constexpr (EPI == EPI_DROPGRAD) {
      if (a.part != nullptr) {
        const int ch = n0 / a.bn_period;
        bnb = a.bias[ch];
        bngi = 1.0f / a.bn_gamma[ch];
        inv_scale = 1.0f / a.drop.scale;
      }
    }
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = m0 + wave * 32 * MI + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      if (m >= a.M || !cok) continue;
      float v = acc[i][j][r];
      int64_t oi = (int64_t)m * a.ldc + col;
      if constexpr (EPI == EPI_PARTIAL) oi += (int64_t)blockIdx.z * a.M * a.ldc;
      if constexpr (EPI == EPI_CONV) {
        v = fmaxf(v + bias, 0.0f);
        st[j][0] += v;
        st[j][1] = fmaf(v, v, st[j][1]);
      } else if constexpr (EPI == EPI_FC1) {
        v = drop_apply(a.drop, oi, fmaxf(v + bias, 0.0f));
      } else if constexpr (EPI == EPI_DROPGRAD) {
        const bool k = a.drop.mask_in[oi] != 0;
        v = v * (k ? a.drop.scale : 0.0f);
        if (a.part != nullptr) {
          st[j][0] += v;
          st[j][1] = fmaf(v, (a.bnp[oi] * inv_scale - bnb) * bngi, st[j][1]);
        }
      }
      a.out[oi] = v;
    }
  }
  }  // tile loop
  if constexpr (EPI == EPI_CONV) {
    if (a.part == nullptr) return;
    // reduce over lane halves, then waves (through LDS)
    float* red = As;  // reuse: [4 waves][NB][2]
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      float s0 = st[j][0] + __shfl_xor(st[j][0], 32, 64);
      float s1 = st[j][1] + __shfl_xor(st[j][1], 32, 64);
      if (lane < 32) {
        red[(wave * NB + j * 32 + lane) * 2 + 0] = s0;
        red[(wave * NB + j * 32 + lane) * 2 + 1] = s1;
      }
    }
    __syncthreads();
    if (tid < NB && n0 + tid < a.N) {
      float s0 = 0.0f, s1 = 0.0f;
      for (int w = 0; w < 4; ++w) {
        s0 += red[(w * NB + tid) * 2 + 0];
        s1 += red[(w * NB + tid) * 2 + 1];
      }
      a.part[((int64_t)0 * a.N + n0 + tid) * a.nblk + blockIdx.x] = s0;
      a.part[((int64_t)1 * a.N + n0 + tid) * a.nblk + blockIdx.x] = s1;
    }
  }
  if constexpr (EPI == EPI_DROPGRAD && NJ == 1) {
    if (a.part == nullptr) return;
    // every column of the block belongs to one BN3 channel: one partial pair per block
    float* red = As;
    const float s0 = abd::wave_sum(st[0][0]), s1 = abd::wave_sum(st[0][1]);
    if (lane == 0) {
      red[wave * 2] = s0;
      red[wave * 2 + 1] = s1;
    }
    __syncthreads();
    if (tid == 0) {
      float t0 = 0.0f, t1 = 0.0f;
      for (int w = 0; w < kT / kWave; ++w) {
        t0 += red[w * 2];
        t1 += red[w * 2 + 1];
      }
      const int cpb = a.bn_period / NB, ch = n0 / a.bn_period, C = a.N / a.bn_period;
      const int slot = blockIdx.x * cpb + (int)(blockIdx.y % cpb), nb = gridDim.x * cpb;
      a.part[((int64_t)0 * C + ch) * nb + slot] = t0;
      a.part[((int64_t)1 * C + ch) * nb + slot] = t1;
    }
  }
}

// Weight-stationary 2x2 conv GEMM, 3-plane split (ABD_PREC_F32_SPLIT), Cs = N = 64, 4 taps, K = 256:
// conv2 forward (EPI_CONV: bias + ReLU + BN2 statistics) and data gradient (EPI_STORE).
//   * the whole weight operand (64 x 256, three exact bf16 planes, 101 KB with conflict-free
//     528-B rows) is staged into LDS ONCE per block: one persistent 512-thread block per CU;
//   * every wave owns a contiguous 1/(8 grid) share of the output rows and walks it in 64-row x
//     64-column tiles (2 x 2 v_mfma_f32_32x32x16_bf16 accumulators) with no block barrier:
//     its A fragments (8 consecutive channels of one tap-shifted source row per lane) come
//     straight from global memory through buffer loads (an out-of-grid tap reads zeros via the
//     descriptor's range check), are split into three bf16 planes in registers and fed to the
//     MFMAs; the K loop (4 taps x 4 channel groups of 16) is unrolled with loads two steps ahead.
// Same six-term product as gemm_nt_bf16_kernel<.., NP = 3> (a2b0 + a0b2 + a1b1 + a1b0 + a0b1 +
// a0b0 per 16-deep step), so the GEMM keeps fp32 accuracy; only the summation grouping differs.
// LDS weight rows are K + 8 bf16 (528 B at K = 256, 272 B at K = 128): the 16 lanes of a
// ds_read_b128 phase start 4 banks apart, conflict-free.
__device__ __forceinline__ void split3_x8(const float4& lo, const float4& hi, bf16x8* pl) {
  const f32x2 in[4] = {f32x2{lo.x, lo.y}, f32x2{lo.z, lo.w}, f32x2{hi.x, hi.y}, f32x2{hi.z, hi.w}};
  uint32_t u[3][4];
#pragma unroll
  for (int h = 0; h < 4; ++h) {
    f32x2 x = in[h];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const bf16x2 r = __builtin_convertvector(x, bf16x2);
      u[q][h] = __builtin_bit_cast(uint32_t, r);
      if (q < 2) {
        const f32x2 back = {__builtin_bit_cast(float, u[q][h] << 16), __builtin_bit_cast(float, u[q][h] & 0xffff0000u)};
        x -= back;  // exact: x - rne(x) fits in fp32
      }
    }
  }
#pragma unroll
  for (int q = 0; q < 3; ++q) pl[q] = __builtin_bit_cast(bf16x8, make_uint4(u[q][0], u[q][1], u[q][2], u[q][3]));
}

// NP = 1 (ABD_PREC_BF16): one plane, the operands rounded to bf16 (RNE) and ONE MFMA term a0 b0
// per step -- the same weight-stationary schedule at a sixth of the MFMA work.
__device__ __forceinline__ void round1_x8(const float4& lo, const float4& hi, bf16x8* pl) {
  const f32x2 in[4] = {f32x2{lo.x, lo.y}, f32x2{lo.z, lo.w}, f32x2{hi.x, hi.y}, f32x2{hi.z, hi.w}};
  uint32_t u[4];
#pragma unroll
  for (int h = 0; h < 4; ++h) u[h] = __builtin_bit_cast(uint32_t, __builtin_convertvector(in[h], bf16x2));
  pl[0] = __builtin_bit_cast(bf16x8, make_uint4(u[0], u[1], u[2], u[3]));
}
template <int NP>
__device__ __forceinline__ void planes_x8(const float4& lo, const float4& hi, bf16x8* pl) {
  if constexpr (NP == 3) split3_x8(lo, hi, pl);
  else round1_x8(lo, hi, pl);
}
// MFMA terms (a plane, b plane) of a product: six for the exact 3-plane split, one for bf16
template <int NP> struct Terms;
template <> struct Terms<3> {
  static constexpr int n = 6;
  static constexpr int A[6] = {2, 0, 1, 1, 0, 0}, B[6] = {0, 2, 1, 0, 1, 0};  // a2b0 a0b2 a1b1 a1b0 a0b1 a0b0
};
template <> struct Terms<1> {
  static constexpr int n = 1;
  static constexpr int A[1] = {0}, B[1] = {0};
};

// Template parameters: NJ = N / 32 output-channel tiles, CS = input channels (K = 4 CS), MI = 32-row
// A fragments per wave tile, PDW = K steps the A loads run ahead (register ring of PDW slots),
// WPB = waves per block, NP = bf16 planes per operand (3: f32split, 1: bf16).  conv2: <2, 64, 2>
// (101 KB of weights, one 8-wave block per CU); conv3 forward <1, 64, 1> and data gradient
// <2, 32, 1> (48 KB, smaller tiles for their 150-180 k rows).
// PA: the A source comes pre-split (NTArgs::srcs, store_planes4): NP 16-B plane loads per fragment
// replace the two fp32 loads and the in-register split.
// KO: K-step order.  false: tap-major (step ks = tap * CS/16 + channel group);  true: channel-
// group-major (ks = group * 4 + tap), so the four taps of one 16-channel group -- the same source
// rows shifted by (0,0) (0,1) (1,0) (1,1) -- are consecutive steps and re-read L1-resident lines
// (a wave's working set per group: ~46 rows x 64 B instead of ~46 rows x 256 B per tap).
template <int EPI, int NJ, int CS, int MI, int PDW, int WPB, int NP = 3, bool PA = false, bool KO = false>
__global__ void __launch_bounds__(WPB * 64, 1) conv_ws_split_kernel(NTArgs a) {
  constexpr int N = 32 * NJ, K = 4 * CS, LD = K + 8, KS = K / 16, TR = 32 * MI;
  static_assert(KS % PDW == 0, "a tile's K steps must be a whole number of ring turns");
  __shared__ __attribute__((aligned(16))) __bf16 Bs[NP][N * LD];
  __shared__ float red[WPB][N][2];
  __shared__ float bfold[N];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // ---- weights -> three exact bf16 planes, [plane][n][k] with k = tap * CS + channel
  for (int idx = tid; idx < N * (K / 8); idx += WPB * 64) {
    const int n = idx / (K / 8), k8 = (idx % (K / 8)) * 8;
    const float4 lo = *reinterpret_cast<const float4*>(a.Bw + (int64_t)n * a.ldb + k8);
    const float4 hi = *reinterpret_cast<const float4*>(a.Bw + (int64_t)n * a.ldb + k8 + 4);
    bf16x8 pl[NP];
    planes_x8<NP>(lo, hi, pl);
#pragma unroll
    for (int q = 0; q < NP; ++q) *reinterpret_cast<bf16x8*>(&Bs[q][n * LD + k8]) = pl[q];
  }
  if (EPI == EPI_CONV && a.fold_t != nullptr) {
    // folded bias b_n + sum_c ft[c][n] (bn_finalize_kernel), 8 lanes per output channel; a.Bw holds
    // the folded weights
    for (int q = tid; q < N * 8; q += WPB * 64) {
      const int n = q / 8, part = q % 8;
      double acc = 0.0;
#pragma unroll
      for (int c = 0; c < CS / 8; ++c) acc += a.fold_t[(int64_t)(part * (CS / 8) + c) * N + n];
#pragma unroll
      for (int o = 4; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
      if (part == 0) bfold[n] = (float)(acc + (double)a.bias[n]);
    }
  }
  __syncthreads();
  // ---- this wave's rows [r_lo, r_hi): an even split of M over every wave of the grid
  const int64_t W = (int64_t)gridDim.x * WPB;
  const int64_t g = (int64_t)blockIdx.x * WPB + __builtin_amdgcn_readfirstlane(wave);  // wave-uniform (SGPR)
  const int r_lo = (int)(a.M * g / W), r_hi = (int)(a.M * (g + 1) / W);
  const int HoWo = a.Ho * a.Wo;
  constexpr uint32_t EB = PA ? 2u : 4u;  // bytes per source element
  const __amdgpu_buffer_rsrc_t arsrc =
      PA ? __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(a.srcs), 0,
                                             (int)std::min<int64_t>((int64_t)NP * a.splane * 2, 0x7ffffff0), 0x00020000)
         : __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.src), 0,
                                             (int)std::min<int64_t>((int64_t)a.Hs * a.Ws * CS * 4 * (a.M / HoWo),
                                                                    0x7ffffff0),
                                             0x00020000);
  const uint32_t pstride = PA ? (uint32_t)(a.splane * 2) : 0u;  // bytes between planes
  constexpr uint32_t kOOB = 0x80000000u;
  const int kq = 8 * (lane >> 5);  // this lane's 8 channels / k inside a 16-deep step
  float st[NJ][2];
  float bias[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    st[j][0] = st[j][1] = 0.0f;
    bias[j] = 0.0f;
    if constexpr (EPI == EPI_CONV) bias[j] = a.fold_t != nullptr ? bfold[32 * j + (lane & 31)] : a.bias[32 * j + (lane & 31)];
  }
  // One continuous stream of K steps over all of this wave's tiles (KS steps per TR-row tile):
  // the A loads run PDW steps ahead ACROSS tile boundaries, so the pipeline never drains at a
  // tile's epilogue.  li: byte offsets (tap 0, channel kq) + tap-validity masks of the MI A rows
  // of the tile the loads are in.
  struct RowInfo {
    uint32_t roff[MI], tm[MI];
  };
  auto rows_of = [&](int m0) {
    RowInfo r;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int m = m0 + 32 * i + (lane & 31);
      const bool ok = m < r_hi;
      const int mm = ok ? m : r_lo;
      const int b = mm / HoWo, rem = mm - b * HoWo;
      const int h = rem / a.Wo, w = rem - h * a.Wo;
      r.roff[i] = (uint32_t)((((int64_t)b * a.Hs + h) * a.Ws + w) * CS + kq) * EB;
      uint32_t mk = 0;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int hs = h + a.dh[t], ws = w + a.dw[t];
        if (ok && hs >= 0 && hs < a.Hs && ws >= 0 && ws < a.Ws) mk |= 1u << t;
      }
      r.tm[i] = mk;
    }
    return r;
  };
  const int ntiles = (r_hi - r_lo + TR - 1) / TR;
  // this wave's output rows [r_lo, r_hi) as one buffer (ldc == N checked by the launcher)
  const __amdgpu_buffer_rsrc_t orsrc = __builtin_amdgcn_make_buffer_rsrc(
      a.out + (int64_t)r_lo * N, 0, (r_hi - r_lo) * N * 4, 0x00020000);
  if (ntiles > 0) {
    constexpr int NR = PA ? NP : 2;  // 16-B registers per A fragment: fp32 lo/hi, or the planes
    uint4 raw[PDW][MI][NR];  // [slot][i][.]: slot ks % PDW, refilled with the step PDW later once used
    auto load = [&](const RowInfo& li, int ks, uint4 (&r)[MI][NR]) {
      const int t = KO ? ks % 4 : ks / (CS / 16), c16 = KO ? ks / 4 : ks % (CS / 16);
      const uint32_t tofs = (uint32_t)(((a.dh[t] * a.Ws + a.dw[t]) * CS + c16 * 16) * EB);
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const uint32_t off = ((li.tm[i] >> t) & 1u) ? li.roff[i] + tofs : kOOB;
#pragma unroll
        for (int q = 0; q < NR; ++q)
          r[i][q] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                                  arsrc, (int)(off + (PA ? q * pstride : 16u * q)), 0, 0));
      }
    };
    f32x16 acc[MI][NJ];
    // B fragments of a K step (identical for every tile), double-buffered: step ks's MFMAs use
    // bvs[ks & 1] while the reads for step ks + 1 are in flight (LDS latency off the MFMA path)
    bf16x8 bvs[2][NJ][NP];
    auto load_b = [&](int ks, bf16x8 (&bv)[NJ][NP]) {
      const int kb = (KO ? (ks % 4) * CS + (ks / 4) * 16 : ks * 16) + kq;  // k = tap * CS + channel
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int q = 0; q < NP; ++q)
          bv[j][q] = *reinterpret_cast<const bf16x8*>(&Bs[q][(32 * j + (lane & 31)) * LD + kb]);
    };
    auto step = [&](int ks, uint4 (&r)[MI][NR], const RowInfo& li, int lks) {
      bf16x8 av[MI][NP];
      bf16x8 (&bv)[NJ][NP] = bvs[ks & 1];
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        if constexpr (PA) {
#pragma unroll
          for (int q = 0; q < NP; ++q) av[i][q] = __builtin_bit_cast(bf16x8, r[i][PA ? q : 0]);
        } else {
          planes_x8<NP>(__builtin_bit_cast(float4, r[i][0]), __builtin_bit_cast(float4, r[i][NR - 1]), av[i]);
        }
      }
      // keep the refill behind the split: hoisted above it, the loads need fresh registers and
      // the loop-carried slot turns into copies that wait for the loads (a synchronous prefetch)
      __builtin_amdgcn_sched_barrier(0);
      load(li, lks, r);  // unconditional: a conditional refill is a phi (copies)
      load_b((ks + 1) % KS, bvs[(ks + 1) & 1]);
      // term-major: independent accumulator chains between dependent MFMAs
#pragma unroll
      for (int term = 0; term < Terms<NP>::n; ++term)
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[i][Terms<NP>::A[term]], bv[j][Terms<NP>::B[term]],
                                                                acc[i][j], 0, 0, 0);
    };
    RowInfo li = rows_of(r_lo);
    // in step order: the scheduler otherwise issues them last-slot-first, slot 0 becomes the
    // youngest load on loop entry, and the waitcnt merged at the tile-loop header (entry edge
    // vs back edge) drains every load in flight at the start of EVERY tile
#pragma unroll
    for (int sl = 0; sl < PDW; ++sl) {
      load(li, sl, raw[sl]);
      __builtin_amdgcn_sched_barrier(0);
    }
    load_b(0, bvs[0]);
#pragma unroll 1
    for (int tile = 0; tile < ntiles; ++tile) {
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;
      // KS unrolled K steps; the last PDW load the next tile's first PDW steps (past the last
      // tile they re-read this tile's final step: harmless, never consumed)
      const bool more = tile + 1 < ntiles;
      const RowInfo cur = li;
      li = rows_of(r_lo + TR * (more ? tile + 1 : tile));  // unconditional (no branch in the stream)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        if (ks + PDW < KS) step(ks, raw[ks % PDW], cur, ks + PDW);
        else step(ks, raw[ks % PDW], li, more ? ks + PDW - KS : KS - 1);
      }
      // branch-free epilogue: rows past r_hi store to an out-of-range buffer offset (dropped by
      // the range check), so the waitcnt pass can count the stores and keep the loads in flight
      const int m0 = r_lo + TR * tile;
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          const bool ok = m < r_hi;
          const uint32_t ob = ok ? (uint32_t)((m - r_lo) * N + (lane & 31)) * 4u : kOOB;
#pragma unroll
          for (int j = 0; j < NJ; ++j) {
            float v = acc[i][j][r];
            if constexpr (EPI == EPI_CONV) {
              v = fmaxf(v + bias[j], 0.0f);
              const float vs = ok ? v : 0.0f;
              st[j][0] += vs;
              st[j][1] = fmaf(vs, vs, st[j][1]);
            }
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), orsrc, (int)(ob + 128u * j), 0, 0);
          }
        }
    }
  }
  if constexpr (EPI == EPI_CONV) {
    if (a.part == nullptr) return;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const float s0 = st[j][0] + __shfl_xor(st[j][0], 32, 64);
      const float s1 = st[j][1] + __shfl_xor(st[j][1], 32, 64);
      if (lane < 32) {
        red[wave][32 * j + lane][0] = s0;
        red[wave][32 * j + lane][1] = s1;
      }
    }
    __syncthreads();
    if (tid < N) {
      float s0 = 0.0f, s1 = 0.0f;
      for (int w = 0; w < WPB; ++w) {
        s0 += red[w][tid][0];
        s1 += red[w][tid][1];
      }
      a.part[((int64_t)0 * a.N + tid) * a.nblk + blockIdx.x] = s0;
      a.part[((int64_t)1 * a.N + tid) * a.nblk + blockIdx.x] = s1;
    }
  }
}

// Weight-stationary conv2 FORWARD with the A operand staged through LDS by DMA (ABD_WS_DMA=1,
// A/B knob).  Same product, tiles, epilogue and summation order as conv_ws_split_kernel<EPI_CONV,
// 2, 64, 1, .., KO = true>; only how the A fragments reach the registers differs.  The direct path
// loads each lane's 32 B of its own output row from global memory: the four lanes of a quad (the
// unit the texture address stage processes together) touch four NHWC rows 256 B apart -- four L1
// lines per quad, ~58 tag lookups per 1-KB load, TA stalled on the L1 in 35 % of the kernel's
// cycles.  Here, per 16-channel group, a wave DMAs the tile's whole source span (the 32 output
// rows' positions plus the taps' +1 / +Ws / +Ws+1 shifts: <= 64 positions x 64 B) into its own
// LDS buffer with `buffer_load_dwordx4 ... lds`, four lanes per position -- one line per quad --
// and the four taps read their fragments from it (2 ds_read_b128 per lane and tap; the 16-B chunk
// is XOR-swizzled by (position >> 2) & 3 so the 16 lanes of a read phase hit distinct banks).
// Forward taps only ((0,0),(0,1),(1,0),(1,1) with Hs = Ho + 1, Ws = Wo + 1: every tap inside the
// source), checked by the launcher.  No block barrier in the loop: each wave waits for its own DMA.
#ifndef ABD_DMA_TRIM
#define ABD_DMA_TRIM 1
#endif
constexpr int kDmaSpan = 64;  // staged positions per tile and group (span <= 31 + 3 + 14 + Ws + 1)
#ifndef ABD_DMA_ABL  // ablation bits (measurement builds only; results wrong): 1 no epilogue stores,
#define ABD_DMA_ABL 0  // 2 no DMA waits, 4 no DMA, 8 no A split
#endif
// PA (bf16 mode's plane operands, NP = 1): the A source is the producer's bf16 plane (NTArgs::srcs,
// store_planes4), staged as 32 B per position and group (two lanes per position, 32 positions per
// DMA instruction: half the instructions and bytes of the fp32 staging), the 16-B half a lane reads
// XOR-swizzled by (position >> 3) & 1, and read straight into the MFMA operand (no split).
template <int EPI, int NP, int NJ = 2, bool PA = false>
__global__ void __launch_bounds__(512, 1) conv_ws_dma_kernel(NTArgs a) {
  static_assert(!PA || NP == 1, "pre-split staging: the single bf16 plane");
  constexpr int CS = 64, N = 32 * NJ, K = 4 * CS, LD = K + 8, WPB = 8, G = CS / 16;
  constexpr int PPI = PA ? 32 : 16;  // staged positions per DMA instruction
  __shared__ __attribute__((aligned(16))) __bf16 Bs[NP][N * LD];
  __shared__ __attribute__((aligned(16))) float stage[WPB][kDmaSpan * 16];
  __shared__ float red[WPB][N][2];
  __shared__ float bfold[N];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int idx = tid; idx < N * (K / 8); idx += WPB * 64) {
    const int n = idx / (K / 8), k8 = (idx % (K / 8)) * 8;
    const float4 lo = *reinterpret_cast<const float4*>(a.Bw + (int64_t)n * a.ldb + k8);
    const float4 hi = *reinterpret_cast<const float4*>(a.Bw + (int64_t)n * a.ldb + k8 + 4);
    bf16x8 pl[NP];
    planes_x8<NP>(lo, hi, pl);
#pragma unroll
    for (int q = 0; q < NP; ++q) *reinterpret_cast<bf16x8*>(&Bs[q][n * LD + k8]) = pl[q];
  }
  if (EPI == EPI_CONV && a.fold_t != nullptr) {
    for (int q = tid; q < N * 8; q += WPB * 64) {
      const int n = q / 8, part = q % 8;
      double acc = 0.0;
#pragma unroll
      for (int c = 0; c < CS / 8; ++c) acc += a.fold_t[(int64_t)(part * (CS / 8) + c) * N + n];
#pragma unroll
      for (int o = 4; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
      if (part == 0) bfold[n] = (float)(acc + (double)a.bias[n]);
    }
  }
  __syncthreads();
  const int64_t W = (int64_t)gridDim.x * WPB;
  const int64_t g = (int64_t)blockIdx.x * WPB + __builtin_amdgcn_readfirstlane(wave);
  const int r_lo = (int)(a.M * g / W), r_hi = (int)(a.M * (g + 1) / W);
  const int HoWo = a.Ho * a.Wo;
  const int npos = a.Hs * a.Ws * (a.M / HoWo);  // source positions
  // taps as linear source offsets; the data gradient's leave the source grid at its edges (masked)
  int tofs[4], tmin = 0, tmax = 0;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    tofs[t] = a.dh[t] * a.Ws + a.dw[t];
    tmin = min(tmin, tofs[t]);
    tmax = max(tmax, tofs[t]);
  }
  const __amdgpu_buffer_rsrc_t arsrc =
      PA ? __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(a.srcs), 0,
                                             (int)std::min<int64_t>((int64_t)npos * CS * 2, 0x7ffffff0), 0x00020000)
         : __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.src), 0,
                                             (int)std::min<int64_t>((int64_t)npos * CS * 4, 0x7ffffff0), 0x00020000);
  const int kq = 8 * (lane >> 5);
  float st[NJ][2];
  float bias[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    st[j][0] = st[j][1] = 0.0f;
    bias[j] = 0.0f;
    if constexpr (EPI == EPI_CONV) bias[j] = a.fold_t != nullptr ? bfold[32 * j + (lane & 31)] : a.bias[32 * j + (lane & 31)];
  }
  // the wave index as a scalar: the DMA's LDS base (M0) is then plain scalar arithmetic, not a
  // v_readfirstlane of a per-lane address before every DMA instruction
  float* sw = stage[__builtin_amdgcn_readfirstlane(wave)];
  // DMA of channel group cg for the span starting at source position p0: instruction i, lane l ->
  // position 16 i + l / 4, LDS slot l % 4 holds global chunk (l % 4) ^ ((pos >> 2) & 3)
  // only the 16-position blocks the tile reads (need: wave-uniform; typically 48 of the 64 slots)
  auto dma1 = [&](int p0, int cg, int need, int i) {
    if (ABD_DMA_ABL & 4) return;
    if (i > 0 && PPI * i >= need) return;
    uint32_t off;
    if constexpr (PA) {  // PA: instruction i, lane l -> position 32 i + l / 2, half (l % 2) ^ ((pos >> 3) & 1)
      const int pos = 32 * i + (lane >> 1);
      const int half = (lane & 1) ^ ((pos >> 3) & 1);
      off = (uint32_t)(((p0 + pos) * CS + cg * 16 + half * 8) * 2);
    } else {
      const int pos = 16 * i + (lane >> 2);
      const int chunk = (lane & 3) ^ ((pos >> 2) & 3);
      off = (uint32_t)(((p0 + pos) * CS + cg * 16 + chunk * 4) * 4);  // past the end: zeros
    }
    __builtin_amdgcn_raw_ptr_buffer_load_lds(arsrc, (__attribute__((address_space(3))) void*)(sw + i * 256), 16,
                                             (int)off, 0, 0, 0);
  };
  auto dma = [&](int p0, int cg, int need) {
#pragma unroll
    for (int i = 0; i < kDmaSpan / PPI; ++i) dma1(p0, cg, need, i);
  };
  const int ntiles = (r_hi - r_lo + 31) / 32;
  const __amdgpu_buffer_rsrc_t orsrc = __builtin_amdgcn_make_buffer_rsrc(
      a.out + (int64_t)r_lo * N, 0, (r_hi - r_lo) * N * 4, 0x00020000);
  constexpr uint32_t kOOB = 0x80000000u;
  auto src_of = [&](int m) {
    const int b = m / HoWo, rem = m - b * HoWo;
    const int h = rem / a.Wo, w = rem - h * a.Wo;
    return (b * a.Hs + h) * a.Ws + w;
  };
  // tap-validity bits of output row m (h + dh in [0, Hs), w + dw in [0, Ws))
  auto taps_of = [&](int m) {
    const int b = m / HoWo, rem = m - b * HoWo;
    const int h = rem / a.Wo, w = rem - h * a.Wo;
    uint32_t mk = 0;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int hs = h + a.dh[t], ws = w + a.dw[t];
      if (hs >= 0 && hs < a.Hs && ws >= 0 && ws < a.Ws) mk |= 1u << t;
    }
    return mk;
  };
  // first staged position of the tile starting at m: the rows' minimum source index (a source
  // image boundary can step it back) plus the most negative tap
  // and the number of staged positions its rows' taps reach (ABD_DMA_TRIM=0: always kDmaSpan)
  auto span_base = [&](int m, int& need) {
    const int s0 = src_of(min(m + (lane & 31), r_hi - 1));
    int v = s0, u = s0;
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) {
      v = min(v, __shfl_xor(v, o, 64));
      u = max(u, __shfl_xor(u, o, 64));
    }
    const int base = __builtin_amdgcn_readfirstlane(v) + tmin;
    need = ABD_DMA_TRIM ? __builtin_amdgcn_readfirstlane(u) + tmax + 1 - base : kDmaSpan;
    return base;
  };
  // B fragments of step (cg, t), double-buffered one step ahead (the LDS latency off the MFMA path)
  bf16x8 bvs[2][NJ][NP];
  auto load_b = [&](int cg, int t, bf16x8 (&bv)[NJ][NP]) {
    const int kb = t * CS + cg * 16 + kq;  // KO order: step = cg * 4 + t
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int q = 0; q < NP; ++q) bv[j][q] = *reinterpret_cast<const bf16x8*>(&Bs[q][(32 * j + (lane & 31)) * LD + kb]);
  };
  int need = kDmaSpan, needn = kDmaSpan;
  int p0 = ntiles > 0 ? span_base(r_lo, need) : 0;
  if (ntiles > 0) dma(p0, 0, need);  // the first tile's group 0; later tiles' group 0 is issued a group ahead
  load_b(0, 0, bvs[0]);
#pragma unroll 1
  for (int tile = 0; tile < ntiles; ++tile) {
    const int m0 = r_lo + 32 * tile;
    const int mr = min(m0 + (lane & 31), r_hi - 1);
    const int prow = src_of(mr) - p0;  // this lane's row inside the span
    const uint32_t tm = taps_of(mr);
    const bool more = tile + 1 < ntiles;
    const int p0n = span_base(more ? m0 + 32 : m0, needn);
    f32x16 acc[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[j][r] = 0.0f;
#pragma unroll
    for (int cg = 0; cg < G; ++cg) {
      // this wave's DMA of group cg has landed; group 0 of a later tile was issued before the
      // previous tile's 16 * NJ epilogue stores, which may stay in flight (vmcnt counts in issue
      // order).  The count must equal the stores per tile exactly: a larger one lets the DMA
      // of group 0 still be in flight (NJ = 1 issues 16 stores: vmcnt(32) would never wait).
      static_assert(NJ == 1 || NJ == 2, "epilogue store count per tile is 16 * NJ");
      if (ABD_DMA_ABL & 6) {
      } else if (cg == 0 && tile > 0) {
        if constexpr (NJ == 2) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      uint4 raw[4][2];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int pos = min(max(prow + tofs[t], 0), kDmaSpan - 1);  // an invalid tap's position is clamped
        if constexpr (PA) {
          const char* rowp = reinterpret_cast<const char*>(sw) + pos * 32;
          raw[t][0] = raw[t][1] = *reinterpret_cast<const uint4*>(rowp + (((lane >> 5) ^ ((pos >> 3) & 1)) * 16));
        } else {
          const int sx = (pos >> 2) & 3;
          const float* rowp = sw + pos * 16;
          raw[t][0] = *reinterpret_cast<const uint4*>(rowp + (((2 * (lane >> 5)) ^ sx) * 4));
          raw[t][1] = *reinterpret_cast<const uint4*>(rowp + (((2 * (lane >> 5) + 1) ^ sx) * 4));
        }
        if constexpr (EPI != EPI_CONV) {  // and zeroed (forward taps never leave the grid)
          if (!((tm >> t) & 1u)) raw[t][0] = raw[t][1] = make_uint4(0u, 0u, 0u, 0u);
        }
      }
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        if (t == 1) {
          // every lane's reads of group cg are complete (tap 0's MFMAs are issued: the wait costs
          // little) before the buffer is refilled: with group cg + 1, or after the last group with
          // the next tile's group 0
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
        if (t == 1) {
          if (cg + 1 < G) dma(p0, cg + 1, need);
          else if (more) dma(p0n, 0, needn);
        }
        const int s = cg * 4 + t;
        // next step's B fragments (past the tile's last step: the next tile's first)
        load_b(((s + 1) % (4 * G)) / 4, (s + 1) % 4, bvs[(s + 1) & 1]);
        bf16x8 av[NP];
        if constexpr (PA) {
          av[0] = __builtin_bit_cast(bf16x8, raw[t][0]);
        } else if (ABD_DMA_ABL & 8) {
#pragma unroll
          for (int q = 0; q < NP; ++q) av[q] = __builtin_bit_cast(bf16x8, q == 1 ? raw[t][1] : raw[t][0]);
        } else {
          planes_x8<NP>(__builtin_bit_cast(float4, raw[t][0]), __builtin_bit_cast(float4, raw[t][1]), av);
        }
        bf16x8 (&bv)[NJ][NP] = bvs[s & 1];
#pragma unroll
        for (int term = 0; term < Terms<NP>::n; ++term)
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[Terms<NP>::A[term]], bv[j][Terms<NP>::B[term]], acc[j], 0, 0, 0);
      }
    }
    p0 = p0n;
    need = needn;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = m0 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      const bool ok = m < r_hi;
      const uint32_t ob = ok ? (uint32_t)((m - r_lo) * N + (lane & 31)) * 4u : kOOB;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        float v = acc[j][r];
        if constexpr (EPI == EPI_CONV) {
          v = fmaxf(v + bias[j], 0.0f);
          const float vs = ok ? v : 0.0f;
          st[j][0] += vs;
          st[j][1] = fmaf(vs, vs, st[j][1]);
        }
        if ((ABD_DMA_ABL & 1) && __builtin_bit_cast(uint32_t, v) != 0x7fc00001u) continue;
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), orsrc, (int)(ob + 128u * j), 0, 0);
      }
    }
  }
  if (EPI != EPI_CONV || a.part == nullptr) return;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const float s0 = st[j][0] + __shfl_xor(st[j][0], 32, 64);
    const float s1 = st[j][1] + __shfl_xor(st[j][1], 32, 64);
    if (lane < 32) {
      red[wave][32 * j + lane][0] = s0;
      red[wave][32 * j + lane][1] = s1;
    }
  }
  __syncthreads();
  if (tid < N) {
    float s0 = 0.0f, s1 = 0.0f;
    for (int w = 0; w < WPB; ++w) {
      s0 += red[w][tid][0];
      s1 += red[w][tid][1];
    }
    a.part[((int64_t)0 * a.N + tid) * a.nblk + blockIdx.x] = s0;
    a.part[((int64_t)1 * a.N + tid) * a.nblk + blockIdx.x] = s1;
  }
}

// Weight-stationary conv2 GEMM in f32split with the A operand staged PRE-SPLIT (round 4).
// conv_ws_dma_kernel<EPI, 3> splits every (row, tap) fragment of a 16-channel group after reading it
// from its fp32 stage -- 32 rows x 4 taps of splits for ~48 distinct positions, 2.7x redundant --
// and its LDS-DMA pieces cost 60-185 issue cycles each beside MFMAs (MI355X_MICROARCH.md); with the
// split's VALU they crowd the issue slots the MFMAs need (forward ablation: no DMA issue 0.131 ->
// 0.083 ms, no split -> 0.106).  Here each wave loads the group's span with plain buffer loads one
// group ahead (units of 8 channels x 1 position, 32 B, <= 2 per lane), splits each unit ONCE into the
// three exact bf16 planes, writes them to its own LDS stage (kPreRow = 56 bf16 = 112 B per position:
// 3 planes x 32 B + 16 B pad, 7 bank groups apart, so 16 consecutive positions hit 16 distinct
// groups), and the taps read the planes straight into the MFMA operands (3 ds_read_b128 per tap).
// Same tiles, K order, products, summation order and epilogue as conv_ws_dma_kernel<EPI, 3>.
// LDS: 101,376 (weights) + 57,344 (stages; the data gradient's 58,240 with a zero position per
// wave) + 256 = 158,976 / 159,872 B of the CU's 163,840 (the statistics' per-wave partials reuse
// each wave's stage after its last tile).
// Ablations (-DABD_PRE_ABL, results discarded; forward / data gradient, ms): 0.121 / 0.123 base; no
// stage writes 0.099 / 0.093; no split 0.103 / 0.100; no loads 0.112 / 0.114; no output stores
// 0.117 / 0.110; no MFMAs 0.093 / 0.088 -- the MFMAs are not what bounds it.
constexpr int kPreRow = 56;
#ifndef ABD_PRE_ABL  // measurement builds (results discarded): 1 no stage writes, 2 no loads, 4 no MFMAs,
#define ABD_PRE_ABL 0  // 8 no output stores, 16 no split (raw bits written to the planes)
#endif
#ifndef ABD_WS_PRE  // measurement builds: 0 conv_ws_dma_kernel<EPI, 3> everywhere, 1 the conv2 forward,
#define ABD_WS_PRE 3  // 2 + the conv2 data gradient (default ABD_WS_DMA=1 too), 3 + the conv3 forward
#endif
template <int EPI, int NJ = 2>
__global__ void __launch_bounds__(512, 1) conv_ws_pre_kernel(NTArgs a) {
  constexpr int NP = 3, CS = 64, N = 32 * NJ, K = 4 * CS, LD = K + 8, WPB = 8, G = CS / 16;
  __shared__ __attribute__((aligned(16))) __bf16 Bs[NP][N * LD];
  // data gradient: an out-of-grid tap reads the stage's zero position (one address select per tap
  // instead of zeroing its 12 fragment registers; dgrad -3 us)
  constexpr bool ZROW = EPI != EPI_CONV;
  constexpr int SPOS = kDmaSpan + (ZROW ? 1 : 0);  // staged positions per wave (+ the zero position)
  __shared__ __attribute__((aligned(16))) __bf16 stage[WPB][SPOS * kPreRow];
  // the statistics' per-wave partials reuse the wave's own stage once its tiles are done
  static_assert(N * 2 * sizeof(float) <= SPOS * kPreRow * sizeof(__bf16), "red fits a stage");
  auto red = [&](int w) { return reinterpret_cast<float (*)[2]>(&stage[w][0]); };
  __shared__ float bfold[N];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int idx = tid; idx < N * (K / 8); idx += WPB * 64) {
    const int n = idx / (K / 8), k8 = (idx % (K / 8)) * 8;
    const float4 lo = *reinterpret_cast<const float4*>(a.Bw + (int64_t)n * a.ldb + k8);
    const float4 hi = *reinterpret_cast<const float4*>(a.Bw + (int64_t)n * a.ldb + k8 + 4);
    bf16x8 pl[NP];
    planes_x8<NP>(lo, hi, pl);
#pragma unroll
    for (int q = 0; q < NP; ++q) *reinterpret_cast<bf16x8*>(&Bs[q][n * LD + k8]) = pl[q];
  }
  if (EPI == EPI_CONV && a.fold_t != nullptr) {
    for (int q = tid; q < N * 8; q += WPB * 64) {
      const int n = q / 8, part = q % 8;
      double acc = 0.0;
#pragma unroll
      for (int c = 0; c < CS / 8; ++c) acc += a.fold_t[(int64_t)(part * (CS / 8) + c) * N + n];
#pragma unroll
      for (int o = 4; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
      if (part == 0) bfold[n] = (float)(acc + (double)a.bias[n]);
    }
  }
  __syncthreads();
  const int64_t W = (int64_t)gridDim.x * WPB;
  const int64_t g = (int64_t)blockIdx.x * WPB + __builtin_amdgcn_readfirstlane(wave);
  const int r_lo = (int)(a.M * g / W), r_hi = (int)(a.M * (g + 1) / W);
  const int HoWo = a.Ho * a.Wo;
  const int npos = a.Hs * a.Ws * (a.M / HoWo);
  int tofs[4], tmin = 0, tmax = 0;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    tofs[t] = a.dh[t] * a.Ws + a.dw[t];
    tmin = min(tmin, tofs[t]);
    tmax = max(tmax, tofs[t]);
  }
  const __amdgpu_buffer_rsrc_t arsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(a.src), 0, (int)std::min<int64_t>((int64_t)npos * CS * 4, 0x7ffffff0), 0x00020000);
  const int kq = 8 * (lane >> 5);
  float st[NJ][2];
  float bias[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    st[j][0] = st[j][1] = 0.0f;
    bias[j] = 0.0f;
    if constexpr (EPI == EPI_CONV) bias[j] = a.fold_t != nullptr ? bfold[32 * j + (lane & 31)] : a.bias[32 * j + (lane & 31)];
  }
  __bf16* sw = stage[__builtin_amdgcn_readfirstlane(wave)];
  if constexpr (ZROW) {
    if (lane < kPreRow / 8) *reinterpret_cast<bf16x8*>(sw + kDmaSpan * kPreRow + lane * 8) = bf16x8{};
  }
  constexpr uint32_t kOOB = 0x80000000u;
  // unit u = lane + 64 k: position u >> 1, channels cg * 16 + 8 (u & 1) .. + 7 of the group
  auto fetch = [&](int p0, int cg, int need, float4 (&r)[2][2]) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int u = lane + 64 * k, pos = u >> 1;
      const uint32_t off = pos < need ? (uint32_t)(((p0 + pos) * CS + cg * 16 + (u & 1) * 8) * 4) : kOOB;
      if constexpr ((ABD_PRE_ABL & 2) != 0) {
        typedef float fv4 __attribute__((ext_vector_type(4)));
        fv4 z;
        asm volatile("; abl" : "=v"(z) : "v"(off));
        r[k][0] = r[k][1] = __builtin_bit_cast(float4, z);
        continue;
      }
      r[k][0] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(arsrc, (int)off, 0, 0));
      r[k][1] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(arsrc, (int)(off + 16u), 0, 0));
    }
  };
  auto put = [&](int need, const float4 (&r)[2][2]) {
    if constexpr ((ABD_PRE_ABL & 1) != 0) {
      typedef float fv4 __attribute__((ext_vector_type(4)));
      const fv4 x0 = __builtin_bit_cast(fv4, r[0][0]), x1 = __builtin_bit_cast(fv4, r[0][1]);
      const fv4 x2 = __builtin_bit_cast(fv4, r[1][0]), x3 = __builtin_bit_cast(fv4, r[1][1]);
      asm volatile("; abl" ::"v"(x0), "v"(x1), "v"(x2), "v"(x3), "v"(need));
      return;
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int u = lane + 64 * k, pos = u >> 1;
      if (pos < need) {
        bf16x8 pl[NP];
        if constexpr ((ABD_PRE_ABL & 16) != 0) {
          pl[0] = __builtin_bit_cast(bf16x8, r[k][0]);
          pl[1] = __builtin_bit_cast(bf16x8, r[k][1]);
          pl[2] = pl[0];
        } else {
          planes_x8<NP>(r[k][0], r[k][1], pl);
        }
#pragma unroll
        for (int q = 0; q < NP; ++q) *reinterpret_cast<bf16x8*>(sw + pos * kPreRow + q * 16 + (u & 1) * 8) = pl[q];
      }
    }
  };
  const int ntiles = (r_hi - r_lo + 31) / 32;
  const __amdgpu_buffer_rsrc_t orsrc = __builtin_amdgcn_make_buffer_rsrc(
      a.out + (int64_t)r_lo * N, 0, (r_hi - r_lo) * N * 4, 0x00020000);
  // this lane's output row m0 + (lane & 31) of the current tile as (b, h, w), stepped 32 rows per
  // tile without dividing (the per-tile divisions of the other kernels' src_of / taps_of cost ~15 %
  // of this kernel's VALU).  Rows past r_hi (the wave's last tile) continue the image pattern: their
  // outputs are dropped, their taps stay inside the staged span (dma_span bounds any 32 rows), and
  // past the last image their positions load zeros (buffer range check).
  const int dH = 32 / a.Wo, dW = 32 - dH * a.Wo;
  int cb, ch, cw;
  {
    const int m = r_lo + (lane & 31);
    cb = m / HoWo;
    const int rem = m - cb * HoWo;
    ch = rem / a.Wo;
    cw = rem - ch * a.Wo;
  }
  auto step32 = [&](int& b, int& h, int& w) {
    w += dW;
    h += dH;
    if (w >= a.Wo) {
      w -= a.Wo;
      ++h;
    }
    while (h >= a.Ho) {
      h -= a.Ho;
      ++b;
    }
  };
  auto src_at = [&](int b, int h, int w) { return (b * a.Hs + h) * a.Ws + w; };
  auto taps_at = [&](int h, int w) {
    uint32_t mk = 0;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int hs = h + a.dh[t], ws = w + a.dw[t];
      if (hs >= 0 && hs < a.Hs && ws >= 0 && ws < a.Ws) mk |= 1u << t;
    }
    return mk;
  };
  // first staged position of the 32 rows whose lane-row source is s0, and the positions they reach
  auto span_of = [&](int s0, int& need) {
    int v = s0, u = s0;
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) {
      v = min(v, __shfl_xor(v, o, 64));
      u = max(u, __shfl_xor(u, o, 64));
    }
    const int base = __builtin_amdgcn_readfirstlane(v) + tmin;
    need = __builtin_amdgcn_readfirstlane(u) + tmax + 1 - base;
    return base;
  };
  // B fragments are loaded BD steps ahead (NBV buffers, a power of two: the 16 steps of a tile keep
  // the buffer order across tiles); 2 steps ahead: forward -2, data gradient -1.5 us against 1
  constexpr int BD = 2, NBV = 4;
  bf16x8 bvs[NBV][NJ][NP];
  auto load_b = [&](int cg, int t, bf16x8 (&bv)[NJ][NP]) {
    const int kb = t * CS + cg * 16 + kq;
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int q = 0; q < NP; ++q) bv[j][q] = *reinterpret_cast<const bf16x8*>(&Bs[q][(32 * j + (lane & 31)) * LD + kb]);
  };
  // Software pipeline over the wave's stream of groups (4 per tile): while group g's MFMAs run, its
  // 12 A fragments are already in registers, group g + 1's planes are written to the stage (LDS
  // executes a wave's DS instructions in order: g's reads precede the writes) and group g + 2's
  // units are loading.
  int need = kDmaSpan, needn = kDmaSpan;
  int p0 = ntiles > 0 ? span_of(src_at(cb, ch, cw), need) : 0;
  float4 raw[2][2];
  fetch(p0, 0, ntiles > 0 ? need : 0, raw);
  put(ntiles > 0 ? need : 0, raw);
  fetch(p0, 1, ntiles > 0 ? need : 0, raw);
#pragma unroll
  for (int s = 0; s < BD; ++s) load_b(s / 4, s % 4, bvs[s]);
#pragma unroll 1
  for (int tile = 0; tile < ntiles; ++tile) {
    const int m0 = r_lo + 32 * tile;
    const int prow = src_at(cb, ch, cw) - p0;
    const uint32_t tm = taps_at(ch, cw);
    const bool more = tile + 1 < ntiles;
    int nb = cb, nh = ch, nw = cw;  // the next tile's row
    step32(nb, nh, nw);
    const int p0n = span_of(src_at(nb, nh, nw), needn);
    const int nn = more ? needn : 0;  // staged positions of the next tile (0: nothing to stage)
    f32x16 acc[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[j][r] = 0.0f;
#pragma unroll
    for (int cg = 0; cg < G; ++cg) {
      __builtin_amdgcn_sched_barrier(0);
      bf16x8 av[4][NP];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        int pos = min(max(prow + tofs[t], 0), kDmaSpan - 1);  // an invalid tap's position is clamped
        if constexpr (ZROW) pos = (tm >> t) & 1u ? pos : kDmaSpan;  // ... or the zero position
        const __bf16* rp = sw + pos * kPreRow + kq;
#pragma unroll
        for (int q = 0; q < NP; ++q) av[t][q] = *reinterpret_cast<const bf16x8*>(rp + q * 16);
      }
      __builtin_amdgcn_sched_barrier(0);
      // group g + 1 into the stage (this tile's next group, or the next tile's group 0)
      put(cg + 1 < G ? need : nn, raw);
      __builtin_amdgcn_sched_barrier(0);
      // group g + 2's loads
      if (cg + 2 < G) fetch(p0, cg + 2, need, raw);
      else fetch(p0n, cg + 2 - G, nn, raw);
      __builtin_amdgcn_sched_barrier(0);  // one group's loads live at a time (hoisted, they spill)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        if constexpr (EPI != EPI_CONV && !ZROW) {  // data-gradient taps leave the source grid at its edges
          if (!((tm >> t) & 1u)) {
#pragma unroll
            for (int q = 0; q < NP; ++q) av[t][q] = bf16x8{};
          }
        }
        const int s = cg * 4 + t;
        load_b(((s + BD) % (4 * G)) / 4, (s + BD) % 4, bvs[(s + BD) % NBV]);
        bf16x8 (&bv)[NJ][NP] = bvs[s % NBV];
#pragma unroll
        for (int term = 0; term < Terms<NP>::n; ++term)
#pragma unroll
          for (int j = 0; j < NJ; ++j) {
            if constexpr ((ABD_PRE_ABL & 4) != 0) {
              asm volatile("; abl" ::"v"(av[t][Terms<NP>::A[term]]), "v"(bv[j][Terms<NP>::B[term]]));
              continue;
            }
            acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[t][Terms<NP>::A[term]], bv[j][Terms<NP>::B[term]], acc[j], 0, 0, 0);
          }
      }
    }
    p0 = p0n;
    need = needn;
    cb = nb;
    ch = nh;
    cw = nw;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = m0 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      const bool ok = m < r_hi;
      const uint32_t ob = ok ? (uint32_t)((m - r_lo) * N + (lane & 31)) * 4u : kOOB;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        float v = acc[j][r];
        if constexpr (EPI == EPI_CONV) {
          v = fmaxf(v + bias[j], 0.0f);
          const float vs = ok ? v : 0.0f;
          st[j][0] += vs;
          st[j][1] = fmaf(vs, vs, st[j][1]);
        }
        if ((ABD_PRE_ABL & 8) && __builtin_bit_cast(uint32_t, v) != 0x7fc00001u) continue;
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), orsrc, (int)(ob + 128u * j), 0, 0);
      }
    }
  }
  if (EPI != EPI_CONV || a.part == nullptr) return;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const float s0 = st[j][0] + __shfl_xor(st[j][0], 32, 64);
    const float s1 = st[j][1] + __shfl_xor(st[j][1], 32, 64);
    if (lane < 32) {
      red(wave)[32 * j + lane][0] = s0;
      red(wave)[32 * j + lane][1] = s1;
    }
  }
  __syncthreads();
  if (tid < N) {
    float s0 = 0.0f, s1 = 0.0f;
    for (int w = 0; w < WPB; ++w) {
      s0 += red(w)[tid][0];
      s1 += red(w)[tid][1];
    }
    a.part[((int64_t)0 * a.N + tid) * a.nblk + blockIdx.x] = s0;
    a.part[((int64_t)1 * a.N + tid) * a.nblk + blockIdx.x] = s1;
  }
}

// Weight-stationary conv GEMM in f32split with WAVE-SPECIALISED staging (round 4).  The ablations of
// conv_ws_pre_kernel (no MFMAs: still 0.093 ms of 0.121) show its every-wave chain -- loads, split,
// LDS writes, fragment reads, MFMAs -- bound by latency at 2 waves per SIMD, with the matrix pipe
// ~45 % busy.  Here the two waves of a SIMD split the roles: waves 0-3 (one per SIMD) only read
// fragments and run the MFMAs and the epilogue; waves 4-7 (their SIMD partners) load the consumer's
// span two groups ahead, split each unit once into the three exact bf16 planes and write them into
// the consumer's double-buffered stage, so the split's VALU co-executes with the partner's MFMAs.
// One block barrier per 16-channel group publishes group q + 1 while the consumer reads group q.
// Every wave runs the same number of groups (the longest consumer's; rows past r_hi are masked).
// Same tiles (32 rows x 32 NJ columns per consumer tile), K order, products and epilogue as
// conv_ws_pre_kernel, so results are identical to it.  LDS: 101,376 (weights) + 57,344 / 58,240
// (4 consumers x 2 buffers x 64 positions x 112 B, + a zero position per buffer in the data
// gradient) + 256 B.
#ifndef ABD_SPEC_ABL  // measurement builds (results discarded): 1 no stage writes, 2 no loads,
#define ABD_SPEC_ABL 0  // 4 no MFMAs, 8 no output stores, 16 no group barriers (every wave runs free),
                        // 32 no B-fragment LDS reads (each register set loaded once)
#endif
#ifndef ABD_SPEC_ILV  // consumer read schedule: 3 (default) A one tap ahead and every step's reads
#define ABD_SPEC_ILV 3  // two per MFMA gap; 2 one per gap; 1 only B interleaved; 0 all 18 reads at the
#endif                 // group start (A/B, 3 alternations: 0 1.0007, 1 0.9916, 2 0.9894 ms per step;
                       // 2 vs 3 on another box: forward 0.1179 vs 0.1164, data gradient 0.1223 vs 0.1207)
#ifndef ABD_WS_SPEC  // conv_ws_spec_kernel replaces conv_ws_pre_kernel: 2 everywhere, 1 the forwards
#define ABD_WS_SPEC 2  // only, 0 nowhere (measurement builds)
#endif
// NP = 1 (bf16 mode, conv2): the A source is the producer layer's bf16 plane (NTArgs::srcs), loaded 16 B
// per unit and stored to the stage unchanged (no split); one MFMA term per step.  Same tiles, K order
// and products as conv_ws_dma_kernel<EPI, 1, 2, true>, whose LDS-DMA pieces stalled the issuing
// waves' MFMAs (r6_bf16abl: without the DMA issue the bf16 forward ran 39 -> 21 us at B = 256).
#ifndef ABD_BF16_SPEC  // measurement builds: 0 keeps bf16's conv2 on conv_ws_dma_kernel
#define ABD_BF16_SPEC 1
#endif
template <int EPI, int NJ = 2, int NP = 3>
__global__ void __launch_bounds__(512, 1) conv_ws_spec_kernel(NTArgs a) {
  static_assert(NP == 3 || (NP == 1 && NJ == 2), "f32split planes, or bf16 planes for conv2");
  constexpr int CS = 64, N = 32 * NJ, K = 4 * CS, LD = K + 8, WPB = 8, NC = 4, G = CS / 16;
  static_assert(G == 4, "the group parity selects the stage buffer; the producer loads one tile ahead");
  constexpr bool ZROW = EPI != EPI_CONV;
  constexpr int SPOS = kDmaSpan + (ZROW ? 1 : 0);
  __shared__ __attribute__((aligned(16))) __bf16 Bs[NP][N * LD];
  __shared__ __attribute__((aligned(16))) __bf16 stage[NC][2][SPOS * kPreRow];
  __shared__ float bfold[N];
  static_assert(N * 2 * sizeof(float) <= SPOS * kPreRow * sizeof(__bf16), "red fits a stage buffer");
  auto red = [&](int w) { return reinterpret_cast<float (*)[2]>(&stage[w][0][0]); };
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int idx = tid; idx < N * (K / 8); idx += WPB * 64) {
    const int n = idx / (K / 8), k8 = (idx % (K / 8)) * 8;
    const float4 lo = *reinterpret_cast<const float4*>(a.Bw + (int64_t)n * a.ldb + k8);
    const float4 hi = *reinterpret_cast<const float4*>(a.Bw + (int64_t)n * a.ldb + k8 + 4);
    bf16x8 pl[NP];
    planes_x8<NP>(lo, hi, pl);
#pragma unroll
    for (int q = 0; q < NP; ++q) *reinterpret_cast<bf16x8*>(&Bs[q][n * LD + k8]) = pl[q];
  }
  if (EPI == EPI_CONV && a.fold_t != nullptr) {
    for (int q = tid; q < N * 8; q += WPB * 64) {
      const int n = q / 8, part = q % 8;
      double acc = 0.0;
#pragma unroll
      for (int c = 0; c < CS / 8; ++c) acc += a.fold_t[(int64_t)(part * (CS / 8) + c) * N + n];
#pragma unroll
      for (int o = 4; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
      if (part == 0) bfold[n] = (float)(acc + (double)a.bias[n]);
    }
  }
  const bool producer = __builtin_amdgcn_readfirstlane(wave) >= NC;
  const int c = __builtin_amdgcn_readfirstlane(wave) & (NC - 1);  // the consumer this wave is or serves
  if constexpr (ZROW) {
    if (!producer && lane < 2 * (kPreRow / 8))
      *reinterpret_cast<bf16x8*>(&stage[c][lane / (kPreRow / 8)][kDmaSpan * kPreRow + (lane % (kPreRow / 8)) * 8]) = bf16x8{};
  }
  const int64_t W = (int64_t)gridDim.x * NC;
  const int64_t g = (int64_t)blockIdx.x * NC + c;
  const int r_lo = (int)(a.M * g / W), r_hi = (int)(a.M * (g + 1) / W);
  const int nt = (int)((a.M + W - 1) / W + 31) / 32;  // tiles of every wave (the longest consumer's)
  const int HoWo = a.Ho * a.Wo;
  const int npos = a.Hs * a.Ws * (a.M / HoWo);
  int tofs[4], tmin = 0, tmax = 0;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    tofs[t] = a.dh[t] * a.Ws + a.dw[t];
    tmin = min(tmin, tofs[t]);
    tmax = max(tmax, tofs[t]);
  }
  constexpr uint32_t kOOB = 0x80000000u;
  // this wave's (consumer's) output row of the current tile, stepped 32 rows per tile as in
  // conv_ws_pre_kernel (rows past r_hi continue the pattern; past the last image they load zeros)
  const int dH = 32 / a.Wo, dW = 32 - dH * a.Wo;
  int cb, ch, cw;
  {
    const int m = r_lo + (lane & 31);
    cb = m / HoWo;
    const int rem = m - cb * HoWo;
    ch = rem / a.Wo;
    cw = rem - ch * a.Wo;
  }
  auto step32 = [&](int& b, int& h, int& w) {
    w += dW;
    h += dH;
    if (w >= a.Wo) {
      w -= a.Wo;
      ++h;
    }
    while (h >= a.Ho) {
      h -= a.Ho;
      ++b;
    }
  };
  auto src_at = [&](int b, int h, int w) { return (b * a.Hs + h) * a.Ws + w; };
  auto span_of = [&](int s0, int& need) {
    int v = s0, u = s0;
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) {
      v = min(v, __shfl_xor(v, o, 64));
      u = max(u, __shfl_xor(u, o, 64));
    }
    const int base = __builtin_amdgcn_readfirstlane(v) + tmin;
    need = __builtin_amdgcn_readfirstlane(u) + tmax + 1 - base;
    return base;
  };
  if (producer) {
    // ---- producer: group q + 1 into buffer (q + 1) & 1 while the consumer reads group q ----
    const __amdgpu_buffer_rsrc_t arsrc =
        NP == 1 ? __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(a.srcs), 0,
                                                    (int)std::min<int64_t>((int64_t)npos * CS * 2, 0x7ffffff0), 0x00020000)
                : __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.src), 0,
                                                    (int)std::min<int64_t>((int64_t)npos * CS * 4, 0x7ffffff0), 0x00020000);
    auto fetch = [&](int p0, int cg, int need, float4 (&r)[2][2]) {
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int pos = (lane & 31) + 32 * k, h = lane >> 5;
        if constexpr (NP == 1) {  // 8 bf16 channels of the plane: one 16-B load (r[k][1] unused)
          const uint32_t off = pos < need ? (uint32_t)(((p0 + pos) * CS + cg * 16 + h * 8) * 2) : kOOB;
          r[k][0] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(arsrc, (int)off, 0, 0));
          r[k][1] = r[k][0];
          continue;
        }
        const uint32_t off = pos < need ? (uint32_t)(((p0 + pos) * CS + cg * 16 + h * 8) * 4) : kOOB;
        if constexpr ((ABD_SPEC_ABL & 2) != 0) {
          typedef float fv4 __attribute__((ext_vector_type(4)));
          fv4 z;
          asm volatile("; abl" : "=v"(z) : "v"(off));
          r[k][0] = r[k][1] = __builtin_bit_cast(float4, z);
          continue;
        }
        r[k][0] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(arsrc, (int)off, 0, 0));
        r[k][1] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(arsrc, (int)(off + 16u), 0, 0));
      }
    };
    // every position of the span buffer is written (past `need` the loads returned zeros).  Unit
    // (lane, k) = channels 8 (lane >> 5) .. + 7 of position (lane & 31) + 32 k: a ds_write_b128's
    // 8-lane bank group then writes 8 consecutive positions 112 B apart, distinct banks (the
    // position-pair order of conv_ws_pre_kernel 2-way conflicts), and a load still touches 32 lines
    auto put = [&](__bf16* sw, const float4 (&r)[2][2]) {
      if constexpr ((ABD_SPEC_ABL & 1) != 0) {
        typedef float fv4 __attribute__((ext_vector_type(4)));
        const fv4 x0 = __builtin_bit_cast(fv4, r[0][0]), x1 = __builtin_bit_cast(fv4, r[0][1]);
        const fv4 x2 = __builtin_bit_cast(fv4, r[1][0]), x3 = __builtin_bit_cast(fv4, r[1][1]);
        asm volatile("; abl" ::"v"(x0), "v"(x1), "v"(x2), "v"(x3), "v"(sw));
        return;
      }
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int pos = (lane & 31) + 32 * k, h = lane >> 5;
        if constexpr (NP == 1) {
          *reinterpret_cast<bf16x8*>(sw + pos * kPreRow + h * 8) = __builtin_bit_cast(bf16x8, r[k][0]);
          continue;
        }
        bf16x8 pl[NP];
        planes_x8<NP>(r[k][0], r[k][1], pl);
#pragma unroll
        for (int q = 0; q < NP; ++q) *reinterpret_cast<bf16x8*>(sw + pos * kPreRow + q * 16 + h * 8) = pl[q];
      }
    };
    // loads run RB = 4 groups ahead of their put (one tile): group q + 1 is put from raw[(q + 1) % 4]
    // and that buffer then loads group q + 5 (the next tile's cg + 1, or the tile after's group 0)
    int need0 = 0, need1 = 0, need2 = 0;
    const int p00 = span_of(src_at(cb, ch, cw), need0);  // tile 0
    step32(cb, ch, cw);
    int p01 = span_of(src_at(cb, ch, cw), need1);  // the tile after the one being put
    step32(cb, ch, cw);
    int p02 = span_of(src_at(cb, ch, cw), need2);  // the one after that
    if (nt < 2) need1 = 0;
    if (nt < 3) need2 = 0;
    float4 raw[4][2][2];
#pragma unroll
    for (int q = 0; q < 4; ++q) fetch(p00, q, need0, raw[q]);
    __syncthreads();  // weights, bfold and the zero positions
    put(stage[c][0], raw[0]);
    fetch(p01, 0, need1, raw[0]);
    __syncthreads();
#pragma unroll 1
    for (int tile = 0; tile < nt; ++tile) {
#pragma unroll
      for (int cg = 0; cg < G; ++cg) {
        if (cg + 1 < G || tile + 1 < nt) put(stage[c][(cg + 1) & 1], raw[(cg + 1) % 4]);
        if (cg + 1 < G) fetch(p01, cg + 1, need1, raw[(cg + 1) % 4]);
        else fetch(p02, 0, need2, raw[0]);
        if constexpr ((ABD_SPEC_ABL & 16) == 0) __syncthreads();
      }
      p01 = p02;
      need1 = need2;
      step32(cb, ch, cw);
      p02 = span_of(src_at(cb, ch, cw), need2);
      if (tile + 3 >= nt) need2 = 0;
    }
  } else {
    // ---- consumer: fragments of group q from buffer q & 1, MFMAs, epilogue per tile ----
    const int kq = 8 * (lane >> 5);
    float st[NJ][2];
    float bias[NJ];
    __syncthreads();  // weights, bfold and the zero positions
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      st[j][0] = st[j][1] = 0.0f;
      bias[j] = 0.0f;
      if constexpr (EPI == EPI_CONV) bias[j] = a.fold_t != nullptr ? bfold[32 * j + (lane & 31)] : a.bias[32 * j + (lane & 31)];
    }
    const __amdgpu_buffer_rsrc_t orsrc = __builtin_amdgcn_make_buffer_rsrc(
        a.out + (int64_t)r_lo * N, 0, (r_hi - r_lo) * N * 4, 0x00020000);
    auto taps_at = [&](int h, int w) {
      uint32_t mk = 0;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int hs = h + a.dh[t], ws = w + a.dw[t];
        if (hs >= 0 && hs < a.Hs && ws >= 0 && ws < a.Ws) mk |= 1u << t;
      }
      return mk;
    };
    constexpr int BD = 2, NBV = 4;  // B fragments two steps ahead (as conv_ws_pre_kernel)
    bf16x8 bvs[NBV][NJ][NP];
    auto load_b = [&](int cg, int t, bf16x8 (&bv)[NJ][NP]) {
      if constexpr ((ABD_SPEC_ABL & 32) != 0) return;  // ablation: B fragments stay in registers
      const int kb = t * CS + cg * 16 + kq;
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int q = 0; q < NP; ++q) bv[j][q] = *reinterpret_cast<const bf16x8*>(&Bs[q][(32 * j + (lane & 31)) * LD + kb]);
    };
    if constexpr ((ABD_SPEC_ABL & 32) != 0) {  // every B register set loaded once
#pragma unroll
      for (int s = 0; s < NBV; ++s)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
          for (int q = 0; q < NP; ++q)
            bvs[s][j][q] = *reinterpret_cast<const bf16x8*>(&Bs[q][(32 * j + (lane & 31)) * LD + s * CS + kq]);
    }
#pragma unroll
    for (int s = 0; s < BD; ++s) load_b(s / 4, s % 4, bvs[s]);
    __syncthreads();  // group 0 staged
#pragma unroll 1
    for (int tile = 0; tile < nt; ++tile) {
      const int m0 = r_lo + 32 * tile;
      int need;
      const int prow = src_at(cb, ch, cw) - span_of(src_at(cb, ch, cw), need);
      const uint32_t tm = taps_at(ch, cw);
      step32(cb, ch, cw);
      f32x16 acc[NJ];
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[j][r] = 0.0f;
#pragma unroll
      for (int cg = 0; cg < G; ++cg) {
        const __bf16* sw = stage[c][cg & 1];
#if ABD_SPEC_ILV >= 2
        // A fragments one tap ahead (two register sets), B two steps ahead; each step's reads go
        // one per MFMA gap
        bf16x8 avb[2][NP];
        auto load_a = [&](int t, bf16x8 (&av)[NP]) {
          int pos = min(max(prow + tofs[t], 0), kDmaSpan - 1);
          if constexpr (ZROW) pos = (tm >> t) & 1u ? pos : kDmaSpan;
          const __bf16* rp = sw + pos * kPreRow + kq;
#pragma unroll
          for (int q = 0; q < NP; ++q) av[q] = *reinterpret_cast<const bf16x8*>(rp + q * 16);
        };
        load_a(0, avb[0]);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int s = cg * 4 + t;
          load_b(((s + BD) % (4 * G)) / 4, (s + BD) % 4, bvs[(s + BD) % NBV]);
          if (t + 1 < 4) load_a(t + 1, avb[(t + 1) & 1]);
          constexpr int PER = ABD_SPEC_ILV >= 3 ? 2 : 1;  // reads per MFMA gap
          constexpr int G1 = (NJ * NP + NP + PER - 1) / PER, G0 = (NJ * NP + PER - 1) / PER;
          if (t + 1 < 4) {
#pragma unroll
            for (int x = 0; x < G1; ++x) {
              __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
              __builtin_amdgcn_sched_group_barrier(0x100, PER, 0);
            }
            __builtin_amdgcn_sched_group_barrier(0x008, Terms<NP>::n * NJ - G1, 0);
          } else {
#pragma unroll
            for (int x = 0; x < G0; ++x) {
              __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
              __builtin_amdgcn_sched_group_barrier(0x100, PER, 0);
            }
            __builtin_amdgcn_sched_group_barrier(0x008, Terms<NP>::n * NJ - G0, 0);
          }
          bf16x8 (&bv)[NJ][NP] = bvs[s % NBV];
          bf16x8 (&av)[NP] = avb[t & 1];
#pragma unroll
          for (int term = 0; term < Terms<NP>::n; ++term)
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
              if constexpr ((ABD_SPEC_ABL & 4) != 0) {
                asm volatile("; abl" ::"v"(av[Terms<NP>::A[term]]), "v"(bv[j][Terms<NP>::B[term]]));
                continue;
              }
              acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[Terms<NP>::A[term]], bv[j][Terms<NP>::B[term]], acc[j], 0, 0, 0);
            }
        }
#else
        bf16x8 av[4][NP];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          int pos = min(max(prow + tofs[t], 0), kDmaSpan - 1);
          if constexpr (ZROW) pos = (tm >> t) & 1u ? pos : kDmaSpan;
          const __bf16* rp = sw + pos * kPreRow + kq;
#pragma unroll
          for (int q = 0; q < NP; ++q) av[t][q] = *reinterpret_cast<const bf16x8*>(rp + q * 16);
        }
        // all 12 A reads issue here (left to itself the compiler sinks each read to its first use
        // and waits on it there: with one MFMA wave per SIMD every LDS latency was exposed)
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int s = cg * 4 + t;
          load_b(((s + BD) % (4 * G)) / 4, (s + BD) % 4, bvs[(s + BD) % NBV]);
#if ABD_SPEC_ILV
          // the step's B reads one per MFMA gap instead of a burst (LDS issue stalls)
#pragma unroll
          for (int x = 0; x < NJ * NP; ++x) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          }
          __builtin_amdgcn_sched_group_barrier(0x008, Terms<NP>::n * NJ - NJ * NP, 0);
#else
          __builtin_amdgcn_sched_barrier(0);
#endif
          bf16x8 (&bv)[NJ][NP] = bvs[s % NBV];
#pragma unroll
          for (int term = 0; term < Terms<NP>::n; ++term)
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
              if constexpr ((ABD_SPEC_ABL & 4) != 0) {
                asm volatile("; abl" ::"v"(av[t][Terms<NP>::A[term]]), "v"(bv[j][Terms<NP>::B[term]]));
                continue;
              }
              acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[t][Terms<NP>::A[term]], bv[j][Terms<NP>::B[term]], acc[j], 0, 0, 0);
            }
        }
#endif
        if ((ABD_SPEC_ABL & 16) == 0 && cg + 1 < G) __syncthreads();  // the last group's barrier follows the epilogue
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const bool ok = m < r_hi;
        const uint32_t ob = ok ? (uint32_t)((m - r_lo) * N + (lane & 31)) * 4u : kOOB;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          float v = acc[j][r];
          if constexpr (EPI == EPI_CONV) {
            v = fmaxf(v + bias[j], 0.0f);
            const float vs = ok ? v : 0.0f;
            st[j][0] += vs;
            st[j][1] = fmaf(vs, vs, st[j][1]);
          }
          if ((ABD_SPEC_ABL & 8) && __builtin_bit_cast(uint32_t, v) != 0x7fc00001u) continue;
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), orsrc, (int)(ob + 128u * j), 0, 0);
        }
      }
      if constexpr ((ABD_SPEC_ABL & 16) == 0) __syncthreads();
    }
    if (EPI == EPI_CONV && a.part != nullptr) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const float s0 = st[j][0] + __shfl_xor(st[j][0], 32, 64);
        const float s1 = st[j][1] + __shfl_xor(st[j][1], 32, 64);
        if (lane < 32) {
          red(c)[32 * j + lane][0] = s0;
          red(c)[32 * j + lane][1] = s1;
        }
      }
    }
  }
  if (EPI != EPI_CONV || a.part == nullptr) return;
  __syncthreads();
  if (tid < N) {
    float s0 = 0.0f, s1 = 0.0f;
    for (int w = 0; w < NC; ++w) {
      s0 += red(w)[tid][0];
      s1 += red(w)[tid][1];
    }
    a.part[((int64_t)0 * a.N + tid) * a.nblk + blockIdx.x] = s0;
    a.part[((int64_t)1 * a.N + tid) * a.nblk + blockIdx.x] = s1;
  }
}

struct TNArgs {
  const float* D;
  int ldd;
  const float* src;
  int Hs, Ws, Cs;
  int Ho, Wo, M;
  int taps;
  int dh[4], dw[4];
  int N, Ktot;
  int mchunk;
  float* slab;
};

template <int NB, int KT>
__global__ void __launch_bounds__(kT) gemm_tn_kernel(TNArgs a) {
  constexpr int MR = 32;
  __shared__ __attribute__((aligned(16))) float Ds[MR * NB];
  __shared__ __attribute__((aligned(16))) float Ss[MR * KT];
  constexpr int KTILES = KT / 32;
  constexpr int TPW = (NB / 32) * KTILES / 4;  // accumulator tiles per wave
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int mstart = blockIdx.x * a.mchunk;
  const int mend = min(a.M, mstart + a.mchunk);
  const int k0 = blockIdx.y * KT;
  const int n0 = blockIdx.z * NB;
  f32x16 acc[TPW];
#pragma unroll
  for (int i = 0; i < TPW; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[i][r] = 0.0f;
  const int tile0 = wave * TPW;
  const int ntile = tile0 / KTILES;  // all of a wave's tiles share one n-tile
  for (int mm = mstart; mm < mend; mm += MR) {
    for (int idx = tid; idx < MR * NB / 4; idx += kT) {
      const int r = idx / (NB / 4), q = idx - r * (NB / 4);
      const int m = mm + r;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (m < mend) v = *reinterpret_cast<const float4*>(a.D + (int64_t)m * a.ldd + n0 + 4 * q);
      *reinterpret_cast<float4*>(Ds + r * NB + 4 * q) = v;
    }
    for (int idx = tid; idx < MR * KT / 4; idx += kT) {
      const int r = idx / (KT / 4), q = idx - r * (KT / 4);
      const int m = mm + r;
      const int kx = k0 + 4 * q;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (m < mend && kx < a.Ktot) {
        const int t = kx / a.Cs, c = kx - t * a.Cs;
        const int b = m / (a.Ho * a.Wo);
        const int rem = m - b * a.Ho * a.Wo;
        const int h = rem / a.Wo + a.dh[t], w = rem % a.Wo + a.dw[t];
        if (h >= 0 && h < a.Hs && w >= 0 && w < a.Ws)
          v = *reinterpret_cast<const float4*>(a.src + (((int64_t)b * a.Hs + h) * a.Ws + w) * a.Cs + c);
      }
      *reinterpret_cast<float4*>(Ss + r * KT + 4 * q) = v;
    }
    __syncthreads();
    const float* ap = Ds + (lane >> 5) * NB + ntile * 32 + (lane & 31);
#pragma unroll
    for (int kk = 0; kk < MR; kk += 2) {
      const float av = ap[kk * NB];
#pragma unroll
      for (int i = 0; i < TPW; ++i) {
        const int kt = (tile0 + i) % KTILES;
        const float bv = Ss[(kk + (lane >> 5)) * KT + kt * 32 + (lane & 31)];
        acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc[i], 0, 0, 0);
      }
    }
    __syncthreads();
  }
  float* slab = a.slab + (int64_t)blockIdx.x * a.N * a.Ktot;
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    const int kt = (tile0 + i) % KTILES;
    const int k = k0 + kt * 32 + (lane & 31);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int n = n0 + ntile * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      if (n < a.N && k < a.Ktot) slab[(int64_t)n * a.Ktot + k] = acc[i][r];
    }
  }
}

// 2x2 convolution weight gradient by output-row chunks.
//   dW[n][t*CIN + ci] = sum_m dz[m][n] * src[row(m) + tap t][ci]
// A chunk is R consecutive output rows of one utterance.  Its R+1 source rows
// ((R+1)*Ws*CIN floats) are contiguous in NHWC and are copied into LDS as is; its dz rows
// are copied row by row to a row stride of Ws (= Wo + 1) positions, leaving a pad
// column that is zeroed once.  On that common grid the reduction index m' = hl*Ws + w
// addresses both operands linearly (dz at m'*NB, tap t's source at (m' + dh*Ws + dw)*CIN),
// so the MFMA loop is pure base + immediate LDS reads; the pad positions contribute
// zero products (Ws/Wo extra MFMAs).  Copies use global_load_lds into one of two buffers
// while the block runs the MFMAs of the previous chunk.  Each wave owns TPW 32x32
// accumulator tiles of one n-tile; each block sums a contiguous range of chunks into its
// slab, reduced later in slab order (deterministic).
struct WGArgs {
  const float* dz;   // (B, Ho, Wo, NB)
  const float* src;  // (B, Hs, Ws, CIN), Hs >= Ho + 1, Ws == Wo + 1
  int Ho, Wo, Hs, Ws;
  int R, cpb, nchunks, per;
  int dsz, bsz;      // LDS floats: dz part (16-B aligned) and one whole buffer
  float* slab;       // [gridDim.x][NB][4*CIN]
  // conv_wgrad_trp_kernel<..., PS = true>: dz and src as NP exact bf16 planes (plane-major)
  const uint16_t* dzs;
  const uint16_t* srcs;
  int64_t dzplane, srcplane;
};

// n16 16-byte pieces from g to l, lane-linear: wave-instruction j of wave w copies pieces
// (j*kT + w*64) .. +63 into the same offsets of l
__device__ __forceinline__ void glds_copy(const float* g, float* l, int n16) {
  const int lane = threadIdx.x & 63, wbase = threadIdx.x & ~63;
  for (int i0 = 0; i0 < n16; i0 += kT) {
    const int i = i0 + wbase + lane;
    if (i < n16)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(g + 4 * i),
                                       (__attribute__((address_space(3))) void*)(l + 4 * (i0 + wbase)), 16, 0, 0);
  }
}

template <int NB, int CIN>
__global__ void __launch_bounds__(kT, 4) conv_wgrad_rows_kernel(WGArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds_wg[];
  constexpr int KT = 4 * CIN / 32, TILES = (NB / 32) * KT, TPW = TILES / 4;
  static_assert(TILES % 4 == 0 && KT % TPW == 0, "a wave's tiles must share one n-tile");
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int half = lane >> 5, col = lane & 31;
  const int nt = (wave * TPW) / KT;
  const int rowd = a.Wo * NB / 4;  // 16-byte pieces per dz row
  int boff[TPW];
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    const int kt = (wave * TPW + i) % KT;
    const int tap = kt / (CIN / 32), cb = kt % (CIN / 32);
    boff[i] = ((tap >> 1) * a.Ws + (tap & 1)) * CIN + cb * 32 + col;
  }
  // zero both buffers once: dz pad columns stay zero (copies never touch them) and every
  // LDS word a pad position can read is finite (0 * finite = 0)
  for (int i = threadIdx.x; i < 2 * a.bsz; i += kT) lds_wg[i] = 0.0f;
  __syncthreads();
  f32x16 acc[TPW];
#pragma unroll
  for (int i = 0; i < TPW; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[i][r] = 0.0f;
  const int c0 = blockIdx.x * a.per, c1 = min(a.nchunks, c0 + a.per);
  auto stage = [&](int c, float* buf) {
    const int b = c / a.cpb, h0 = (c - b * a.cpb) * a.R;
    const int rows = min(a.R, a.Ho - h0);
    const float* g = a.dz + ((int64_t)b * a.Ho + h0) * a.Wo * NB;
    for (int r = 0; r < rows; ++r) glds_copy(g + r * a.Wo * NB, buf + r * a.Ws * NB, rowd);
    glds_copy(a.src + ((int64_t)b * a.Hs + h0) * a.Ws * CIN, buf + a.dsz, (rows + 1) * a.Ws * CIN / 4);
  };
  if (c0 < c1) stage(c0, lds_wg);
  for (int c = c0; c < c1; ++c) {
    float* cur = lds_wg + ((c - c0) & 1) * a.bsz;
    __syncthreads();  // chunk c landed (vmcnt(0) + barrier); the other buffer is free
    if (c + 1 < c1) stage(c + 1, lds_wg + ((c + 1 - c0) & 1) * a.bsz);
    const int h0 = (c % a.cpb) * a.R;
    const int rows = min(a.R, a.Ho - h0);
    // m' over the rows*Ws grid positions in pairs; an odd count leaves out only the last
    // position, which is a pad column (zero dz)
    const int mcount = (rows * a.Ws) & ~1;
    const float* D = cur + half * NB + nt * 32 + col;
    const float* S = cur + a.dsz + half * CIN;
    // software-pipelined one pair ahead (the read past the end lands in slack / zeros)
    float av = D[0];
    float bv[TPW];
#pragma unroll
    for (int i = 0; i < TPW; ++i) bv[i] = S[boff[i]];
    for (int mp = 0; mp < mcount; mp += 2) {
      const float avn = D[(mp + 2) * NB];
      float bvn[TPW];
#pragma unroll
      for (int i = 0; i < TPW; ++i) bvn[i] = S[(mp + 2) * CIN + boff[i]];
#pragma unroll
      for (int i = 0; i < TPW; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv[i], acc[i], 0, 0, 0);
      av = avn;
#pragma unroll
      for (int i = 0; i < TPW; ++i) bv[i] = bvn[i];
    }
  }
  float* slab = a.slab + (int64_t)blockIdx.x * NB * (4 * CIN);
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    const int k = ((wave * TPW + i) % KT) * 32 + col;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int n = nt * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
      slab[(int64_t)n * (4 * CIN) + k] = acc[i][r];
    }
  }
}

// sum slabs in order; conv layout maps (n=co, k=t*Cin+ci) -> torch (co, ci, kh, kw)
// Exact three-way bf16 split of 8 fp32 values (x = p0 + p1 + p2, see gemm_nt_bf16_kernel).
__device__ __forceinline__ void split3_x8(const float (&x)[8], bf16x8& p0, bf16x8& p1, bf16x8& p2) {
  // pairs: v_cvt_pk_bf16_f32 (RNE), widen by bit moves, a float2 subtraction for the exact residual
  // (two v_sub_f32: no packed FP32 in this library, Makefile PKFLAGS)
  uint32_t u[3][4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    f32x2 v = {x[2 * e], x[2 * e + 1]};
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) {
      u[pl][e] = __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2));
      if (pl < 2) {
        const f32x2 back = {__builtin_bit_cast(float, u[pl][e] << 16), __builtin_bit_cast(float, u[pl][e] & 0xffff0000u)};
        v -= back;
      }
    }
  }
  p0 = __builtin_bit_cast(bf16x8, make_uint4(u[0][0], u[0][1], u[0][2], u[0][3]));
  p1 = __builtin_bit_cast(bf16x8, make_uint4(u[1][0], u[1][1], u[1][2], u[1][3]));
  p2 = __builtin_bit_cast(bf16x8, make_uint4(u[2][0], u[2][1], u[2][2], u[2][3]));
}

// conv2 weight gradient on bf16 MFMA with fp32-accurate products (ABD_PREC_F32_SPLIT; round 2).
// dW[n][t*64 + c] = sum_q dz[q][n] * src[q + off(t)][c]: the reduction index q (positions) is the
// outer NHWC index of both operands, so the MFMA operands are column reads of row-major images.
// Per chunk of R output rows of one utterance, dz rows (at the source row stride Ws = Wo + 1, pad
// column and tail zeroed) and the R + 1 source rows are staged ONCE, split into three exact bf16
// planes, as row-major LDS images (one 448-B row per position: planes at +0/+128/+256 B, 64 B pad --
// a 16-bank row step, so the four rows of a transposed read's 32-lane half land on distinct banks),
// and the fragments are read with ds_read_b64_tr_b16 (gfx950 transpose read: lane i of a 16-lane
// group receives column i of 4 rows).  Wave w owns tap w: 2 x 2 accumulator tiles (64 n x 64 c),
// six MFMA terms per 16-position step.  Chunk c + 1's global loads are in flight while chunk c's
// MFMAs run (registers), then split into the other LDS buffer.  Slabs as conv_wgrad_rows_kernel.
constexpr int kTrRow = 448;  // bytes per staged position (3 planes x 64 bf16 + pad)
typedef __bf16 bf16x4v __attribute__((ext_vector_type(4)));
// Software-pipelined transpose-read weight gradient (the round-2 kernel, conv_wgrad_tr_kernel, had
// the same staging without the pipeline; it is gone).  One 4-wave block per CU (the double-buffered images take 104 KB), so a wave has
// no partner on its SIMD to hide its non-MFMA work: every chunk's staging is moved inside the
// previous chunk's MFMA stream instead.
//   * chunk c + 2's global loads are issued at the top of chunk c (two chunks ahead: a whole
//     chunk of MFMAs covers their latency);
//   * chunk c + 1's registers are split and written to the other image buffer slot by slot
//     between chunk c's MFMAs (the MFMA pipe leaves 24 of its 32 cycles to vector issue);
//   * the next 16-position step's fragments are read after the current step's first term, so the
//     LDS latency is off the MFMA path and the lgkmcnt range (15) still covers the older reads.
// NS = Qd / 16 steps and MAXS staging slots are compile-time (checked by the launcher); slots
// past the images write a trash row (row Qd + Qs of each buffer).
#ifndef ABD_TRP_ILV  // the next step's fragment reads PER per MFMA gap (0: one burst after term 0);
#define ABD_TRP_ILV 2  // conv2 weight gradient 0.109 -> 0.104 ms (A/B, 3 alternations; PER 1: 0.1045)
#endif
#ifndef ABD_TRP_ABL  // ablation bits (measurement builds): 1 no MFMAs, 2 no staging writes, 4 no loads
#define ABD_TRP_ABL 0
#endif
// NP = 1 (ABD_PREC_BF16): one RNE-rounded bf16 plane per operand and one MFMA term (a0 b0); the
// staging of chunk c + 1 then rides on each step's single term.
// PS: dz and src come pre-split (WGArgs::dzs / srcs, store_planes4): a slot loads its 4 channels'
// NP planes (8 B each) and stores them as they are -- no split in the staging.
template <int NP> struct PlaneSlot {
  uint2 v[NP];
};
template <int R, int NB, int NS, int MAXS, int NP = 3, bool PS = false>
__global__ void __launch_bounds__(kT, 1) conv_wgrad_trp_kernel(WGArgs a) {
  constexpr int CIN = 64, NT = NB / 32, D4 = NB / 4, Qd = 16 * NS;
  constexpr uint32_t EB = PS ? 2u : 4u;  // bytes per staged element
  using SlotT = typename std::conditional<PS, PlaneSlot<NP>, float4>::type;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_tr[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int Ws = a.Ws, Wo = a.Wo;
  const int Qs = Qd + Ws + 1;
  const int nd4 = Qd * D4, ns4 = Qs * 16;
  const int bufb = (Qd + Qs + 1) * kTrRow;
  constexpr uint32_t kOOB = 0x80000000u;
  uint32_t off0[MAXS], loff[MAXS];
  bool isdz[MAXS];
#pragma unroll
  for (int k = 0; k < MAXS; ++k) {
    const int i = threadIdx.x + k * kT;
    isdz[k] = __builtin_amdgcn_readfirstlane(threadIdx.x & ~63) + k * kT < nd4;
    int row, c4;
    if (i < nd4) {
      const int q = i / D4, r = q / Ws, w = q - r * Ws;
      c4 = i % D4;
      row = q;
      off0[k] = (r < R && w < Wo) ? (uint32_t)(((r * Wo + w) * NB + 4 * c4) * EB) : kOOB;
    } else {
      const int q = (i - nd4) >> 4;
      c4 = (i - nd4) & 15;
      const bool ok = i < nd4 + ns4;
      row = ok ? Qd + q : Qd + Qs;  // trash row
      off0[k] = (ok && q < (R + 1) * Ws) ? (uint32_t)((q * CIN + 4 * c4) * EB) : kOOB;
    }
    loff[k] = (uint32_t)(row * kTrRow + c4 * 8);
  }
  f32x16 acc[NT][2];
#pragma unroll
  for (int i = 0; i < NT; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;
  const int c0 = blockIdx.x * a.per, c1 = min(a.nchunks, c0 + a.per);
  auto fetch = [&](int c, SlotT (&st)[MAXS]) {
    const int b = c / a.cpb, h0 = (c - b * a.cpb) * R;
    const uint32_t hdz = (uint32_t)(h0 * Wo * NB * EB), hsr = (uint32_t)(h0 * Ws * CIN * EB);
    if constexpr (PS) {
      // one descriptor per plane and utterance: rows past the utterance read zeros
      __amdgpu_buffer_rsrc_t rdz[NP], rsr[NP];
#pragma unroll
      for (int q = 0; q < NP; ++q) {
        rdz[q] = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(a.dzs) + q * a.dzplane + (int64_t)b * a.Ho * Wo * NB,
                                                   0, a.Ho * Wo * NB * 2, 0x00020000);
        rsr[q] = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(a.srcs) + q * a.srcplane +
                                                       (int64_t)b * a.Hs * Ws * CIN,
                                                   0, a.Hs * Ws * CIN * 2, 0x00020000);
      }
#pragma unroll
      for (int k = 0; k < MAXS; ++k) {
        const uint32_t o = off0[k] == kOOB ? kOOB : off0[k] + (isdz[k] ? hdz : hsr);
#pragma unroll
        for (int q = 0; q < NP; ++q)
          st[k].v[q] = __builtin_bit_cast(uint2, isdz[k] ? __builtin_amdgcn_raw_buffer_load_b64(rdz[q], (int)o, 0, 0)
                                                         : __builtin_amdgcn_raw_buffer_load_b64(rsr[q], (int)o, 0, 0));
      }
    } else {
    const __amdgpu_buffer_rsrc_t rdz = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(a.dz) + (int64_t)b * a.Ho * Wo * NB, 0, a.Ho * Wo * NB * 4, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(a.src) + (int64_t)b * a.Hs * Ws * CIN, 0, a.Hs * Ws * CIN * 4, 0x00020000);
#pragma unroll
    for (int k = 0; k < MAXS; ++k) {
      if constexpr (ABD_TRP_ABL & 4) {
        st[k] = make_float4((float)c, 1.f, 2.f, 3.f);
        continue;
      }
      const uint32_t o = off0[k] == kOOB ? kOOB : off0[k] + (isdz[k] ? hdz : hsr);
      st[k] = __builtin_bit_cast(float4, isdz[k] ? __builtin_amdgcn_raw_buffer_load_b128(rdz, (int)o, 0, 0)
                                                 : __builtin_amdgcn_raw_buffer_load_b128(rsr, (int)o, 0, 0));
    }
    }
  };
  auto put_slot = [&](int k, const SlotT& vv, unsigned char* buf) {
    if constexpr (ABD_TRP_ABL & 2) return;
    if constexpr (PS) {
#pragma unroll
      for (int pl = 0; pl < NP; ++pl) *reinterpret_cast<uint2*>(buf + loff[k] + pl * 128) = vv.v[pl];
      return;
    }
    const float4& v = reinterpret_cast<const float4&>(vv);
    f32x2 x[2] = {f32x2{v.x, v.y}, f32x2{v.z, v.w}};
#pragma unroll
    for (int pl = 0; pl < NP; ++pl) {
      uint32_t u[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        u[h] = __builtin_bit_cast(uint32_t, __builtin_convertvector(x[h], bf16x2));
        if (pl < NP - 1) {
          const f32x2 back = {__builtin_bit_cast(float, u[h] << 16), __builtin_bit_cast(float, u[h] & 0xffff0000u)};
          x[h] -= back;
        }
      }
      *reinterpret_cast<uint2*>(buf + loff[k] + pl * 128) = make_uint2(u[0], u[1]);
    }
  };
  const int g = (lane >> 4) & 1, h = lane >> 5, qq = (lane & 15) >> 2, pp = lane & 3;
  auto frag = [&](const unsigned char* img, int row0, int tile, int pl) -> bf16x8 {
    const int col = 32 * tile + 16 * g + 4 * pp;
    const unsigned char* p = img + (row0 + 8 * h + qq) * kTrRow + pl * 128 + col * 2;
    const bf16x4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) bf16x4v*)(p));
    const bf16x4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) bf16x4v*)(p + 4 * kTrRow));
    return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  };
  const int toff = (wave >> 1) * Ws + (wave & 1);
  struct Frags {
    bf16x8 av[NT][NP], bv[2][NP];
  };
  auto load_frags = [&](const unsigned char* cur, int s, Frags& F) {
#pragma unroll
    for (int pl = 0; pl < NP; ++pl) {
#pragma unroll
      for (int t = 0; t < NT; ++t) F.av[t][pl] = frag(cur, 16 * s, t, pl);
#pragma unroll
      for (int t = 0; t < 2; ++t) F.bv[t][pl] = frag(cur + Qd * kTrRow, 16 * s + toff, t, pl);
    }
  };
  constexpr int NTERM = Terms<NP>::n;
  auto term = [&](const Frags& F, int tm) {
    if constexpr (ABD_TRP_ABL & 1) return;
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(F.av[i][Terms<NP>::A[tm]], F.bv[j][Terms<NP>::B[tm]],
                                                            acc[i][j], 0, 0, 0);
  };
  // chunk c from `cur`; chunk c + 1's registers stP -> `nxt`; chunk c + 2 -> stF
  auto body = [&](int c, const unsigned char* cur, unsigned char* nxt, const SlotT (&stP)[MAXS],
                  SlotT (&stF)[MAXS]) {
    __syncthreads();  // chunk c's images complete; every wave is done with chunk c - 1 (= nxt)
    fetch(min(c + 2, c1 - 1), stF);
    Frags F[2];
    load_frags(cur, 0, F[0]);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      term(F[s & 1], 0);
      __builtin_amdgcn_sched_barrier(0);
      // every read of this step's fragments done (they have had a step to land): otherwise the
      // 24 reads issued next push the older ones past lgkmcnt's range and the waits for terms
      // 1-5 also wait for most of the new reads
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
      if (s + 1 < NS) load_frags(cur, s + 1, F[(s + 1) & 1]);
#if ABD_TRP_ILV
      if constexpr (NTERM > 1) {
        // the next step's reads spread over this step's MFMA gaps instead of one burst
        constexpr int MF = (NTERM - 1) * NT * 2, RD = (NT + 2) * NP * 2, PER = ABD_TRP_ILV;
        constexpr int NG = (RD + PER - 1) / PER < MF ? (RD + PER - 1) / PER : MF;
        if (s + 1 < NS) {
#pragma unroll
          for (int x = 0; x < NG; ++x) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, PER, 0);
          }
        }
      } else {
        __builtin_amdgcn_sched_barrier(0);
      }
#else
      __builtin_amdgcn_sched_barrier(0);
#endif
      if constexpr (NTERM == 1) {
#pragma unroll
        for (int k = 0; k < MAXS; ++k)  // slot k rides on step k % NS
          if (k % NS == s) put_slot(k, stP[k], nxt);
      } else {
#pragma unroll
        for (int tm = 1; tm < NTERM; ++tm) {
          term(F[s & 1], tm);
#pragma unroll
          for (int k = 0; k < MAXS; ++k)  // slot k rides on step k % NS, term 1 + (k / NS) % 5
            if (k % NS == s && 1 + (k / NS) % (NTERM - 1) == tm) put_slot(k, stP[k], nxt);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  SlotT stA[MAXS], stB[MAXS];
  unsigned char* buf0 = lds_tr;
  unsigned char* buf1 = lds_tr + bufb;
  if (c0 < c1) {
    fetch(c0, stA);
#pragma unroll
    for (int k = 0; k < MAXS; ++k) put_slot(k, stA[k], buf0);
    fetch(min(c0 + 1, c1 - 1), stA);
  }
  for (int c = c0; c < c1; c += 2) {
    body(c, buf0, buf1, stA, stB);
    if (c + 1 < c1) body(c + 1, buf1, buf0, stB, stA);
  }
  float* slab = a.slab + (int64_t)blockIdx.x * NB * (4 * CIN);
#pragma unroll
  for (int i = 0; i < NT; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int n = 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        slab[(int64_t)n * (4 * CIN) + wave * CIN + 32 * j + (lane & 31)] = acc[i][j][r];
      }
}

__global__ void __launch_bounds__(kT) slab_reduce_kernel(const float* slab, int nslab, int N, int Ktot, int conv_cin,
                                                         float* out, const float4* fold, const float* fold_db) {
  const int64_t total = (int64_t)N * Ktot;
  for (int64_t e = blockIdx.x * (int64_t)kT + threadIdx.x; e < total; e += (int64_t)gridDim.x * kT) {
    const float s = ordered_sum(slab + e, total, nslab);
    const int n = (int)(e / Ktot), k = (int)(e % Ktot);
    if (conv_cin > 0) {
      const int t = k / conv_cin, ci = k % conv_cin;
      out[((int64_t)n * conv_cin + ci) * 4 + t] = unfold_wgrad(s, fold, fold_db, n, ci);
    } else {
      out[e] = s;
    }
  }
}

// ------------------------------------------------------------------ fc2 + loss + metrics
struct LossArgs {
  const float* d2;   // (B,128)
  const float* w;    // fc2.weight (K,128)
  const float* b;    // (K)
  const int64_t* labels;
  const int64_t* ind;
  int B, K;
  float inv_batch;   // 1 / global batch (dL/dz normaliser)
  float* logprobs;   // (B,K)
  float* dz;         // (B,K) or null
  float* rowinfo;    // (B,4): loss, correct, poisoned, asr_hit
};

__global__ void __launch_bounds__(kT) fc2_loss_kernel(LossArgs a) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (kT / kWave) + (threadIdx.x >> 6);
  if (row >= a.B) return;
  const bool act = lane < a.K;
  float z = -INFINITY;
  if (act) {
    float acc = a.b[lane];
    const float* x = a.d2 + (int64_t)row * 128;
    const float* wr = a.w + (int64_t)lane * 128;
    for (int j = 0; j < 128; ++j) acc = fmaf(x[j], wr[j], acc);
    z = acc;
  }
  // o = log_softmax(z) (model output); loss = CE(o) = logsumexp(o) - o[y]
  const float mz = abd::wave_max(z);
  const float ez = act ? expf(z - mz) : 0.0f;
  const float lse = mz + logf(abd::wave_sum(ez));
  const float o = act ? z - lse : -INFINITY;
  const float mo = abd::wave_max(o);
  const float eo = act ? expf(o - mo) : 0.0f;
  const float so = abd::wave_sum(eo);
  const float lse2 = mo + logf(so);
  const int y = a.labels ? (int)a.labels[row] : -1;
  const float oy = __shfl(o, y < 0 ? 0 : y, 64);
  // first index of the maximum (torch max(dim=1))
  const unsigned long long ball = __ballot(act && o == mo);
  const int pred = __ffsll((long long)ball) - 1;
  float dov = 0.0f;
  if (act && a.dz) dov = (eo / so - (lane == y ? 1.0f : 0.0f)) * a.inv_batch;
  const float sdo = abd::wave_sum(dov);  // every lane takes part
  if (act) {
    a.logprobs[(int64_t)row * a.K + lane] = o;
    if (a.dz) a.dz[(int64_t)row * a.K + lane] = dov - expf(o) * sdo;
  }
  if (lane == 0 && y >= 0) {
    const bool pois = a.ind != nullptr && a.ind[row] == 1;
    float* ri = a.rowinfo + (int64_t)row * 4;
    ri[0] = lse2 - oy;
    ri[1] = (pred == y) ? 1.0f : 0.0f;
    ri[2] = pois ? 1.0f : 0.0f;
    ri[3] = (pois && pred == y) ? 1.0f : 0.0f;
  }
}

// one block: deterministic batch reduction -> metrics (loss mean as double bits, counts)
// lw: the batch-mean loss is weighted by lw before it is accumulated -- data parallelism passes
// B_local / B_global, so the per-rank words SUM over ranks to the global batch mean even when
// the last batch of an epoch splits unevenly (parallel_dp.reduce_metrics)
__device__ __forceinline__ void metrics_body(const float* rowinfo, int B, int64_t* metrics, double lw = 1.0) {
  double s = 0.0;
  long long c = 0, p = 0, h = 0;
  for (int i = threadIdx.x; i < B; i += kT) {
    s += rowinfo[i * 4 + 0];
    c += (long long)rowinfo[i * 4 + 1];
    p += (long long)rowinfo[i * 4 + 2];
    h += (long long)rowinfo[i * 4 + 3];
  }
  __shared__ double rs[kT];
  __shared__ long long rc[3][kT];
  rs[threadIdx.x] = s;
  rc[0][threadIdx.x] = c;
  rc[1][threadIdx.x] = p;
  rc[2][threadIdx.x] = h;
  __syncthreads();
  for (int o = kT / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      rs[threadIdx.x] += rs[threadIdx.x + o];
      for (int j = 0; j < 3; ++j) rc[j][threadIdx.x] += rc[j][threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    double acc = __longlong_as_double(metrics[0]);
    acc += rs[0] * lw / B;
    metrics[0] = __double_as_longlong(acc);
    metrics[1] += B;
    metrics[2] += rc[0][0];
    metrics[3] += rc[1][0];
    metrics[4] += rc[2][0];
    metrics[5] += 1;
  }
}
__global__ void __launch_bounds__(kT) metrics_kernel(const float* rowinfo, int B, int64_t* metrics) {
  metrics_body(rowinfo, B, metrics);
}

#include "fc_head.inc"

// fc2 data gradient through dropout2/ReLU: da = (dz . W2) * scale2 * [d2 > 0]
__device__ __forceinline__ void fc2_bwd_body(const float* dz, const float* d2, const float* w2, int B, int K,
                                             float scale2, float* da, int bx, int nb) {
  const int64_t nd = (int64_t)B * 128;
  for (int64_t f = bx * (int64_t)kT + threadIdx.x; f < nd; f += (int64_t)nb * kT) {
    const int b = (int)(f / 128), j = (int)(f % 128);
    float s = 0.0f;
    for (int k = 0; k < K; ++k) s = fmaf(dz[(int64_t)b * K + k], w2[(int64_t)k * 128 + j], s);
    da[f] = d2[f] > 0.0f ? s * scale2 : 0.0f;
  }
}
__global__ void __launch_bounds__(kT) fc2_bwd_kernel(const float* dz, const float* d2, const float* w2, int B, int K,
                                                     float scale2, float* da) {
  fc2_bwd_body(dz, d2, w2, B, K, scale2, da, blockIdx.x, gridDim.x);
}

// fc1: sum the split-K partials in order, + bias, ReLU, dropout2 -> d2
__global__ void __launch_bounds__(kT) fc1_epilogue_kernel(const float* part, int ks, int B, const float* bias,
                                                          DropArgs drop, float* d2) {
  const int64_t e = blockIdx.x * (int64_t)kT + threadIdx.x;
  if (e >= (int64_t)B * 128) return;
  const float v = ordered_sum(part + e, (int64_t)B * 128, ks);
  d2[e] = drop_apply(drop, e, fmaxf(v + bias[e & 127], 0.0f));
}

// fc2 weight/bias gradient partials: grid (K, nsplit); 128 threads = hidden units
__device__ __forceinline__ void fc2_wgrad_body(const float* dz, const float* d2, int B, int K, int rows, float* part,
                                               int k, int sp, int j) {
  const int b0 = sp * rows, b1 = min(B, b0 + rows);
  float s = 0.0f, sb = 0.0f;
#pragma unroll 4
  for (int b = b0; b < b1; ++b) {
    const float g = dz[(int64_t)b * K + k];
    s = fmaf(g, d2[(int64_t)b * 128 + j], s);
    sb += g;
  }
  part[((int64_t)sp * K + k) * 129 + j] = s;
  if (j == 0) part[((int64_t)sp * K + k) * 129 + 128] = sb;
}
__global__ void __launch_bounds__(128) fc2_wgrad_kernel(const float* dz, const float* d2, int B, int K, int rows,
                                                       float* part) {
  fc2_wgrad_body(dz, d2, B, K, rows, part, blockIdx.x, blockIdx.y, threadIdx.x);
}

// fc2_wgrad_kernel and fc2_bwd_kernel in one launch (independent: both only read dz and d2):
// blocks [0, nw) run two 128-thread (k, split) groups each, the rest fc2_bwd's grid-stride loop
// metrics != nullptr: the last block reduces the loss kernel's per-row flags into the counters
__global__ void __launch_bounds__(kT) fc2_grads_kernel(const float* dz, const float* d2, const float* w2, int B, int K,
                                                       int rows, int nsplit, float* part, float scale2, float* da,
                                                       int nw, const float* rowinfo, int64_t* metrics, double lw) {
  const int nb = (int)gridDim.x - (metrics ? 1 : 0);
  if (metrics && (int)blockIdx.x == nb) {
    metrics_body(rowinfo, B, metrics, lw);
    return;
  }
  if ((int)blockIdx.x < nw) {
    const int pr = (int)blockIdx.x * 2 + (int)(threadIdx.x >> 7);
    if (pr < K * nsplit) fc2_wgrad_body(dz, d2, B, K, rows, part, pr % K, pr / K, threadIdx.x & 127);
    return;
  }
  fc2_bwd_body(dz, d2, w2, B, K, scale2, da, (int)blockIdx.x - nw, nb - nw);
}

__device__ __forceinline__ void fc2_wgrad_reduce_body(const float* part, int nsplit, int K, float* gw, float* gb, int e) {
  if (e >= K * 129) return;
  float s = 0.0f;
  for (int i = 0; i < nsplit; ++i) s += part[(int64_t)i * K * 129 + e];
  const int k = e / 129, j = e % 129;
  if (j < 128) gw[k * 128 + j] = s;
  else gb[k] = s;
}
__global__ void __launch_bounds__(kT) fc2_wgrad_reduce_kernel(const float* part, int nsplit, int K, float* gw,
                                                              float* gb) {
  fc2_wgrad_reduce_body(part, nsplit, K, gw, gb, blockIdx.x * kT + threadIdx.x);
}

// stage 1 of the slab reduction: group sums (each group = up to 32 slabs, in order)
// bs.part != nullptr: the last grid row (blockIdx.y == gridDim.y - 1) instead computes the
// independent bias-gradient column sums, one block per column
__global__ void __launch_bounds__(kT) slab_group_kernel(const float* slab, int nslab, int64_t total, int gsize,
                                                        float* part, BiasSum bs) {
  if (bs.part != nullptr && blockIdx.y == gridDim.y - 1) {
    if ((int)blockIdx.x < bs.ncols) partial_sum_body(bs.part, bs.nblk, bs.out, nullptr, nullptr, blockIdx.x);
    return;
  }
  const int64_t e = blockIdx.x * (int64_t)kT + threadIdx.x;
  if (e >= total) return;
  const int g = blockIdx.y;
  const int i0 = g * gsize, i1 = min(nslab, i0 + gsize);
  part[(int64_t)g * total + e] = ordered_sum(slab + (int64_t)i0 * total + e, total, i1 - i0);
}

// column sums of a (rows, cols) matrix: one block per column, fixed reduction tree
__device__ __forceinline__ void colsum_body(const float* x, int rows, int cols, float* out, int c) {
  double s = 0.0;
  for (int r = threadIdx.x; r < rows; r += kT) s += x[(int64_t)r * cols + c];
  __shared__ double red[kT / kWave];
  s = abd::wave_sum_d(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) out[c] = (float)(red[0] + red[1] + red[2] + red[3]);
}
__global__ void __launch_bounds__(kT) colsum_kernel(const float* x, int rows, int cols, float* out) {
  colsum_body(x, rows, cols, out, blockIdx.x);
}
// fc2_wgrad_reduce_kernel and colsum_kernel (fc1 bias gradient) in one launch: blocks [0, cols)
// are the column sums, the rest the split reduction
__global__ void __launch_bounds__(kT) fc2_reduce_colsum_kernel(const float* part, int nsplit, int K, float* gw,
                                                               float* gb, const float* x, int rows, int cols,
                                                               float* out) {
  if ((int)blockIdx.x < cols) {
    colsum_body(x, rows, cols, out, blockIdx.x);
    return;
  }
  fc2_wgrad_reduce_body(part, nsplit, K, gw, gb, ((int)blockIdx.x - cols) * kT + threadIdx.x);
}

// ------------------------------------------------------------------ Adam (torch single-tensor semantics)
struct AdamArgs {
  float* p;
  const float* g;
  float* m;
  float* v;
  int64_t n;
  float omb1, beta2, omb2, step_size, bc2_sqrt, eps;
};
__device__ __forceinline__ void adam_elem(const AdamArgs& a, int64_t i) {
  const float gi = a.g[i];
  const float mi = a.m[i] + a.omb1 * (gi - a.m[i]);
  const float vi = a.v[i] * a.beta2 + a.omb2 * gi * gi;
  a.m[i] = mi;
  a.v[i] = vi;
  const float denom = sqrtf(vi) / a.bc2_sqrt + a.eps;
  a.p[i] = a.p[i] + (-a.step_size) * (mi / denom);
}
__global__ void __launch_bounds__(kT) adam_kernel(AdamArgs a) {
  for (int64_t i = blockIdx.x * (int64_t)kT + threadIdx.x; i < a.n; i += (int64_t)gridDim.x * kT) adam_elem(a, i);
}
// The single-rank train step's last two launches in one: blocks [0, 320) reduce one conv1 weight /
// bias gradient column each from conv1_wgrad_kernel's partials (partial_sum_body: the gradient
// buffer gets the same value) and apply Adam to that parameter; the other blocks run Adam over
// parameters [320, n).  conv1.weight / conv1.bias are the flat buffer's first 256 + 64 entries.
__global__ void __launch_bounds__(kT) adam_c1_kernel(AdamArgs a, const float* part, int nblk) {
  constexpr int kC1 = 5 * 64;
  if ((int)blockIdx.x < kC1) {
    const int col = blockIdx.x;
    float* g = const_cast<float*>(a.g);
    partial_sum_body(part, nblk, nullptr, g, g + 4 * 64, col);
    if (threadIdx.x == 0) adam_elem(a, col < 4 * 64 ? (col % 64) * 4 + col / 64 : col);
    return;
  }
  const int64_t nb = (int64_t)gridDim.x - kC1;
  for (int64_t i = kC1 + ((int64_t)blockIdx.x - kC1) * kT + threadIdx.x; i < a.n; i += nb * kT) adam_elem(a, i);
}

// d z = d o - exp(o) * sum(d o)   (o = log_softmax(z))
__global__ void __launch_bounds__(kT) logsoftmax_bwd_kernel(const float* dlp, const float* lp, int B, int K, float* dz) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (kT / kWave) + (threadIdx.x >> 6);
  if (row >= B) return;
  const bool act = lane < K;
  const float d = act ? dlp[(int64_t)row * K + lane] : 0.0f;
  const float sd = abd::wave_sum(d);
  if (act) dz[(int64_t)row * K + lane] = d - expf(lp[(int64_t)row * K + lane]) * sd;
}

int grid_for(int64_t total, int cap = 4096) {
  return (int)std::max<int64_t>(1, std::min<int64_t>((total + kT - 1) / kT, cap));
}

}  // namespace

// ======================================================================= host orchestration
struct abd_cnn {
  Geo g;
  int max_batch;
  int64_t off[P_COUNT + 1];
  int precision = ABD_PREC_F32_SPLIT;  // abd_smallcnn_set_precision (include/abd.h)
};

namespace {

struct Work {
  float *p1, *r2, *p2, *r3, *p3d, *d2, *logp, *dz, *rowinfo;
  float *dp3, *da, *dz3, *dp2, *dz2, *dp1;
  float *w2f, *w2d, *w3f, *w3d, *f1t;
  float* part;
  float *partb3, *partb2;  // BN3 / BN2 backward-apply bias partials (read by the side stream's slab reduction)
  float* xh3;              // fused fc head: xhat of each pool3-selected element (B x flat)
  float* hslab;            // fused fc head: fc1 split-K partials (ks x B x 128)
  float* part3;            // fused fc head: BN3 backward sums per (row block, feature tile, channel slot)
  float* daT;              // fused fc head: da transposed (128 x B), head_dgrad's A operand
  uint16_t* p1s;           // conv2 plane mode: pool1 output m as exact bf16 planes [3][n_p1]
  uint16_t* dz2s;          // conv2 plane mode: BN2-backward output dz2 as planes [3][n_r2]
  unsigned* tickets;       // guarded BN fallbacks' arrival tickets (zeroed by the prep blocks)
  int ntickets;
  float* w2fold;           // BN1 fold (bn_finalize_kernel): conv2 forward weights times alpha
  double* ft2;             //   and the beta' bias terms [ci][co]
  float* slab;
  float* slab2;   // group sums of slab (hierarchical reduce) / fc1 split-K partials
  float4* coef;   // 3 x 64
  BCoef* bcoef;   // 3 x 64
  uint8_t *mask1, *mask2;
  size_t bytes;
};

constexpr int kConv2Slabs = 1024, kConv3Slabs = 1024, kFc1MSplit = 8, kFc1KSplit = 48, kFc2Split = 16;
constexpr int kSlabGroup = 32;

// conv1 kernels loop over (utterance, rows) chunks; the capped grid keeps the BN partial count small.
// ABD_C1_ROWS / ABD_C1_CAP override (tuning).
int env_int(const char* name, int dflt) {
  const char* v = getenv(name);
  return v ? atoi(v) : dflt;
}
int c1_rows() { return kR1; }
int64_t nchunks_conv1(const Geo& g, int64_t B) { return B * ((g.H1 + c1_rows() - 1) / c1_rows()); }
int64_t nblk_conv1(const Geo& g, int64_t B) { return std::min<int64_t>(nchunks_conv1(g, B), 2048); }
// resident blocks of conv1_stats_fold_kernel over the device
int64_t c1f_blocks() {
  static int64_t n = 0;
  if (n == 0) {
    int dev = 0, cu = 256, per = 1;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, reinterpret_cast<const void*>(&conv1_stats_fold_kernel),
                                                       kT, 0);
    n = (int64_t)cu * std::max(1, per);
  }
  return n;
}
// resident blocks of conv1_wgrad_kernel over the device (ABD_C1W_CAP overrides)
template <bool FULL>
int64_t c1w_blocks() {
  static int64_t n = 0;
  if (n == 0) {
    int dev = 0, cu = 256, per = 1;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, reinterpret_cast<const void*>(&conv1_wgrad_kernel<FULL>),
                                                       kT, 0);
    n = (int64_t)cu * std::max(1, per);
  }
  return n;
}

// fused fc head launch geometry (fc_head.inc): head_fwd row tiles of 32 x position splits of pp pooled
// positions (pp a power of two <= 8, the smallest that keeps the grid <= 512 blocks), head_dgrad
// 32-feature tiles x 128-row blocks
struct HeadPlan {
  int rt, ks, pp, nft, nrb;
};
HeadPlan head_plan(const Geo& g, int64_t B) {
  HeadPlan h;
  h.rt = (int)((B + 31) / 32);
  const int P = g.flat / 32;
  h.pp = 1;
  while (h.pp < 8 && (int64_t)h.rt * ((P + h.pp - 1) / h.pp) > 512) h.pp *= 2;
  h.ks = (P + h.pp - 1) / h.pp;
  h.nft = g.flat / 32;
  h.nrb = (int)((B + kHeadRB - 1) / kHeadRB);
  return h;
}
// the single-rank train step runs the fused fc head; SyncBN steps keep the round-2 launches (BN3's
// sums are all-reduced between the loss and the BN3 backward)
bool head_on() { return true; }

PoolArgs pool_args(const Geo& g, int layer, int64_t B);
int head_napply(const PoolArgs& a, int64_t B);

Work layout(const abd_cnn* net, int64_t B, char* base) {
  const Geo& g = net->g;
  Work w{};
  size_t off = 0;
  auto take = [&](size_t bytes) -> char* {
    char* p = base ? base + off : nullptr;
    off += (bytes + 255) & ~(size_t)255;
    return p;
  };
  auto F = [&](int64_t n) { return reinterpret_cast<float*>(take((size_t)n * sizeof(float))); };
  const int64_t n_p1 = B * g.H1 * g.W1p * 64, n_r2 = B * g.H2 * g.W2 * 64, n_p2 = B * g.H2p * g.W2p * 64;
  const int64_t n_r3 = B * g.H3 * g.W3 * 32;
  w.p1 = F(n_p1);
  w.r2 = F(n_r2);
  w.p2 = F(n_p2);
  w.r3 = F(n_r3);
  w.p3d = F(B * g.flat);
  w.d2 = F(B * 128);
  w.logp = F(B * g.K);
  w.dz = F(B * g.K);
  w.rowinfo = F(B * 4);
  w.dp3 = F(B * g.flat);
  w.da = F(B * 128);
  w.dz3 = F(n_r3);
  w.dp2 = F(n_p2);
  w.dz2 = F(n_r2);
  w.dp1 = F(n_p1);
  w.w2f = F(64 * 256);
  w.w2d = F(64 * 256);
  w.w3f = F(32 * 256);
  w.w3d = F(64 * 128);
  w.f1t = F(128LL * g.flat);
  // partial buffers: max over users (5 values x 64 channels x blocks)
  const int64_t pb = std::max<int64_t>({nblk_conv1(g, B) * 64 * 5, 4096LL * 64 * 2,
                                        ((B * g.H2 * g.W2 + kBM - 1) / kBM) * 64 * 2});
  w.part = F(pb);
  const int64_t slab = std::max<int64_t>({(int64_t)kConv2Slabs * 64 * 256, (int64_t)kConv3Slabs * 32 * 256,
                                          (int64_t)kFc1MSplit * 128 * g.flat});
  w.slab = F(slab);
  w.slab2 = F(std::max<int64_t>({(int64_t)(kConv2Slabs / kSlabGroup + 1) * 64 * 256, (int64_t)kFc1KSplit * B * 128,
                                 (int64_t)kFc2Split * 64 * 129}));
  w.coef = reinterpret_cast<float4*>(take(3 * 64 * sizeof(float4)));
  w.bcoef = reinterpret_cast<BCoef*>(take(3 * 64 * sizeof(BCoef)));
  w.mask1 = reinterpret_cast<uint8_t*>(take((size_t)B * g.flat));
  w.mask2 = reinterpret_cast<uint8_t*>(take((size_t)B * 128));
  // grid_for caps the apply grids at 4096 blocks; the fused head's apply grid is uncapped
  w.partb3 = F(std::max<int64_t>(4096, head_napply(pool_args(g, 3, B), B)) * 64);
  w.partb2 = F(4096LL * 64);
  w.w2fold = F(64 * 256);     // BN1 fold: conv2 weights times alpha, bias terms (double)
  w.ft2 = reinterpret_cast<double*>(take(64 * 64 * sizeof(double)));
  {
    const HeadPlan hp = head_plan(g, B);
    w.xh3 = F(B * g.flat);
    w.hslab = F((int64_t)hp.ks * B * 128);
    w.part3 = F((int64_t)hp.nrb * hp.nft * 64);
    w.daT = F(128 * B);
  }
  w.p1s = reinterpret_cast<uint16_t*>(take((size_t)3 * n_p1 * sizeof(uint16_t)));
  w.dz2s = reinterpret_cast<uint16_t*>(take((size_t)3 * n_r2 * sizeof(uint16_t)));
  w.ntickets = kGuardTickets;
  w.tickets = reinterpret_cast<unsigned*>(take((size_t)w.ntickets * sizeof(unsigned)));
  w.bytes = off;
  return w;
}

struct Params {
  const float* p[P_COUNT];
};

Params params_of(const abd_cnn* net, const float* flat) {
  Params r;
  for (int i = 0; i < P_COUNT; ++i) r.p[i] = flat + net->off[i];
  return r;
}

PrepArgs prep_args(const Params& P, const Work& w, const Geo& g) {
  return PrepArgs{P.p[P_C2W], P.p[P_C3W], P.p[P_F1W], g.flat, w.w2f, w.w2d, w.w3f, w.w3d, w.f1t, w.tickets, w.ntickets};
}
unsigned prep_blocks(const Geo& g) { return (unsigned)grid_for(64 * 256 + 32 * 256 + 128LL * g.flat); }

PoolArgs pool_args(const Geo& g, int layer, int64_t B) {
  PoolArgs a{};
  a.B = (int)B;
  if (layer == 2) {
    a.H = g.H2;
    a.W = g.W2;
    a.C = 64;
    a.Ho = g.H2p;
    a.Wo = g.W2p;
    a.kh = a.kw = 2;
    a.sh = a.sw = 2;
    a.ph = 1;
    a.pw = 1;
  } else {
    a.H = g.H3;
    a.W = g.W3;
    a.C = 32;
    a.Ho = g.H3p;
    a.Wo = g.W3p;
    a.kh = a.kw = 2;
    a.sh = a.sw = 2;
    a.ph = 0;
    a.pw = 1;
    a.flat_n = g.flat;
  }
  return a;
}

// extended window grid of bn_bwd_apply_kernel (windows tile the input: kernel == stride)
int win_ext_h(const PoolArgs& a) { return std::max(a.Ho, (a.H + a.ph + a.sh - 1) / a.sh); }
int win_ext_w(const PoolArgs& a) { return std::max(a.Wo, (a.W + a.pw + a.sw - 1) / a.sw); }
// head_bwd_kernel's BN3 apply blocks: kHeadIT windows x 4 channels per thread, no grid stride
int head_napply(const PoolArgs& a, int64_t B) {
  return (int)((B * win_ext_h(a) * win_ext_w(a) * 32 / 4 + kHeadIT * kT - 1) / (kHeadIT * kT));
}

// ---- fused fc head (fc_head.inc): arguments and the three launches
HeadArgs head_args(const abd_cnn* net, const Work& w, const Params& P, float* grads, int64_t B,
                   const DropArgs& d1, const DropArgs& d2, const int64_t* labels, const int64_t* ind, float inv_batch,
                   float* logprobs_out, int64_t* metrics, double loss_w) {
  const Geo& g = net->g;
  const HeadPlan hp = head_plan(g, B);
  HeadArgs a{};
  a.B = (int)B;
  a.F = g.flat;
  a.P = g.flat / 32;
  a.K = g.K;
  a.ks = hp.ks;
  a.nft = hp.nft;
  a.nrb = hp.nrb;
  a.pool = pool_args(g, 3, B);
  a.pool.r = w.r3;
  a.pool.coef = w.coef + 128;
  a.pool.dp = w.dp3;
  a.drop1 = d1;
  a.drop1.mask_out = w.mask1;
  a.drop2 = d2;
  a.drop2.mask_out = w.mask2;
  a.f1t = w.f1t;
  a.w1 = P.p[P_F1W];
  a.b1 = P.p[P_F1B];
  a.w2 = P.p[P_F2W];
  a.b2 = P.p[P_F2B];
  a.bn3w = P.p[P_BN3W];
  a.labels = labels;
  a.ind = ind;
  a.inv_batch = inv_batch;
  a.p3d = w.p3d;
  a.xh3 = w.xh3;
  a.slab = w.hslab;
  a.d2 = w.d2;
  a.logp = logprobs_out ? logprobs_out : w.logp;
  a.dz = w.dz;
  a.rowinfo = w.rowinfo;
  a.da = w.da;
  a.dp3 = w.dp3;
  a.daT = w.daT;
  a.mask1 = w.mask1;
  a.part3 = w.part3;
  float* G[P_COUNT];
  for (int i = 0; i < P_COUNT; ++i) G[i] = grads ? grads + net->off[i] : nullptr;
  a.g_f1w = G[P_F1W];
  a.g_f1b = G[P_F1B];
  a.g_f2w = G[P_F2W];
  a.g_f2b = G[P_F2B];
  a.g_bn3w = G[P_BN3W];
  a.g_bn3b = G[P_BN3B];
  a.metrics = metrics;
  a.loss_w = loss_w;
  a.dz3 = w.dz3;
  a.partb3 = w.partb3;
  a.hx = win_ext_h(a.pool);
  a.wx = win_ext_w(a.pool);
  a.n_w1 = 4 * ((g.flat + 31) / 32);
  a.n_w2 = 4 * ((g.K + 31) / 32) + (g.K + 128 + kHeadW2 - 1) / kHeadW2;  // fc2 weight tiles + bias sums
  a.n_apply = head_napply(a.pool, B);
  return a;
}

// launch 1 (forward: pool3 + dropout1 + fc1 partials) / 2 (row head, then dp3 + BN3 sums) /
// 3 (gradients + BN3 apply)
int launch_head(int which, const HeadArgs& a, hipStream_t s) {
  if (which == 1) {
    const dim3 grid((unsigned)((a.B + 31) / 32), (unsigned)a.ks);
    const int pp = (a.P + a.ks - 1) / a.ks;
    abd::prof_begin(abd::PH_HEAD_FWD, s);
    if (pp <= 1) head_fwd_kernel<1><<<grid, kT, 0, s>>>(a);
    else if (pp <= 2) head_fwd_kernel<2><<<grid, kT, 0, s>>>(a);
    else if (pp <= 4) head_fwd_kernel<4><<<grid, kT, 0, s>>>(a);
    else head_fwd_kernel<8><<<grid, kT, 0, s>>>(a);
    abd::prof_end(abd::PH_HEAD_FWD, s);
  } else if (which == 2) {
    abd::prof_begin(abd::PH_HEAD_MID, s);
    head_row_kernel<<<(unsigned)((a.B + kHeadRows - 1) / kHeadRows), kT, 0, s>>>(a);
    abd::prof_end(abd::PH_HEAD_MID, s);
    ABD_LAUNCH_CHECK();
    abd::prof_begin(abd::PH_HEAD_DGRAD, s);
    head_dgrad_kernel<<<dim3((unsigned)a.nft, (unsigned)a.nrb), kT, 0, s>>>(a);
    abd::prof_end(abd::PH_HEAD_DGRAD, s);
  } else {
    abd::prof_begin(abd::PH_HEAD_BWD, s);
    head_bwd_kernel<<<(unsigned)(a.n_w1 + a.n_w2 + 1 + a.n_apply), kT, 0, s>>>(a);
    abd::prof_end(abd::PH_HEAD_BWD, s);
  }
  ABD_LAUNCH_CHECK();
  return 0;
}

NTArgs conv_fwd_args(const float* src, int Hs, int Ws, int Cs, int Ho, int Wo, int64_t B, const float* Bw, int N,
                     const float* bias, float* out) {
  NTArgs a{};
  a.src = src;
  a.Hs = Hs;
  a.Ws = Ws;
  a.Cs = Cs;
  a.Ho = Ho;
  a.Wo = Wo;
  a.M = (int)(B * Ho * Wo);
  a.taps = 4;
  for (int t = 0; t < 4; ++t) {
    a.dh[t] = t >> 1;
    a.dw[t] = t & 1;
  }
  a.Bw = Bw;
  a.ldb = 4 * Cs;
  a.N = N;
  a.bias = bias;
  a.out = out;
  a.ldc = N;
  return a;
}

NTArgs conv_dgrad_args(const float* dz, int Hd, int Wd, int Cd, int Ho, int Wo, int64_t B, const float* Wdg, int N,
                       float* out) {
  NTArgs a = conv_fwd_args(dz, Hd, Wd, Cd, Ho, Wo, B, Wdg, N, nullptr, out);
  for (int t = 0; t < 4; ++t) {
    a.dh[t] = -(t >> 1);
    a.dw[t] = -(t & 1);
  }
  return a;
}

TNArgs conv_wgrad_args(const float* dz, int Cout, const float* src, int Hs, int Ws, int Cs, int Ho, int Wo, int64_t B,
                       int nslab, float* slab) {
  TNArgs a{};
  a.D = dz;
  a.ldd = Cout;
  a.src = src;
  a.Hs = Hs;
  a.Ws = Ws;
  a.Cs = Cs;
  a.Ho = Ho;
  a.Wo = Wo;
  a.M = (int)(B * Ho * Wo);
  a.taps = 4;
  for (int t = 0; t < 4; ++t) {
    a.dh[t] = t >> 1;
    a.dw[t] = t & 1;
  }
  a.N = Cout;
  a.Ktot = 4 * Cs;
  a.mchunk = (a.M + nslab - 1) / nslab;
  a.mchunk = (a.mchunk + 31) / 32 * 32;
  a.slab = slab;
  return a;
}

// conv_wgrad_trp_kernel<R, NB, NS, MAXS> launch; -1 when the geometry is not this instantiation's
// geometry check of conv_wgrad_trp_kernel<R, NB, NS, MAXS, ...> (also used to decide the plane mode)
template <int R, int NB, int NS, int MAXS>
bool trp_fits(int Ho, int Wo, int Hs, int Ws) {
  if (Ws != Wo + 1 || Hs < Ho + 1) return false;
  const int Qd = ((R * Ws + 15) / 16) * 16, Qs = Qd + Ws + 1;
  if (Qd != 16 * NS || (Qd * (NB / 4) + Qs * 16 + kT - 1) / kT > MAXS) return false;
  return 2 * (size_t)(Qd + Qs + 1) * kTrRow <= 160 * 1024;
}
// pl: pre-split planes (dzs / srcs, plane strides) for the PS instantiation, else nullptr
struct WgPlanes {
  const uint16_t* dzs;
  const uint16_t* srcs;
  int64_t dzplane, srcplane;
};
template <int R, int NB, int NS, int MAXS, int NP = 3, bool PS = false>
int launch_wgrad_trp_n(const float* dz, const float* src, int Ho, int Wo, int Hs, int Ws, int64_t B, int max_slabs,
                       float* slab, int phase, hipStream_t s, const WgPlanes* pl = nullptr) {
  if (!trp_fits<R, NB, NS, MAXS>(Ho, Wo, Hs, Ws)) return -1;
  if (PS && pl == nullptr) return -1;
  const int Qd = ((R * Ws + 15) / 16) * 16, Qs = Qd + Ws + 1;
  WGArgs a{};
  a.dz = dz;
  a.src = src;
  if (PS) {
    a.dzs = pl->dzs;
    a.srcs = pl->srcs;
    a.dzplane = pl->dzplane;
    a.srcplane = pl->srcplane;
  }
  a.Ho = Ho;
  a.Wo = Wo;
  a.Hs = Hs;
  a.Ws = Ws;
  a.R = R;
  a.cpb = (Ho + R - 1) / R;
  a.nchunks = (int)(B * a.cpb);
  a.slab = slab;
  const size_t lds = 2 * (size_t)(Qd + Qs + 1) * kTrRow;
  if (lds > 160 * 1024) return -1;
  auto* kern = &conv_wgrad_trp_kernel<R, NB, NS, MAXS, NP, PS>;
  static size_t cached = 0;
  static int per_cu = 1, n_cu = 256;
  if (cached != lds) {
    ABD_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds));
    int dev = 0;
    ABD_HIP(hipGetDevice(&dev));
    ABD_HIP(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
    ABD_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(kern), kT, lds));
    per_cu = std::max(1, per_cu);
    cached = lds;
  }
  int grid = (int)std::min<int64_t>({(int64_t)a.nchunks, (int64_t)n_cu * per_cu, (int64_t)max_slabs});
  a.per = (a.nchunks + grid - 1) / grid;
  grid = (a.nchunks + a.per - 1) / a.per;
  if (phase >= 0) abd::prof_begin(phase, s);
  kern<<<grid, kT, lds, s>>>(a);
  if (phase >= 0) abd::prof_end(phase, s);
  ABD_LAUNCH_CHECK();
  return grid;
}

// conv2's pre-split weight gradient: the first trp instantiation launch_wgrad_tr<.., 64> would pick
template <int R>
bool trp_planes_fit(int Ho, int Wo, int Hs, int Ws) {
  return trp_fits<6, 64, 5, 11>(Ho, Wo, Hs, Ws) || trp_fits<R, 64, 2, 5>(Ho, Wo, Hs, Ws) ||
         trp_fits<R, 64, 3, 8>(Ho, Wo, Hs, Ws) || trp_fits<R, 64, 1, 4>(Ho, Wo, Hs, Ws);
}
template <int R, int NP>
int launch_wgrad_tr_planes(int Ho, int Wo, int Hs, int Ws, int64_t B, int max_slabs, float* slab, int phase,
                           hipStream_t s, const WgPlanes& pl) {
  int r = launch_wgrad_trp_n<6, 64, 5, 11, NP, true>(nullptr, nullptr, Ho, Wo, Hs, Ws, B, max_slabs, slab, phase, s, &pl);
  if (r < 0) r = launch_wgrad_trp_n<R, 64, 2, 5, NP, true>(nullptr, nullptr, Ho, Wo, Hs, Ws, B, max_slabs, slab, phase, s, &pl);
  if (r < 0) r = launch_wgrad_trp_n<R, 64, 3, 8, NP, true>(nullptr, nullptr, Ho, Wo, Hs, Ws, B, max_slabs, slab, phase, s, &pl);
  if (r < 0) r = launch_wgrad_trp_n<R, 64, 1, 4, NP, true>(nullptr, nullptr, Ho, Wo, Hs, Ws, B, max_slabs, slab, phase, s, &pl);
  return r;
}
// the transpose-read weight gradient for the f32split / bf16 modes: the first trp instantiation
// whose staging fits the geometry (conv2 at W = 40, Ws = 13: 6-row chunks fill 72 of 80 staged
// positions; 2-row: 24 of 32), -1 when none does (the caller then takes conv_wgrad_rows_kernel)
template <int R, int NB, int NP = 3>
int launch_wgrad_tr(const float* dz, const float* src, int Ho, int Wo, int Hs, int Ws, int64_t B, int max_slabs,
                    float* slab, int phase, hipStream_t s) {
  int r = -1;
  if constexpr (NB == 64) {
    r = launch_wgrad_trp_n<6, NB, 5, 11, NP>(dz, src, Ho, Wo, Hs, Ws, B, max_slabs, slab, phase, s);
    if (r < 0) r = launch_wgrad_trp_n<R, NB, 2, 5, NP>(dz, src, Ho, Wo, Hs, Ws, B, max_slabs, slab, phase, s);
    if (r < 0) r = launch_wgrad_trp_n<R, NB, 3, 8, NP>(dz, src, Ho, Wo, Hs, Ws, B, max_slabs, slab, phase, s);
    if (r < 0) r = launch_wgrad_trp_n<R, NB, 1, 4, NP>(dz, src, Ho, Wo, Hs, Ws, B, max_slabs, slab, phase, s);
  } else {
    r = launch_wgrad_trp_n<R, NB, 2, 4, NP>(dz, src, Ho, Wo, Hs, Ws, B, max_slabs, slab, phase, s);
    if (r < 0) r = launch_wgrad_trp_n<R, NB, 3, 6, NP>(dz, src, Ho, Wo, Hs, Ws, B, max_slabs, slab, phase, s);
    if (r < 0) r = launch_wgrad_trp_n<R, NB, 1, 2, NP>(dz, src, Ho, Wo, Hs, Ws, B, max_slabs, slab, phase, s);
  }
  return r;
}

template <int NB, int CIN>
int launch_wgrad_rows(const float* dz, const float* src, int Ho, int Wo, int Hs, int Ws, int64_t B, int R,
                      int max_slabs, float* slab, int phase, hipStream_t s) {
  ABD_CHECK(Ws == Wo + 1 && Hs >= Ho + 1, ABD_E_UNSUPPORTED, "wgrad geometry");
  WGArgs a{};
  a.dz = dz;
  a.src = src;
  a.Ho = Ho;
  a.Wo = Wo;
  a.Hs = Hs;
  a.Ws = Ws;
  a.R = std::max(1, std::min(R, Ho));
  a.cpb = (Ho + a.R - 1) / a.R;
  a.nchunks = (int)(B * a.cpb);
  // dz on the Ws-strided grid; source rows + one slack row (a pad position's dh = 1 tap
  // reads one row past the chunk)
  a.dsz = ((a.R * Ws + 2) * NB + 3) & ~3;  // + positions for the one-ahead read
  a.bsz = (a.dsz + (a.R + 2) * Ws * CIN + 3) & ~3;
  a.slab = slab;
  const size_t lds = 2 * (size_t)a.bsz * sizeof(float);
  auto* kern = &conv_wgrad_rows_kernel<NB, CIN>;
  static size_t cached_lds = 0;
  static int per_cu = 1, n_cu = 256;
  if (cached_lds != lds) {
    ABD_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds));
    int dev = 0;
    ABD_HIP(hipGetDevice(&dev));
    ABD_HIP(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
    ABD_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(kern), kT, lds));
    per_cu = std::max(1, per_cu);
    cached_lds = lds;
  }
  int grid = (int)std::min<int64_t>({(int64_t)a.nchunks, (int64_t)n_cu * per_cu, (int64_t)max_slabs});
  a.per = (a.nchunks + grid - 1) / grid;
  grid = (a.nchunks + a.per - 1) / a.per;
  if (phase >= 0) abd::prof_begin(phase, s);
  kern<<<grid, kT, lds, s>>>(a);
  if (phase >= 0) abd::prof_end(phase, s);
  ABD_LAUNCH_CHECK();
  return grid;
}


// conv_ws_split_kernel / conv_ws_dma_kernel: persistent blocks, one per CU
int ws_grid() {
  static int n = 0;
  if (n == 0) {
    int dev = 0, cu = 256;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, dev);
    n = std::max(1, cu);
  }
  return n;
}
// blocks of a launch: one 8-wave block per CU (conv3's 48 KB of weights and 132-190 VGPRs also fit
// only one).  Small problems (FlowMur's 32 x 13 input: conv2 has 23 k rows at B = 256) get no more
// blocks than give every wave one 32-row tile: each block stages the whole weight operand into its
// LDS, so the full grid would stage it 256 times for ~11 rows per wave.
// rows_per_block: 32 per computing wave -- 8 for the split / DMA / pre-split kernels, 4 for the
// wave-specialised kernel (4 consumers + 4 producers; round 5: FlowMur's conv3 forward, M = 3,840,
// ran 15 blocks of two serial tiles per consumer instead of 30 of one)
int ws_blocks(int64_t M, int rows_per_block = 8 * 32) {
  const int64_t need = (M + rows_per_block - 1) / rows_per_block;
  return (int)std::max<int64_t>(1, std::min<int64_t>(ws_grid(), need));
}
// 32-bit buffer offsets of the weight-stationary kernels (their A operand is one buffer resource)
bool ws_fits(const NTArgs& a) {
  return a.taps == 4 && a.ksplit <= 1 && a.ldb == 4 * a.Cs && a.ldc == a.N &&
         (int64_t)a.Hs * a.Ws * a.Cs * 4 * (a.M / (a.Ho * a.Wo)) < 0x7ffffff0LL;
}
// ABD_WS_DMA: 0 direct-load kernel everywhere, 1 (default) LDS-DMA kernel for the forward GEMMs,
// 2 LDS-DMA for the data gradients too (read at each launch: tests/test_gpu_conv_tiles.py runs all three)
int ws_dma_mode() { return env_int("ABD_WS_DMA", 1); }
// Largest staged span (positions) of any 32 consecutive output rows of conv_ws_dma_kernel: the
// rows' source indices repeat with the image (period Ho*Wo), so every window over two images plus
// one tile is scanned once per geometry (cached).
int dma_span(const NTArgs& a) {
  static std::mutex mu;
  static std::map<std::array<int, 12>, int> cache;
  const std::array<int, 12> key{a.Hs, a.Ws, a.Ho, a.Wo, a.dh[0], a.dh[1], a.dh[2], a.dh[3], a.dw[0], a.dw[1], a.dw[2], a.dw[3]};
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  const int HoWo = a.Ho * a.Wo, n = 2 * HoWo + 32;
  int tmin = 0, tmax = 0;
  for (int t = 0; t < 4; ++t) {
    tmin = std::min(tmin, a.dh[t] * a.Ws + a.dw[t]);
    tmax = std::max(tmax, a.dh[t] * a.Ws + a.dw[t]);
  }
  auto src = [&](int m) {
    const int b = m / HoWo, rem = m % HoWo, h = rem / a.Wo, w = rem % a.Wo;
    return (b * a.Hs + h) * a.Ws + w;
  };
  int span = 0;
  for (int m0 = 0; m0 + 32 <= n; ++m0) {
    int lo = INT32_MAX, hi = INT32_MIN;
    for (int r = 0; r < 32; ++r) {
      lo = std::min(lo, src(m0 + r));
      hi = std::max(hi, src(m0 + r));
    }
    span = std::max(span, hi + tmax - (lo + tmin) + 1);
  }
  cache[key] = span;
  return span;
}
// Which weight-stationary kernel launch_conv_ws_split takes for these arguments (its grid -- and
// EPI_CONV's partial count a.nblk -- depends on it: ws_nblk)
enum WsKind { WS_SPEC, WS_PRE, WS_DMA, WS_SPLIT };
template <int EPI, int NP, bool PA>
WsKind ws_kind(const NTArgs& a) {
  const int dma_mode = ws_dma_mode();
  const bool dma = dma_mode == 2 || (dma_mode == 1 && (EPI == EPI_CONV || (PA && NP == 1) ||
                                                      (ABD_WS_PRE >= 2 && NP == 3 && !PA && a.N == 64)));
  // the forward's taps never leave the source grid; the data gradient's are masked in the kernel
  const bool fwd_taps = a.dh[0] == 0 && a.dw[0] == 0 && a.dh[1] == 0 && a.dw[1] == 1 && a.dh[2] == 1 && a.dw[2] == 0 &&
                        a.dh[3] == 1 && a.dw[3] == 1 && a.Hs == a.Ho + 1 && a.Ws == a.Wo + 1;
  const bool dg_taps = a.dh[0] == 0 && a.dw[0] == 0 && a.dh[1] == 0 && a.dw[1] == -1 && a.dh[2] == -1 && a.dw[2] == 0 &&
                       a.dh[3] == -1 && a.dw[3] == -1;
  if ((!PA || NP == 1) && dma && (a.N == 64 || (a.N == 32 && !PA)) && a.Cs == 64 &&
      (EPI == EPI_CONV ? fwd_taps : (EPI == EPI_STORE && dg_taps)) && dma_span(a) <= kDmaSpan) {
    constexpr bool spec = ABD_WS_SPEC >= 2 || (ABD_WS_SPEC == 1 && EPI == EPI_CONV);
    if (PA && NP == 1) return ABD_BF16_SPEC ? WS_SPEC : WS_DMA;
    if (NP == 3 && a.N == 64 && ABD_WS_PRE) return spec ? WS_SPEC : WS_PRE;
    if (NP == 3 && a.N == 32 && ABD_WS_PRE >= 3) return spec ? WS_SPEC : WS_PRE;
    return WS_DMA;
  }
  return WS_SPLIT;
}
template <int EPI, int NP, bool PA>
int ws_nblk(const NTArgs& a) {
  return ws_blocks(a.M, ws_kind<EPI, NP, PA>(a) == WS_SPEC ? 4 * 32 : 8 * 32);
}
template <int EPI, int NP = 3, bool PA = false>
int launch_conv_ws_split(const NTArgs& a, hipStream_t s, int phase) {
  if (!ws_fits(a)) return -1;
  if (PA && (a.srcs == nullptr || a.N != 64 || a.Cs != 64)) return -1;
  const WsKind kind = ws_kind<EPI, NP, PA>(a);
  const int nb = ws_blocks(a.M, kind == WS_SPEC ? 4 * 32 : 8 * 32);
  if (EPI == EPI_CONV && a.part != nullptr && a.nblk != nb) return -1;
  if (phase >= 0) abd::prof_begin(phase, s);
  // K-step order (see the kernel): channel-group-major for the forward (conv2 0.147 -> 0.141 ms),
  // tap-major for the data gradient (0.133 vs 0.136 ms channel-major)
  const bool ko = EPI == EPI_CONV;
  // LDS-DMA A operand (conv_ws_dma_kernel): the forward 0.140 -> 0.130-0.134 ms; the f32split data
  // gradient measured no faster through it (r4_v4: 0.1309 direct vs 0.1316 staged), so it stays on
  // the direct kernel by default (ws_dma_mode); bf16's plane-operand data gradient is staged
  // (0.0702 -> 0.0683 ms).  conv3 (N = 32) runs the same kernels with one 32-column tile per wave.
  if (kind != WS_SPLIT) {
    if constexpr (PA && NP == 1) {
      if (kind == WS_SPEC) conv_ws_spec_kernel<EPI, 2, 1><<<dim3(nb), dim3(512), 0, s>>>(a);
      else conv_ws_dma_kernel<EPI, 1, 2, true><<<dim3(nb), dim3(512), 0, s>>>(a);
    } else if (kind == WS_SPEC && a.N == 64) conv_ws_spec_kernel<EPI><<<dim3(nb), dim3(512), 0, s>>>(a);
    else if (kind == WS_SPEC) conv_ws_spec_kernel<EPI, 1><<<dim3(nb), dim3(512), 0, s>>>(a);
    else if (kind == WS_PRE && a.N == 64) conv_ws_pre_kernel<EPI><<<dim3(nb), dim3(512), 0, s>>>(a);
    else if (kind == WS_PRE) conv_ws_pre_kernel<EPI, 1><<<dim3(nb), dim3(512), 0, s>>>(a);
    else if (a.N == 64) conv_ws_dma_kernel<EPI, NP><<<dim3(nb), dim3(512), 0, s>>>(a);
    else conv_ws_dma_kernel<EPI, NP, 1><<<dim3(nb), dim3(512), 0, s>>>(a);
  } else if (PA) {
    if (ko) conv_ws_split_kernel<EPI, 2, 64, 1, 8, 8, NP, true, true><<<dim3(nb), dim3(512), 0, s>>>(a);
    else conv_ws_split_kernel<EPI, 2, 64, 1, 8, 8, NP, true><<<dim3(nb), dim3(512), 0, s>>>(a);
  } else if (a.N == 64 && a.Cs == 64) {
    if (ko) conv_ws_split_kernel<EPI, 2, 64, 1, 8, 8, NP, false, true><<<dim3(nb), dim3(512), 0, s>>>(a);
    else conv_ws_split_kernel<EPI, 2, 64, 1, 8, 8, NP><<<dim3(nb), dim3(512), 0, s>>>(a);
  } else if (a.N == 32 && a.Cs == 64) {
    if (ko) conv_ws_split_kernel<EPI, 1, 64, 1, 4, 8, NP, false, true><<<dim3(nb), dim3(512), 0, s>>>(a);
    else conv_ws_split_kernel<EPI, 1, 64, 1, 4, 8, NP><<<dim3(nb), dim3(512), 0, s>>>(a);
  } else if (a.N == 64 && a.Cs == 32) {
    if (ko) conv_ws_split_kernel<EPI, 2, 32, 1, 4, 8, NP, false, true><<<dim3(nb), dim3(512), 0, s>>>(a);
    else conv_ws_split_kernel<EPI, 2, 32, 1, 4, 8, NP><<<dim3(nb), dim3(512), 0, s>>>(a);
  } else {
    if (phase >= 0) abd::prof_end(phase, s);
    return -1;
  }
  if (phase >= 0) abd::prof_end(phase, s);
  ABD_LAUNCH_CHECK();
  return 0;
}

// grid.x of an NT launch: one block per 128*MI-row tile (EPI_CONV's a.nblk must match)
template <int NB, int EPI, int MI = 1>
int nt_grid_x(const NTArgs& a) {
  return (a.M + kBM * MI - 1) / (kBM * MI);
}

template <int NB, int EPI, int MI = 1, int KC = kKC>
int launch_nt(const NTArgs& a, hipStream_t s, int phase) {
  if (a.Cs % KC != 0) return -1;
  dim3 grid(nt_grid_x<NB, EPI, MI>(a), (a.N + NB - 1) / NB, a.ksplit > 1 ? a.ksplit : 1);
  if (phase >= 0) abd::prof_begin(phase, s);
  gemm_nt_kernel<NB, EPI, MI, KC><<<grid, dim3(kT), 0, s>>>(a);
  if (phase >= 0) abd::prof_end(phase, s);
  ABD_LAUNCH_CHECK();
  return 0;
}

// dv != nullptr (conv weight gradients): the final reduction also derives the BatchNorm feeding the
// conv (slab_reduce_derive_kernel)
// fold (conv2 under the BN1 fold): the gradient is unfolded with the bias gradient bias.out
// gd: the small-gamma guard riding on the derivation (its partial count must be conv_cin, the grid)
template <class Guard = NoGuard>
int reduce_slabs(const Work& w, int nsl, int N, int Ktot, int conv_cin, float* out, hipStream_t s,
                 BiasSum bias = BiasSum{}, const DeriveArgs* dv = nullptr, const float4* fold = nullptr,
                 Guard gd = Guard{}) {
  const int64_t total = (int64_t)N * Ktot;
  const float* src = w.slab;
  int n = nsl;
  const unsigned gx = (unsigned)((total + kT - 1) / kT);
  const bool carry = bias.part != nullptr && nsl > kSlabGroup && (int64_t)gx >= bias.ncols;
  if (bias.part != nullptr && !carry) {
    partial_sum_kernel<<<(unsigned)bias.ncols, kT, 0, s>>>(bias.part, bias.nblk, bias.ncols, bias.out);
    ABD_LAUNCH_CHECK();
  }
  if (nsl > kSlabGroup) {
    const int G = (nsl + kSlabGroup - 1) / kSlabGroup;
    slab_group_kernel<<<dim3(gx, (unsigned)(G + (carry ? 1 : 0))), kT, 0, s>>>(w.slab, nsl, total, kSlabGroup,
                                                                                w.slab2, carry ? bias : BiasSum{});
    ABD_LAUNCH_CHECK();
    src = w.slab2;
    n = G;
  }
  if (dv != nullptr && conv_cin > 0)
    slab_reduce_derive_kernel<Guard><<<conv_cin, kT, 0, s>>>(src, n, N, Ktot, conv_cin, out, *dv, gd);
  else
    slab_reduce_kernel<<<grid_for(total), kT, 0, s>>>(src, n, N, Ktot, conv_cin, out, fold, bias.out);
  ABD_LAUNCH_CHECK();
  return 0;
}

// -------------------------------------------------------------- synchronised BatchNorm (host)
struct BnSync {
  double* buf = nullptr;
  int (*fn)(void*, int, int64_t, int64_t) = nullptr;
  void* ctx = nullptr;
  bool on() const { return buf != nullptr && fn != nullptr; }
};

BnSync bn_sync_of(const abd_train_args* a) {
  BnSync y;
  if (a && a->bn_sync_buf && a->bn_sync) {
    y.buf = a->bn_sync_buf;
    y.fn = a->bn_sync;
    y.ctx = a->bn_sync_ctx;
  }
  return y;
}

// point 0..2: forward bn1..bn3; 3..5: backward bn3..bn1
int sync_point(const BnSync& y, int point, int C) {
  const int rc = y.fn(y.ctx, point, (int64_t)point * ABD_BN_SYNC_STRIDE, 2 * C + 1);
  ABD_CHECK(rc == 0, ABD_E_INVALID, "bn_sync callback failed at point %d (%d)", point, rc);
  return 0;
}

// train-mode BatchNorm statistics -> coefficients (+ running statistics), per rank or synchronised
// fw / fwo / ft: BN1 fold outputs (bn_finalize_kernel; single rank only: bn1_fold_ok excludes SyncBN)
int bn_fwd_finalize(const BnSync& y, int point, const float* part, int nblk, int C, double count, const float* gamma,
                    const float* beta, float* rm, float* rv, float4* coef, int64_t* nbt, hipStream_t s,
                    const float* fw = nullptr, float* fwo = nullptr, double* ft = nullptr) {
  ABD_CHECK(fw == nullptr || !y.on(), ABD_E_UNSUPPORTED, "BN1 fold with SyncBN");
  if (!y.on()) {
    bn_finalize_kernel<<<C, kT, 0, s>>>(part, nblk, C, count, gamma, beta, rm, rv, coef, nbt, fw, fwo, ft);
    ABD_LAUNCH_CHECK();
    return 0;
  }
  double* buf = y.buf + (int64_t)point * ABD_BN_SYNC_STRIDE;
  bn_local_sums_kernel<<<C, kT, 0, s>>>(part, nblk, C, count, buf, nullptr, nullptr);
  ABD_LAUNCH_CHECK();
  if (sync_point(y, point, C)) return -1;
  bn_sync_finalize_kernel<<<1, 64, 0, s>>>(buf, C, gamma, beta, rm, rv, coef, nbt);
  ABD_LAUNCH_CHECK();
  return 0;
}

int bn_bwd_finalize(const BnSync& y, int point, const float* part, int nblk, int C, double count, const float* gamma,
                    const float4* coef, float* dgamma, float* dbeta, BCoef* bcoef, hipStream_t s) {
  if (!y.on()) {
    bn_bwd_finalize_kernel<<<C, kT, 0, s>>>(part, nblk, C, count, gamma, coef, dgamma, dbeta, bcoef);
    ABD_LAUNCH_CHECK();
    return 0;
  }
  double* buf = y.buf + (int64_t)point * ABD_BN_SYNC_STRIDE;
  bn_local_sums_kernel<<<C, kT, 0, s>>>(part, nblk, C, count, buf, dgamma, dbeta);
  ABD_LAUNCH_CHECK();
  if (sync_point(y, point, C)) return -1;
  bn_sync_bwd_finalize_kernel<<<1, 64, 0, s>>>(buf, C, gamma, coef, bcoef);
  ABD_LAUNCH_CHECK();
  return 0;
}

// -------------------------------------------------------------- forward (train or eval)
int forward(abd_cnn* net, const Work& w, const Params& P, const float* x, int64_t B, const float* running_in,
            float* running_upd, bool train, const DropArgs& drop1, const DropArgs& drop2, hipStream_t s,
            int64_t* nbt = nullptr, float4* inst_coef = nullptr, const BnSync& sy = BnSync{},
            const PrepArgs* prep = nullptr, bool fold1 = false, const HeadArgs* head = nullptr, int planes = 0) {
  // planes > 0: conv2 plane mode (conv2_planes): conv1_stats_fold_kernel writes m as planes, conv2
  // reads them
  // inst_coef != nullptr: every utterance is its own BatchNorm batch (B x 160 float4 of
  // coefficients), running statistics untouched -- a batch of batch-1 train-mode forwards
  const Geo& g = net->g;
  const bool inst = inst_coef != nullptr;
  C1Args c1{};
  c1.x = x;
  c1.w = P.p[P_C1W];
  c1.b = P.p[P_C1B];
  c1.coef = w.coef;
  c1.p1 = w.p1;
  c1.part = w.part;
  c1.g = g;
  c1.B = (int)B;
  c1.nblk = (int)nblk_conv1(g, B);
  c1.rows = c1_rows();
  const float* rm[3] = {running_in, running_in + 128, running_in + 256};
  const float* rv[3] = {running_in + 64, running_in + 192, running_in + 288};
  float* rmu[3] = {nullptr, nullptr, nullptr};
  float* rvu[3] = {nullptr, nullptr, nullptr};
  if (running_upd) {
    rmu[0] = running_upd;
    rvu[0] = running_upd + 64;
    rmu[1] = running_upd + 128;
    rvu[1] = running_upd + 192;
    rmu[2] = running_upd + 256;
    rvu[2] = running_upd + 288;
  }
  // ---- layer 1
  if (inst) {
    inst_conv1_coef_kernel<<<(unsigned)B, kT, 0, s>>>(c1, P.p[P_BN1W], P.p[P_BN1B], inst_coef);
    c1.coef = inst_coef;
    c1.coef_bstride = 64;
  } else if (train) {
    // prep != nullptr: the first nprep blocks do the weight repacks (prep_weights_body) instead
    if (prep) {
      c1.prep = *prep;
      c1.nprep = (int)std::min<unsigned>(prep_blocks(g), 256u);
    }
    abd::prof_begin(abd::PH_CONV1_STATS, s);
    if (fold1) {
      c1.gamma = P.p[P_BN1W];
      if (planes > 0) {
        c1.p1s = w.p1s;
        c1.plane = B * g.H1 * g.W1p * 64;
        c1.np = planes;
      }
      c1.nblk = (int)std::min<int64_t>(c1.nblk, c1f_blocks());  // one resident round
      conv1_stats_fold_kernel<<<c1.nblk + c1.nprep, kT, 0, s>>>(c1);
    } else {
      conv1_stats_kernel<<<c1.nblk + c1.nprep, kT, 0, s>>>(c1);
    }
    abd::prof_end(abd::PH_CONV1_STATS, s);
    ABD_LAUNCH_CHECK();
    if (bn_fwd_finalize(sy, 0, w.part, c1.nblk, 64, (double)B * g.H1 * g.W1, P.p[P_BN1W], P.p[P_BN1B], rmu[0],
                        rvu[0], w.coef, running_upd ? nbt : nullptr, s, fold1 ? w.w2f : nullptr,
                        fold1 ? w.w2fold : nullptr, fold1 ? w.ft2 : nullptr))
      return -1;
  } else {
    bn_eval_coef_kernel<<<1, 64, 0, s>>>(P.p[P_BN1W], P.p[P_BN1B], rm[0], rv[0], 64, w.coef);
  }
  ABD_LAUNCH_CHECK();
  if (!fold1) {
    abd::prof_begin(abd::PH_CONV1_POOL, s);
    conv1_bn_pool_kernel<<<(unsigned)nchunks_conv1(g, B), kT, 0, s>>>(c1);  // no partials: one chunk per block
    abd::prof_end(abd::PH_CONV1_POOL, s);
    ABD_LAUNCH_CHECK();
  }
  // ---- layer 2: conv2 (MFMA) + relu + stats -> BN2 -> pool2
  {
    NTArgs a = conv_fwd_args(w.p1, g.H1, g.W1p, 64, g.H2, g.W2, B, w.w2f, 64, P.p[P_C2B], w.r2);
    const bool bf = net->precision == ABD_PREC_BF16, sp = net->precision == ABD_PREC_F32_SPLIT;
    // f32split / bf16: the weight-stationary kernels (bf16 on one plane); fp32 MFMA otherwise, and
    // for a batch past their 32-bit buffer offsets
    const bool ws = (sp || bf) && ws_fits(a);
    if (planes > 0) {   // (set before the grid: the plane-operand kernel takes its own grid)
      a.srcs = w.p1s;
      a.splane = B * g.H1 * g.W1p * 64;
    }
    a.nblk = !ws ? nt_grid_x<64, EPI_CONV>(a)
             : planes == 1 ? ws_nblk<EPI_CONV, 1, true>(a)
             : bf ? ws_nblk<EPI_CONV, 1, false>(a) : ws_nblk<EPI_CONV, 3, false>(a);
    a.part = (train && !inst) ? w.part : nullptr;
    // p1 holds m under the BN1 fold: only the weight-stationary split kernel applies it (bn1_fold_ok)
    ABD_CHECK(!fold1 || ws, ABD_E_UNSUPPORTED, "BN1 fold needs the weight-stationary conv2 kernel");
    if (fold1) {
      a.Bw = w.w2fold;
      a.fold_t = w.ft2;
    }
    if (planes == 1 ? launch_conv_ws_split<EPI_CONV, 1, true>(a, s, abd::PH_CONV2_FWD)
        : ws ? (bf ? launch_conv_ws_split<EPI_CONV, 1>(a, s, abd::PH_CONV2_FWD)
                   : launch_conv_ws_split<EPI_CONV>(a, s, abd::PH_CONV2_FWD))
             : launch_nt<64, EPI_CONV>(a, s, abd::PH_CONV2_FWD))
      return -1;
    if (inst)
      inst_coef_kernel<<<(unsigned)B, kT, 0, s>>>(w.r2, g.H2 * g.W2, 64, P.p[P_BN2W], P.p[P_BN2B],
                                                  inst_coef + B * 64);
    else if (train) {
      if (bn_fwd_finalize(sy, 1, w.part, a.nblk, 64, (double)a.M, P.p[P_BN2W], P.p[P_BN2B], rmu[1], rvu[1],
                          w.coef + 64, nullptr, s))
        return -1;
    } else
      bn_eval_coef_kernel<<<1, 64, 0, s>>>(P.p[P_BN2W], P.p[P_BN2B], rm[1], rv[1], 64, w.coef + 64);
    ABD_LAUNCH_CHECK();
    PoolArgs pa = pool_args(g, 2, B);
    pa.r = w.r2;
    pa.coef = inst ? inst_coef + B * 64 : w.coef + 64;
    pa.coef_bstride = inst ? 64 : 0;
    pa.out = w.p2;
    abd::prof_begin(abd::PH_BN2_POOL, s);
    bn_pool_fwd_kernel<<<grid_for(B * pa.Ho * pa.Wo * 64 / 4), kT, 0, s>>>(pa);
    abd::prof_end(abd::PH_BN2_POOL, s);
    ABD_LAUNCH_CHECK();
  }
  // ---- layer 3
  {
    NTArgs a = conv_fwd_args(w.p2, g.H2p, g.W2p, 64, g.H3, g.W3, B, w.w3f, 32, P.p[P_C3B], w.r3);
    const bool bf3 = net->precision == ABD_PREC_BF16, sp3 = net->precision == ABD_PREC_F32_SPLIT;
    const bool ws3 = (sp3 || bf3) && ws_fits(a);
    a.nblk = !ws3 ? nt_grid_x<32, EPI_CONV>(a) : bf3 ? ws_nblk<EPI_CONV, 1, false>(a) : ws_nblk<EPI_CONV, 3, false>(a);
    a.part = (train && !inst) ? w.part : nullptr;
    if (ws3 ? (bf3 ? launch_conv_ws_split<EPI_CONV, 1>(a, s, abd::PH_CONV3_FWD)
                   : launch_conv_ws_split<EPI_CONV>(a, s, abd::PH_CONV3_FWD))
            : launch_nt<32, EPI_CONV>(a, s, abd::PH_CONV3_FWD))
      return -1;
    if (inst)
      inst_coef_kernel<<<(unsigned)B, kT, 0, s>>>(w.r3, g.H3 * g.W3, 32, P.p[P_BN3W], P.p[P_BN3B],
                                                  inst_coef + B * 128);
    else if (train) {
      if (bn_fwd_finalize(sy, 2, w.part, a.nblk, 32, (double)a.M, P.p[P_BN3W], P.p[P_BN3B], rmu[2], rvu[2],
                          w.coef + 128, nullptr, s))
        return -1;
    } else
      bn_eval_coef_kernel<<<1, 64, 0, s>>>(P.p[P_BN3W], P.p[P_BN3B], rm[2], rv[2], 32, w.coef + 128);
    ABD_LAUNCH_CHECK();
    if (head) return launch_head(1, *head, s);  // BN3 + pool3 + dropout1 + fc1 partials (fc_head.inc)
    PoolArgs pa = pool_args(g, 3, B);
    pa.r = w.r3;
    pa.coef = inst ? inst_coef + B * 128 : w.coef + 128;
    pa.coef_bstride = inst ? 32 : 0;
    pa.out = w.p3d;
    pa.drop = drop1;
    abd::prof_begin(abd::PH_BN3_POOL, s);
    bn_pool_fwd_kernel<<<grid_for(B * pa.Ho * pa.Wo * 32 / 4), kT, 0, s>>>(pa);
    abd::prof_end(abd::PH_BN3_POOL, s);
    ABD_LAUNCH_CHECK();
  }
  // ---- fc1 (MFMA, split-K over the flat features) -> in-order sum + bias + relu + dropout2
  {
    NTArgs a{};
    a.src = w.p3d;
    a.Hs = a.Ws = a.Ho = a.Wo = 1;
    a.Cs = g.flat;
    a.M = (int)B;
    a.taps = 1;
    a.Bw = P.p[P_F1W];
    a.ldb = g.flat;
    a.N = 128;
    a.out = w.slab2;
    a.ldc = 128;
    a.ksplit = std::min(g.flat / kKC, kFc1KSplit);
    abd::prof_begin(abd::PH_FC1_FWD, s);
    if (launch_nt<128, EPI_PARTIAL>(a, s, -1)) return -1;
    fc1_epilogue_kernel<<<(unsigned)((B * 128 + kT - 1) / kT), kT, 0, s>>>(w.slab2, a.ksplit, (int)B, P.p[P_F1B], drop2,
                                                                           w.d2);
    abd::prof_end(abd::PH_FC1_FWD, s);
    ABD_LAUNCH_CHECK();
  }
  return 0;
}

int loss_and_metrics(abd_cnn* net, const Work& w, const Params& P, const int64_t* labels, const int64_t* ind,
                     int64_t B, float inv_batch, bool want_dz, float* logprobs_out, int64_t* metrics,
                     hipStream_t s) {
  LossArgs la{};
  la.d2 = w.d2;
  la.w = P.p[P_F2W];
  la.b = P.p[P_F2B];
  la.labels = labels;
  la.ind = ind;
  la.B = (int)B;
  la.K = net->g.K;
  la.inv_batch = inv_batch;
  la.logprobs = logprobs_out ? logprobs_out : w.logp;
  la.dz = want_dz ? w.dz : nullptr;
  la.rowinfo = w.rowinfo;
  abd::prof_begin(abd::PH_FC2_LOSS, s);
    fc2_loss_kernel<<<(unsigned)((B + 3) / 4), kT, 0, s>>>(la);
    abd::prof_end(abd::PH_FC2_LOSS, s);
  ABD_LAUNCH_CHECK();
  if (metrics && labels) {
    abd::prof_begin(abd::PH_METRICS, s);
    metrics_kernel<<<1, kT, 0, s>>>(w.rowinfo, (int)B, metrics);
    abd::prof_end(abd::PH_METRICS, s);
    ABD_LAUNCH_CHECK();
  }
  return 0;
}

// The train step folds BN1 into conv2 (conv1_stats_fold_kernel; the separate conv1_bn_pool pass
// remains for f32, SyncBN and per-utterance steps) when conv2's forward runs on the
// weight-stationary split kernel (ws_fits: 32-bit buffer offsets).
bool bn1_fold_ok(const abd_cnn* net, const Geo& g, int64_t B) {
  return (net->precision == ABD_PREC_F32_SPLIT || net->precision == ABD_PREC_BF16) &&
         (int64_t)g.H1 * g.W1p * 64 * 4 * B < 0x7ffffff0LL;
}
// conv2 plane mode: the train step keeps conv2's two activation operands -- the pool1 output m (BN1
// fold) and the BN2-backward output dz2 -- as exact bf16 planes written by their producers
// (conv1_stats_fold_kernel, bn_bwd_apply_kernel), and conv2's forward, data- and weight-gradient
// kernels read the planes as MFMA operands (no per-use split).  Returns the plane count (3 in
// f32split, 1 in bf16) or 0 (fp32 buffers).  Measured (r3_v2, B = 512 ultrasonic): in f32split the
// planes are 6 B per element against fp32's 4, and the weight-stationary GEMMs re-read every operand
// row for 4 taps from L2 -- conv2 forward 0.144 -> 0.235 ms, data gradient 0.129 -> 0.184, weight
// gradient 0.121 -> 0.152, BN2 backward +11 us: bf16 only (one 2-B plane halves the operand bytes).
int conv2_planes(const abd_cnn* net, const Geo& g, int64_t B, bool fold1) {
  if (!fold1) return 0;
  const int np = net->precision == ABD_PREC_BF16 ? 1 : 0;
  if (np == 0) return 0;
  const int64_t n_p1 = B * g.H1 * g.W1p * 64, n_r2 = B * g.H2 * g.W2 * 64;
  if ((int64_t)3 * std::max(n_p1, n_r2) * 2 >= 0x7ffffff0LL) return 0;  // 32-bit buffer offsets
  if (!trp_planes_fit<2>(g.H2, g.W2, g.H1, g.W1p)) return 0;
  return np;
}

constexpr int kGuardBlocks = 64;
int bn_bwd_guard(const PoolArgs& pa_in, const float* gamma, const float* beta, double count, const float4* coef,
                 float* dgamma, float* dbeta, BCoef* bcoef, unsigned* ticket, hipStream_t s) {
  PoolArgs pa = pa_in;
  pa.nblk = std::min(grid_for((int64_t)pa.B * pa.Ho * pa.Wo * pa.C / 4), kGuardBlocks);
  bn_pool_bwd_stats_guard_kernel<<<pa.nblk, kT, 0, s>>>(
      PoolGuard{pa, gamma, beta, GuardOut{count, coef, dgamma, dbeta, bcoef, ticket}});
  ABD_LAUNCH_CHECK();
  return 0;
}

int backward(abd_cnn* net, const Work& w, const Params& P, float* grads, const float* x, int64_t B,
             const DropArgs& drop1, hipStream_t s, void* fc_grads_event, const BnSync& sy = BnSync{},
             int64_t* metrics = nullptr, bool fold1 = false, double loss_w = 1.0, const HeadArgs* head = nullptr,
             int planes = 0, int* c1_defer = nullptr) {
  // c1_defer != nullptr: conv1's weight / bias gradient columns are left as partials in w.part (their
  // count in *c1_defer) for adam_c1_kernel to reduce in the optimizer launch
  // fold1: the forward ran conv1_stats_fold_kernel (p1 holds m); conv2's weight gradient is unfolded
  // head: the fused fc head ran its forward and row launches (fc_head.inc); its third launch -- fc
  // gradients, counters, BN3 backward -- replaces everything down to conv3's weight gradient
  // SyncBN steps take the activation passes: the derived sums' small-gamma fallback (below) is decided
  // on the device, where the host-issued all-reduce of a second set of sums cannot follow it.
  // Single-rank steps derive BN2 / BN1's backward sums in the next conv's final weight-gradient
  // reduction (slab_reduce_derive_kernel).
  const bool derive = !sy.on();
  int bn3_parts = 0;  // > 0: BN3 backward partials from the fc1 data-gradient epilogue
  const Geo& g = net->g;
  float* G[P_COUNT];
  for (int i = 0; i < P_COUNT; ++i) G[i] = grads + net->off[i];
  const float s2 = 1.0f / (1.0f - kP2);
  if (head) {
    if (launch_head(3, *head, s)) return -1;
    // fc1/fc2 gradients are final here (see below)
    if (fc_grads_event) ABD_HIP(hipEventRecord(static_cast<hipEvent_t>(fc_grads_event), s));
  } else {
  // ---- fc2 + dropout2/relu
  abd::prof_begin(abd::PH_FC2_BWD, s);
  {
    const int rows = (int)((B + kFc2Split - 1) / kFc2Split);
    // two launches instead of four: [fc2 weight-grad partials | da] then [their reduction | fc1 bias]
    const int nw = (g.K * kFc2Split + 1) / 2;
    fc2_grads_kernel<<<(unsigned)(nw + grid_for(B * 128) + (metrics ? 1 : 0)), kT, 0, s>>>(
        w.dz, w.d2, P.p[P_F2W], (int)B, g.K, rows, kFc2Split, w.slab2, s2, w.da, nw, w.rowinfo, metrics, loss_w);
    fc2_reduce_colsum_kernel<<<(unsigned)(128 + (g.K * 129 + kT - 1) / kT), kT, 0, s>>>(
        w.slab2, kFc2Split, g.K, G[P_F2W], G[P_F2B], w.da, (int)B, 128, G[P_F1B]);
  }
  abd::prof_end(abd::PH_FC2_BWD, s);
  ABD_LAUNCH_CHECK();
  // ---- fc1 weight grad (TN: n = 128 units, k = flat features, reduce over batch)
  {
    TNArgs a{};
    a.D = w.da;
    a.ldd = 128;
    a.src = w.p3d;
    a.Hs = a.Ws = a.Ho = a.Wo = 1;
    a.Cs = g.flat;
    a.M = (int)B;
    a.taps = 1;
    a.N = 128;
    a.Ktot = g.flat;
    a.mchunk = (int)((B + kFc1MSplit - 1) / kFc1MSplit);
    a.mchunk = (a.mchunk + 31) / 32 * 32;
    const int nsl = (int)((B + a.mchunk - 1) / a.mchunk);
    a.slab = w.slab;
    dim3 grid(nsl, (g.flat + 127) / 128, 1);
    abd::prof_begin(abd::PH_FC1_WGRAD, s);
    gemm_tn_kernel<128, 128><<<grid, kT, 0, s>>>(a);
    abd::prof_end(abd::PH_FC1_WGRAD, s);
    ABD_LAUNCH_CHECK();
    if (reduce_slabs(w, nsl, 128, g.flat, 0, G[P_F1W], s)) return -1;
  }
  // fc1/fc2 gradients (the tail of the flat buffer, 94 % of it) are final here: a DP caller
  // all-reduces them on a side stream while the conv backward below keeps this one busy
  if (fc_grads_event) {
    ABD_HIP(hipEventRecord(static_cast<hipEvent_t>(fc_grads_event), s));
  }
  // ---- fc1 data grad (NT against fc1.weight^T) * dropout1 mask
  {
    NTArgs a{};
    a.src = w.da;
    a.Hs = a.Ws = a.Ho = a.Wo = 1;
    a.Cs = 128;
    a.M = (int)B;
    a.taps = 1;
    a.Bw = w.f1t;
    a.ldb = 128;
    a.N = g.flat;
    a.out = w.dp3;
    a.ldc = g.flat;
    a.drop = drop1;
    a.drop.mask_in = drop1.enabled ? w.mask1 : nullptr;
    // BN3's backward sums in this epilogue (32-column tiles within one channel)
    const int per3 = g.flat / 32;  // columns per BN3 channel (flatten order c, h, w)
    if (!sy.on() && drop1.enabled && per3 % 32 == 0) {
      a.part = w.part;
      a.bias = P.p[P_BN3B];
      a.bn_gamma = P.p[P_BN3W];
      a.bnp = w.p3d;
      a.bn_period = per3;
      bn3_parts = ((a.M + kBM - 1) / kBM) * (per3 / 32);
    }
    // 32-column tiles: M = B rows is short (4 row tiles at B = 512), so 128-column tiles leave
    // most CUs idle (96 blocks)
    if (drop1.enabled ? launch_nt<32, EPI_DROPGRAD>(a, s, abd::PH_FC1_DGRAD)
                      : launch_nt<32, EPI_STORE>(a, s, abd::PH_FC1_DGRAD))
      return -1;
  }
  }  // !head
  // ---- pool3 / BN3 / relu backward -> dz3; conv3 wgrad + dgrad
  {
    PoolArgs pa = pool_args(g, 3, B);
    pa.r = w.r3;
    pa.coef = w.coef + 128;
    pa.dp = w.dp3;
    pa.part = w.part;
    if (head) {  // dz3 and the conv3 bias partials came from head_bwd_kernel
      pa.nblk = head->n_apply;
    } else {
    if (bn3_parts > 0) {  // partials from the fc1 data-gradient epilogue
      pa.nblk = bn3_parts;
    } else {
      pa.nblk = grid_for(B * pa.Ho * pa.Wo * 32 / 4);
      bn_pool_bwd_stats_kernel<<<pa.nblk, kT, 0, s>>>(pa);
      ABD_LAUNCH_CHECK();
    }
    if (bn_bwd_finalize(sy, 3, w.part, pa.nblk, 32, (double)B * g.H3 * g.W3, P.p[P_BN3W], w.coef + 128, G[P_BN3W],
                        G[P_BN3B], w.bcoef + 128, s))
      return -1;
    if (bn3_parts > 0 && bn_bwd_guard(pa, P.p[P_BN3W], P.p[P_BN3B], (double)B * g.H3 * g.W3, w.coef + 128, G[P_BN3W],
                                      G[P_BN3B], w.bcoef + 128, w.tickets + 2, s))
      return -1;
    pa.bcoef = w.bcoef + 128;
    pa.dz = w.dz3;
    pa.part = w.partb3;
    pa.nblk = grid_for(B * win_ext_h(pa) * win_ext_w(pa) * 32 / 4);
    abd::prof_begin(abd::PH_BN3_BWD, s);
    bn_bwd_apply_kernel<<<pa.nblk, kT, 0, s>>>(pa, win_ext_h(pa), win_ext_w(pa));
    abd::prof_end(abd::PH_BN3_BWD, s);
    ABD_LAUNCH_CHECK();
    }  // !head
    int nsl = net->precision == ABD_PREC_BF16
                  ? launch_wgrad_tr<4, 32, 1>(w.dz3, w.p2, g.H3, g.W3, g.H2p, g.W2p, B, kConv3Slabs, w.slab,
                                              abd::PH_CONV3_WGRAD, s)
              : net->precision == ABD_PREC_F32_SPLIT
                  ? launch_wgrad_tr<4, 32>(w.dz3, w.p2, g.H3, g.W3, g.H2p, g.W2p, B, kConv3Slabs, w.slab,
                                           abd::PH_CONV3_WGRAD, s)
                  : -1;
    if (nsl < 0)
      nsl = launch_wgrad_rows<32, 64>(w.dz3, w.p2, g.H3, g.W3, g.H2p, g.W2p, B, 4, kConv3Slabs, w.slab,
                                      abd::PH_CONV3_WGRAD, s);
    // conv3's data gradient first: the BN2 guard riding on the reduction below reads dp2
    NTArgs da = conv_dgrad_args(w.dz3, g.H3, g.W3, 32, g.H2p, g.W2p, B, w.w3d, 64, w.dp2);
    const bool ws3 = net->precision != ABD_PREC_F32 && ws_fits(da);
    if (ws3 ? (net->precision == ABD_PREC_BF16 ? launch_conv_ws_split<EPI_STORE, 1>(da, s, abd::PH_CONV3_DGRAD)
                                               : launch_conv_ws_split<EPI_STORE>(da, s, abd::PH_CONV3_DGRAD))
            : launch_nt<64, EPI_STORE>(da, s, abd::PH_CONV3_DGRAD))
      return -1;
    // conv3 bias gradient (BN3-backward partials) rides on the slab reduction's launch
    // BN2's backward coefficients come out of the same final reduction (derive_fused), with BN2's
    // small-gamma guard (PoolGuard: one partial per derivation block)
    const DeriveArgs dv2{nullptr, P.p[P_C3W], G[P_C3B], P.p[P_BN2W], P.p[P_BN2B], w.coef + 64, (double)B * g.H2 * g.W2,
                         G[P_BN2W], G[P_BN2B], w.bcoef + 64};
    PoolArgs pg = pool_args(g, 2, B);
    pg.r = w.r2;
    pg.coef = w.coef + 64;
    pg.dp = w.dp2;
    pg.part = w.part;
    pg.nblk = 64;  // = reduce_slabs' conv_cin (the derivation grid)
    const PoolGuard guard2{pg, P.p[P_BN2W], P.p[P_BN2B],
                           GuardOut{(double)B * g.H2 * g.W2, w.coef + 64, G[P_BN2W], G[P_BN2B], w.bcoef + 64,
                                    w.tickets + 1}};
    if (nsl < 0 || (derive ? reduce_slabs(w, nsl, 32, 256, 64, G[P_C3W], s, BiasSum{w.partb3, pa.nblk, 32, G[P_C3B]},
                                          &dv2, nullptr, guard2)
                           : reduce_slabs(w, nsl, 32, 256, 64, G[P_C3W], s, BiasSum{w.partb3, pa.nblk, 32, G[P_C3B]})))
      return -1;
  }
  // ---- pool2 / BN2 / relu backward -> dz2; conv2 wgrad + dgrad
  int nsl2 = -1, pa_nblk2 = 0;  // conv2's weight-gradient slabs and bias partials (reduced with BN1 below)
  {
    PoolArgs pa = pool_args(g, 2, B);
    pa.r = w.r2;
    pa.coef = w.coef + 64;
    pa.dp = w.dp2;
    pa.part = w.part;
    pa.nblk = grid_for(B * pa.Ho * pa.Wo * 64 / 4);
    if (!derive) {  // derived: conv3's weight / bias gradients, BN2's sums and its guard are final here
      bn_pool_bwd_stats_kernel<<<pa.nblk, kT, 0, s>>>(pa);
      ABD_LAUNCH_CHECK();
      if (bn_bwd_finalize(sy, 4, w.part, pa.nblk, 64, (double)B * g.H2 * g.W2, P.p[P_BN2W], w.coef + 64, G[P_BN2W],
                          G[P_BN2B], w.bcoef + 64, s))
        return -1;
    }
    pa.bcoef = w.bcoef + 64;
    pa.dz = w.dz2;
    if (planes > 0) {  // conv2 plane mode: dz2 as planes for conv2's data and weight gradients
      pa.dzs = w.dz2s;
      pa.dzplane = B * g.H2 * g.W2 * 64;
      pa.dznp = planes;
    }
    pa.part = w.partb2;
    pa.nblk = grid_for(B * win_ext_h(pa) * win_ext_w(pa) * 64 / 4);
    abd::prof_begin(abd::PH_BN2_BWD, s);
    bn_bwd_apply_kernel<<<pa.nblk, kT, 0, s>>>(pa, win_ext_h(pa), win_ext_w(pa));
    abd::prof_end(abd::PH_BN2_BWD, s);
    ABD_LAUNCH_CHECK();
    pa_nblk2 = pa.nblk;
    const WgPlanes wpl{w.dz2s, w.p1s, B * g.H2 * g.W2 * 64, B * g.H1 * g.W1p * 64};
    int nsl = planes == 1 ? launch_wgrad_tr_planes<2, 1>(g.H2, g.W2, g.H1, g.W1p, B, kConv2Slabs, w.slab,
                                                         abd::PH_CONV2_WGRAD, s, wpl)
              : net->precision == ABD_PREC_BF16
                  ? launch_wgrad_tr<2, 64, 1>(w.dz2, w.p1, g.H2, g.W2, g.H1, g.W1p, B, kConv2Slabs, w.slab,
                                              abd::PH_CONV2_WGRAD, s)
              : net->precision == ABD_PREC_F32_SPLIT
                  ? launch_wgrad_tr<2, 64>(w.dz2, w.p1, g.H2, g.W2, g.H1, g.W1p, B, kConv2Slabs, w.slab,
                                           abd::PH_CONV2_WGRAD, s)
                  : -1;
    ABD_CHECK(planes == 0 || nsl >= 0, ABD_E_UNSUPPORTED, "conv2 plane-mode weight gradient geometry");
    if (nsl < 0)
      nsl = launch_wgrad_rows<64, 64>(w.dz2, w.p1, g.H2, g.W2, g.H1, g.W1p, B, 1, kConv2Slabs, w.slab,
                                      abd::PH_CONV2_WGRAD, s);
    nsl2 = nsl;
    // conv2's data gradient first: the BN1 guard riding on the reduction below reads dp1
    NTArgs da = conv_dgrad_args(w.dz2, g.H2, g.W2, 64, g.H1, g.W1p, B, w.w2d, 64, w.dp1);
    if (planes > 0) {
      da.srcs = w.dz2s;
      da.splane = B * g.H2 * g.W2 * 64;
    }
    const bool ws2 = net->precision != ABD_PREC_F32 && ws_fits(da);
    if ((planes == 1 ? launch_conv_ws_split<EPI_STORE, 1, true>(da, s, abd::PH_CONV2_DGRAD)
         : ws2 ? (net->precision == ABD_PREC_BF16 ? launch_conv_ws_split<EPI_STORE, 1>(da, s, abd::PH_CONV2_DGRAD)
                                                  : launch_conv_ws_split<EPI_STORE>(da, s, abd::PH_CONV2_DGRAD))
               : launch_nt<64, EPI_STORE>(da, s, abd::PH_CONV2_DGRAD)))
      return -1;
  }
  // ---- pool1 / BN1 / relu backward fused with the conv1 weight gradient
  {
    C1Args c1{};
    c1.x = x;
    c1.w = P.p[P_C1W];
    c1.b = P.p[P_C1B];
    c1.coef = w.coef;
    c1.dp1 = w.dp1;
    c1.part = w.part;
    c1.g = g;
    c1.B = (int)B;
    c1.nblk = (int)nblk_conv1(g, B);
    c1.rows = c1_rows();
    const DeriveArgs dv1{fold1 ? w.coef : nullptr, P.p[P_C2W], G[P_C2B], P.p[P_BN1W], P.p[P_BN1B], w.coef, (double)B * g.H1 * g.W1,
                         G[P_BN1W], G[P_BN1B], w.bcoef};
    if (derive) {
      // conv2's weight / bias gradients, BN1's derived sums and its small-gamma guard in one launch.
      // Guard: (p - beta) / gamma unfolded; folded, the derivation is division-free but routes dy to
      // the window's max / min r, while pool1 picks the first maximum of fl(alpha r + beta') -- the
      // same element unless alpha is so small that the rounded values tie (at gamma = 0 every window
      // ties and the reference routes to its first element)
      C1Args c1g = c1;
      c1g.nblk = 64;  // = reduce_slabs' conv_cin (the derivation grid)
      const C1Guard guard1{c1g, P.p[P_BN1W], P.p[P_BN1B],
                           GuardOut{(double)B * g.H1 * g.W1, w.coef, G[P_BN1W], G[P_BN1B], w.bcoef, w.tickets + 0}};
      if (nsl2 < 0 || reduce_slabs(w, nsl2, 64, 256, 64, G[P_C2W], s, BiasSum{w.partb2, pa_nblk2, 64, G[P_C2B]}, &dv1,
                                  fold1 ? w.coef : nullptr, guard1))
        return -1;
    } else {
      if (nsl2 < 0 || reduce_slabs(w, nsl2, 64, 256, 64, G[P_C2W], s, BiasSum{w.partb2, pa_nblk2, 64, G[P_C2B]}, nullptr,
                                  fold1 ? w.coef : nullptr))
        return -1;
      conv1_bwd_stats_kernel<<<c1.nblk, kT, 0, s>>>(c1);
      ABD_LAUNCH_CHECK();
      if (bn_bwd_finalize(sy, 5, w.part, c1.nblk, 64, (double)B * g.H1 * g.W1, P.p[P_BN1W], w.coef, G[P_BN1W],
                          G[P_BN1B], w.bcoef, s))
        return -1;
    }
    c1.bcoef = w.bcoef;
    // one resident round: the grid-stride chunk loop otherwise runs a second, partial round of
    // blocks (occupancy 5 blocks/CU < the 8 of the stats kernels' 2048-block grid)
    c1.nblk = (int)std::min<int64_t>(c1.nblk, g.W1 % 3 == 0 ? c1w_blocks<true>() : c1w_blocks<false>());
    abd::prof_begin(abd::PH_CONV1_BWD, s);
    if (g.W1 % 3 == 0)
      conv1_wgrad_kernel<true><<<c1.nblk, kT, 0, s>>>(c1);
    else
      conv1_wgrad_kernel<false><<<c1.nblk, kT, 0, s>>>(c1);
    abd::prof_end(abd::PH_CONV1_BWD, s);
    ABD_LAUNCH_CHECK();
    // part rows: j*64 + c, j = 0..3 weights (kh,kw), 4 bias -> conv1.w is (c,1,kh,kw): transpose via tiny pass
    if (c1_defer != nullptr) {
      *c1_defer = c1.nblk;
    } else {
      partial_sum_kernel<<<5 * 64, kT, 0, s>>>(w.part, c1.nblk, 5 * 64, nullptr, G[P_C1W], G[P_C1B]);
      ABD_LAUNCH_CHECK();
    }
  }
  return 0;
}

DropArgs make_drop(const abd_train_args* a, int which, uint8_t* ws_mask, int64_t cols) {
  DropArgs d{};
  d.enabled = 1;
  d.p = which == 1 ? kP1 : kP2;
  d.scale = 1.0f / (1.0f - d.p);
  d.seed = a->seed;
  d.stream = a->counter * 2 + (uint64_t)(which - 1);
  d.base = (uint64_t)a->row_offset * (uint64_t)cols;
  d.mask_in = which == 1 ? a->mask1_in : a->mask2_in;
  d.mask_out = ws_mask;
  return d;
}

void copy_masks(const abd_train_args* a, const Work& w, const Geo& g, int64_t B, hipStream_t s) {
  if (a->mask1_out) (void)hipMemcpyAsync(a->mask1_out, w.mask1, (size_t)B * g.flat, hipMemcpyDeviceToDevice, s);
  if (a->mask2_out) (void)hipMemcpyAsync(a->mask2_out, w.mask2, (size_t)B * 128, hipMemcpyDeviceToDevice, s);
}

}  // namespace

extern "C" {

int abd_smallcnn_create(int H0, int W0, int num_classes, int max_batch, abd_cnn** net) {
  ABD_CHECK(net != nullptr, ABD_E_INVALID, "NULL out pointer");
  ABD_CHECK(num_classes >= 1 && num_classes <= 64, ABD_E_UNSUPPORTED, "num_classes must be in [1, 64]");
  Geo g = make_geo(H0, W0, num_classes);
  ABD_CHECK(H0 >= 8 && W0 >= 8 && W0 <= 128 && g.W3 >= 1 && g.H3 >= 2, ABD_E_UNSUPPORTED,
            "input %dx%d too small/large for smallcnn", H0, W0);
  ABD_CHECK(g.flat % 32 == 0, ABD_E_UNSUPPORTED, "flat features %d not a multiple of 32", g.flat);
  auto* n = new abd_cnn();
  n->g = g;
  n->max_batch = max_batch;
  int64_t sz[P_COUNT];
  param_sizes(g, sz);
  n->off[0] = 0;
  for (int i = 0; i < P_COUNT; ++i) n->off[i + 1] = n->off[i] + sz[i];
  *net = n;
  return ABD_OK;
}

void abd_smallcnn_destroy(abd_cnn* net) { delete net; }

int abd_smallcnn_set_precision(abd_cnn* net, int precision) {
  ABD_CHECK(net != nullptr, ABD_E_INVALID, "NULL net");
  ABD_CHECK(precision == ABD_PREC_F32 || precision == ABD_PREC_BF16 || precision == ABD_PREC_F32_SPLIT, ABD_E_INVALID, "unknown precision %d", precision);
  net->precision = precision;
  return ABD_OK;
}

int64_t abd_smallcnn_param_count(const abd_cnn* net) { return net ? net->off[P_COUNT] : -1; }

int abd_smallcnn_param_offsets(const abd_cnn* net, int64_t* offsets) {
  ABD_CHECK(net && offsets, ABD_E_INVALID, "NULL argument");
  for (int i = 0; i <= P_COUNT; ++i) offsets[i] = net->off[i];
  return ABD_OK;
}

int abd_smallcnn_flat_features(const abd_cnn* net) { return net ? net->g.flat : -1; }

size_t abd_smallcnn_workspace_bytes(const abd_cnn* net, int64_t batch) {
  if (!net) return 0;
  return layout(net, batch, nullptr).bytes;
}

int abd_smallcnn_bn1_folded(const abd_cnn* net, int64_t batch) {
  return (net && batch >= 1 && bn1_fold_ok(net, net->g, batch)) ? 1 : 0;
}

int abd_smallcnn_conv2_planes(const abd_cnn* net, int64_t batch) {
  if (!net || batch < 1) return 0;
  return conv2_planes(net, net->g, batch, bn1_fold_ok(net, net->g, batch));
}

int64_t abd_smallcnn_workspace_offset(const abd_cnn* net, int64_t batch, const char* name) {
  if (!net || !name) return -1;
  char* base = reinterpret_cast<char*>(static_cast<uintptr_t>(4096));  // any non-null base: offsets only
  const Work w = layout(net, batch, base);
  const struct {
    const char* n;
    const void* p;
  } tab[] = {{"p1", w.p1},     {"r2", w.r2},       {"p2", w.p2},     {"r3", w.r3},       {"p3d", w.p3d},
             {"d2", w.d2},     {"logp", w.logp},   {"dz", w.dz},     {"dp3", w.dp3},     {"da", w.da},
             {"dz3", w.dz3},   {"dp2", w.dp2},     {"dz2", w.dz2},   {"dp1", w.dp1},     {"coef", w.coef},
             {"bcoef", w.bcoef}, {"mask1", w.mask1}, {"mask2", w.mask2}, {"rowinfo", w.rowinfo},
             {"p1s", w.p1s},   {"dz2s", w.dz2s},   {"xh3", w.xh3}};
  for (const auto& t : tab)
    if (strcmp(t.n, name) == 0) return (int64_t)(static_cast<const char*>(t.p) - base);
  return -1;
}

int abd_smallcnn_train_step(abd_cnn* net, const abd_train_args* a, void* workspace, size_t workspace_bytes,
                            abd_stream_t stream) {
  ABD_CHECK(net && a && a->x && a->labels && a->params && a->grads && a->running, ABD_E_INVALID, "NULL argument");
  const int64_t B = a->batch;
  // BatchNorm2d normalises over N x H x W, so one row is a valid train-mode batch (the loader's
  // 1-row tail, drop_last=False)
  ABD_CHECK(B >= 1, ABD_E_INVALID, "train step needs batch >= 1, got %lld", (long long)B);
  ABD_CHECK(B * net->g.H1 * net->g.W1p * 64 < (1LL << 31), ABD_E_INVALID, "batch too large (int32 activation offsets)");
  const Work w = layout(net, B, static_cast<char*>(workspace));
  ABD_CHECK(workspace && workspace_bytes >= w.bytes, ABD_E_WORKSPACE, "workspace too small (%zu < %zu)",
            workspace_bytes, w.bytes);
  ABD_CHECK(!a->do_update || (a->exp_avg && a->exp_avg_sq && a->adam_step >= 1), ABD_E_INVALID, "Adam state missing");
  hipStream_t s = static_cast<hipStream_t>(stream);
  const Geo& g = net->g;
  Params P = params_of(net, a->params);
  // the weight repacks ride on conv1_stats_kernel's launch (forward(..., prep))
  const PrepArgs prep = prep_args(P, w, g);
  const bool fold1 = bn1_fold_ok(net, g, B) && !bn_sync_of(a).on();  // the fold rides on the single-rank finalize
  DropArgs d1 = make_drop(a, 1, w.mask1, g.flat), d2 = make_drop(a, 2, w.mask2, 128);
  const BnSync sy = bn_sync_of(a);
  const float inv = (a->grad_scale > 0.0f ? a->grad_scale : 1.0f) / (float)B;
  const double loss_w = a->grad_scale > 0.0f ? (double)a->grad_scale : 1.0;
  // fused fc head (3 launches); SyncBN steps keep the round-2 launches (BN3's sums are all-reduced
  // between the loss and the BN3 backward)
  const bool use_head = head_on() && !sy.on();
  HeadArgs ha{};
  if (use_head)
    ha = head_args(net, w, P, a->grads, B, d1, d2, a->labels, a->indicators, inv, a->logprobs_out, a->metrics, loss_w);
  const int planes = conv2_planes(net, g, B, fold1);
  if (forward(net, w, P, a->x, B, a->running, a->running, true, d1, d2, s, a->num_batches_tracked, nullptr, sy, &prep,
              fold1, use_head ? &ha : nullptr, planes))
    return -1;
  if (use_head) {
    if (launch_head(2, ha, s)) return -1;
  } else {
    // the metrics reduction rides on backward()'s fc2 gradient launch
    if (loss_and_metrics(net, w, P, a->labels, a->indicators, B, inv, true, a->logprobs_out, nullptr, s)) return -1;
  }
  // single-rank update: conv1's gradient reduction rides on the Adam launch (one launch fewer)
  const bool defer = a->do_update && !sy.on() && net->off[P_C1W] == 0 && net->off[P_C1B] == 4 * 64 &&
                     net->off[P_BN1W] == 5 * 64;
  int c1_nblk = 0;
  if (backward(net, w, P, a->grads, a->x, B, d1, s, a->fc_grads_event, sy, a->metrics, fold1, loss_w,
               use_head ? &ha : nullptr, planes, defer ? &c1_nblk : nullptr))
    return -1;
  copy_masks(a, w, g, B, s);
  if (defer) {
    const double bc1 = 1.0 - pow((double)a->beta1, (double)a->adam_step);
    const double bc2 = 1.0 - pow((double)a->beta2, (double)a->adam_step);
    const int64_t n = net->off[P_COUNT];
    const AdamArgs aa{a->params, a->grads, a->exp_avg, a->exp_avg_sq, n, (float)(1.0 - (double)a->beta1), a->beta2,
                      (float)(1.0 - (double)a->beta2), (float)((double)a->lr / bc1), (float)sqrt(bc2), a->eps};
    abd::prof_begin(abd::PH_ADAM, s);
    adam_c1_kernel<<<5 * 64 + (unsigned)grid_for(n - 5 * 64, 2048), kT, 0, s>>>(aa, w.part, c1_nblk);
    abd::prof_end(abd::PH_ADAM, s);
    ABD_LAUNCH_CHECK();
  } else if (a->do_update) {
    int rc = abd_smallcnn_apply(net, a, workspace, workspace_bytes, stream);
    if (rc) return rc;
  }
  return ABD_OK;
}

int abd_smallcnn_forward(abd_cnn* net, const abd_train_args* a, int train_mode, void* workspace,
                         size_t workspace_bytes, abd_stream_t stream) {
  ABD_CHECK(net && a && a->x && a->params && a->running && a->logprobs_out, ABD_E_INVALID, "NULL argument");
  const int64_t B = a->batch;
  ABD_CHECK(B >= 1, ABD_E_INVALID, "bad batch %lld", (long long)B);  // 1 row: BatchNorm2d counts N x H x W
  ABD_CHECK(B * net->g.H1 * net->g.W1p * 64 < (1LL << 31), ABD_E_INVALID, "batch too large (int32 activation offsets)");
  const Work w = layout(net, B, static_cast<char*>(workspace));
  ABD_CHECK(workspace && workspace_bytes >= w.bytes, ABD_E_WORKSPACE, "workspace too small (%zu < %zu)",
            workspace_bytes, w.bytes);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const Geo& g = net->g;
  Params P = params_of(net, a->params);
  prep_weights_kernel<<<prep_blocks(g), kT, 0, s>>>(prep_args(P, w, g));
  ABD_LAUNCH_CHECK();
  DropArgs d1{}, d2{};
  if (train_mode) {
    d1 = make_drop(a, 1, w.mask1, g.flat);
    d2 = make_drop(a, 2, w.mask2, 128);
  }
  if (forward(net, w, P, a->x, B, a->running, train_mode ? a->running : nullptr, train_mode != 0, d1, d2, s,
              train_mode ? a->num_batches_tracked : nullptr, nullptr, train_mode ? bn_sync_of(a) : BnSync{}))
    return -1;
  if (loss_and_metrics(net, w, P, nullptr, nullptr, B, 1.0f, false, w.logp, nullptr, s)) return -1;
  (void)hipMemcpyAsync(a->logprobs_out, w.logp, (size_t)B * g.K * sizeof(float), hipMemcpyDeviceToDevice, s);
  if (train_mode) {
    copy_masks(a, w, g, B, s);
  }
  return ABD_OK;
}

int abd_smallcnn_backward(abd_cnn* net, const abd_train_args* a, const float* dlogprobs, void* workspace,
                          size_t workspace_bytes, abd_stream_t stream) {
  ABD_CHECK(net && a && a->x && a->params && a->grads && dlogprobs, ABD_E_INVALID, "NULL argument");
  const int64_t B = a->batch;
  ABD_CHECK(B >= 1, ABD_E_INVALID, "backward needs batch >= 1, got %lld", (long long)B);
  ABD_CHECK(B * net->g.H1 * net->g.W1p * 64 < (1LL << 31), ABD_E_INVALID, "batch too large (int32 activation offsets)");
  const Work w = layout(net, B, static_cast<char*>(workspace));
  ABD_CHECK(workspace && workspace_bytes >= w.bytes, ABD_E_WORKSPACE, "workspace too small");
  hipStream_t s = static_cast<hipStream_t>(stream);
  Params P = params_of(net, a->params);
  logsoftmax_bwd_kernel<<<(unsigned)((B + 3) / 4), kT, 0, s>>>(dlogprobs, w.logp, (int)B, net->g.K, w.dz);
  ABD_LAUNCH_CHECK();
  DropArgs d1{};
  d1.enabled = 1;
  d1.p = kP1;
  d1.scale = 1.0f / (1.0f - kP1);
  if (backward(net, w, P, a->grads, a->x, B, d1, s, a->fc_grads_event, bn_sync_of(a))) return -1;
  return ABD_OK;
}

int abd_smallcnn_apply(abd_cnn* net, const abd_train_args* a, void* workspace, size_t workspace_bytes,
                       abd_stream_t stream) {
  (void)workspace;
  (void)workspace_bytes;
  ABD_CHECK(net && a && a->params && a->grads && a->exp_avg && a->exp_avg_sq, ABD_E_INVALID, "NULL argument");
  return abd_adam_f32(a->params, a->grads, a->exp_avg, a->exp_avg_sq, net->off[P_COUNT], a->adam_step, a->lr,
                      a->beta1, a->beta2, a->eps, stream);
}

int abd_smallcnn_eval(abd_cnn* net, const float* x, int64_t batch, const float* params, const float* running,
                      const int64_t* labels, const int64_t* indicators, float* logprobs, int64_t* metrics,
                      void* workspace, size_t workspace_bytes, abd_stream_t stream) {
  ABD_CHECK(net && x && params && running && logprobs, ABD_E_INVALID, "NULL argument");
  if (batch == 0) return ABD_OK;
  ABD_CHECK(batch * net->g.H1 * net->g.W1p * 64 < (1LL << 31), ABD_E_INVALID, "batch too large (int32 activation offsets)");
  const Work w = layout(net, batch, static_cast<char*>(workspace));
  ABD_CHECK(workspace && workspace_bytes >= w.bytes, ABD_E_WORKSPACE, "workspace too small (%zu < %zu)",
            workspace_bytes, w.bytes);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const Geo& g = net->g;
  Params P = params_of(net, params);
  prep_weights_kernel<<<prep_blocks(g), kT, 0, s>>>(prep_args(P, w, g));
  ABD_LAUNCH_CHECK();
  DropArgs off{};
  if (forward(net, w, P, x, batch, running, nullptr, false, off, off, s)) return -1;
  return loss_and_metrics(net, w, P, labels, indicators, batch, 1.0f / (float)batch, false, logprobs,
                          labels ? metrics : nullptr, s);
}

static size_t inst_coef_bytes(int64_t batch) { return ((size_t)batch * 160 * sizeof(float4) + 255) & ~(size_t)255; }

size_t abd_smallcnn_forward_per_utterance_workspace_bytes(const abd_cnn* net, int64_t batch) {
  if (!net) return 0;
  return layout(net, batch, nullptr).bytes + inst_coef_bytes(batch);
}

int abd_smallcnn_forward_per_utterance(abd_cnn* net, const float* x, int64_t batch, const float* params,
                                       uint64_t seed, uint64_t counter, const uint8_t* mask1_in,
                                       const uint8_t* mask2_in, float* logprobs, void* workspace,
                                       size_t workspace_bytes, abd_stream_t stream) {
  ABD_CHECK(net && x && params && logprobs, ABD_E_INVALID, "NULL argument");
  if (batch == 0) return ABD_OK;
  ABD_CHECK(batch > 0 && batch * net->g.H1 * net->g.W1p * 64 < (1LL << 31), ABD_E_INVALID,
            "bad batch %lld (int32 activation offsets)", (long long)batch);
  const Work w = layout(net, batch, static_cast<char*>(workspace));
  const size_t need = w.bytes + inst_coef_bytes(batch);
  ABD_CHECK(workspace && workspace_bytes >= need, ABD_E_WORKSPACE, "workspace too small (%zu < %zu)", workspace_bytes,
            need);
  float4* icoef = reinterpret_cast<float4*>(static_cast<char*>(workspace) + w.bytes);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const Geo& g = net->g;
  Params P = params_of(net, params);
  prep_weights_kernel<<<prep_blocks(g), kT, 0, s>>>(prep_args(P, w, g));
  ABD_LAUNCH_CHECK();
  abd_train_args a{};
  a.seed = seed;
  a.counter = counter;
  a.mask1_in = mask1_in;
  a.mask2_in = mask2_in;
  DropArgs d1 = make_drop(&a, 1, w.mask1, net->g.flat), d2 = make_drop(&a, 2, w.mask2, 128);
  if (forward(net, w, P, x, batch, nullptr, nullptr, true, d1, d2, s, nullptr, icoef)) return -1;
  return loss_and_metrics(net, w, P, nullptr, nullptr, batch, 1.0f, false, logprobs, nullptr, s);
}

static size_t dz1_bytes(const abd_cnn* net, int64_t batch) {
  return ((size_t)batch * net->g.H1 * net->g.W1 * 64 * sizeof(float) + 255) & ~(size_t)255;
}

size_t abd_smallcnn_input_grad_workspace_bytes(const abd_cnn* net, int64_t batch) {
  if (!net) return 0;
  return layout(net, batch, nullptr).bytes + dz1_bytes(net, batch);
}

int abd_smallcnn_input_grad(abd_cnn* net, const float* x, int64_t batch, const float* params, const float* running,
                            const int64_t* labels, float loss_scale, float* logprobs, float* dx, int64_t* metrics,
                            void* workspace, size_t workspace_bytes, abd_stream_t stream) {
  ABD_CHECK(net && x && params && running && labels && dx, ABD_E_INVALID, "NULL argument");
  const int64_t B = batch;
  ABD_CHECK(B >= 1, ABD_E_INVALID, "bad batch %lld", (long long)B);
  ABD_CHECK(B * net->g.H1 * net->g.W1 * 64 < (1LL << 31), ABD_E_INVALID, "batch too large (int32 activation offsets)");
  const Work w = layout(net, B, static_cast<char*>(workspace));
  const size_t need = w.bytes + dz1_bytes(net, B);
  ABD_CHECK(workspace && workspace_bytes >= need, ABD_E_WORKSPACE, "workspace too small (%zu < %zu)", workspace_bytes,
            need);
  float* dz1 = reinterpret_cast<float*>(static_cast<char*>(workspace) + w.bytes);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const Geo& g = net->g;
  Params P = params_of(net, params);
  prep_weights_kernel<<<prep_blocks(g), kT, 0, s>>>(prep_args(P, w, g));
  ABD_LAUNCH_CHECK();
  DropArgs off{};
  if (forward(net, w, P, x, B, running, nullptr, false, off, off, s)) return -1;
  if (loss_and_metrics(net, w, P, labels, nullptr, B, loss_scale / (float)B, true, logprobs ? logprobs : w.logp,
                       metrics, s))
    return -1;
  // fc2 -> ReLU (no dropout in eval) -> fc1 data gradient
  fc2_bwd_kernel<<<grid_for(B * 128), kT, 0, s>>>(w.dz, w.d2, P.p[P_F2W], (int)B, g.K, 1.0f, w.da);
  ABD_LAUNCH_CHECK();
  {
    NTArgs a{};
    a.src = w.da;
    a.Hs = a.Ws = a.Ho = a.Wo = 1;
    a.Cs = 128;
    a.M = (int)B;
    a.taps = 1;
    a.Bw = w.f1t;
    a.ldb = 128;
    a.N = g.flat;
    a.out = w.dp3;
    a.ldc = g.flat;
    if (launch_nt<128, EPI_STORE>(a, s, -1)) return -1;
  }
  // pool / eval BN / ReLU backward and conv data gradients, layers 3 and 2
  for (int layer = 3; layer >= 2; --layer) {
    const int C = layer == 3 ? 32 : 64;
    const int co = layer == 3 ? 128 : 64;
    bn_eval_bcoef_kernel<<<1, 64, 0, s>>>(w.coef + co, C, w.bcoef + co);
    ABD_LAUNCH_CHECK();
    PoolArgs pa = pool_args(g, layer, B);
    pa.r = layer == 3 ? w.r3 : w.r2;
    pa.coef = w.coef + co;
    pa.dp = layer == 3 ? w.dp3 : w.dp2;
    pa.bcoef = w.bcoef + co;
    pa.dz = layer == 3 ? w.dz3 : w.dz2;
    pa.part = w.part;
    pa.nblk = grid_for(B * win_ext_h(pa) * win_ext_w(pa) * C / 4);
    bn_bwd_apply_kernel<<<pa.nblk, kT, 0, s>>>(pa, win_ext_h(pa), win_ext_w(pa));
    ABD_LAUNCH_CHECK();
    NTArgs da = layer == 3 ? conv_dgrad_args(w.dz3, g.H3, g.W3, 32, g.H2p, g.W2p, B, w.w3d, 64, w.dp2)
                           : conv_dgrad_args(w.dz2, g.H2, g.W2, 64, g.H1, g.W1p, B, w.w2d, 64, w.dp1);
    if (launch_nt<64, EPI_STORE>(da, s, -1)) return -1;
  }
  // layer 1: dz1 (NHWC) then the conv1 data gradient
  C1Args c1{};
  c1.x = x;
  c1.w = P.p[P_C1W];
  c1.b = P.p[P_C1B];
  c1.coef = w.coef;
  c1.dp1 = w.dp1;
  c1.g = g;
  c1.B = (int)B;
  conv1_dz_eval_kernel<<<grid_for(B * g.H1 * ((g.W1 + 2) / 3) * 16), kT, 0, s>>>(c1, dz1);
  ABD_LAUNCH_CHECK();
  conv1_dx_kernel<<<grid_for(B * g.H0 * g.W0), kT, 0, s>>>(P.p[P_C1W], dz1, (int)B, g, dx);
  ABD_LAUNCH_CHECK();
  return ABD_OK;
}

int abd_adam_f32(float* params, const float* grads, float* exp_avg, float* exp_avg_sq, int64_t n, int64_t step,
                 float lr, float beta1, float beta2, float eps, abd_stream_t stream) {
  ABD_CHECK(params && grads && exp_avg && exp_avg_sq && step >= 1, ABD_E_INVALID, "bad Adam arguments");
  const double bc1 = 1.0 - pow((double)beta1, (double)step);
  const double bc2 = 1.0 - pow((double)beta2, (double)step);
  const float step_size = (float)((double)lr / bc1);
  const float bc2s = (float)sqrt(bc2);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const AdamArgs aa{params, grads, exp_avg, exp_avg_sq, n, (float)(1.0 - (double)beta1), beta2,
                    (float)(1.0 - (double)beta2), step_size, bc2s, eps};
  abd::prof_begin(abd::PH_ADAM, s);
  adam_kernel<<<grid_for(n, 2048), kT, 0, s>>>(aa);
  abd::prof_end(abd::PH_ADAM, s);
  ABD_LAUNCH_CHECK();
  return ABD_OK;
}

}  // extern "C"
