// Fused trigger-injection + STFT + mel + dB + DCT (MFCC) for gfx950.
//
// Replaces prepare_dataset.py:35-47 (torchaudio T.MFCC) and
// utils/daba_selection_tools.py:16-22 (librosa feature.mfcc); the injection modes
// replace ultrasonic.py:75, flowmur.py:77-85/101-106,
// utils/flowmur_generate_trigger.py:49-62 and utils/badnet_trigger.py:18-27.
//
// Design (DESIGN.md "Feature stage"):
//   kernel stft_mel : grid = batch x chunks, one 256-thread workgroup handles PPB
//       *pairs* of frames of one utterance.  Two real frames are packed into one
//       complex FFT (z = a + i b) held in LDS; Stockham radix-{2,3,4,5} passes
//       ping-pong between two LDS buffers.  Non-smooth n_fft (ultrasonic: 1103 is
//       prime) goes through Bluestein with a {2,3,5}-smooth M >= 2N-1.  Power ->
//       sparse mel projection -> 10 log10 -> per-chunk max, written to workspace.
//   kernel db_dct   : grid = batch x frame-tiles: per-utterance top_db clamp and the
//       ortho DCT-II, written straight into the (B,1,T,C) model layout, BadNets patch
//       in the epilogue.
// Waveform injection is applied in the sample loader, so the poisoned waveform never
// round-trips through HBM.
#include "abd_common.h"
#include "prof.h"

#include <algorithm>
#include <cmath>
#include <complex>
#include <cstdlib>
#include <mutex>
#include <utility>
#include <vector>

namespace {

constexpr int kThreads = 256;
using abd::kWave;
constexpr int kMaxComplexPerBlock = 6144;  // ppb * M  (LDS: 2 * 8 B * this = 96 KiB max)
constexpr int kTT = 8;                     // frames per db_dct block
constexpr int kQueues = 8;                 // fast-kernel item queues (one per XCD)
constexpr int kQueueStride = 64;           // unsigned words between queue counters (256 B)

// ABD_STFT_ABLATE (diagnostic builds only: -DABD_STFT_ABLATE_BUILD): the fast kernel's ablation
// switches; compiled out otherwise (their wave-uniform tests cost SGPRs the kernel spills)
#ifdef ABD_STFT_ABLATE_BUILD
constexpr bool kAblate = true;
#else
constexpr bool kAblate = false;
#endif
#ifdef ABD_GATHER_SCALAR
constexpr bool kGatherV4 = false;  // A/B build: the per-element gather everywhere
#else
constexpr bool kGatherV4 = true;
#endif

struct MfccDev {
  int N, hop, pad, pad_mode, M, bluestein, n_freqs, n_mels, n_mfcc, T, ppb, chunks, n_pass, fast;
  int dct_lds;  // db_dct_lds_kernel allowed (every plan but ABD_GENERIC_FFT's, when dct_tiles == 0)
  int ablate;  // diagnostics only (0 in the library; measurement builds set it): 1 skip sample loads, 2 skip FFTs, 4 skip mel
  int64_t L;
  float top_db;
  int radix[16], ns[16];
  const float2* tw;
  const float2* chirp_in;
  const float2* vhat;
  const float2* chirp_out;
  const float* window;
  const int* mel_start;
  const int* mel_count;
  const int* mel_off;
  const float* mel_w;
  const float* dct;
  const float4* dct_frag;  // db_dct_mfma_kernel B fragments: [s][q][tile][col] = dct[16s+4q+j][16 tile+col], j<4
  int dct_tiles;           // ceil(n_mfcc / 16) when the MFMA DCT applies (n_mels % 16 == 0, n_mfcc <= 48), else 0
  // fast (specialised) kernel tables
  const float2* ftw;      // [W_{R0 R1}^e] ++ [W_M^k], e, k < R0 R1
  const float4* chirp_out2;  // Bluestein fast kernel: (chirp_out[k], chirp_out[k ? N - k : 0]), k <= N/2
  const float4* ftw4;     // fast kernel pass 2: [p][k] (W_{R0 R1}^{k (1+2p)}, W_{R0 R1}^{k (2+2p)}), p < R1/2
  const float4* vhat4;    // Bluestein fast kernel: [p][j] (vhat[j + 2p M/R0], vhat[j + (2p+1) M/R0]), p < R0/2
  const float2* ftw2;     // fast forward kernel: [r][k] tables W_{R0 R1}^{k r} (k < R0, r < R1) ++
                          // W_M^{k r} (k < R0 R1, r < R2): every twiddle load is base + immediate
  const int4* mel2_meta;  // per half-filter slot 2m+h: (first bin, count, weight offset, 0)
  const float* mel2_w;    // compact slot weights
  int mel2_total, mel2_hp;  // #weights, max slot count rounded up to 8
  const float* mel3_w;      // Bluestein fast path: kMelHP zero-padded weights per slot (NULL = unused)
  // non-Bluestein fast path: every filter's support cut into segments of <= kMelSeg bins (a segment
  // near the top shifted down so its kMelSeg reads stay below n_freqs, its weights offset to match)
  const int* mseg_start;    // first bin read by segment s
  const float4* mseg_w;     // [s][kMelSeg / 4] zero-padded weights
  const int2* mfilt_seg;    // filter m: (first segment, segment count)
  int nseg;                 // segments (0 = use the half-slot loop)
  // backward (mel^T): the <= 2 filters that touch each bin (-1 = none) and their weights
  const int2* bin_mel;
  const float2* bin_w;
  int bwd_ok;  // every bin lies in at most two filters
};

struct InjDev {
  int mode;
  const float* trig;
  int64_t trig_len;
  const uint8_t* poison;
  const int32_t* position;
  float snr_db;
  int patch, pt0, pt1, pc0, pc1;
  float pval;
  const int32_t* frames;  // ragged rows: valid frames per row (NULL = all T)
  float fpad;             // value written to frames >= frames[row]
  bool scale_by_row;      // rowscale is indexed by the table row (abd_inject.row_scale), not the batch row
};

// Ragged rows (utils/daba_selection_tools.py:70-76: librosa MFCC of a shorter clip, then
// np.pad(..., constant_values=-200) to 32 frames): the clip sits zero-extended in its row,
// which leaves frames < 1 + len/hop exactly as librosa computes them on the short clip
// (constant centre padding), but the top_db reference max must only see those frames.
__device__ float ragged_db_max(const float* __restrict__ row_db, int n, float* red) {
  float m = -INFINITY;
  for (int i = threadIdx.x; i < n; i += kThreads) m = fmaxf(m, row_db[i]);
  m = abd::wave_max(m);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x / kWave] = m;
  __syncthreads();
  m = red[0];
  for (int i = 1; i < kThreads / kWave; ++i) m = fmaxf(m, red[i]);
  return m;
}

__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
// -i * a
__device__ __forceinline__ float2 cmi(float2 a) { return make_float2(a.y, -a.x); }

template <int R>
__device__ __forceinline__ void dft(float2* v);

template <>
__device__ __forceinline__ void dft<2>(float2* v) {
  float2 a = v[0], b = v[1];
  v[0] = cadd(a, b);
  v[1] = csub(a, b);
}
template <>
__device__ __forceinline__ void dft<4>(float2* v) {
  float2 t0 = cadd(v[0], v[2]), t1 = csub(v[0], v[2]);
  float2 t2 = cadd(v[1], v[3]), t3 = cmi(csub(v[1], v[3]));
  v[0] = cadd(t0, t2);
  v[2] = csub(t0, t2);
  v[1] = cadd(t1, t3);
  v[3] = csub(t1, t3);
}
template <>
__device__ __forceinline__ void dft<3>(float2* v) {
  const float h = 0.86602540378443864676f;  // sqrt(3)/2
  float2 s = cadd(v[1], v[2]);
  float2 t = make_float2(v[0].x - 0.5f * s.x, v[0].y - 0.5f * s.y);
  float2 d = csub(v[1], v[2]);
  d = make_float2(d.x * h, d.y * h);
  v[0] = cadd(v[0], s);
  v[1] = make_float2(t.x + d.y, t.y - d.x);
  v[2] = make_float2(t.x - d.y, t.y + d.x);
}
template <>
__device__ __forceinline__ void dft<5>(float2* v) {
  const float c1 = 0.30901699437494742410f, c2 = -0.80901699437494742410f;
  const float s1 = 0.95105651629515357212f, s2 = 0.58778525229247312917f;
  float2 b1 = cadd(v[1], v[4]), b2 = cadd(v[2], v[3]);
  float2 d1 = csub(v[1], v[4]), d2 = csub(v[2], v[3]);
  float2 a0 = v[0];
  float2 t1 = make_float2(a0.x + c1 * b1.x + c2 * b2.x, a0.y + c1 * b1.y + c2 * b2.y);
  float2 t2 = make_float2(a0.x + c2 * b1.x + c1 * b2.x, a0.y + c2 * b1.y + c1 * b2.y);
  float2 u1 = make_float2(s1 * d1.x + s2 * d2.x, s1 * d1.y + s2 * d2.y);
  float2 u2 = make_float2(s2 * d1.x - s1 * d2.x, s2 * d1.y - s1 * d2.y);
  v[0] = make_float2(a0.x + b1.x + b2.x, a0.y + b1.y + b2.y);
  v[1] = make_float2(t1.x + u1.y, t1.y - u1.x);
  v[4] = make_float2(t1.x - u1.y, t1.y + u1.x);
  v[2] = make_float2(t2.x + u2.y, t2.y - u2.x);
  v[3] = make_float2(t2.x - u2.y, t2.y + u2.x);
}

// One Stockham pass over nfft FFTs of length M stored back to back (src -> dst).
template <int R>
__device__ __forceinline__ void stockham_pass(const float2* __restrict__ src, float2* __restrict__ dst,
                                              int nfft, int M, int Ns, const float2* __restrict__ tw) {
  const int MR = M / R;
  const int tstep = M / (Ns * R);
  const int total = nfft * MR;
  for (int g = threadIdx.x; g < total; g += kThreads) {
    const int f = g / MR;
    const int j = g - f * MR;
    const float2* s = src + f * M;
    float2* d = dst + f * M;
    const int k = j % Ns;
    float2 v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      float2 a = s[j + r * MR];
      if (r > 0) a = cmul(a, tw[k * r * tstep]);
      v[r] = a;
    }
    dft<R>(v);
    const int base = (j - k) * R + k;
#pragma unroll
    for (int r = 0; r < R; ++r) d[base + r * Ns] = v[r];
  }
}

// Runs all passes; returns the buffer holding the result (0 = a, 1 = b).
__device__ int run_fft(float2* a, float2* b, int nfft, const MfccDev& p) {
  float2* src = a;
  float2* dst = b;
  int cur = 0;
  for (int ps = 0; ps < p.n_pass; ++ps) {
    const int R = p.radix[ps], Ns = p.ns[ps];
    if (R == 4) stockham_pass<4>(src, dst, nfft, p.M, Ns, p.tw);
    else if (R == 2) stockham_pass<2>(src, dst, nfft, p.M, Ns, p.tw);
    else if (R == 3) stockham_pass<3>(src, dst, nfft, p.M, Ns, p.tw);
    else stockham_pass<5>(src, dst, nfft, p.M, Ns, p.tw);
    __syncthreads();
    float2* t = src;
    src = dst;
    dst = t;
    cur ^= 1;
  }
  return cur;
}

__device__ __forceinline__ bool row_poisoned(const InjDev& inj, int64_t u) {
  return inj.mode != ABD_INJECT_NONE && (inj.poison == nullptr || inj.poison[u] != 0);
}

// deploy_trigger_to_waveform (utils/flowmur_generate_trigger.py:56-59) in torch's op order
// (s*w, + t, / (s+1): each rounded, no contraction), then clamp(-1, 1) (:92) if CLAMP.
__device__ __forceinline__ float deploy_mix(float v, float t, bool in, float rs, bool clamp) {
  const float sv = __fmul_rn(rs, v);
  float r = (in ? __fadd_rn(sv, t) : sv) / (rs + 1.0f);
  if (clamp) r = fminf(fmaxf(r, -1.0f), 1.0f);
  return r;
}

__device__ __forceinline__ bool is_deploy(int mode) {
  return mode == ABD_INJECT_DEPLOY || mode == ABD_INJECT_DEPLOY_CLAMP;
}

// Injected sample s (0 <= s < L) of batch position u.  rs = per-row scale from the
// norm pre-pass (SNR: trigger gain, DEPLOY: s).
__device__ __forceinline__ float inj_sample(const float* __restrict__ x, int64_t s, const InjDev& inj,
                                            bool pois, int pos, float rs) {
  float v = x[s];
  if (!pois) return v;
  switch (inj.mode) {
    case ABD_INJECT_ADD:
      return (s < inj.trig_len) ? v + inj.trig[s] : v;
    case ABD_INJECT_SNR_WINDOW: {
      int64_t o = s - pos;
      return (o >= 0 && o < inj.trig_len) ? v + rs * inj.trig[o] : v;
    }
    case ABD_INJECT_HALF_MIX: {
      int64_t o = s - pos;
      return (o >= 0 && o < inj.trig_len) ? (v + inj.trig[o]) / 2.0f : v / 2.0f;
    }
    case ABD_INJECT_DEPLOY:
    case ABD_INJECT_DEPLOY_CLAMP: {
      int64_t o = s - pos;
      const bool in = o >= 0 && o < inj.trig_len;
      return deploy_mix(v, in ? inj.trig[o] : 0.0f, in, rs, inj.mode == ABD_INJECT_DEPLOY_CLAMP);
    }
    default:
      return v;
  }
}

__device__ __forceinline__ float padded_sample(const float* __restrict__ x, int64_t i, const MfccDev& p,
                                               const InjDev& inj, bool pois, int pos, float rs) {
  // i: index into the centre-padded signal; map to the original sample.
  int64_t s = i - p.pad;
  if (s < 0 || s >= p.L) {
    if (p.pad_mode == ABD_PAD_CONSTANT) return 0.0f;
    if (s < 0) s = -s;
    if (s >= p.L) s = 2 * (p.L - 1) - s;
  }
  return inj_sample(x, s, inj, pois, pos, rs);
}

// Per-row scale for the SNR / DEPLOY modes (flowmur.py:77-80, flowmur_generate_trigger.py:50-52).
__global__ void __launch_bounds__(kThreads) row_scale_kernel(const float* __restrict__ wave, int64_t row_stride,
                                                             int64_t L, const int32_t* __restrict__ rows,
                                                             InjDev inj, float* __restrict__ scale) {
  const int64_t u = blockIdx.x;
  // the scale is read for poisoned rows only (inj_sample / fsample mix only those; the backward
  // passes poison == NULL): a clean row's block leaves at once -- ~90 % of a training batch
  if (!row_poisoned(inj, u)) {
    if (threadIdx.x == 0) scale[u] = 0.0f;
    return;
  }
  const int64_t row = rows ? rows[u] : u;
  const float* x = wave + row * row_stride;
  // float4 loads (16-B aligned rows and trigger) with four independent double chains; the loads of
  // 8 strides are issued before their sums (the loop alone waited on one load per stride: 12 us
  // for 256 rows of 16,000 samples), the sums keep the per-stride order of the plain loop
  auto sumsq = [&](const float* p, int64_t n) -> double {
    double s4[4] = {0.0, 0.0, 0.0, 0.0};
    const bool al = (reinterpret_cast<uintptr_t>(p) & 15) == 0;
    int64_t i0 = 0;
    if (al) {
      const float4* p4 = reinterpret_cast<const float4*>(p);
      const int64_t n4 = n / 4;
      constexpr int U = 8;
      int64_t i = threadIdx.x;
      for (; i + (U - 1) * kThreads < n4; i += U * kThreads) {
        float4 v[U];
#pragma unroll
        for (int q = 0; q < U; ++q) v[q] = p4[i + q * kThreads];
#pragma unroll
        for (int q = 0; q < U; ++q) {
          s4[0] += (double)v[q].x * v[q].x;
          s4[1] += (double)v[q].y * v[q].y;
          s4[2] += (double)v[q].z * v[q].z;
          s4[3] += (double)v[q].w * v[q].w;
        }
      }
      for (; i < n4; i += kThreads) {
        const float4 v = p4[i];
        s4[0] += (double)v.x * v.x;
        s4[1] += (double)v.y * v.y;
        s4[2] += (double)v.z * v.z;
        s4[3] += (double)v.w * v.w;
      }
      i0 = n4 * 4;
    }
    for (int64_t i = i0 + threadIdx.x; i < n; i += kThreads) s4[0] += (double)p[i] * p[i];
    return (s4[0] + s4[1]) + (s4[2] + s4[3]);
  };
  double sx = sumsq(x, L), st = sumsq(inj.trig, inj.trig_len);
  __shared__ double red[2][kThreads / kWave];
  sx = abd::wave_sum_d(sx);
  st = abd::wave_sum_d(st);
  const int w = threadIdx.x / kWave;
  if ((threadIdx.x & 63) == 0) {
    red[0][w] = sx;
    red[1][w] = st;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0, b = 0;
    for (int i = 0; i < kThreads / kWave; ++i) {
      a += red[0][i];
      b += red[1][i];
    }
    const float wn = (float)sqrt(a), tn = (float)sqrt(b);
    float r = 0.0f;
    if (inj.mode == ABD_INJECT_SNR_WINDOW) {
      r = sqrtf((wn * wn) / (tn * tn) * (float)pow(10.0, -(double)inj.snr_db / 10.0));
    } else if (is_deploy(inj.mode)) {
      r = (float)pow(10.0, 30.0 / 20.0) * (tn / wn);
    }
    scale[u] = r;
  }
}

__global__ void __launch_bounds__(kThreads) stft_mel_kernel(MfccDev p, const float* __restrict__ wave,
                                                            int64_t row_stride, const int32_t* __restrict__ rows,
                                                            int64_t batch, InjDev inj,
                                                            const float* __restrict__ rowscale,
                                                            float* __restrict__ ws_db, float* __restrict__ ws_max) {
  extern __shared__ __attribute__((aligned(16))) float2 lds[];
  const int nblocks = gridDim.x;
  const int lb = abd::xcd_remap(blockIdx.x, nblocks);
  const int64_t u = lb / p.chunks;
  const int c = lb - (int)(u * p.chunks);
  if (u >= batch) return;
  const int64_t row = rows ? rows[u] : u;
  const float* x = wave + row * row_stride;
  const bool pois = row_poisoned(inj, u);
  const int pos = (inj.position != nullptr) ? inj.position[u] : 0;
  const float rs = (rowscale != nullptr) ? rowscale[inj.scale_by_row ? row : u] : 0.0f;

  const int P = (p.T + 1) / 2;
  const int p0 = c * p.ppb;
  const int np = min(p.ppb, P - p0);
  float2* A = lds;
  float2* Bf = lds + p.ppb * p.M;

  // ---- load two frames per FFT (packed as real + imag), window / chirp
  const int tot = np * p.M;
  for (int idx = threadIdx.x; idx < tot; idx += kThreads) {
    const int f = idx / p.M;
    const int n = idx - f * p.M;
    float2 z = make_float2(0.0f, 0.0f);
    if (n < p.N) {
      const int t0 = 2 * (p0 + f), t1 = t0 + 1;
      const float a = padded_sample(x, (int64_t)t0 * p.hop + n, p, inj, pois, pos, rs);
      const float b = (t1 < p.T) ? padded_sample(x, (int64_t)t1 * p.hop + n, p, inj, pois, pos, rs) : 0.0f;
      if (p.bluestein) {
        z = cmul(make_float2(a, b), p.chirp_in[n]);
      } else {
        const float w = p.window[n];
        z = make_float2(a * w, b * w);
      }
    }
    A[idx] = z;
  }
  __syncthreads();

  int cur = run_fft(A, Bf, np, p);
  float2* Z = cur ? Bf : A;
  float2* other = cur ? A : Bf;
  if (p.bluestein) {
    for (int idx = threadIdx.x; idx < tot; idx += kThreads) {
      const int n = idx % p.M;
      float2 v = Z[idx];
      Z[idx] = cmul(make_float2(v.x, -v.y), p.vhat[n]);
    }
    __syncthreads();
    const int cur2 = run_fft(Z, other, np, p);
    float2* R = cur2 ? other : Z;
    other = cur2 ? Z : other;
    Z = R;
  }

  // ---- unpack the two real spectra -> power, into `other` (as floats)
  float* pw = reinterpret_cast<float*>(other);
  const int nf = p.n_freqs;
  for (int idx = threadIdx.x; idx < np * nf; idx += kThreads) {
    const int f = idx / nf;
    const int k = idx - f * nf;
    const int kn = (k == 0) ? 0 : p.N - k;
    float2 P1 = Z[f * p.M + k], Q = Z[f * p.M + kn];
    if (p.bluestein) {
      float2 a = cmul(p.chirp_out[k], P1);
      float2 b = cmul(p.chirp_out[kn], Q);
      P1 = make_float2(a.x, -a.y);
      Q = make_float2(b.x, -b.y);
    }
    const float ar = 0.5f * (P1.x + Q.x), ai = 0.5f * (P1.y - Q.y);
    const float br = 0.5f * (P1.y + Q.y), bi = 0.5f * (Q.x - P1.x);
    pw[(2 * f) * nf + k] = ar * ar + ai * ai;
    pw[(2 * f + 1) * nf + k] = br * br + bi * bi;
  }
  __syncthreads();

  // ---- sparse mel projection + dB
  float lmax = -INFINITY;
  const int nfr = 2 * np;
  for (int idx = threadIdx.x; idx < nfr * p.n_mels; idx += kThreads) {
    const int fl = idx / p.n_mels;
    const int m = idx - fl * p.n_mels;
    const int t = 2 * p0 + fl;
    if (t >= p.T) continue;
    const float* src = pw + fl * nf + p.mel_start[m];
    const float* w = p.mel_w + p.mel_off[m];
    const int cnt = p.mel_count[m];
    float acc = 0.0f;
    for (int i = 0; i < cnt; ++i) acc = fmaf(src[i], w[i], acc);
    const float db = 10.0f * log10f(fmaxf(acc, 1e-10f));
    ws_db[((int64_t)u * p.T + t) * p.n_mels + m] = db;
    lmax = fmaxf(lmax, db);
  }
  __shared__ float red[kThreads / kWave];
  lmax = abd::wave_max(lmax);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x / kWave] = lmax;
  __syncthreads();
  if (threadIdx.x == 0) {
    float m = red[0];
    for (int i = 1; i < kThreads / kWave; ++i) m = fmaxf(m, red[i]);
    ws_max[u * p.chunks + c] = m;
  }
}

__global__ void __launch_bounds__(kThreads) db_dct_kernel(MfccDev p, const float* __restrict__ ws_db,
                                                          const float* __restrict__ ws_max, InjDev inj,
                                                          float* __restrict__ out) {
  __shared__ float db[kTT * 256];
  const int64_t u = blockIdx.x;
  const int t0 = blockIdx.y * kTT;
  const int nt = min(kTT, p.T - t0);
  const int nv = inj.frames ? min(max(inj.frames[u], 0), p.T) : p.T;
  float mx = -INFINITY;
  if (nv < p.T) {
    __shared__ float rred[kThreads / kWave];
    mx = ragged_db_max(ws_db + u * p.T * p.n_mels, nv * p.n_mels, rred);
  } else {
    for (int i = 0; i < p.chunks; ++i) mx = fmaxf(mx, ws_max[u * p.chunks + i]);
  }
  const float floor_db = (p.top_db >= 0.0f) ? mx - p.top_db : -INFINITY;
  for (int idx = threadIdx.x; idx < nt * p.n_mels; idx += kThreads)
    db[idx] = fmaxf(ws_db[((int64_t)u * p.T + t0) * p.n_mels + idx], floor_db);
  __syncthreads();
  const bool pois = inj.patch && row_poisoned(inj, u);
  for (int o = threadIdx.x; o < nt * p.n_mfcc; o += kThreads) {
    const int t = o / p.n_mfcc;
    const int c = o - t * p.n_mfcc;
    const float* d = db + t * p.n_mels;
    float acc = 0.0f;
    for (int m = 0; m < p.n_mels; ++m) acc = fmaf(d[m], p.dct[m * p.n_mfcc + c], acc);
    const int tt = t0 + t;
    if (pois && tt >= inj.pt0 && tt < inj.pt1 && c >= inj.pc0 && c < inj.pc1) acc = inj.pval;
    if (tt >= nv) acc = inj.fpad;
    out[((int64_t)u * p.T + tt) * p.n_mfcc + c] = acc;
  }
}

// db_dct with the DCT matrix in LDS: block = (utterance, 16 frames); thread = (frame, 4
// consecutive coefficients); the dB tile is read with broadcasts, the matrix row as float4.
constexpr int kTT2 = 16;  // frames per db_dct_lds block (52 measured equal: 0.039 ms at B = 512, 100 frames)
__global__ void __launch_bounds__(kThreads) db_dct_lds_kernel(MfccDev p, const float* __restrict__ ws_db,
                                                              const float* __restrict__ ws_max, InjDev inj,
                                                              float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* dct = sm;                           // n_mels x n_mfcc (row-major, n_mfcc % 4 == 0)
  float* db = sm + p.n_mels * p.n_mfcc;      // kTT2 x n_mels
  __shared__ float red[kThreads / kWave];
  const int64_t u = blockIdx.x;
  const int t0 = blockIdx.y * kTT2;
  const int nt = min(kTT2, p.T - t0);
  const int nv = inj.frames ? min(max(inj.frames[u], 0), p.T) : p.T;
  float mx = -INFINITY;
  if (nv < p.T) {
    for (int i = threadIdx.x; i < nv * p.n_mels; i += kThreads) mx = fmaxf(mx, ws_db[u * p.T * p.n_mels + i]);
  } else {
    for (int i = threadIdx.x; i < p.chunks; i += kThreads) mx = fmaxf(mx, ws_max[u * p.chunks + i]);
  }
  mx = abd::wave_max(mx);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x / kWave] = mx;
  const int nd4 = p.n_mels * p.n_mfcc / 4;
  for (int i = threadIdx.x; i < nd4; i += kThreads)
    reinterpret_cast<float4*>(dct)[i] = reinterpret_cast<const float4*>(p.dct)[i];
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  const float floor_db = (p.top_db >= 0.0f) ? mx - p.top_db : -INFINITY;
  const float* src = ws_db + ((int64_t)u * p.T + t0) * p.n_mels;
  for (int i = threadIdx.x; i < nt * p.n_mels; i += kThreads) db[i] = fmaxf(src[i], floor_db);
  __syncthreads();
  const int cg4 = p.n_mfcc / 4;
  const bool pois = inj.patch && row_poisoned(inj, u);
  for (int o = threadIdx.x; o < nt * cg4; o += kThreads) {
    const int t = o / cg4, c0 = (o - t * cg4) * 4;
    const float* d = db + t * p.n_mels;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int m = 0; m < p.n_mels; ++m) {
      const float x = d[m];
      const float4 w = *reinterpret_cast<const float4*>(dct + m * p.n_mfcc + c0);
      acc.x = fmaf(x, w.x, acc.x);
      acc.y = fmaf(x, w.y, acc.y);
      acc.z = fmaf(x, w.z, acc.z);
      acc.w = fmaf(x, w.w, acc.w);
    }
    const int tt = t0 + t;
    if (pois && tt >= inj.pt0 && tt < inj.pt1) {
      float* a = &acc.x;
      for (int q = 0; q < 4; ++q)
        if (c0 + q >= inj.pc0 && c0 + q < inj.pc1) a[q] = inj.pval;
    }
    if (tt >= nv) acc = make_float4(inj.fpad, inj.fpad, inj.fpad, inj.fpad);
    *reinterpret_cast<float4*>(out + ((int64_t)u * p.T + tt) * p.n_mfcc + c0) = acc;
  }
}

// dB clamp + DCT on the matrix cores: block = (utterance, 64 frames), wave = 16 frames x 16 NT
// coefficients, v_mfma_f32_16x16x4_f32 (exact fp32 products, fp32 accumulation) over the mels.
// Lane l feeds A[frame l & 15][mel] from one float4 of its frame's dB row per 16 mels (the K order
// inside a 16-mel group is permuted identically in the host-built B fragments, MfccDev::dct_frag),
// clamped at the utterance's top_db floor on the fly.  Replaces db_dct_lds_kernel, whose per-block
// staging of the 20 KB DCT matrix and LDS float4 row reads bound it (36 us at B = 512, 100 frames).
typedef float f32x4v __attribute__((ext_vector_type(4)));
template <int NT>
__global__ void __launch_bounds__(kThreads) db_dct_mfma_kernel(MfccDev p, const float* __restrict__ ws_db,
                                                               const float* __restrict__ ws_max, InjDev inj,
                                                               float* __restrict__ out) {
  __shared__ float red[kThreads / kWave];
  const int64_t u = blockIdx.x;
  const int nv = inj.frames ? min(max(inj.frames[u], 0), p.T) : p.T;
  float mx = -INFINITY;
  if (nv < p.T) {
    for (int i = threadIdx.x; i < nv * p.n_mels; i += kThreads) mx = fmaxf(mx, ws_db[u * p.T * p.n_mels + i]);
  } else {
    for (int i = threadIdx.x; i < p.chunks; i += kThreads) mx = fmaxf(mx, ws_max[u * p.chunks + i]);
  }
  mx = abd::wave_max(mx);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x / kWave] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  const float floor_db = (p.top_db >= 0.0f) ? mx - p.top_db : -INFINITY;
  const int lane = threadIdx.x & 63;
  const int t0 = (blockIdx.y * (kThreads / kWave) + (threadIdx.x >> 6)) * 16;
  if (t0 >= p.T) return;
  const int q = lane >> 4, col = lane & 15;
  const float* arow = ws_db + ((int64_t)u * p.T + min(t0 + col, p.T - 1)) * p.n_mels + 4 * q;
  const float4* bf = p.dct_frag + q * NT * 16 + col;
  f32x4v acc[NT];
#pragma unroll
  for (int n = 0; n < NT; ++n) acc[n] = f32x4v{0.0f, 0.0f, 0.0f, 0.0f};
  const int ns = p.n_mels / 16;
  for (int sg = 0; sg < ns; ++sg) {
    float4 a = *reinterpret_cast<const float4*>(arow + 16 * sg);
    a.x = fmaxf(a.x, floor_db);
    a.y = fmaxf(a.y, floor_db);
    a.z = fmaxf(a.z, floor_db);
    a.w = fmaxf(a.w, floor_db);
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      const float4 b = bf[(sg * 4 * NT + n) * 16];
      acc[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b.x, acc[n], 0, 0, 0);
      acc[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b.y, acc[n], 0, 0, 0);
      acc[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b.z, acc[n], 0, 0, 0);
      acc[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b.w, acc[n], 0, 0, 0);
    }
  }
  // D: lane holds frames t0 + 4q + i (i < 4) of coefficient 16 n + col
  const bool pois = inj.patch && row_poisoned(inj, u);
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    const int c = 16 * n + col;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int t = t0 + 4 * q + i;
      if (t < p.T && c < p.n_mfcc) {
        float v = acc[n][i];
        if (pois && t >= inj.pt0 && t < inj.pt1 && c >= inj.pc0 && c < inj.pc1) v = inj.pval;
        if (t >= nv) v = inj.fpad;
        out[((int64_t)u * p.T + t) * p.n_mfcc + c] = v;
      }
    }
  }
}

__global__ void __launch_bounds__(kThreads) inject_wave_kernel(const float* __restrict__ wave, int64_t row_stride,
                                                               int64_t L, const int32_t* __restrict__ rows,
                                                               InjDev inj, const float* __restrict__ rowscale,
                                                               float* __restrict__ out) {
  const int64_t u = blockIdx.y;
  const int64_t row = rows ? rows[u] : u;
  const float* x = wave + row * row_stride;
  const bool pois = row_poisoned(inj, u);
  const int pos = inj.position ? inj.position[u] : 0;
  const float rs = rowscale ? rowscale[inj.scale_by_row ? row : u] : 0.0f;
  for (int64_t s = blockIdx.x * (int64_t)kThreads + threadIdx.x; s < L; s += (int64_t)gridDim.x * kThreads)
    out[u * L + s] = inj_sample(x, s, inj, pois, pos, rs);
}

// =====================================================================================
// Specialised STFT+mel kernel for the attack geometries (compile-time radix plans).
//   n_fft 1103 (ultrasonic, Bluestein M = 2304 = 16*12*12), 2048 = 16*16*8 (flowmur, daba),
//   400 = 16*25 (badnets, jingleback).
// vs the generic kernel: radix-16/25/9/8 butterflies in registers (2-3 LDS passes instead of
// 4-6), divisions by compile-time constants, twiddle table in LDS (persistent blocks load it
// once), in-place passes (read -> barrier -> write), Bluestein's pointwise spectrum product
// fused into the second FFT's first pass, mel projection straight from the packed spectrum.
// =====================================================================================
constexpr double cx_pi = 3.14159265358979323846264338327950288;
constexpr double cx_sin_small(double x) {
  double x2 = x * x, term = x, sum = x;
  for (int i = 1; i < 14; ++i) {
    term *= -x2 / ((2.0 * i) * (2.0 * i + 1.0));
    sum += term;
  }
  return sum;
}
constexpr double cx_cos_small(double x) {
  double x2 = x * x, term = 1.0, sum = 1.0;
  for (int i = 1; i < 14; ++i) {
    term *= -x2 / ((2.0 * i - 1.0) * (2.0 * i));
    sum += term;
  }
  return sum;
}
// (cos, sin)(2 pi m / N) by octant reduction (exact at octant boundaries)
constexpr double cx_trig2pi(int m, int N, bool want_sin) {
  m %= N;
  if (m < 0) m += N;
  const int o = (8 * m) / N;
  const double a = 2.0 * cx_pi * m / N - o * (cx_pi / 4.0);
  const double ca = cx_cos_small(a), sa = cx_sin_small(a);
  const double r = 0.70710678118654752440084436210485;
  const double cb[8] = {1, r, 0, -r, -1, -r, 0, r}, sb[8] = {0, r, 1, r, 0, -r, -1, -r};
  return want_sin ? sb[o] * ca + cb[o] * sa : cb[o] * ca - sb[o] * sa;
}
template <int N>
struct TwTab {
  float c[N];
  float s[N];  // exp(-2 pi i m / N) = (c, s)
  constexpr TwTab() : c(), s() {
    for (int m = 0; m < N; ++m) {
      c[m] = (float)cx_trig2pi(m, N, false);
      s[m] = (float)-cx_trig2pi(m, N, true);
    }
  }
};
template <int N>
__device__ constexpr TwTab<N> kTw{};

// ---- butterflies on ext_vector_type(2) complex values.  Every multiplication by -i / +i is
// written as fma(swap(d), {1,-1}, t) (exact: *1 and *-1 are exact).  With packed FP32 the backend
// emitted one v_pk_fma_f32 with op_sel/neg modifiers; this library is built without packed FP32
// (Makefile PKFLAGS: op_sel-swapped v_pk_* low lanes go wrong under GPU sharing),
// so each is two v_fma_f32 / v_sub_f32 on the halves.
typedef float f2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2v vswap(f2v a) { return __builtin_shufflevector(a, a, 1, 0); }
__device__ __forceinline__ f2v fmav(f2v a, f2v b, f2v c) { return __builtin_elementwise_fma(a, b, c); }
constexpr f2v kPM = {1.0f, -1.0f};
// t + (-i) d  and  t + i d
__device__ __forceinline__ f2v add_mi(f2v t, f2v d) { return fmav(vswap(d), kPM, t); }
__device__ __forceinline__ f2v add_pi(f2v t, f2v d) { return fmav(vswap(d), -kPM, t); }
// a * w (compile-time w: the backend folds (-w.y, w.x) into an SGPR-pair literal, 2 instructions)
__device__ __forceinline__ f2v cmulv(f2v a, f2v w) {
  const f2v ax = __builtin_shufflevector(a, a, 0, 0), ay = __builtin_shufflevector(a, a, 1, 1);
  return fmav(ay, __builtin_shufflevector(w, -w, 3, 0), ax * w);
}
// a * w and conj(a) * w for run-time w (table twiddles, chirps), lane by lane:
//   t = (a.x w.x, a.x w.y);  r.lo = -a.y w.y + t.lo,  r.hi = a.y w.x + t.hi   (conj: signs of a.y flip)
// The library is built without packed-FP32 instructions (Makefile, PKFLAGS): round 3's v_pk_mul /
// v_pk_fma pair with op_sel modifiers gave the same roundings, and the scalar build measured no
// slower (r4: STFT 0.249 vs 0.251 ms).
__device__ __forceinline__ f2v cmul_rt(f2v a, f2v w) {
  return f2v{__builtin_fmaf(-a.y, w.y, a.x * w.x), __builtin_fmaf(a.y, w.x, a.x * w.y)};
}
__device__ __forceinline__ f2v cmul_conj_rt(f2v a, f2v w) {  // conj(a) * w
  return f2v{__builtin_fmaf(a.y, w.y, a.x * w.x), __builtin_fmaf(-a.y, w.x, a.x * w.y)};
}
// value the compiler must treat as defined without materialising it (skip paths of the
// wave-uniform pass guards: otherwise the backend zero-fills every register of the butterfly)
// An opaque unspecified value.  (freeze(poison) -- __builtin_nondeterministic_value -- removes the
// s_nop the hazard recognizer puts before each empty asm, but lets the compiler turn the
// wave-uniform skip branches into selects: the idle waves of a partial pass then computed their
// clamped butterflies, +23 % VALU instructions in the Bluestein kernel, measured.)
__device__ __forceinline__ f2v undef_f2v() {
  f2v v;
  asm volatile("" : "=v"(v));
  return v;
}

template <int R>
__device__ __forceinline__ void dftv(f2v* v);
template <>
__device__ __forceinline__ void dftv<2>(f2v* v) {
  const f2v a = v[0], b = v[1];
  v[0] = a + b;
  v[1] = a - b;
}
template <>
__device__ __forceinline__ void dftv<4>(f2v* v) {
  const f2v t0 = v[0] + v[2], t1 = v[0] - v[2], t2 = v[1] + v[3], d = v[1] - v[3];
  v[0] = t0 + t2;
  v[2] = t0 - t2;
  v[1] = add_mi(t1, d);
  v[3] = add_pi(t1, d);
}
template <>
__device__ __forceinline__ void dftv<3>(f2v* v) {
  const float h = 0.86602540378443864676f;  // sqrt(3)/2
  const f2v s = v[1] + v[2];
  const f2v t = fmav(s, f2v{-0.5f, -0.5f}, v[0]);
  const f2v d = (v[1] - v[2]) * h;
  v[0] = v[0] + s;
  v[1] = add_mi(t, d);
  v[2] = add_pi(t, d);
}
template <>
__device__ __forceinline__ void dftv<5>(f2v* v) {
  const float c1 = 0.30901699437494742410f, c2 = -0.80901699437494742410f;
  const float s1 = 0.95105651629515357212f, s2 = 0.58778525229247312917f;
  const f2v b1 = v[1] + v[4], b2 = v[2] + v[3], d1 = v[1] - v[4], d2 = v[2] - v[3];
  const f2v a0 = v[0];
  const f2v t1 = fmav(b2, f2v{c2, c2}, fmav(b1, f2v{c1, c1}, a0));
  const f2v t2 = fmav(b2, f2v{c1, c1}, fmav(b1, f2v{c2, c2}, a0));
  const f2v u1 = fmav(d2, f2v{s2, s2}, d1 * s1);
  const f2v u2 = fmav(d2, f2v{-s1, -s1}, d1 * s2);
  v[0] = a0 + b1 + b2;
  v[1] = add_mi(t1, u1);
  v[4] = add_pi(t1, u1);
  v[2] = add_mi(t2, u2);
  v[3] = add_pi(t2, u2);
}

// t * W_N^e with compile-time e: trivial angles need no multiply
template <int N, int E>
__device__ __forceinline__ f2v twc(f2v t) {
  constexpr int e = E % N;
  if constexpr (e == 0) {
    return t;
  } else if constexpr (4 * e == N) {  // -i
    return __builtin_shufflevector(t, -t, 1, 2);
  } else if constexpr (2 * e == N) {
    return -t;
  } else if constexpr (4 * e == 3 * N) {  // +i
    return __builtin_shufflevector(-t, t, 1, 2);
  } else if constexpr (8 * e == N) {  // (1 - i)/sqrt2
    return add_mi(t, t) * 0.70710678118654752440f;
  } else if constexpr (8 * e == 3 * N) {  // (-1 - i)/sqrt2
    return add_mi(-t, t) * 0.70710678118654752440f;
  } else {
    return cmulv(t, f2v{kTw<N>.c[e], kTw<N>.s[e]});
  }
}

template <int N1, int N2, int N2I>
__device__ __forceinline__ void dftv_tw_col(f2v* t) {
#pragma unroll
  for (int k1 = 1; k1 < N1; ++k1) {
    // k1 runtime in the unrolled loop: dispatch through a switch the compiler folds
    switch (k1 * N2I) {
#define ABD_TWC(E) \
  case E: t[k1] = twc<N1 * N2, E>(t[k1]); break;
      ABD_TWC(1) ABD_TWC(2) ABD_TWC(3) ABD_TWC(4) ABD_TWC(5) ABD_TWC(6) ABD_TWC(7) ABD_TWC(8) ABD_TWC(9)
      ABD_TWC(10) ABD_TWC(11) ABD_TWC(12) ABD_TWC(13) ABD_TWC(14) ABD_TWC(15) ABD_TWC(16)
#undef ABD_TWC
      default: break;
    }
  }
}

// Cooley-Tukey N = N1*N2 in registers, natural-order in and out.
template <int N1, int N2>
__device__ __forceinline__ void dftv_comp(f2v* v);

#ifndef ABD_R12_N1
#define ABD_R12_N1 4  // radix-12 butterfly as 4 x 3 (ABD_R12_N1=3: 3 x 4)
#endif
template <int R>
struct DftV {
  static __device__ __forceinline__ void run(f2v* v) { dftv<R>(v); }
};
template <>
struct DftV<8> {
  static __device__ __forceinline__ void run(f2v* v) { dftv_comp<2, 4>(v); }
};
template <>
struct DftV<9> {
  static __device__ __forceinline__ void run(f2v* v) { dftv_comp<3, 3>(v); }
};
template <>
struct DftV<12> {
  static __device__ __forceinline__ void run(f2v* v) { dftv_comp<ABD_R12_N1, 12 / ABD_R12_N1>(v); }
};
template <>
struct DftV<16> {
  static __device__ __forceinline__ void run(f2v* v) { dftv_comp<4, 4>(v); }
};
template <>
struct DftV<20> {
  static __device__ __forceinline__ void run(f2v* v) { dftv_comp<4, 5>(v); }
};
template <>
struct DftV<25> {
  static __device__ __forceinline__ void run(f2v* v) { dftv_comp<5, 5>(v); }
};

template <int N1, int N2, int N2I>
__device__ __forceinline__ void dftv_col(f2v* v) {
  constexpr int N = N1 * N2;
  f2v t[N1];
#pragma unroll
  for (int n1 = 0; n1 < N1; ++n1) t[n1] = v[N2 * n1 + N2I];
  dftv<N1>(t);
  dftv_tw_col<N1, N2, N2I>(t);
#pragma unroll
  for (int k1 = 0; k1 < N1; ++k1) v[N2 * k1 + N2I] = t[k1];
  (void)N;
}

template <int N1, int N2, int... I>
__device__ __forceinline__ void dftv_cols(f2v* v, std::integer_sequence<int, I...>) {
  (dftv_col<N1, N2, I>(v), ...);
}

template <int N1, int N2>
__device__ __forceinline__ void dftv_comp(f2v* v) {
  constexpr int N = N1 * N2;
  dftv_cols<N1, N2>(v, std::make_integer_sequence<int, N2>{});
#pragma unroll
  for (int k1 = 0; k1 < N1; ++k1) dftv<N2>(v + N2 * k1);
  f2v o[N];
#pragma unroll
  for (int k1 = 0; k1 < N1; ++k1)
#pragma unroll
    for (int k2 = 0; k2 < N2; ++k2) o[k1 + N1 * k2] = v[N2 * k1 + k2];
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] = o[i];
}

// threadIdx.x behind an opaque move.  The persistent item loop would otherwise hoist every
// thread-invariant LDS/global address of all passes out of the loop and keep them live
// (~150 extra VGPRs, occupancy 1-2); recomputing them per use costs a few VALU ops.
__device__ __forceinline__ int ltid() {
  int t;
  asm volatile("v_mov_b32 %0, %1" : "=v"(t) : "v"((int)threadIdx.x));
  __builtin_assume(t >= 0 && t < kThreads);
  return t;
}

// LDS layout of the fast kernel's FFT buffers: element i lives at i + (i >> 4) (one pad
// slot per 16 complex).  The first Stockham pass writes j*R + r across lanes (stride 16
// complex = 128 B: a 16-way conflict on ds_write_b64's 16-lane groups); padded, those
// writes hit distinct banks, and offsets that are multiples of 16 stay affine
// (pidx(i + 16q) = pidx(i) + 17q) so the passes keep base + immediate addressing.
__device__ __forceinline__ int pidx(int i) { return i + (i >> 4); }
// w[r] = w1^r for r < R by repeated squaring / one multiply (<= 4 roundings deep).
template <int R>
__device__ __forceinline__ void tw_powers(f2v w1, f2v* w) {
  w[1] = w1;
#pragma unroll
  for (int r = 2; r < R; ++r) w[r] = (r % 2 == 0) ? cmul_rt(w[r / 2], w[r / 2]) : cmul_rt(w[r - 1], w1);
}

// One in-place Stockham pass over PP FFTs of length M: every thread reads its butterflies
// into registers, barrier, writes them back in Stockham order, barrier.
//   TWK 0: first pass (no twiddles)
//   TWK 1: tw = W_{NS*R}^e table, factor W_{NS*R}^{k r} read directly (k < NS, r < R)
//   TWK 2: tw = W_M^k table (k < NS, NS*R == M), factor (W_M^k)^r by tw_powers
//   TWK 3: tw = [k][r] table of W_{NS*R}^{k r} (k < NS, r < R): one load per factor, no VALU
//   VMUL : fold Bluestein's pointwise product conj(a) * vhat into the loads
//   ZT   : rows r >= ZT are known zero (Bluestein's zero-padded input): not loaded, and the
//          butterfly arithmetic on them folds away (mfcc.hip builds with -fno-signed-zeros)
//   RS   : only rows r < RS of the output are stored (Bluestein's last pass: outputs >= N are
//          never read; the arithmetic feeding only unstored rows is dead and folds away)
template <int M, int R, int NS, int PP, int TWK, bool VMUL, int ZT = R, int RS = R>
__device__ __forceinline__ void spass(float2* __restrict__ bufs, const float2* __restrict__ tws,
                                      const float2* __restrict__ vhats) {
  constexpr int MR = M / R;
  constexpr int NB = PP * MR;
  constexpr int ROUNDS = (NB + kThreads - 1) / kThreads;
  f2v* buf = reinterpret_cast<f2v*>(bufs);
  const f2v* tw = reinterpret_cast<const f2v*>(tws);
  const f2v* vhat = reinterpret_cast<const f2v*>(vhats);
  f2v v[ROUNDS][R];
  const int tid = ltid();  // one value for both phases: the guards below provably agree
#pragma unroll
  for (int rd = 0; rd < ROUNDS; ++rd) {
    // wave-uniform guard: waves wholly past NB skip; the partial wave computes clamped
    // (duplicate) butterflies and only its store is lane-guarded -- a lane-divergent guard
    // here makes the backend zero-fill all R registers on the skip path
    const int g = min(tid + rd * kThreads, NB - 1);
    if (ROUNDS * kThreads == NB || __builtin_amdgcn_readfirstlane(tid & ~63) + rd * kThreads < NB) {
      const int f = g / MR;
      const int j = g - f * MR;
      const int rb = f * M + j;
      const int prb = pidx(rb);
      const int k = (NS == 1) ? 0 : j % NS;
      f2v w[R];
      if constexpr (TWK == 2) tw_powers<R>(tw[k], w);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if (r >= ZT) {
          v[rd][r] = f2v{0.0f, 0.0f};
          continue;
        }
        // MR % 16 == 0: pidx(rb + r MR) = pidx(rb) + r (MR + MR/16) -> base + immediate
        f2v a = buf[(MR % 16 == 0) ? prb + r * (MR + MR / 16) : pidx(rb + r * MR)];
        if constexpr (VMUL) a = cmul_conj_rt(a, vhat[j + r * MR]);
        if constexpr (TWK == 1) {
          if (r > 0) a = cmul_rt(a, tw[k * r]);
        } else if constexpr (TWK == 2) {
          if (r > 0) a = cmul_rt(a, w[r]);
        } else if constexpr (TWK == 3) {
          if (r > 0) a = cmul_rt(a, tw[r * NS + k]);
        }
        v[rd][r] = a;
      }
      DftV<R>::run(v[rd]);
    } else {
#pragma unroll
      for (int r = 0; r < R; ++r) v[rd][r] = undef_f2v();
    }
  }
  __syncthreads();
#pragma unroll
  for (int rd = 0; rd < ROUNDS; ++rd) {
    // wave-uniform guard: waves wholly past NB skip; the partial wave computes clamped
    // (duplicate) butterflies and only its store is lane-guarded -- a lane-divergent guard
    // here makes the backend zero-fill all R registers on the skip path
    const int g = min(tid + rd * kThreads, NB - 1);
    if (ROUNDS * kThreads == NB || __builtin_amdgcn_readfirstlane(tid & ~63) + rd * kThreads < NB) {
      const int f = g / MR;
      const int j = g - f * MR;
      const int k = (NS == 1) ? 0 : j % NS;
      const int dst = f * M + (j - k) * R + k;
      const int pd = pidx(dst);
      // first pass: dst = j*16, r < 16; later passes: NS % 16 == 0 -> affine as above
      constexpr bool AFF = (NS == 1) ? (R == 16) : (NS % 16 == 0);
#pragma unroll
      for (int r = 0; r < RS; ++r)
        buf[AFF ? pd + r * (NS + NS / 16) : pidx(dst + r * NS)] = v[rd][r];
    }
  }
  __syncthreads();
}

// tw: [W_{R0 R1}^e, e < R0 R1] ++ [W_M^k, k < R0 R1]
// NZ: the input is zero beyond its first NZ elements (per FFT)
// NO: only outputs k < NO are read afterwards (three-pass plans: the last pass writes k = j + r R0 R1)
// KR: tw is the [k][r] layout (MfccDev::ftw2) instead of ftw
template <int M, int R0, int R1, int R2, int PP, bool VMUL, int NZ = M, int NO = M, bool KR = false>
__device__ __forceinline__ void fft_plan(float2* buf, const float2* tw, const float2* vhat) {
  static_assert(R0 * R1 * R2 == M, "radix plan must factor M");
  static_assert(NO == M || R2 > 1, "output pruning needs a third pass");
  constexpr int MR0 = M / R0;
  spass<M, R0, 1, PP, 0, VMUL, (NZ + MR0 - 1) / MR0>(buf, nullptr, vhat);
  spass<M, R1, R0, PP, KR ? 3 : 1, false>(buf, tw, nullptr);
  if constexpr (R2 > 1)
    spass<M, R2, R0 * R1, PP, KR ? 3 : 2, false, R2, (NO + R0 * R1 - 1) / (R0 * R1)>(buf, tw + R0 * R1, nullptr);
}

// Fast-kernel pass with the global loads moved ahead of the barrier: the pass's twiddle / vhat
// loads are issued BEFORE the barrier that publishes the previous pass's LDS writes (the
// registers are free there: the previous pass's values are already stored), so their latency
// overlaps the barrier wait instead of stalling the DFT; then LDS reads -> DFT -> barrier ->
// writes.  No trailing barrier: the next pass (or the caller) opens with one.
//   TWK 0: none;  2: W_M^k base (ftw2 pass-3 table column r = 1) + tw_powers;  3: [r][k] table;
//        4: [pair][k] float4 table (MfccDev::ftw4: rows 1 + 2p and 2 + 2p in one 16-B load)
//   V4 (with VMUL): Bluestein's vhat as [pair][j] float4 (MfccDev::vhat4: rows 2p, 2p + 1)
//   PF: rows r < PF are prefetched, the rest loaded after the barrier (VGPR budget of 8 blocks/CU)
// The pair tables halve the pass's vector-memory instructions: the kernel's vector-memory data
// path (TD) was ~90 % busy, its wave-load count -- not bytes or L1 misses -- the limit.
constexpr int kPrefetchRows = 8;
// TWK 5: the first L = ceil((R - 1) / 2) rows (rounded up to whole pairs) from the pair table, the
// rest as one product each -- half the pass-2 twiddle bytes, factors one rounding from the table
template <int R>
constexpr int kTw5Rows = (((R - 1 + 1) / 2) + 1) / 2 * 2;
template <int R, int PF, int ZT, int LO>
__device__ __forceinline__ void pair_rows(f2v* pre, const float4* __restrict__ t4, int idx, int stride, bool after) {
  // rows LO + 2p and LO + 1 + 2p from t4[p * stride + idx]; `after`: only pairs whose first row is
  // past the prefetch budget, else only those within it
#pragma unroll
  for (int p = 0; p < R / 2; ++p) {
    const int r0 = LO + 2 * p;
    if (r0 >= R || r0 >= ZT || (after ? r0 < PF : r0 >= PF)) continue;
    const float4 q = t4[p * stride + idx];
    pre[r0] = f2v{q.x, q.y};
    if (r0 + 1 < R) pre[r0 + 1] = f2v{q.z, q.w};
  }
}
//   PS: shared-column pairs -- the item's PS FFTs (buffers FS apart) are transformed by the same
//       threads, butterfly column j of every FFT with ONE set of twiddle / vhat loads (PP == 1)
template <int M, int R, int NS, int PP, int TWK, bool VMUL, int ZT = R, int RS = R, int PF = kPrefetchRows,
          bool V4 = false, int PS = 1>
__device__ __forceinline__ void spass_pf(float2* __restrict__ bufs, const float2* __restrict__ tws,
                                         const float2* __restrict__ vhats, const float4* __restrict__ t4 = nullptr) {
  static_assert(!(VMUL && TWK != 0), "vhat product and twiddles never share a pass");
  static_assert(!V4 || VMUL, "V4 is the vhat pair table");
  static_assert(PS == 1 || PP == 1, "shared-column pairs (PS) or distinct pairs (PP), not both");
  constexpr int MR = M / R;
  constexpr int NB = PP * MR;
  constexpr int ROUNDS = (NB + kThreads - 1) / kThreads;
  constexpr int FS = M + M / 16;  // one padded FFT buffer
  f2v* buf = reinterpret_cast<f2v*>(bufs);
  const f2v* tw = reinterpret_cast<const f2v*>(tws);
  const f2v* vhat = reinterpret_cast<const f2v*>(vhats);
  const int tid = ltid();
  f2v pre[ROUNDS][R];
#pragma unroll
  for (int rd = 0; rd < ROUNDS; ++rd) {
    const int g = min(tid + rd * kThreads, NB - 1);
    const int f = g / MR;
    const int j = g - f * MR;
    const int k = (NS == 1) ? 0 : j % NS;
    if (ROUNDS * kThreads == NB || __builtin_amdgcn_readfirstlane(tid & ~63) + rd * kThreads < NB) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if constexpr (VMUL && !V4) pre[rd][r] = (r < ZT && r < PF) ? vhat[j + r * MR] : undef_f2v();
        else if constexpr (TWK == 3) pre[rd][r] = (r > 0 && r < PF) ? tw[r * NS + k] : undef_f2v();
        else if constexpr (TWK == 2) pre[rd][r] = (r == 1) ? tw[NS + k] : undef_f2v();
        else pre[rd][r] = undef_f2v();
      }
      if constexpr (TWK == 4) pair_rows<R, PF, R, 1>(pre[rd], t4, k, NS, false);
      if constexpr (TWK == 5) pair_rows<kTw5Rows<R> + 1, PF, R, 1>(pre[rd], t4, k, NS, false);
      if constexpr (V4) pair_rows<R, PF, ZT, 0>(pre[rd], t4, j, MR, false);
    } else {
#pragma unroll
      for (int r = 0; r < R; ++r) pre[rd][r] = undef_f2v();
    }
  }
  __syncthreads();
  f2v v[ROUNDS][PS][R];
#pragma unroll
  for (int rd = 0; rd < ROUNDS; ++rd) {
    const int g = min(tid + rd * kThreads, NB - 1);
    if (ROUNDS * kThreads == NB || __builtin_amdgcn_readfirstlane(tid & ~63) + rd * kThreads < NB) {
      const int f = g / MR;
      const int j = g - f * MR;
      const int rb = f * M + j;
      const int prb = pidx(rb);
      const int k = (NS == 1) ? 0 : j % NS;
      if constexpr (TWK == 2) tw_powers<R>(pre[rd][1], pre[rd]);
#pragma unroll
      for (int r = PF; r < R; ++r) {  // rows past the prefetch budget
        if constexpr (VMUL && !V4) {
          if (r < ZT) pre[rd][r] = vhat[j + r * MR];
        } else if constexpr (TWK == 3) {
          pre[rd][r] = tw[r * NS + k];
        }
      }
      if constexpr (TWK == 4) pair_rows<R, PF, R, 1>(pre[rd], t4, k, NS, true);
      if constexpr (TWK == 5) {
        pair_rows<kTw5Rows<R> + 1, PF, R, 1>(pre[rd], t4, k, NS, true);
        // rows past the loaded ones: one product of two table entries each (a + b = r, a, b <= L)
#pragma unroll
        for (int r = kTw5Rows<R> + 1; r < R; ++r) pre[rd][r] = cmul_rt(pre[rd][r / 2], pre[rd][r - r / 2]);
      }
      if constexpr (V4) pair_rows<R, PF, ZT, 0>(pre[rd], t4, j, MR, true);
#pragma unroll
      for (int q = 0; q < PS; ++q) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
          if (r >= ZT) {
            v[rd][q][r] = f2v{0.0f, 0.0f};
            continue;
          }
          f2v a = buf[q * FS + ((MR % 16 == 0) ? prb + r * (MR + MR / 16) : pidx(rb + r * MR))];
          if constexpr (VMUL) a = cmul_conj_rt(a, pre[rd][r]);
          if constexpr (TWK != 0) {
            if (r > 0) a = cmul_rt(a, pre[rd][r]);
          }
          v[rd][q][r] = a;
        }
        DftV<R>::run(v[rd][q]);
      }
    } else {
#pragma unroll
      for (int q = 0; q < PS; ++q)
#pragma unroll
        for (int r = 0; r < R; ++r) v[rd][q][r] = undef_f2v();
    }
  }
  __syncthreads();
#pragma unroll
  for (int rd = 0; rd < ROUNDS; ++rd) {
    const int g = min(tid + rd * kThreads, NB - 1);
    if (ROUNDS * kThreads == NB || __builtin_amdgcn_readfirstlane(tid & ~63) + rd * kThreads < NB) {
      const int f = g / MR;
      const int j = g - f * MR;
      const int k = (NS == 1) ? 0 : j % NS;
      const int dst = f * M + (j - k) * R + k;
      const int pd = pidx(dst);
      constexpr bool AFF = (NS == 1) ? (R == 16) : (NS % 16 == 0);
#pragma unroll
      for (int q = 0; q < PS; ++q)
#pragma unroll
        for (int r = 0; r < RS; ++r)
          if (ROUNDS * kThreads == NB || tid + rd * kThreads < NB)
            buf[q * FS + (AFF ? pd + r * (NS + NS / 16) : pidx(dst + r * NS))] = v[rd][q][r];
    }
  }
}

// fft_plan over spass_pf with the [k][r] tables (MfccDev::ftw2); no trailing barrier.
//   ABD_TW3_TABLE: the third pass reads all R2 - 1 factors from the table instead of one base + powers
#ifdef ABD_TW3_TABLE
constexpr int kTw3 = 3;
#else
constexpr int kTw3 = 2;
#endif
// pass 2: 4 = the [pair][k] float4 table (default); 3 = the [r][k] table; 2 = one W_{R0 R1}^k load
// (ftw2 row 1) + tw_powers (A/B builds: -DABD_TW2=3 / 2).  The powers measured as fast as the pair
// table (0.239 vs 0.240 ms) but their ~6-rounding-deep factors moved a FlowMur top_db clamp
// decision: the trigger gradient left the autograd golden by 8.5e-3 (tests/test_gpu_flowmur.py)
#ifdef ABD_TW2
constexpr int kTw2 = ABD_TW2;
#else
constexpr int kTw2 = 4;
#endif
// PS > 1 (PP == 1): shared-column pairs, every row's table loads prefetched (the 4-block budget)
template <int M, int R0, int R1, int R2, int PP, bool VMUL, int NZ = M, int NO = M, int PS = 1>
__device__ __forceinline__ void fft_plan_pf(float2* buf, const float2* tw, const float2* vhat, const float4* tw4,
                                            const float4* vhat4) {
  static_assert(R0 * R1 * R2 == M, "radix plan must factor M");
  static_assert(NO == M || R2 > 1, "output pruning needs a third pass");
  constexpr int MR0 = M / R0;
  constexpr int ZT0 = (NZ + MR0 - 1) / MR0;
  constexpr int PF0 = PS > 1 ? R0 : kPrefetchRows, PF1 = PS > 1 ? R1 : kPrefetchRows,
                PF2 = PS > 1 ? R2 : kPrefetchRows;
  spass_pf<M, R0, 1, PP, 0, VMUL, ZT0, R0, PF0, VMUL, PS>(buf, nullptr, vhat, vhat4);
  spass_pf<M, R1, R0, PP, kTw2, false, R1, R1, PF1, false, PS>(buf, tw, nullptr, tw4);
  if constexpr (R2 > 1)
    spass_pf<M, R2, R0 * R1, PP, kTw3, false, R2, (NO + R0 * R1 - 1) / (R0 * R1), PF2, false, PS>(buf, tw + R0 * R1,
                                                                                              nullptr);
}

// Injected sample at signal index s (already clamped into [0, L)); branch-free so the
// gather below can keep every load of a group in flight.  Same arithmetic as inj_sample.
template <int MODE>
__device__ __forceinline__ float fsample(const float* __restrict__ x, const InjDev& inj, int s, int pos, float rs) {
  const float v = x[s];
  if constexpr (MODE == ABD_INJECT_ADD) {
    const int tl = (int)inj.trig_len;
    const float t = inj.trig[min(s, tl - 1)];
    return (s < tl) ? v + t : v;
  } else if constexpr (MODE == ABD_INJECT_SNR_WINDOW || MODE == ABD_INJECT_HALF_MIX || MODE == ABD_INJECT_DEPLOY ||
                       MODE == ABD_INJECT_DEPLOY_CLAMP) {
    const int tl = (int)inj.trig_len;
    const int o = s - pos;
    const bool in = o >= 0 && o < tl;
    const float t = inj.trig[min(max(o, 0), tl - 1)];
    if constexpr (MODE == ABD_INJECT_SNR_WINDOW) {
      return in ? v + rs * t : v;
    } else if constexpr (MODE == ABD_INJECT_HALF_MIX) {
      return in ? (v + t) / 2.0f : v / 2.0f;
    } else {
      return deploy_mix(v, t, in, rs, MODE == ABD_INJECT_DEPLOY_CLAMP);
    }
  } else {
    return v;
  }
}

// Frames 2(p0+f), 2(p0+f)+1 of one utterance -> z = (a + i b) * (chirp | window), f < np,
// zero-padded to M.  Groups of G elements per thread: all sample / chirp loads of a group
// are issued before the first LDS store.  INTERIOR: every frame of the item lies inside the
// signal (no padding, both frames of every pair exist), so sample addresses are affine.
template <int M, int NN, int PP, bool BLUE, int MODE, bool INTERIOR, int NZW = M>
__device__ __forceinline__ void load_frames(float2* __restrict__ buf, const float* __restrict__ x, const MfccDev& p,
                                            const InjDev& inj, int pos, float rs, int p0, int np) {
  static_assert(PP == 1 || NZW == M, "store pruning assumes one FFT per item");
  constexpr int TOT = PP * NZW;  // elements n >= NZW are never read by the first pass
  constexpr int ITERS = (TOT + kThreads - 1) / kThreads;
  constexpr int G = 8;
  const int L = (int)p.L;
  const bool refl = p.pad_mode != ABD_PAD_CONSTANT;
  const int hop = p.hop;
#pragma unroll
  for (int g0 = 0; g0 < ITERS; g0 += G) {
    float a[G], b[G];
    float2 c[G];
    bool ok[G];
#pragma unroll
    for (int q = 0; q < G; ++q) {
      const int idx = ltid() + (g0 + q) * kThreads;
      const int f = (PP == 1) ? 0 : idx / M;
      const int n = idx - f * M;
      ok[q] = (g0 + q < ITERS) && (idx < TOT) && (n < NN) && (PP == 1 || INTERIOR || f < np);
      const int t0 = 2 * (p0 + f);
      const int i0 = t0 * hop + n - p.pad, i1 = i0 + hop;
      if (kAblate && (p.ablate & 1)) {
        a[q] = (float)n;
        b[q] = (float)t0;
      } else if constexpr (INTERIOR) {
        // PP == 1: iterations wholly below NN load at base + immediate, wholly above NN load
        // nothing; only the straddling one clamps (its n >= NN lanes are discarded).
        const int it = g0 + q;
        const bool full = PP == 1 && (it + 1) * kThreads <= NN;
        const bool dead = PP == 1 && it * kThreads >= NN;
        if (dead) {
          a[q] = 0.0f;
          b[q] = 0.0f;
        } else {
          const int s0 = full ? i0 : min(i0, L - 1 - hop);
          a[q] = fsample<MODE>(x, inj, s0, pos, rs);
          b[q] = fsample<MODE>(x, inj, s0 + hop, pos, rs);
        }
      } else {
        const bool okb = t0 + 1 < p.T;
        int s0 = refl ? abs(i0) : i0, s1 = refl ? abs(i1) : i1;
        if (refl) {
          s0 = (s0 >= L) ? 2 * (L - 1) - s0 : s0;
          s1 = (s1 >= L) ? 2 * (L - 1) - s1 : s1;
        }
        const bool in0 = refl || (i0 >= 0 && i0 < L), in1 = refl || (i1 >= 0 && i1 < L);
        s0 = min(max(s0, 0), L - 1);
        s1 = min(max(s1, 0), L - 1);
        a[q] = in0 ? fsample<MODE>(x, inj, s0, pos, rs) : 0.0f;
        b[q] = (in1 && okb) ? fsample<MODE>(x, inj, s1, pos, rs) : 0.0f;
      }
      const int nn = min(n, NN - 1);
      if constexpr (BLUE) {
        c[q] = p.chirp_in[nn];
      } else {
        const float w = p.window[nn];
        c[q] = make_float2(w, w);
      }
    }
#pragma unroll
    for (int q = 0; q < G; ++q) {
      const int idx = ltid() + (g0 + q) * kThreads;
      if ((g0 + q < ITERS) && idx < TOT) {
        float2 z;
        if constexpr (BLUE) {
          const f2v zz = cmul_rt(f2v{a[q], b[q]}, f2v{c[q].x, c[q].y});
          z = make_float2(zz.x, zz.y);
        }
        else z = make_float2(a[q] * c[q].x, b[q] * c[q].y);
        buf[pidx(idx)] = ok[q] ? z : make_float2(0.0f, 0.0f);
      }
    }
  }
}

// Interior Bluestein items (one frame pair, every sample inside the signal) with no injection or
// the additive trigger: each thread takes 4 consecutive elements n..n+3, so a frame's samples come
// as one (dword-aligned) 16-B load, the chirp as two, the trigger as one -- a quarter of the
// per-element path's vector-memory instructions, which bound the kernel (TD busy ~85-90 %).
// Same arithmetic per element as load_frames / fsample.
// PS > 1: the item's PS consecutive pairs (frames 2(p0+q), 2(p0+q)+1) into buffers FS apart, one
// chirp load per element group for all of them.
template <int M, int NN, int MODE, int NZW, int PS = 1>
__device__ __forceinline__ void load_frames_v4(float2* __restrict__ buf, const float* __restrict__ x, const MfccDev& p,
                                               const InjDev& inj, int p0) {
  static_assert(MODE == ABD_INJECT_NONE || MODE == ABD_INJECT_ADD, "vector gather: no / additive injection");
  static_assert(NZW % 4 == 0, "element groups of 4");
  constexpr int GROUPS = NZW / 4;
  constexpr int ITERS = (GROUPS + kThreads - 1) / kThreads;
  constexpr int FS = M + M / 16;
  const int hop = p.hop;
  const int base = 2 * p0 * hop - p.pad;  // sample of frame a's element 0
  const int tl = (int)inj.trig_len;
  const float4* ci4 = reinterpret_cast<const float4*>(p.chirp_in);
#pragma unroll
  for (int it = 0; it < ITERS; ++it) {
    const int gi = ltid() + it * kThreads;
    if (ITERS * kThreads != GROUPS && gi >= GROUPS) break;
    const int n = 4 * gi;
    float a[PS][4], b[PS][4];
    float2 c[4];
    if (kAblate && (p.ablate & 1)) {  // measurement builds: no sample / trigger / chirp loads
#pragma unroll
      for (int q = 0; q < PS; ++q)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          a[q][e] = (float)(n + e);
          b[q][e] = (float)(p0 + q);
        }
#pragma unroll
      for (int e = 0; e < 4; ++e) c[e] = make_float2(1.0f, (float)e);
    } else if (n + 3 < NN) {
      const float4 c01 = ci4[2 * gi], c23 = ci4[2 * gi + 1];
#pragma unroll
      for (int q = 0; q < PS; ++q) {
        const int s0 = base + 2 * q * hop + n, s1 = s0 + hop;
        float4 va, vb;
        __builtin_memcpy(&va, x + s0, 16);
        __builtin_memcpy(&vb, x + s1, 16);
        a[q][0] = va.x; a[q][1] = va.y; a[q][2] = va.z; a[q][3] = va.w;
        b[q][0] = vb.x; b[q][1] = vb.y; b[q][2] = vb.z; b[q][3] = vb.w;
        if constexpr (MODE == ABD_INJECT_ADD) {
          // v + t for samples s < tl (fsample): whole groups by one 16-B trigger load each
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int sb = h ? s1 : s0;
            float* v = h ? b[q] : a[q];
            if (sb + 3 < tl) {
              float4 tv;
              __builtin_memcpy(&tv, inj.trig + sb, 16);
              v[0] += tv.x; v[1] += tv.y; v[2] += tv.z; v[3] += tv.w;
            } else if (sb < tl) {
#pragma unroll
              for (int e = 0; e < 4; ++e)
                if (sb + e < tl) v[e] += inj.trig[sb + e];
            }
          }
        }
      }
      c[0] = make_float2(c01.x, c01.y); c[1] = make_float2(c01.z, c01.w);
      c[2] = make_float2(c23.x, c23.y); c[3] = make_float2(c23.z, c23.w);
    } else {  // the group straddling NN: per element, zero past the frame
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const bool ok = n + e < NN;
#pragma unroll
        for (int q = 0; q < PS; ++q) {
          const int s0 = base + 2 * q * hop + min(n + e, NN - 1);
          a[q][e] = ok ? fsample<MODE>(x, inj, s0, 0, 0.0f) : 0.0f;
          b[q][e] = ok ? fsample<MODE>(x, inj, s0 + hop, 0, 0.0f) : 0.0f;
        }
        c[e] = p.chirp_in[min(n + e, NN - 1)];
      }
    }
#pragma unroll
    for (int q = 0; q < PS; ++q)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const f2v zz = cmul_rt(f2v{a[q][e], b[q][e]}, f2v{c[e].x, c[e].y});
        buf[q * FS + pidx(n + e)] = (n + e < NN) ? make_float2(zz.x, zz.y) : make_float2(0.0f, 0.0f);
      }
  }
}

// BLUE: the item's PP pairs are shared-column FFTs (spass_pf PS = PP), loaded pair by pair into
// buffers M + M/16 apart (the vector gather takes all PP at once)
template <int M, int NN, int PP, bool BLUE, int MODE, int NZW = M>
__device__ __forceinline__ void load_item(float2* buf, const float* x, const MfccDev& p, const InjDev& inj, int pos,
                                          float rs, int p0, int np) {
  const int first = 2 * p0 * p.hop - p.pad;
  const int last_t = 2 * (p0 + PP) - 1;
  const bool interior = np == PP && first >= 0 && last_t < p.T && last_t * p.hop - p.pad + NN <= (int)p.L;
  if constexpr (BLUE && (MODE == ABD_INJECT_NONE || MODE == ABD_INJECT_ADD) && NZW % 4 == 0) {
    if (interior && kGatherV4) {
      load_frames_v4<M, NN, MODE, NZW, PP>(buf, x, p, inj, p0);
      return;
    }
  }
  if constexpr (BLUE && PP > 1) {
#pragma unroll
    for (int q = 0; q < PP; ++q) {  // pairs past the utterance (q >= np) load clamped frames, never stored
      float2* bq = buf + q * (M + M / 16);
      if (interior) load_frames<M, NN, 1, BLUE, MODE, true, NZW>(bq, x, p, inj, pos, rs, p0 + q, 1);
      else load_frames<M, NN, 1, BLUE, MODE, false, NZW>(bq, x, p, inj, pos, rs, p0 + q, 1);
    }
  } else {
    if (interior) load_frames<M, NN, PP, BLUE, MODE, true, NZW>(buf, x, p, inj, pos, rs, p0, np);
    else load_frames<M, NN, PP, BLUE, MODE, false, NZW>(buf, x, p, inj, pos, rs, p0, np);
  }
}

// Persistent blocks walk a contiguous range of (utterance, chunk) work items; each item is
// PP pairs of frames of one utterance.  Per item:
//   gather + inject + chirp/window -> FFT (-> pointwise * vhat -> FFT, Bluestein)
//   -> in-place power |A_k|^2, |B_k|^2 (Bluestein output chirp fused)
//   -> mel by half-filter slots (2 per filter, balanced), halves combined by a lane swap
//   -> 10 log10 -> ws_db, per-item max -> ws_max.
// Twiddles are read through the L1 from the [k][r] tables (MfccDev::ftw2): the block's LDS is its
// FFT buffer alone (19.6 KB for Bluestein), so 8 blocks (32 waves, the CU maximum) fit; the kernel
// is latency-bound (46 % of wave cycles parked at barriers / waitcnt), so residency is what pays.
// the L1 instead, the Bluestein block's LDS drops from 23.7 to 19.6 KB and 8 blocks (32 waves, the
// CU maximum) fit instead of 6 -- the kernel is latency-bound (46 % of wave cycles parked at
// barriers / waitcnt, profiles/r2_stft_pmc.txt), so the extra residency is what pays.
constexpr int kBlueBlocks = 8;

// Bluestein item (one pair of frames) after the second FFT: power -> mel -> dB.
//   power: bin k of frames a / b from Z[k], Z[N-k] (output chirp fused), written as one float2
//          per bin into a contiguous array placed past the FFT outputs that are still read
//          (Z[k], k < N), so the reads and writes need no barrier between them;
//   mel:   thread = half-filter slot (2 m + h, 2 n_mels == kThreads), kMelHP zero-padded weights
//          per slot (p.mel3_w), every read base + immediate, one float2 FMA per bin for both
//          frames (two v_fma_f32 in the scalar build); the halves are combined by a lane swap, lane h writes frame 2 p0 + h.
constexpr int kMelHP = 16;  // padded bins per half-filter slot of the Bluestein fast path
// bins per mel segment of the non-Bluestein fast path (MfccDev::mseg_*); ABD_MEL_SEG=0 builds the
// half-slot loop instead (measurement builds)
constexpr int kMelSeg = 8;
#ifndef ABD_MEL_SEG
#define ABD_MEL_SEG 1
#endif
// float2 slot of a pair's FFT buffer where the segmented mel's partials start (past pidx(nf - 1))
constexpr int mel_seg_offset(int nf) { return ((nf + nf / 16) + 15) / 16 * 16; }
// PS pairs (buffers FS apart, frames t0 + 2q, t0 + 2q + 1): one chirp / weight load for all of them.
template <int M, int NN, int PS = 1>
__device__ __forceinline__ float power_mel_blue(float2* __restrict__ bufs, const MfccDev& p, float* __restrict__ db_u,
                                                int t0) {
  constexpr int NF = NN / 2 + 1;
  constexpr int POFF = ((NN + NN / 16) + 15) / 16 * 16;  // >= pidx(N - 1) + 1
  constexpr int FS = M + M / 16;
  static_assert(POFF + NF + kMelHP <= M + M / 16, "power array must fit the FFT buffer");
  f2v* buf = reinterpret_cast<f2v*>(bufs);
  f2v* pw = buf + POFF;
  constexpr int PR = (NF + kMelHP + kThreads - 1) / kThreads;
  f2v cq[PR][2];  // output chirps, loaded ahead of the barrier that publishes the last FFT pass
#pragma unroll
  for (int rd = 0; rd < PR; ++rd) {
    const int k = min(ltid() + rd * kThreads, NF - 1);
    const float4 c2 = p.chirp_out2[k];  // (w[k] / M, w[N - k] / M): one 16-B load per bin
    cq[rd][0] = f2v{c2.x, c2.y};
    cq[rd][1] = f2v{c2.z, c2.w};
  }
  __syncthreads();
#pragma unroll
  for (int rd = 0; rd < PR; ++rd) {
    const int k = ltid() + rd * kThreads;
    if (k < NF + kMelHP) {
#pragma unroll
      for (int q = 0; q < PS; ++q) {
        f2v e = f2v{0.0f, 0.0f};
        if (k < NF) {
          const int kn = (k == 0) ? 0 : NN - k;
          // X[k] = conj(w[k] R[k]) / M  (chirp_out = w / M)
          f2v P1 = cmul_rt(buf[q * FS + pidx(k)], cq[rd][0]), Q = cmul_rt(buf[q * FS + pidx(kn)], cq[rd][1]);
          P1.y = -P1.y;
          Q.y = -Q.y;
          const float ar = 0.5f * (P1.x + Q.x), ai = 0.5f * (P1.y - Q.y);
          const float br = 0.5f * (P1.y + Q.y), bi = 0.5f * (Q.x - P1.x);
          e = f2v{ar * ar + ai * ai, br * br + bi * bi};
        }
        pw[q * FS + k] = e;  // bins NF .. NF + kMelHP - 1: zeros under the slots' padded weights
      }
    }
  }
  __syncthreads();
  const int sl = ltid();
  const int start = p.mel2_meta[sl].x;
  const float4* wq = reinterpret_cast<const float4*>(p.mel3_w) + sl;  // [q][slot], 2 n_mels == kThreads slots
  float w[kMelHP];
#pragma unroll
  for (int q = 0; q < kMelHP / 4; ++q) {
    const float4 v = wq[q * kThreads];
    w[4 * q] = v.x;
    w[4 * q + 1] = v.y;
    w[4 * q + 2] = v.z;
    w[4 * q + 3] = v.w;
  }
  float lmax = -INFINITY;
#pragma unroll
  for (int q = 0; q < PS; ++q) {
    const f2v* ps = pw + q * FS + start;
    f2v s = f2v{0.0f, 0.0f};
#pragma unroll
    for (int i = 0; i < kMelHP; ++i) s = fmav(ps[i], f2v{w[i], w[i]}, s);
    s.x += __shfl_xor(s.x, 1);
    s.y += __shfl_xor(s.y, 1);
    const int h = sl & 1;
    const int t = t0 + 2 * q + h;
    if (t < p.T) {
      const float d = 10.0f * log10f(fmaxf(h ? s.y : s.x, 1e-10f));
      db_u[(int64_t)t * p.n_mels + (sl >> 1)] = d;
      lmax = fmaxf(lmax, d);
    }
  }
  return lmax;
}

// NBLK: blocks per CU the Bluestein build is register-budgeted for (8: 64 VGPRs and <= 80 SGPRs, the
// compiler spills SGPRs into VGPR lanes; 7: 72 VGPRs / 96 SGPRs, no spills, one block fewer)
template <int M, int NN, int R0, int R1, int R2, int PP, bool BLUE, int NBLK = kBlueBlocks>
__global__ void __launch_bounds__(kThreads, NBLK) stft_mel_fast_kernel(MfccDev p, const float* __restrict__ wave,
                                                                 int64_t row_stride,
                                                                 const int32_t* __restrict__ rows, int64_t batch,
                                                                 InjDev inj, const float* __restrict__ rowscale,
                                                                 float* __restrict__ ws_db,
                                                                 float* __restrict__ ws_max,
                                                                 unsigned* __restrict__ queue) {
  // first FFT's first pass reads rows r < ceil(N / (M/R0)) only: the rest is never stored
  constexpr int kNZW = BLUE ? ((NN + M / R0 - 1) / (M / R0)) * (M / R0) : M;
  // Bluestein: the item's PP pairs are shared-column FFTs (one twiddle / vhat / chirp / mel-weight
  // load per element for all of them); the other plans map PP pairs onto distinct threads
  constexpr int PS = BLUE ? PP : 1, PG = BLUE ? 1 : PP;
  extern __shared__ __attribute__((aligned(16))) float2 lds[];
  constexpr int NTL = 0;
  float2* buf = lds + NTL;
#ifdef ABD_MEL_W_LDS
  float* wl = reinterpret_cast<float*>(lds + NTL + PP * (M + M / 16));
#else
  const float* wl = p.mel2_w;  // 4-5 KB, L1-resident: keeps the block's LDS to its FFT buffer
#endif
  __shared__ float red[kThreads / kWave];
  const float2* tw = p.ftw2;
#ifdef ABD_MEL_W_LDS
  for (int i = ltid(); i < p.mel2_total; i += kThreads) wl[i] = p.mel2_w[i];
#endif
  __shared__ unsigned s_item;
  const int chunks = p.chunks;
  const unsigned n_items = (unsigned)(batch * chunks);
  const int P = (p.T + 1) / 2;
  constexpr int nf = NN / 2 + 1;
  const int S = 2 * p.n_mels;
  // Block b's first item is item b (grid <= items); the rest, [gridDim.x, n_items), come from
  // dynamic queues: no static split, so blocks that become resident late cannot leave a tail.
  // kQueues counters on separate 256-B lines, each owning a contiguous 1/kQueues of those items; a
  // block pulls from its home queue, then steals from the others.  Thread 0 grabs the next item in
  // the middle of the current one (after its first FFT: the atomic's latency still hides behind the
  // rest of the item).  Block 0 zeroes the counters as it starts (no host memset launch); a grid of
  // resident blocks is dispatched within ~1 us (MI355X_MICROARCH.md, workgroup dispatch), and no
  // block grabs before it has loaded and transformed its first item (>= 5 us), so the zeroing has
  // landed before the first grab.  That is a timing argument, not a guarantee: a grab that still
  // beat the store would read the workspace's previous counters and either take an item that is
  // handed out again after the zeroing (both passes write the same values -- every item overwrites,
  // none accumulates) or see an exhausted queue and leave its share to the other blocks; never skip
  // one, since block 0 itself runs on after its store.  (Round 6 measured the alternative -- the
  // last block to finish resets the counters, so a used workspace always starts at zero -- at
  // +7 us per launch: 2,048 same-address atomics at the kernel's tail, profiles/r6_stft/queue_ab.txt.)
  const unsigned g0 = gridDim.x;
  const unsigned rest = n_items > g0 ? n_items - g0 : 0u;
  const unsigned qlen = (rest + kQueues - 1) / kQueues;
  if (blockIdx.x == 0 && threadIdx.x < kQueues)
    __hip_atomic_store(queue + threadIdx.x * kQueueStride, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  unsigned home = blockIdx.x % kQueues;
  auto grab = [&]() -> unsigned {
    for (int t = 0; t < kQueues; ++t) {
      const unsigned q = (home + t) % kQueues;
      const unsigned v = atomicAdd(queue + q * kQueueStride, 1u);
      const unsigned it = q * qlen + v;
      if (v < qlen && it < rest) {
        home = q;
        return g0 + it;
      }
    }
    return ~0u;
  };
  if (threadIdx.x == 0) s_item = blockIdx.x < n_items ? blockIdx.x : ~0u;
  __syncthreads();  // also publishes the staged tables
  unsigned item = s_item;
  while (item != ~0u) {
    unsigned next = 0;
    const int64_t u = item / chunks;
    const int c = (int)(item - u * chunks);
    const int64_t row = rows ? rows[u] : u;
    const float* x = wave + row * row_stride;
    const bool pois = row_poisoned(inj, u);
    const int pos = (inj.position != nullptr) ? inj.position[u] : 0;
    const float rs = (rowscale != nullptr) ? rowscale[inj.scale_by_row ? row : u] : 0.0f;
    const int p0 = c * PP;
    const int np = min(PP, P - p0);
    switch (pois ? inj.mode : ABD_INJECT_NONE) {
      case ABD_INJECT_ADD: load_item<M, NN, PP, BLUE, ABD_INJECT_ADD, kNZW>(buf, x, p, inj, pos, rs, p0, np); break;
      case ABD_INJECT_SNR_WINDOW:
        load_item<M, NN, PP, BLUE, ABD_INJECT_SNR_WINDOW, kNZW>(buf, x, p, inj, pos, rs, p0, np);
        break;
      case ABD_INJECT_HALF_MIX:
        load_item<M, NN, PP, BLUE, ABD_INJECT_HALF_MIX, kNZW>(buf, x, p, inj, pos, rs, p0, np);
        break;
      case ABD_INJECT_DEPLOY: load_item<M, NN, PP, BLUE, ABD_INJECT_DEPLOY, kNZW>(buf, x, p, inj, pos, rs, p0, np); break;
      case ABD_INJECT_DEPLOY_CLAMP:
        load_item<M, NN, PP, BLUE, ABD_INJECT_DEPLOY_CLAMP, kNZW>(buf, x, p, inj, pos, rs, p0, np);
        break;
      default: load_item<M, NN, PP, BLUE, ABD_INJECT_NONE, kNZW>(buf, x, p, inj, pos, rs, p0, np); break;
    }
    // no barrier here: the first pass opens with the one that publishes the loaded frames
    if (!(kAblate && (p.ablate & 2)))
      fft_plan_pf<M, R0, R1, R2, PG, false, BLUE ? NN : M, M, PS>(buf, tw, nullptr, p.ftw4, nullptr);
    if (threadIdx.x == 0) next = grab();  // mid-item: see the queue comment above
    if constexpr (BLUE) {
      if (!(kAblate && (p.ablate & 2))) fft_plan_pf<M, R0, R1, R2, PG, true, M, NN, PS>(buf, tw, p.vhat, p.ftw4, p.vhat4);
    }
    float lmax = -INFINITY;
    if constexpr (BLUE) {
      if (p.mel3_w != nullptr && !(kAblate && (p.ablate & 4))) {
        lmax = power_mel_blue<M, NN, PS>(buf, p, ws_db + (int64_t)u * p.T * p.n_mels, 2 * p0);
        goto item_done;
      }
    }
    __syncthreads();  // the last pass's writes (fft_plan_pf leaves no trailing barrier)
    if (!(kAblate && (p.ablate & 4))) {
      // Power of the two real spectra, written over Z[k] (k <= N/2).  Z[k] is read only by
      // the thread that owns bin k (Z[N-k] with N-k > N/2 is never written), so no barrier
      // is needed between the reads and the in-place writes.
      for (int idx = ltid(); idx < np * nf; idx += kThreads) {
        const int f = idx / nf;
        const int k = idx - f * nf;
        const int kn = (k == 0) ? 0 : NN - k;
        float2* Z = buf + f * (M + M / 16);
        float2 P1 = Z[pidx(k)], Q = Z[pidx(kn)];
        if constexpr (BLUE) {  // X[k] = conj(w[k] R[k]) / M
          const float2 a = cmul(p.chirp_out[k], P1), b = cmul(p.chirp_out[kn], Q);
          P1 = make_float2(a.x, -a.y);
          Q = make_float2(b.x, -b.y);
        }
        const float ar = 0.5f * (P1.x + Q.x), ai = 0.5f * (P1.y - Q.y);
        const float br = 0.5f * (P1.y + Q.y), bi = 0.5f * (Q.x - P1.x);
        Z[pidx(k)] = make_float2(ar * ar + ai * ai, br * br + bi * bi);
      }
      __syncthreads();
      if (p.nseg > 0) {
        // segmented mel (MfccDev::mseg_*): task = (pair f, segment) -> the segment's kMelSeg bins
        // of both frames into a partial past the power values (Z[k > N/2] is dead after the power
        // stage), then task = (pair f, filter m) sums its segments in order -> dB of both frames
        constexpr int PSO = mel_seg_offset(nf);
        const int nseg = p.nseg;
        for (int g = ltid(); g < np * nseg; g += kThreads) {
          const int f = g / nseg, sg = g - f * nseg;
          const float2* Z = buf + f * (M + M / 16);
          const int st = p.mseg_start[sg];
          f2v acc = f2v{0.0f, 0.0f};
#pragma unroll
          for (int q = 0; q < kMelSeg / 4; ++q) {
            const float4 w4 = p.mseg_w[sg * (kMelSeg / 4) + q];
            const float wq[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float2 pw = Z[pidx(st + 4 * q + e)];
              acc = fmav(f2v{pw.x, pw.y}, f2v{wq[e], wq[e]}, acc);
            }
          }
          reinterpret_cast<f2v*>(buf + f * (M + M / 16) + PSO)[sg] = acc;
        }
        __syncthreads();
        for (int h = ltid(); h < np * p.n_mels; h += kThreads) {
          const int f = h / p.n_mels, m = h - f * p.n_mels;
          const f2v* part = reinterpret_cast<const f2v*>(buf + f * (M + M / 16) + PSO);
          const int2 fs = p.mfilt_seg[m];
          f2v sum = part[fs.x];
          for (int j = 1; j < fs.y; ++j) sum += part[fs.x + j];
          const int t = 2 * (p0 + f);
          if (t < p.T) {
            const float d = 10.0f * log10f(fmaxf(sum.x, 1e-10f));
            ws_db[((int64_t)u * p.T + t) * p.n_mels + m] = d;
            lmax = fmaxf(lmax, d);
          }
          if (t + 1 < p.T) {
            const float d = 10.0f * log10f(fmaxf(sum.y, 1e-10f));
            ws_db[((int64_t)u * p.T + t + 1) * p.n_mels + m] = d;
            lmax = fmaxf(lmax, d);
          }
        }
      } else {
        const int tot = np * S;
        const int rounds = (tot + kThreads - 1) / kThreads;
        const int hp = p.mel2_hp;
        const int wlast = p.mel2_total - 1;
        for (int rd = 0; rd < rounds; ++rd) {  // uniform: every lane reaches the shuffles
          const int g = ltid() + rd * kThreads;
          const bool act = g < tot;
          const int gg = act ? g : 0;
          const int f = gg / S;
          const int sl = gg - f * S;
          const int4 meta = p.mel2_meta[sl];  // (start, count, weight offset, -)
          const float2* Z = buf + f * (M + M / 16);
          float sa = 0.0f, sb = 0.0f;
          for (int i0 = 0; i0 < hp; i0 += 8) {
  #pragma unroll
            for (int q = 0; q < 8; ++q) {
              const int i = i0 + q;
              const int k = min(meta.x + i, nf - 1);
              const float w = (i < meta.y) ? wl[min(meta.z + i, wlast)] : 0.0f;
              const float2 pw = Z[pidx(k)];
              sa = fmaf(pw.x, w, sa);
              sb = fmaf(pw.y, w, sb);
            }
          }
          sa += __shfl_xor(sa, 1);
          sb += __shfl_xor(sb, 1);
          const int h = sl & 1;
          const int t = 2 * (p0 + f) + h;
          if (act && t < p.T) {
            const float d = 10.0f * log10f(fmaxf(h ? sb : sa, 1e-10f));
            ws_db[((int64_t)u * p.T + t) * p.n_mels + (sl >> 1)] = d;
            lmax = fmaxf(lmax, d);
          }
        }
      }
    }
  item_done:
    lmax = abd::wave_max(lmax);
    if ((ltid() & 63) == 0) red[ltid() / kWave] = lmax;
    __syncthreads();
    if (threadIdx.x == 0) {
      float mm = red[0];
      for (int i = 1; i < kThreads / kWave; ++i) mm = fmaxf(mm, red[i]);
      ws_max[u * chunks + c] = mm;
      s_item = next;
    }
    __syncthreads();  // s_item published; this item's LDS reads are complete
    item = s_item;
  }
}

// =====================================================================================
// Backward of the MFCC w.r.t. the trigger of a DEPLOY mix: FlowMur trigger optimisation
// (utils/flowmur_generate_trigger.py:89-104: clamp(deploy(w, t)) -> MFCC -> frozen CNN -> CE,
// loss.backward() to t).  After a recomputed forward (stft_mel_fast_kernel -> dB, per-item max):
//   mfcc_db_bwd_kernel : dMFCC -> d dB (DCT^T) -> top_db clamp adjoint (torch.maximum gives a
//       tie half the gradient; amax hands the clamped mass to the maxima, split evenly) ->
//       d mel power (10 / (ln10 x)), in place over the dB workspace
//   stft_bwd_kernel    : per item (PP frame pairs of one utterance): the frames' FFT again,
//       dP_k = sum_m fb[k][m] dmel[m] (<= 2 filters per bin), Y_k = dP_k conj(X_k), and
//       g_n = 2 Re sum_{k<=N/2} Y_k W^{kn} as ONE forward FFT of the Hermitian extension of the
//       packed pair (H_k = Y_k, H_{N-k} = conj(Y_k), H_0 = 2 Y_0, H_{N/2} = 2 Y_{N/2}: real
//       output, frame a in .x, frame b in .y), times the window -> per-frame sample gradients
//   wave_bwd_kernel    : overlap-add of the frames, reflect-pad adjoint, clamp mask, mix
//       adjoint: window part dx/(s+1) per row, SNR-scale part sum dx (w - t_in)/(s+1)^2
//   trig_coef_kernel / trig_grad_kernel : rows summed in order, plus t |t|^-2 sum_u s_u dS_u
//       (s_u = 10^(30/20) |t| / |w_u|)
// =====================================================================================
constexpr float kDbAmin = -99.999f;
constexpr int kWaveSpan = 1024;  // samples per wave_bwd block  // 10 log10(amin = 1e-10) = -100: clamped, no gradient

__global__ void __launch_bounds__(kThreads) mfcc_db_bwd_kernel(MfccDev p, const float* __restrict__ ws_max,
                                                               const float* __restrict__ dout, float* __restrict__ db_io) {
  extern __shared__ __attribute__((aligned(16))) float smb[];
  float* dct = smb;                       // n_mels x n_mfcc
  float* g = smb + p.n_mels * p.n_mfcc;   // T x n_mels: gradient kept by the top_db clamp
  __shared__ double redd[kThreads / kWave];
  __shared__ int redi[kThreads / kWave];
  __shared__ float redm[kThreads / kWave];
  const int64_t u = blockIdx.x;
  const int tid = threadIdx.x;
  for (int i = tid; i < p.n_mels * p.n_mfcc; i += kThreads) dct[i] = p.dct[i];
  float mx = -INFINITY;
  for (int i = tid; i < p.chunks; i += kThreads) mx = fmaxf(mx, ws_max[u * p.chunks + i]);
  mx = abd::wave_max(mx);
  if ((tid & 63) == 0) redm[tid >> 6] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(redm[0], redm[1]), fmaxf(redm[2], redm[3]));
  const float thr = (p.top_db >= 0.0f) ? mx - p.top_db : -INFINITY;
  const int n = p.T * p.n_mels;
  float* db = db_io + u * (int64_t)n;
  const float* d = dout + u * (int64_t)p.T * p.n_mfcc;
  double clamped = 0.0;
  int nmax = 0;
  for (int e = tid; e < n; e += kThreads) {
    const int t = e / p.n_mels, m = e - t * p.n_mels;
    float acc = 0.0f;
    for (int c = 0; c < p.n_mfcc; ++c) acc = fmaf(dct[m * p.n_mfcc + c], d[t * p.n_mfcc + c], acc);
    const float v = db[e];
    float keep = acc;
    if (v < thr) {
      clamped += (double)acc;
      keep = 0.0f;
    } else if (v == thr) {
      clamped += 0.5 * (double)acc;
      keep = 0.5f * acc;
    }
    nmax += (v == mx) ? 1 : 0;
    g[e] = keep;
  }
  clamped = abd::wave_sum_d(clamped);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) nmax += __shfl_xor(nmax, o, 64);
  if ((tid & 63) == 0) {
    redd[tid >> 6] = clamped;
    redi[tid >> 6] = nmax;
  }
  __syncthreads();
  const double cs = redd[0] + redd[1] + redd[2] + redd[3];
  const int nm = redi[0] + redi[1] + redi[2] + redi[3];
  const float share = (float)(cs / (double)max(nm, 1));
  for (int e = tid; e < n; e += kThreads) {
    const float v = db[e];
    const float ge = g[e] + ((v == mx) ? share : 0.0f);
    // d/dx 10 log10(max(x, amin)) = 10 / (ln10 x) above amin; x is the mel power behind v
    const float x = exp10f(0.1f * v);
    db[e] = (v > kDbAmin) ? ge * (4.3429448190325182f / x) : 0.0f;
  }
}

template <int M, int R0, int R1, int R2, int PP>
__global__ void __launch_bounds__(kThreads) stft_bwd_kernel(MfccDev p, const float* __restrict__ wave,
                                                            int64_t row_stride, const int32_t* __restrict__ rows,
                                                            InjDev inj, const float* __restrict__ rowscale,
                                                            const float* __restrict__ dmel,
                                                            float* __restrict__ gframes) {
  constexpr int NT = 2 * R0 * R1;
  constexpr int N = M, NF = N / 2 + 1, MP = M + M / 16;
  extern __shared__ __attribute__((aligned(16))) float2 lds[];
  float2* tw = lds;
  float2* buf = lds + NT;
  for (int i = ltid(); i < NT; i += kThreads) tw[i] = p.ftw[i];
  const int64_t u = blockIdx.x / p.chunks;
  const int c = (int)(blockIdx.x - u * p.chunks);
  const int64_t row = rows ? rows[u] : u;
  const float* x = wave + row * row_stride;
  const bool pois = row_poisoned(inj, u);
  const int pos = inj.position ? inj.position[u] : 0;
  const float rs = rowscale ? rowscale[u] : 0.0f;
  const int P = (p.T + 1) / 2;
  const int p0 = c * PP;
  const int np = min(PP, P - p0);
  switch (pois ? inj.mode : ABD_INJECT_NONE) {
    case ABD_INJECT_DEPLOY: load_item<M, N, PP, false, ABD_INJECT_DEPLOY>(buf, x, p, inj, pos, rs, p0, np); break;
    case ABD_INJECT_DEPLOY_CLAMP:
      load_item<M, N, PP, false, ABD_INJECT_DEPLOY_CLAMP>(buf, x, p, inj, pos, rs, p0, np);
      break;
    default: load_item<M, N, PP, false, ABD_INJECT_NONE>(buf, x, p, inj, pos, rs, p0, np); break;
  }
  __syncthreads();
  fft_plan<M, R0, R1, R2, PP, false>(buf, tw, nullptr);
  // packed spectra -> Hermitian-extended packed adjoint, in place: the thread of bin k is the
  // only reader and writer of positions k and N-k
  for (int idx = ltid(); idx < np * NF; idx += kThreads) {
    const int f = idx / NF, k = idx - f * NF;
    const int kn = (k == 0) ? 0 : N - k;
    float2* Z = buf + f * MP;
    const float2 P1 = Z[pidx(k)], Q = Z[pidx(kn)];
    const float ar = 0.5f * (P1.x + Q.x), ai = 0.5f * (P1.y - Q.y);
    const float br = 0.5f * (P1.y + Q.y), bi = 0.5f * (Q.x - P1.x);
    const int ta = 2 * (p0 + f);
    const int2 mm = p.bin_mel[k];
    const float2 ww = p.bin_w[k];
    const float* da = dmel + ((int64_t)u * p.T + ta) * p.n_mels;
    float dpa = 0.0f, dpb = 0.0f;
    if (mm.x >= 0) dpa = ww.x * da[mm.x];
    if (mm.y >= 0) dpa = fmaf(ww.y, da[mm.y], dpa);
    if (ta + 1 < p.T) {
      const float* dbp = da + p.n_mels;
      if (mm.x >= 0) dpb = ww.x * dbp[mm.x];
      if (mm.y >= 0) dpb = fmaf(ww.y, dbp[mm.y], dpb);
    }
    // Y = dP conj(X)
    const float yar = dpa * ar, yai = -dpa * ai, ybr = dpb * br, ybi = -dpb * bi;
    if (k == 0 || 2 * k == N) {
      Z[pidx(k)] = make_float2(2.0f * yar, 2.0f * ybr);  // X_0, X_{N/2} are real
    } else {
      Z[pidx(k)] = make_float2(yar - ybi, yai + ybr);   // Y_a + i Y_b
      Z[pidx(kn)] = make_float2(yar + ybi, ybr - yai);  // conj(Y_a) + i conj(Y_b)
    }
  }
  __syncthreads();
  fft_plan<M, R0, R1, R2, PP, false>(buf, tw, nullptr);
  for (int idx = ltid(); idx < np * N; idx += kThreads) {
    const int f = idx / N, nn = idx - f * N;
    const float2 v = buf[f * MP + pidx(nn)];
    const float w = p.window[nn];
    const int ta = 2 * (p0 + f);
    gframes[((int64_t)u * p.T + ta) * N + nn] = v.x * w;
    if (ta + 1 < p.T) gframes[((int64_t)u * p.T + ta + 1) * N + nn] = v.y * w;
  }
}

// block = (kWaveSpan samples, utterance), kWaveSpan / 256 samples per thread: overlap-add +
// padding adjoint + clamp mask + mix adjoint; the SNR-scale term is reduced per block
__global__ void __launch_bounds__(kThreads) wave_bwd_kernel(MfccDev p, const float* __restrict__ gframes,
                                                            const float* __restrict__ wave, int64_t row_stride,
                                                            const int32_t* __restrict__ rows, InjDev inj,
                                                            const float* __restrict__ rowscale,
                                                            float* __restrict__ wgrad, double* __restrict__ spart) {
  const int64_t u = blockIdx.y;
  const int64_t row = rows ? rows[u] : u;
  const float* x = wave + row * row_stride;
  const int pos = inj.position[u];
  const float rs = rowscale[u];
  const int L = (int)p.L, N = p.N, hop = p.hop, pad = p.pad, T = p.T;
  const int tl = (int)inj.trig_len;
  const float* G = gframes + u * (int64_t)T * N;
  const double sp1 = (double)rs + 1.0;
  double part = 0.0;
#pragma unroll
  for (int j = 0; j < kWaveSpan / kThreads; ++j) {
    const int s = blockIdx.x * kWaveSpan + j * kThreads + threadIdx.x;
    if (s >= L) break;
    // centre-padded positions that read sample s (torch reflect padding / constant)
    int ip[3];
    int ni = 0;
    ip[ni++] = s + pad;
    if (p.pad_mode != ABD_PAD_CONSTANT) {
      if (s >= 1 && s <= pad) ip[ni++] = pad - s;
      if (s >= L - 1 - pad && s <= L - 2) ip[ni++] = pad + 2 * (L - 1) - s;
    }
    float dx = 0.0f;
    for (int q = 0; q < ni; ++q) {
      const int i = ip[q];
      const int a = i - N + 1;
      const int tlo = a > 0 ? (a + hop - 1) / hop : 0;
      const int thi = min(T - 1, i / hop);
      for (int t = tlo; t <= thi; ++t) dx += G[(int64_t)t * N + (i - t * hop)];
    }
    const float v = x[s];
    const int o = s - pos;
    const bool in = o >= 0 && o < tl;
    const float tv = in ? inj.trig[o] : 0.0f;
    // torch.clamp passes the gradient for -1 <= y <= 1 only
    if (inj.mode == ABD_INJECT_DEPLOY_CLAMP) {
      const float y = deploy_mix(v, tv, in, rs, false);
      if (y < -1.0f || y > 1.0f) dx = 0.0f;
    }
    if (in) wgrad[u * (int64_t)tl + o] = dx / (rs + 1.0f);
    part += (double)dx * ((double)v - (double)tv) / (sp1 * sp1);
  }
  __shared__ double red[kThreads / kWave];
  part = abd::wave_sum_d(part);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = part;
  __syncthreads();
  if (threadIdx.x == 0) spart[u * gridDim.x + blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// coef = sum_u s_u dS_u / |t|^2, where dS_u = d loss / d s_u (one block, fixed order)
__global__ void __launch_bounds__(kThreads) trig_coef_kernel(const double* __restrict__ spart, int nbx, int64_t B,
                                                             const float* __restrict__ rowscale,
                                                             const float* __restrict__ trig, int64_t tl,
                                                             double* __restrict__ coef) {
  double acc = 0.0, tt = 0.0;
  for (int64_t u = threadIdx.x; u < B; u += kThreads) {
    double su = 0.0;
#pragma unroll 8
    for (int b = 0; b < nbx; ++b) su += spart[u * nbx + b];
    acc += (double)rowscale[u] * su;
  }
  for (int64_t k = threadIdx.x; k < tl; k += kThreads) tt += (double)trig[k] * (double)trig[k];
  __shared__ double red[2][kThreads / kWave];
  acc = abd::wave_sum_d(acc);
  tt = abd::wave_sum_d(tt);
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = acc;
    red[1][threadIdx.x >> 6] = tt;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const double a = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    const double t2 = red[1][0] + red[1][1] + red[1][2] + red[1][3];
    coef[0] = t2 > 0.0 ? a / t2 : 0.0;
  }
}

// dtrigger[k] = sum_u wgrad[u][k] + coef * t[k]; block = 64 consecutive k x 4 row groups, the
// four partial sums combined in a fixed order (deterministic)
__global__ void __launch_bounds__(kThreads) trig_grad_kernel(const float* __restrict__ wgrad, int64_t B, int64_t tl,
                                                             const float* __restrict__ trig,
                                                             const double* __restrict__ coef,
                                                             float* __restrict__ dtrig, int accumulate) {
  __shared__ float red[4][64];
  const int kq = threadIdx.x & 63, ug = threadIdx.x >> 6;
  const int64_t k = blockIdx.x * (int64_t)64 + kq;
  float s0 = 0.0f, s1 = 0.0f;
  if (k < tl) {
    int64_t u = ug;
    for (; u + 4 < B; u += 8) {
      s0 += wgrad[u * tl + k];
      s1 += wgrad[(u + 4) * tl + k];
    }
    if (u < B) s0 += wgrad[u * tl + k];
  }
  red[ug][kq] = s0 + s1;
  __syncthreads();
  if (ug == 0 && k < tl) {
    const float s = (red[0][kq] + red[1][kq]) + (red[2][kq] + red[3][kq]);
    const float g = s + (float)(coef[0] * (double)trig[k]);
    dtrig[k] = accumulate ? dtrig[k] + g : g;
  }
}

struct FastPlan {
  int M, N, bluestein, pp, r0, r1;
};
// Bluestein 2304 = R0 * R1 * R2
#ifndef ABD_BLUE_R0
#define ABD_BLUE_R0 16
#endif
#ifndef ABD_BLUE_R1
#define ABD_BLUE_R1 12
#endif
constexpr int kBlueR0 = ABD_BLUE_R0, kBlueR1 = ABD_BLUE_R1, kBlueR2 = 2304 / (ABD_BLUE_R0 * ABD_BLUE_R1);
// Bluestein frame pairs per item (shared-column FFTs: one set of table loads for all of them) and
// the blocks per CU the build is register-budgeted for (PP 2: 39 KB of LDS per block, 4 blocks)
#ifndef ABD_BLUE_PP
#define ABD_BLUE_PP 1
#endif
#ifndef ABD_BLUE_NBLK
#define ABD_BLUE_NBLK (ABD_BLUE_PP == 1 ? 8 : 4)
#endif
// 2048-point (FlowMur / DABA) and 400-point (BadNets / JingleBack) plans: frame pairs per item and
// blocks per CU the build is register-budgeted for (measurement builds override them).  Round 5
// (scripts/stft_plan_ab.sh, feature stage at B = 256, two alternations on one box): 2048 points
// PP 4 / 1 block-budget 0.0495 ms -> PP 2 / 4 blocks 0.0437 (PP 1: 0.058, PP 3: 0.051); 400 points
// PP 13 / 1 0.0590 -> PP 8 / 4 0.0504 (PP 6: 0.055, 9: 0.052, 10: 0.054, 17: 0.066; a 20 x 20
// radix plan at PP 12: 0.058).  Both also take the segmented mel (before it: 400 points 0.0705,
// 2048 points 0.0576 ms).
#ifndef ABD_F2048_PP
#define ABD_F2048_PP 2
#endif
#ifndef ABD_F2048_NBLK
#define ABD_F2048_NBLK 4
#endif
#ifndef ABD_F400_PP
#define ABD_F400_PP 8
#endif
#ifndef ABD_F400_R0
#define ABD_F400_R0 16
#endif
#ifndef ABD_F400_NBLK
#define ABD_F400_NBLK 4
#endif
constexpr int kF400R0 = ABD_F400_R0, kF400R1 = 400 / ABD_F400_R0;
constexpr FastPlan kFastPlans[] = {{2304, 1103, 1, ABD_BLUE_PP, kBlueR0, kBlueR1},
                                   {2048, 2048, 0, ABD_F2048_PP, 16, 16},
                                   {400, 400, 0, ABD_F400_PP, kF400R0, kF400R1}};

const FastPlan* find_fast(int M, int N, int blue) {
  for (const auto& f : kFastPlans)
    if (f.M == M && f.N == N && f.bluestein == blue) return &f;
  return nullptr;
}

template <int M, int NN, int R0, int R1, int R2, int PP, bool BLUE, int NBLK = kBlueBlocks>
int launch_fast(const MfccDev& d, const float* wave, int64_t row_stride, const int32_t* rows, int64_t batch,
                const InjDev& ij, const float* rowscale, float* ws_db, float* ws_max, unsigned* queue,
                hipStream_t s) {
  auto* kern = &stft_mel_fast_kernel<M, NN, R0, R1, R2, PP, BLUE, NBLK>;
  static_assert(M % 16 == 0, "padded LDS layout needs M % 16 == 0");
  size_t lds = (size_t)(PP * (M + M / 16)) * sizeof(float2);
#ifdef ABD_MEL_W_LDS
  lds += (size_t)((d.mel2_total + 3) & ~3) * 4;
#endif
  // residency from the occupancy API (VGPRs + LDS), cached per LDS size (host threads may launch
  // concurrently on different streams: the cache is guarded, the launch itself holds no state)
  static std::mutex mu;
  static size_t cached_lds = 0;
  static int cached_blocks = 0, cached_cu = 0;
  int resident = 0;
  {
    std::lock_guard<std::mutex> lk(mu);
    if (cached_lds != lds) {
      ABD_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds));
      int dev = 0, nb = 0, ncu = 0;
      ABD_HIP(hipGetDevice(&dev));
      ABD_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
      ABD_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, reinterpret_cast<const void*>(kern), kThreads, lds));
      cached_blocks = std::max(1, nb);
      cached_cu = ncu;
      cached_lds = lds;
    }
    resident = cached_cu * cached_blocks;
  }
  // ABD_STFT_MAX_BLOCKS caps the persistent grid (tests: every block then walks many items, the
  // loop-carried path -- next-item hand-off, stealing, LDS reuse across items -- at any batch)
  if (const char* cap = getenv("ABD_STFT_MAX_BLOCKS")) resident = std::max(1, std::min(resident, atoi(cap)));
  const int64_t items = batch * d.chunks;
  const int grid = (int)std::min<int64_t>(items, (int64_t)resident);
  kern<<<grid, kThreads, lds, s>>>(d, wave, row_stride, rows, batch, ij, rowscale, ws_db, ws_max, queue);
  ABD_LAUNCH_CHECK();
  return 0;
}

int dispatch_fast(const MfccDev& d, const float* wave, int64_t row_stride, const int32_t* rows, int64_t batch,
                  const InjDev& ij, const float* rowscale, float* ws_db, float* ws_max, unsigned* queue,
                  hipStream_t s) {
  if (d.M == 2304 && d.N == 1103 && d.bluestein)
    return launch_fast<2304, 1103, kBlueR0, kBlueR1, kBlueR2, ABD_BLUE_PP, true, ABD_BLUE_NBLK>(
        d, wave, row_stride, rows, batch, ij, rowscale, ws_db, ws_max, queue, s);
  if (d.M == 2048 && d.N == 2048 && !d.bluestein)
    return launch_fast<2048, 2048, 16, 16, 8, ABD_F2048_PP, false, ABD_F2048_NBLK>(d, wave, row_stride, rows, batch, ij,
                                                                                  rowscale, ws_db, ws_max, queue, s);
  if (d.M == 400 && d.N == 400 && !d.bluestein)
    return launch_fast<400, 400, kF400R0, kF400R1, 1, ABD_F400_PP, false, ABD_F400_NBLK>(d, wave, row_stride, rows, batch,
                                                                                         ij, rowscale, ws_db, ws_max,
                                                                                         queue, s);
  return -1;
}

template <int M, int R0, int R1, int R2, int PP>
int launch_stft_bwd(const MfccDev& d, const float* wave, int64_t row_stride, const int32_t* rows, int64_t batch,
                    const InjDev& ij, const float* rowscale, const float* dmel, float* gframes, hipStream_t s) {
  auto* kern = &stft_bwd_kernel<M, R0, R1, R2, PP>;
  const size_t lds = (size_t)(2 * R0 * R1 + PP * (M + M / 16)) * sizeof(float2);
  static bool attr = false;
  if (!attr) {
    ABD_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds));
    attr = true;
  }
  kern<<<(unsigned)(batch * d.chunks), kThreads, lds, s>>>(d, wave, row_stride, rows, ij, rowscale, dmel, gframes);
  ABD_LAUNCH_CHECK();
  return 0;
}

int dispatch_stft_bwd(const MfccDev& d, const float* wave, int64_t row_stride, const int32_t* rows, int64_t batch,
                      const InjDev& ij, const float* rowscale, const float* dmel, float* gframes, hipStream_t s) {
  if (d.M == 2048 && d.N == 2048 && !d.bluestein && d.ppb == ABD_F2048_PP)
    return launch_stft_bwd<2048, 16, 16, 8, ABD_F2048_PP>(d, wave, row_stride, rows, batch, ij, rowscale, dmel, gframes,
                                                          s);
  if (d.M == 400 && d.N == 400 && !d.bluestein && d.ppb == ABD_F400_PP)
    return launch_stft_bwd<400, kF400R0, kF400R1, 1, ABD_F400_PP>(d, wave, row_stride, rows, batch, ij, rowscale, dmel,
                                                                  gframes, s);
  return -1;
}

// ------------------------------------------------------------------ host side
bool smooth235(int n) {
  for (int f : {2, 3, 5})
    while (n % f == 0) n /= f;
  return n == 1;
}

std::vector<int> factorize(int M) {
  std::vector<int> r;
  int n = M;
  while (n % 4 == 0) {
    r.push_back(4);
    n /= 4;
  }
  while (n % 2 == 0) {
    r.push_back(2);
    n /= 2;
  }
  while (n % 3 == 0) {
    r.push_back(3);
    n /= 3;
  }
  while (n % 5 == 0) {
    r.push_back(5);
    n /= 5;
  }
  return r;
}

double fft_cost(int M) {
  double c = 0;
  for (int r : factorize(M)) c += M * (1.0 + (r == 2 ? 5.0 : r == 3 ? 8.0 : r == 4 ? 8.5 : 11.2) / 8.0);
  return c;
}

int choose_bluestein_M(int N) {
  const int lo = 2 * N - 1;
  int best = 0;
  double bc = 1e300;
  for (int m = lo; m <= 4 * lo; ++m) {
    if (!smooth235(m)) continue;
    const double c = fft_cost(m);
    if (c < bc) {
      bc = c;
      best = m;
    }
  }
  return best;
}

void host_fft(std::vector<std::complex<double>>& x) {  // forward, O(M^2) fine at plan time
  const int M = (int)x.size();
  std::vector<std::complex<double>> y(M), tw(M);
  for (int k = 0; k < M; ++k) tw[k] = std::polar(1.0, -2.0 * M_PI * k / M);
  for (int k = 0; k < M; ++k) {
    std::complex<double> acc = 0;
    for (int n = 0; n < M; ++n) acc += x[n] * tw[(int64_t)k * n % M];
    y[k] = acc;
  }
  x.swap(y);
}

}  // namespace

struct abd_mfcc_plan {
  MfccDev dev;
  int sr, mel_kind;
  int64_t length;
  void* block = nullptr;
};

extern "C" {

int abd_mfcc_plan_create(int sample_rate, int n_fft, int hop_length, int n_mels, int n_mfcc, int mel_kind,
                         int pad_mode, float top_db, int64_t length, abd_mfcc_plan** plan) {
  ABD_CHECK(plan != nullptr, ABD_E_INVALID, "plan out-pointer is NULL");
  ABD_CHECK(n_fft >= 2 && hop_length >= 1 && n_mels >= 1 && n_mfcc >= 1 && n_mfcc <= n_mels, ABD_E_INVALID,
            "bad MFCC geometry n_fft=%d hop=%d n_mels=%d n_mfcc=%d", n_fft, hop_length, n_mels, n_mfcc);
  ABD_CHECK(n_mels <= 256, ABD_E_UNSUPPORTED, "n_mels > 256 unsupported");
  ABD_CHECK(length > n_fft / 2, ABD_E_INVALID, "length %lld too short for reflect padding of %d",
            (long long)length, n_fft / 2);
  ABD_CHECK(mel_kind == ABD_MEL_HTK || mel_kind == ABD_MEL_SLANEY, ABD_E_INVALID, "bad mel kind");
  const int N = n_fft;
  const bool blue = !smooth235(N);
  const int M = blue ? choose_bluestein_M(N) : N;
  ABD_CHECK(M > 0 && M <= kMaxComplexPerBlock, ABD_E_UNSUPPORTED, "FFT length %d too large", M);
  auto* pl = new abd_mfcc_plan();
  MfccDev& d = pl->dev;
  d.N = N;
  d.hop = hop_length;
  d.pad = N / 2;
  d.pad_mode = pad_mode;
  d.M = M;
  d.bluestein = blue ? 1 : 0;
  d.n_freqs = N / 2 + 1;
  d.n_mels = n_mels;
  d.n_mfcc = n_mfcc;
  d.L = length;
  d.T = (int)(1 + (length + 2 * (N / 2) - N) / hop_length);
  d.top_db = top_db;
  const int P = (d.T + 1) / 2;
  const FastPlan* fp = find_fast(M, N, blue ? 1 : 0);
  // ABD_GENERIC_FFT: every MFCC stage on its generic kernel (runtime-radix STFT, LDS mel, VALU DCT),
  // the fallbacks of geometries without a specialised plan (tests/test_gpu_mfcc.py runs both)
  const bool generic = getenv("ABD_GENERIC_FFT") != nullptr;
  if (fp != nullptr && !generic) {
    d.ppb = fp->pp;  // fixed pairs per work item (compile-time in the fast kernel)
    d.chunks = (P + d.ppb - 1) / d.ppb;
    d.fast = 1;
    d.ablate = 0;
  } else {
    int ppb_max = std::max(1, kMaxComplexPerBlock / M);
    int chunks = (P + ppb_max - 1) / ppb_max;
    d.ppb = (P + chunks - 1) / chunks;
    d.chunks = (P + d.ppb - 1) / d.ppb;
    d.fast = 0;
  }
  auto rad = factorize(M);
  d.n_pass = (int)rad.size();
  int Ns = 1;
  for (int i = 0; i < d.n_pass; ++i) {
    d.radix[i] = rad[i];
    d.ns[i] = Ns;
    Ns *= rad[i];
  }
  pl->sr = sample_rate;
  pl->mel_kind = mel_kind;
  pl->length = length;

  // ---- host tables (double precision, rounded once to fp32)
  std::vector<float2> tw(M), chirp_in(N), vhat(M), chirp_out(N);
  std::vector<float> win(N);
  for (int k = 0; k < M; ++k) {
    const double a = -2.0 * M_PI * k / M;
    tw[k] = make_float2((float)cos(a), (float)sin(a));
  }
  std::vector<double> hann(N);
  for (int n = 0; n < N; ++n) {
    hann[n] = 0.5 - 0.5 * cos(2.0 * M_PI * n / N);
    win[n] = (float)hann[n];
  }
  if (blue) {
    std::vector<std::complex<double>> w(N), v(M, 0.0);
    for (int n = 0; n < N; ++n) {
      const int64_t q = ((int64_t)n * n) % (2 * (int64_t)N);
      w[n] = std::polar(1.0, M_PI * (double)q / N);
      const std::complex<double> ci = hann[n] * std::conj(w[n]);
      chirp_in[n] = make_float2((float)ci.real(), (float)ci.imag());
      const std::complex<double> co = w[n] / (double)M;
      chirp_out[n] = make_float2((float)co.real(), (float)co.imag());
    }
    v[0] = w[0];
    for (int m = 1; m < N; ++m) {
      v[m] = w[m];
      v[M - m] = w[m];
    }
    host_fft(v);
    for (int m = 0; m < M; ++m) vhat[m] = make_float2((float)v[m].real(), (float)(-v[m].imag()));
  }
  // mel filterbank (n_freqs x n_mels), sparse per mel
  const int nf = d.n_freqs;
  std::vector<double> fb((size_t)nf * n_mels, 0.0);
  if (mel_kind == ABD_MEL_HTK) {
    // torchaudio.functional.melscale_fbanks(norm=None, mel_scale="htk"), f_max = sr // 2
    auto h2m = [](double f) { return 2595.0 * log10(1.0 + f / 700.0); };
    auto m2h = [](double m) { return 700.0 * (pow(10.0, m / 2595.0) - 1.0); };
    const double fmax = (double)(sample_rate / 2);
    std::vector<double> fpts(n_mels + 2);
    const double m0 = h2m(0.0), m1 = h2m(fmax);
    for (int i = 0; i < n_mels + 2; ++i) fpts[i] = m2h(m0 + (m1 - m0) * i / (n_mels + 1));
    for (int k = 0; k < nf; ++k) {
      const double f = fmax * k / (nf - 1);
      for (int m = 0; m < n_mels; ++m) {
        const double down = (f - fpts[m]) / (fpts[m + 1] - fpts[m]);
        const double up = (fpts[m + 2] - f) / (fpts[m + 2] - fpts[m + 1]);
        fb[(size_t)k * n_mels + m] = std::max(0.0, std::min(down, up));
      }
    }
  } else {
    // librosa.filters.mel(htk=False, norm="slaney"), stored as float32 like librosa
    auto h2m = [](double f) {
      const double fsp = 200.0 / 3.0, minlog = 1000.0, minmel = minlog / fsp, step = log(6.4) / 27.0;
      return f >= minlog ? minmel + log(f / minlog) / step : f / fsp;
    };
    auto m2h = [](double m) {
      const double fsp = 200.0 / 3.0, minlog = 1000.0, minmel = minlog / fsp, step = log(6.4) / 27.0;
      return m >= minmel ? minlog * exp(step * (m - minmel)) : fsp * m;
    };
    const double fmax = sample_rate / 2.0;
    std::vector<double> melf(n_mels + 2);
    const double m0 = h2m(0.0), m1 = h2m(fmax);
    for (int i = 0; i < n_mels + 2; ++i) melf[i] = m2h(m0 + (m1 - m0) * i / (n_mels + 1));
    for (int m = 0; m < n_mels; ++m) {
      const double enorm = 2.0 / (melf[m + 2] - melf[m]);
      for (int k = 0; k < nf; ++k) {
        const double f = (double)k * sample_rate / N;
        const double lower = -(melf[m] - f) / (melf[m + 1] - melf[m]);
        const double upper = (melf[m + 2] - f) / (melf[m + 2] - melf[m + 1]);
        fb[(size_t)k * n_mels + m] = (double)(float)(std::max(0.0, std::min(lower, upper)) * enorm);
      }
    }
  }
  std::vector<int> mstart(n_mels), mcount(n_mels), moff(n_mels);
  std::vector<float> mw;
  for (int m = 0; m < n_mels; ++m) {
    int lo = -1, hi = -1;
    for (int k = 0; k < nf; ++k)
      if (fb[(size_t)k * n_mels + m] != 0.0) {
        if (lo < 0) lo = k;
        hi = k;
      }
    moff[m] = (int)mw.size();
    if (lo < 0) {
      mstart[m] = 0;
      mcount[m] = 0;
      continue;
    }
    mstart[m] = lo;
    mcount[m] = hi - lo + 1;
    for (int k = lo; k <= hi; ++k) mw.push_back((float)fb[(size_t)k * n_mels + m]);
  }
  if (mw.empty()) mw.push_back(0.0f);
  // half-filter slots for the fast kernel: filter m's support split into two contiguous halves
  std::vector<int4> meta2(2 * (size_t)n_mels);
  std::vector<float> mw2;
  int hmax = 0;
  for (int m = 0; m < n_mels; ++m) {
    const int lo = mstart[m], cnt = mcount[m], c0 = (cnt + 1) / 2;
    for (int h = 0; h < 2; ++h) {
      const int st = lo + (h ? c0 : 0), c = h ? cnt - c0 : c0;
      meta2[2 * m + h] = make_int4(st, c, (int)mw2.size(), 0);
      for (int k = st; k < st + c; ++k) mw2.push_back((float)fb[(size_t)k * n_mels + m]);
      hmax = std::max(hmax, c);
    }
  }
  if (mw2.empty()) mw2.push_back(0.0f);
  // backward (mel^T): the filters touching each bin, at most two for triangular banks
  std::vector<int2> bmel(nf, make_int2(-1, -1));
  std::vector<float2> bw(nf, make_float2(0.0f, 0.0f));
  d.bwd_ok = 1;
  for (int k = 0; k < nf; ++k) {
    int cnt = 0;
    for (int m = 0; m < n_mels; ++m) {
      const double v = fb[(size_t)k * n_mels + m];
      if (v == 0.0) continue;
      if (cnt == 0) {
        bmel[k].x = m;
        bw[k].x = (float)v;
      } else if (cnt == 1) {
        bmel[k].y = m;
        bw[k].y = (float)v;
      } else {
        d.bwd_ok = 0;
      }
      ++cnt;
    }
  }
  d.mel2_total = (int)mw2.size();
  d.mel2_hp = std::max(8, (hmax + 7) / 8 * 8);
  // padded slot weights for the Bluestein fast path (power_mel_blue): one slot per thread
  const bool mel3 = blue && d.fast && 2 * n_mels == kThreads && hmax <= kMelHP;
  std::vector<float> mw3(mel3 ? (size_t)2 * n_mels * kMelHP : 0, 0.0f);
  // [q][slot] float4 groups: the q-th float4 load of the mel stage is one contiguous 4 KB sweep
  // across the 256 slots (lanes) instead of 64-B pieces 64 B apart
  if (mel3)
    for (int sl = 0; sl < 2 * n_mels; ++sl)
      for (int i = 0; i < meta2[sl].y; ++i)
        mw3[(((size_t)(i / 4) * (2 * n_mels) + sl) * 4) + (i % 4)] = mw2[meta2[sl].z + i];
  // segmented mel for the non-Bluestein fast kernel: filter m's support [lo, lo + cnt) as
  // ceil(cnt / kMelSeg) segments (one for an empty filter), summed per filter in segment order
  bool mseg = !blue && d.fast && nf >= kMelSeg && ABD_MEL_SEG;
  std::vector<int> seg_start;
  std::vector<float> seg_w;
  std::vector<int2> filt_seg(mseg ? n_mels : 0);
  if (mseg)
    for (int m = 0; m < n_mels; ++m) {
      const int lo = mstart[m], cnt = mcount[m];
      const int ns = std::max(1, (cnt + kMelSeg - 1) / kMelSeg);
      filt_seg[m] = make_int2((int)seg_start.size(), ns);
      for (int g = 0; g < ns; ++g) {
        const int b0 = lo + g * kMelSeg, c = std::max(0, std::min(kMelSeg, cnt - g * kMelSeg));
        const int st = std::min(b0, nf - kMelSeg);  // reads st .. st + kMelSeg - 1 < nf
        seg_start.push_back(st);
        for (int i = 0; i < kMelSeg; ++i) {
          const int k = st + i;
          seg_w.push_back((k >= b0 && k < b0 + c) ? (float)fb[(size_t)k * n_mels + m] : 0.0f);
        }
      }
    }
  if (mseg && mel_seg_offset(nf) + (int)seg_start.size() > M + M / 16) {  // partials must fit the buffer
    mseg = false;
    seg_start.clear();
    seg_w.clear();
    filt_seg.clear();
  }
  // fast-kernel twiddles: W_{R0 R1}^e and W_M^k, e, k < R0 R1
  const int r01 = fp ? fp->r0 * fp->r1 : 1;
  std::vector<float2> ftw(2 * (size_t)r01);
  for (int e = 0; e < r01; ++e) {
    const double a = -2.0 * M_PI * e / r01, b = -2.0 * M_PI * e / M;
    ftw[e] = make_float2((float)cos(a), (float)sin(a));
    ftw[r01 + e] = make_float2((float)cos(b), (float)sin(b));
  }
  std::vector<float2> ftw2;
  if (fp) {
    const int r0 = fp->r0, r1 = fp->r1, r2 = M / (r0 * r1);
    // [r][k]: for a fixed row r the lanes of a wave (consecutive butterflies j, k = j mod NS) read
    // consecutive entries -- one or two cache lines per wave load instead of one line per lane
    // group at a 96-B stride ([k][r] kept the vector-memory data path 89 % busy)
    for (int r = 0; r < r1; ++r)
      for (int k = 0; k < r0; ++k) {
        const double a = -2.0 * M_PI * (double)((k * r) % r01) / r01;
        ftw2.push_back(make_float2((float)cos(a), (float)sin(a)));
      }
    for (int r = 0; r < r2; ++r)
      for (int k = 0; k < r01; ++k) {
        const double a = -2.0 * M_PI * (double)(((int64_t)k * r) % M) / M;
        ftw2.push_back(make_float2((float)cos(a), (float)sin(a)));
      }
  }
  if (ftw2.empty()) ftw2.push_back(make_float2(1.0f, 0.0f));
  // pair tables of the fast kernel (spass_pf TWK 4 / V4): two rows per 16-B load
  std::vector<float4> ftw4, vhat4;
  if (fp) {
    const int r0 = fp->r0, r1 = fp->r1;
    auto w = [&](int k, int r) {
      const double a = -2.0 * M_PI * (double)((k * r) % r01) / r01;
      return std::make_pair((float)cos(a), (float)sin(a));
    };
    for (int p2 = 0; p2 < r1 / 2; ++p2)
      for (int k = 0; k < r0; ++k) {
        const auto a = w(k, 1 + 2 * p2);
        const auto b = 2 + 2 * p2 < r1 ? w(k, 2 + 2 * p2) : std::make_pair(1.0f, 0.0f);
        ftw4.push_back(make_float4(a.first, a.second, b.first, b.second));
      }
    if (blue) {
      const int mr0 = M / r0;
      for (int p2 = 0; p2 < r0 / 2; ++p2)
        for (int j = 0; j < mr0; ++j) {
          const float2 a = vhat[j + 2 * p2 * mr0], b = vhat[j + (2 * p2 + 1) * mr0];
          vhat4.push_back(make_float4(a.x, a.y, b.x, b.y));
        }
    }
  }
  if (ftw4.empty()) ftw4.push_back(make_float4(1.0f, 0.0f, 1.0f, 0.0f));
  std::vector<float4> co2((size_t)N / 2 + 1);
  for (int k = 0; k <= N / 2; ++k) {
    const float2 a = chirp_out[k], b = chirp_out[k == 0 ? 0 : N - k];
    co2[k] = make_float4(a.x, a.y, b.x, b.y);
  }
  if (vhat4.empty()) vhat4.push_back(make_float4(1.0f, 0.0f, 1.0f, 0.0f));
  std::vector<float> dct((size_t)n_mels * n_mfcc);
  for (int m = 0; m < n_mels; ++m)
    for (int c = 0; c < n_mfcc; ++c) {
      double v = cos(M_PI / n_mels * (m + 0.5) * c) * sqrt(2.0 / n_mels);
      if (c == 0) v *= 1.0 / sqrt(2.0);
      dct[(size_t)m * n_mfcc + c] = (float)v;
    }
  // B fragments of db_dct_mfma_kernel: [s][q][tile][col] -> float4 over j of dct[16 s + 4 q + j][16 tile + col]
  d.dct_tiles = (n_mels % 16 == 0 && n_mfcc <= 48 && !generic) ? (n_mfcc + 15) / 16 : 0;
  d.dct_lds = generic ? 0 : 1;
  std::vector<float4> dfrag;
  if (d.dct_tiles > 0)
    for (int sg = 0; sg < n_mels / 16; ++sg)
      for (int q = 0; q < 4; ++q)
        for (int tile = 0; tile < d.dct_tiles; ++tile)
          for (int col = 0; col < 16; ++col) {
            const int c = 16 * tile + col;
            float e[4];
            for (int j = 0; j < 4; ++j) e[j] = c < n_mfcc ? dct[(size_t)(16 * sg + 4 * q + j) * n_mfcc + c] : 0.0f;
            dfrag.push_back(make_float4(e[0], e[1], e[2], e[3]));
          }
  if (dfrag.empty()) dfrag.push_back(make_float4(0.f, 0.f, 0.f, 0.f));

  // ---- one device block for every table
  auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
  size_t off_tw = 0, sz = al(M * sizeof(float2));
  size_t off_ci = sz;
  sz += al(N * sizeof(float2));
  size_t off_vh = sz;
  sz += al(M * sizeof(float2));
  size_t off_co = sz;
  sz += al(N * sizeof(float2));
  size_t off_win = sz;
  sz += al(N * sizeof(float));
  size_t off_ms = sz;
  sz += al(n_mels * sizeof(int));
  size_t off_mc = sz;
  sz += al(n_mels * sizeof(int));
  size_t off_mo = sz;
  sz += al(n_mels * sizeof(int));
  size_t off_mw = sz;
  sz += al(mw.size() * sizeof(float));
  size_t off_dct = sz;
  sz += al(dct.size() * sizeof(float));
  size_t off_ftw = sz;
  sz += al(ftw.size() * sizeof(float2));
  size_t off_dfrag = sz;
  sz += al(dfrag.size() * sizeof(float4));
  size_t off_ftw2 = sz;
  sz += al(ftw2.size() * sizeof(float2));
  size_t off_co2 = sz;
  sz += al(co2.size() * sizeof(float4));
  size_t off_ftw4 = sz;
  sz += al(ftw4.size() * sizeof(float4));
  size_t off_vh4 = sz;
  sz += al(vhat4.size() * sizeof(float4));
  size_t off_m2 = sz;
  sz += al(meta2.size() * sizeof(int4));
  size_t off_w2 = sz;
  sz += al(mw2.size() * sizeof(float));
  size_t off_w3 = sz;
  sz += al(mw3.size() * sizeof(float));
  size_t off_sst = sz;
  sz += al(seg_start.size() * sizeof(int));
  size_t off_sw = sz;
  sz += al(seg_w.size() * sizeof(float));
  size_t off_fs = sz;
  sz += al(filt_seg.size() * sizeof(int2));
  size_t off_bm = sz;
  sz += al(nf * sizeof(int2));
  size_t off_bw = sz;
  sz += al(nf * sizeof(float2));
  std::vector<char> host(sz, 0);
  memcpy(&host[off_bm], bmel.data(), nf * sizeof(int2));
  memcpy(&host[off_bw], bw.data(), nf * sizeof(float2));
  memcpy(&host[off_tw], tw.data(), M * sizeof(float2));
  memcpy(&host[off_ci], chirp_in.data(), N * sizeof(float2));
  memcpy(&host[off_vh], vhat.data(), M * sizeof(float2));
  memcpy(&host[off_co], chirp_out.data(), N * sizeof(float2));
  memcpy(&host[off_win], win.data(), N * sizeof(float));
  memcpy(&host[off_ms], mstart.data(), n_mels * sizeof(int));
  memcpy(&host[off_mc], mcount.data(), n_mels * sizeof(int));
  memcpy(&host[off_mo], moff.data(), n_mels * sizeof(int));
  memcpy(&host[off_mw], mw.data(), mw.size() * sizeof(float));
  memcpy(&host[off_dct], dct.data(), dct.size() * sizeof(float));
  memcpy(&host[off_ftw], ftw.data(), ftw.size() * sizeof(float2));
  memcpy(&host[off_dfrag], dfrag.data(), dfrag.size() * sizeof(float4));
  memcpy(&host[off_ftw2], ftw2.data(), ftw2.size() * sizeof(float2));
  memcpy(&host[off_co2], co2.data(), co2.size() * sizeof(float4));
  memcpy(&host[off_ftw4], ftw4.data(), ftw4.size() * sizeof(float4));
  memcpy(&host[off_vh4], vhat4.data(), vhat4.size() * sizeof(float4));
  memcpy(&host[off_m2], meta2.data(), meta2.size() * sizeof(int4));
  memcpy(&host[off_w2], mw2.data(), mw2.size() * sizeof(float));
  if (!mw3.empty()) memcpy(&host[off_w3], mw3.data(), mw3.size() * sizeof(float));
  if (mseg) {
    memcpy(&host[off_sst], seg_start.data(), seg_start.size() * sizeof(int));
    memcpy(&host[off_sw], seg_w.data(), seg_w.size() * sizeof(float));
    memcpy(&host[off_fs], filt_seg.data(), filt_seg.size() * sizeof(int2));
  }
  hipError_t e = hipMalloc(&pl->block, sz);
  if (e != hipSuccess) {
    delete pl;
    abd::set_last_error("hipMalloc(%zu) for MFCC tables: %s", sz, hipGetErrorString(e));
    return (int)e;
  }
  e = hipMemcpy(pl->block, host.data(), sz, hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    (void)hipFree(pl->block);
    delete pl;
    abd::set_last_error("hipMemcpy MFCC tables: %s", hipGetErrorString(e));
    return (int)e;
  }
  char* b = static_cast<char*>(pl->block);
  d.tw = reinterpret_cast<const float2*>(b + off_tw);
  d.chirp_in = reinterpret_cast<const float2*>(b + off_ci);
  d.vhat = reinterpret_cast<const float2*>(b + off_vh);
  d.chirp_out = reinterpret_cast<const float2*>(b + off_co);
  d.window = reinterpret_cast<const float*>(b + off_win);
  d.mel_start = reinterpret_cast<const int*>(b + off_ms);
  d.mel_count = reinterpret_cast<const int*>(b + off_mc);
  d.mel_off = reinterpret_cast<const int*>(b + off_mo);
  d.mel_w = reinterpret_cast<const float*>(b + off_mw);
  d.dct = reinterpret_cast<const float*>(b + off_dct);
  d.ftw = reinterpret_cast<const float2*>(b + off_ftw);
  d.dct_frag = reinterpret_cast<const float4*>(b + off_dfrag);
  d.ftw2 = reinterpret_cast<const float2*>(b + off_ftw2);
  d.ftw4 = reinterpret_cast<const float4*>(b + off_ftw4);
  d.chirp_out2 = reinterpret_cast<const float4*>(b + off_co2);
  d.vhat4 = reinterpret_cast<const float4*>(b + off_vh4);
  d.mel2_meta = reinterpret_cast<const int4*>(b + off_m2);
  d.mel2_w = reinterpret_cast<const float*>(b + off_w2);
  d.mel3_w = mw3.empty() || generic ? nullptr : reinterpret_cast<const float*>(b + off_w3);
  d.mseg_start = mseg ? reinterpret_cast<const int*>(b + off_sst) : nullptr;
  d.mseg_w = mseg ? reinterpret_cast<const float4*>(b + off_sw) : nullptr;
  d.mfilt_seg = mseg ? reinterpret_cast<const int2*>(b + off_fs) : nullptr;
  d.nseg = mseg ? (int)seg_start.size() : 0;
  d.bin_mel = reinterpret_cast<const int2*>(b + off_bm);
  d.bin_w = reinterpret_cast<const float2*>(b + off_bw);
  *plan = pl;
  return ABD_OK;
}

void abd_mfcc_plan_destroy(abd_mfcc_plan* plan) {
  if (!plan) return;
  if (plan->block) (void)hipFree(plan->block);
  delete plan;
}

int abd_mfcc_plan_frames(const abd_mfcc_plan* plan) { return plan ? plan->dev.T : -1; }

int abd_mfcc_plan_describe(const abd_mfcc_plan* plan, int* fft_size, int* bluestein, int* n_passes, int* radices) {
  ABD_CHECK(plan != nullptr, ABD_E_INVALID, "NULL plan");
  if (fft_size) *fft_size = plan->dev.M;
  if (bluestein) *bluestein = plan->dev.bluestein;
  if (n_passes) *n_passes = plan->dev.n_pass;
  if (radices)
    for (int i = 0; i < plan->dev.n_pass; ++i) radices[i] = plan->dev.radix[i];
  return ABD_OK;
}

size_t abd_mfcc_workspace_bytes(const abd_mfcc_plan* plan, int64_t batch) {
  if (!plan) return 0;
  const MfccDev& d = plan->dev;
  auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
  return al((size_t)batch * d.T * d.n_mels * sizeof(float)) + al((size_t)batch * d.chunks * sizeof(float)) +
         al((size_t)batch * sizeof(float)) + kQueues * kQueueStride * sizeof(unsigned);  // + item queues
}

static InjDev make_inj(const abd_inject* inj) {
  InjDev r{};
  if (!inj) {
    r.mode = ABD_INJECT_NONE;
    return r;
  }
  r.mode = inj->mode;
  r.trig = inj->trigger;
  r.trig_len = inj->trigger_len;
  r.poison = inj->poison;
  r.position = inj->position;
  r.snr_db = inj->snr_db;
  r.patch = inj->patch;
  r.pt0 = inj->patch_t0;
  r.pt1 = inj->patch_t1;
  r.pc0 = inj->patch_c0;
  r.pc1 = inj->patch_c1;
  r.pval = inj->patch_value;
  r.frames = inj->frames;
  r.fpad = inj->frame_pad;
  r.scale_by_row = false;
  if (r.mode == ABD_INJECT_NONE && r.patch) r.mode = -1;  // patch-only: rows still selected by poison
  return r;
}

static int check_inj(const InjDev& r) {
  if (r.mode > 0) {
    ABD_CHECK(r.trig != nullptr && r.trig_len > 0, ABD_E_INVALID, "injection mode %d needs a trigger", r.mode);
    if (r.mode >= ABD_INJECT_SNR_WINDOW)
      ABD_CHECK(r.position != nullptr, ABD_E_INVALID, "windowed injection needs per-row positions");
  }
  return ABD_OK;
}

#ifndef ABD_ROW_SCALE_TAB  // measurement builds: 0 ignores abd_inject.row_scale (per-call scales)
#define ABD_ROW_SCALE_TAB 1
#endif
int abd_mfcc_f32(const abd_mfcc_plan* plan, const float* wave, int64_t row_stride, const int32_t* rows,
                 int64_t batch, const abd_inject* inj, float* out, void* workspace, size_t workspace_bytes,
                 abd_stream_t stream) {
  ABD_CHECK(batch >= 0, ABD_E_INVALID, "negative batch");
  if (batch == 0) return ABD_OK;
  ABD_CHECK(plan && wave && out, ABD_E_INVALID, "NULL argument");
  ABD_CHECK(row_stride >= plan->length, ABD_E_INVALID, "row_stride < length");
  ABD_CHECK(workspace && workspace_bytes >= abd_mfcc_workspace_bytes(plan, batch), ABD_E_WORKSPACE,
            "workspace too small (%zu < %zu)", workspace_bytes, abd_mfcc_workspace_bytes(plan, batch));
  const MfccDev& d = plan->dev;
  InjDev ij = make_inj(inj);
  int rc = check_inj(ij);
  if (rc) return rc;
  auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
  char* ws = static_cast<char*>(workspace);
  float* ws_db = reinterpret_cast<float*>(ws);
  float* ws_max = reinterpret_cast<float*>(ws + al((size_t)batch * d.T * d.n_mels * sizeof(float)));
  float* ws_scale = reinterpret_cast<float*>(ws + al((size_t)batch * d.T * d.n_mels * sizeof(float)) +
                                             al((size_t)batch * d.chunks * sizeof(float)));
  unsigned* queue = reinterpret_cast<unsigned*>(ws + al((size_t)batch * d.T * d.n_mels * sizeof(float)) +
                                                al((size_t)batch * d.chunks * sizeof(float)) +
                                                al((size_t)batch * sizeof(float)));
  hipStream_t s = static_cast<hipStream_t>(stream);
  const float* rowscale = nullptr;
  if (ij.mode == ABD_INJECT_SNR_WINDOW || ij.mode == ABD_INJECT_DEPLOY || ij.mode == ABD_INJECT_DEPLOY_CLAMP) {
    if (ABD_ROW_SCALE_TAB && inj->row_scale != nullptr) {  // the table's scales, computed once (abd_inject_row_scales)
      rowscale = inj->row_scale;
      ij.scale_by_row = true;
    } else {
      row_scale_kernel<<<dim3((unsigned)batch), dim3(kThreads), 0, s>>>(wave, row_stride, d.L, rows, ij, ws_scale);
      ABD_LAUNCH_CHECK();
      rowscale = ws_scale;
    }
  }
  const int64_t nblk = batch * d.chunks;
  ABD_CHECK(nblk < (1LL << 31), ABD_E_INVALID, "batch too large");
  const size_t lds = 2 * (size_t)d.ppb * d.M * sizeof(float2);
  abd::prof_begin(abd::PH_STFT_MEL, s);
  if (d.fast) {
    if constexpr (kAblate) {  // measurement builds only: ABD_STFT_ABLATE bits (MfccDev::ablate) per launch
      MfccDev da = d;
      const char* e = getenv("ABD_STFT_ABLATE");
      da.ablate = e ? atoi(e) : 0;
      if (dispatch_fast(da, wave, row_stride, rows, batch, ij, rowscale, ws_db, ws_max, queue, s) != 0) return -1;
    } else if (dispatch_fast(d, wave, row_stride, rows, batch, ij, rowscale, ws_db, ws_max, queue, s) != 0) {
      return -1;
    }
  } else {
    stft_mel_kernel<<<dim3((unsigned)nblk), dim3(kThreads), lds, s>>>(d, wave, row_stride, rows, batch, ij, rowscale,
                                                                    ws_db, ws_max);
  }
  abd::prof_end(abd::PH_STFT_MEL, s);
  ABD_LAUNCH_CHECK();
  abd::prof_begin(abd::PH_DB_DCT, s);
  const size_t dct_lds = ((size_t)d.n_mels * d.n_mfcc + (size_t)kTT2 * d.n_mels) * sizeof(float);
  if (d.dct_tiles > 0) {
    const dim3 g((unsigned)batch, (unsigned)((d.T + 63) / 64));
    if (d.dct_tiles == 1) db_dct_mfma_kernel<1><<<g, dim3(kThreads), 0, s>>>(d, ws_db, ws_max, ij, out);
    else if (d.dct_tiles == 2) db_dct_mfma_kernel<2><<<g, dim3(kThreads), 0, s>>>(d, ws_db, ws_max, ij, out);
    else db_dct_mfma_kernel<3><<<g, dim3(kThreads), 0, s>>>(d, ws_db, ws_max, ij, out);
  } else if (d.n_mfcc % 4 == 0 && dct_lds <= 64 * 1024 &&
      (reinterpret_cast<uintptr_t>(out) & 15) == 0 && d.dct_lds) {
    db_dct_lds_kernel<<<dim3((unsigned)batch, (unsigned)((d.T + kTT2 - 1) / kTT2)), dim3(kThreads), dct_lds, s>>>(
        d, ws_db, ws_max, ij, out);
  } else {
    db_dct_kernel<<<dim3((unsigned)batch, (unsigned)((d.T + kTT - 1) / kTT)), dim3(kThreads), 0, s>>>(d, ws_db, ws_max,
                                                                                                     ij, out);
  }
  abd::prof_end(abd::PH_DB_DCT, s);
  ABD_LAUNCH_CHECK();
  return ABD_OK;
}

size_t abd_inject_workspace_bytes(int64_t batch) { return ((size_t)batch * sizeof(float) + 255) & ~(size_t)255; }

int abd_inject_waveform_f32(const float* wave, int64_t row_stride, int64_t length, const int32_t* rows, int64_t batch,
                            const abd_inject* inj, float* out, void* workspace, size_t workspace_bytes,
                            abd_stream_t stream) {
  if (batch == 0) return ABD_OK;
  ABD_CHECK(wave && out, ABD_E_INVALID, "NULL argument");
  InjDev ij = make_inj(inj);
  int rc = check_inj(ij);
  if (rc) return rc;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const float* rowscale = nullptr;
  if (ij.mode == ABD_INJECT_SNR_WINDOW || ij.mode == ABD_INJECT_DEPLOY || ij.mode == ABD_INJECT_DEPLOY_CLAMP) {
    if (inj->row_scale != nullptr) {
      rowscale = inj->row_scale;
      ij.scale_by_row = true;
    } else {
      ABD_CHECK(workspace && workspace_bytes >= abd_inject_workspace_bytes(batch), ABD_E_WORKSPACE,
                "workspace too small");
      row_scale_kernel<<<dim3((unsigned)batch), dim3(kThreads), 0, s>>>(wave, row_stride, length, rows, ij,
                                                                        static_cast<float*>(workspace));
      ABD_LAUNCH_CHECK();
      rowscale = static_cast<const float*>(workspace);
    }
  }
  const unsigned gx = (unsigned)std::min<int64_t>((length + kThreads - 1) / kThreads, 64);
  inject_wave_kernel<<<dim3(gx, (unsigned)batch), dim3(kThreads), 0, s>>>(wave, row_stride, length, rows, ij,
                                                                         rowscale, out);
  ABD_LAUNCH_CHECK();
  return ABD_OK;
}

int abd_inject_row_scales(const float* wave, int64_t row_stride, int64_t length, int64_t n_rows,
                          const abd_inject* inj, float* scales, abd_stream_t stream) {
  ABD_CHECK(n_rows >= 0 && n_rows < (1LL << 31), ABD_E_INVALID, "n_rows out of range");
  if (n_rows == 0) return ABD_OK;
  ABD_CHECK(wave && inj && scales, ABD_E_INVALID, "NULL argument");
  ABD_CHECK(row_stride >= length && length > 0, ABD_E_INVALID, "row_stride < length");
  InjDev ij = make_inj(inj);
  ABD_CHECK(ij.mode == ABD_INJECT_SNR_WINDOW || ij.mode == ABD_INJECT_DEPLOY || ij.mode == ABD_INJECT_DEPLOY_CLAMP,
            ABD_E_INVALID, "row scales exist for the SNR_WINDOW / DEPLOY modes only (got mode %d)", ij.mode);
  ij.poison = nullptr;  // every table row (positions are not needed: the scale is the whole clip's)
  ABD_CHECK(ij.trig != nullptr && ij.trig_len > 0, ABD_E_INVALID, "row scales need a trigger");
  row_scale_kernel<<<dim3((unsigned)n_rows), dim3(kThreads), 0, static_cast<hipStream_t>(stream)>>>(
      wave, row_stride, length, nullptr, ij, scales);
  ABD_LAUNCH_CHECK();
  return ABD_OK;
}

static int wave_blocks(const abd_mfcc_plan* plan) { return (int)((plan->dev.L + kWaveSpan - 1) / kWaveSpan); }

size_t abd_mfcc_deploy_backward_workspace_bytes(const abd_mfcc_plan* plan, int64_t batch, int64_t trigger_len) {
  if (!plan) return 0;
  const MfccDev& d = plan->dev;
  auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
  return abd_mfcc_workspace_bytes(plan, batch) + al((size_t)batch * d.T * d.N * sizeof(float)) +
         al((size_t)batch * trigger_len * sizeof(float)) + al((size_t)batch * wave_blocks(plan) * sizeof(double)) +
         al(sizeof(double));
}

int abd_mfcc_deploy_backward(const abd_mfcc_plan* plan, const float* wave, int64_t row_stride, const int32_t* rows,
                             int64_t batch, const abd_inject* inj, const float* dmfcc, float* dtrigger, int flags,
                             void* workspace, size_t workspace_bytes, abd_stream_t stream) {
  ABD_CHECK(batch >= 1, ABD_E_INVALID, "batch must be >= 1");
  ABD_CHECK(plan && wave && inj && dmfcc && dtrigger, ABD_E_INVALID, "NULL argument");
  const MfccDev& d = plan->dev;
  ABD_CHECK(d.fast && !d.bluestein && d.bwd_ok, ABD_E_UNSUPPORTED,
            "MFCC backward needs a specialised non-Bluestein FFT plan (n_fft 2048 or 400), got n_fft %d", d.N);
  ABD_CHECK(row_stride >= plan->length, ABD_E_INVALID, "row_stride < length");
  InjDev ij = make_inj(inj);
  ABD_CHECK(ij.mode == ABD_INJECT_DEPLOY || ij.mode == ABD_INJECT_DEPLOY_CLAMP, ABD_E_INVALID,
            "MFCC backward is defined for the DEPLOY / DEPLOY_CLAMP mix only (got mode %d)", ij.mode);
  ABD_CHECK(ij.poison == nullptr && !ij.patch, ABD_E_INVALID, "MFCC backward injects every row (poison must be NULL)");
  ABD_CHECK(ij.frames == nullptr, ABD_E_UNSUPPORTED, "MFCC backward does not take ragged rows");
  int rc = check_inj(ij);
  if (rc) return rc;
  ABD_CHECK(ij.trig_len <= d.L, ABD_E_INVALID, "trigger longer than the clip");
  const size_t need = abd_mfcc_deploy_backward_workspace_bytes(plan, batch, ij.trig_len);
  ABD_CHECK(workspace && workspace_bytes >= need, ABD_E_WORKSPACE, "workspace too small (%zu < %zu)", workspace_bytes,
            need);
  const size_t dblds = ((size_t)d.n_mels * d.n_mfcc + (size_t)d.T * d.n_mels) * sizeof(float);
  ABD_CHECK(dblds <= 64 * 1024, ABD_E_UNSUPPORTED, "MFCC backward: %d frames x %d mels exceed the LDS tile", d.T,
            d.n_mels);
  auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
  char* ws = static_cast<char*>(workspace);
  size_t off = 0;
  float* ws_db = reinterpret_cast<float*>(ws + off);
  off += al((size_t)batch * d.T * d.n_mels * sizeof(float));
  float* ws_max = reinterpret_cast<float*>(ws + off);
  off += al((size_t)batch * d.chunks * sizeof(float));
  float* ws_scale = reinterpret_cast<float*>(ws + off);
  off += al((size_t)batch * sizeof(float));
  unsigned* queue = reinterpret_cast<unsigned*>(ws + off);
  off = abd_mfcc_workspace_bytes(plan, batch);
  float* gframes = reinterpret_cast<float*>(ws + off);
  off += al((size_t)batch * d.T * d.N * sizeof(float));
  float* wgrad = reinterpret_cast<float*>(ws + off);
  off += al((size_t)batch * ij.trig_len * sizeof(float));
  double* spart = reinterpret_cast<double*>(ws + off);
  off += al((size_t)batch * wave_blocks(plan) * sizeof(double));
  double* coef = reinterpret_cast<double*>(ws + off);
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (!(flags & ABD_BWD_FORWARD_IN_WORKSPACE)) {
    // forward recompute: SNR scale, then dB + per-item maxima (the values the clamp adjoint needs)
    row_scale_kernel<<<dim3((unsigned)batch), dim3(kThreads), 0, s>>>(wave, row_stride, d.L, rows, ij, ws_scale);
    ABD_LAUNCH_CHECK();
    if (dispatch_fast(d, wave, row_stride, rows, batch, ij, ws_scale, ws_db, ws_max, queue, s) != 0) return -1;
  }
  mfcc_db_bwd_kernel<<<dim3((unsigned)batch), dim3(kThreads), dblds, s>>>(d, ws_max, dmfcc, ws_db);
  ABD_LAUNCH_CHECK();
  ABD_CHECK(dispatch_stft_bwd(d, wave, row_stride, rows, batch, ij, ws_scale, ws_db, gframes, s) == 0,
            ABD_E_UNSUPPORTED, "no backward FFT plan for n_fft %d", d.N);
  wave_bwd_kernel<<<dim3((unsigned)wave_blocks(plan), (unsigned)batch), dim3(kThreads), 0, s>>>(
      d, gframes, wave, row_stride, rows, ij, ws_scale, wgrad, spart);
  ABD_LAUNCH_CHECK();
  trig_coef_kernel<<<1, kThreads, 0, s>>>(spart, wave_blocks(plan), batch, ws_scale, ij.trig, ij.trig_len, coef);
  ABD_LAUNCH_CHECK();
  trig_grad_kernel<<<(unsigned)((ij.trig_len + 63) / 64), kThreads, 0, s>>>(
      wgrad, batch, ij.trig_len, ij.trig, coef, dtrigger, flags & ABD_BWD_ACCUMULATE);
  ABD_LAUNCH_CHECK();
  return ABD_OK;
}


}  // extern "C"
