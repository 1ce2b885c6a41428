// JingleBack style boards (utils/styles_trigger.py:8-53, jingleback.py:38-119) on the device.
//
// pedalboard runs JUCE dsp processors in float32, one clip per call with reset=True, so every
// clip starts from zeroed filter state and snapped parameter smoothers.  The effects the
// default board (style 5: Gain(12) -> LadderFilter(HPF12, 1 kHz) -> Phaser()) and style 1
// (Distortion(30)) use are restated from the JUCE algorithms:
//   Gain          x * Decibels::decibelsToGain(dB)                       (float pow)
//   Distortion    tanh(x * decibelsToGain(drive_db))                     (Gain -> WaveShaper)
//   LadderFilter  juce::dsp::LadderFilter<float>::processSample: tanh saturation through a
//                 128-point LookupTableTransform over [-5, 5], a 4-pole one-sample-delay
//                 ladder with resonance feedback from the last pole, mode mix A[0..4]
//   Phaser        juce::dsp::Phaser<float>: a 1 Hz sine LFO evaluated every 4th sample
//                 (juce::dsp::Oscillator at sr/4, float phase accumulator), mapped log-wise
//                 to a cutoff in [20, min(20000, 0.49 sr)] Hz that sets 6 first-order TPT
//                 allpass stages, output feedback, then a linear dry/wet mix
// The LFO -> allpass coefficient sequence depends on the sample index only (all clips start at
// phase 0), so the plan precomputes it once on the host, with JUCE's float arithmetic, as a
// table of G = g / (1 + g) per update step; the ladder saturation table is precomputed likewise.
//
// Kernel: one thread per clip, the whole chain per sample in registers (the IIR recursions are
// sequential in time and independent across clips).  Each lane streams its own row as float4
// loads/stores: a 128-B line serves the lane for 8 consecutive loads from L1/L2, and the
// ~60 dependent flops per sample, not HBM, bound the kernel (latency-bound: a thread's chain
// of 16000 steps).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <vector>

#include "abd_common.h"

namespace {

constexpr int kMaxFx = 8;
constexpr int kLut = 128;  // LadderFilter saturationLUT points

struct FxDev {
  int n;
  int kind[kMaxFx];
  float gain[kMaxFx];        // GAIN / DISTORTION linear gain
  // ladder (one instance)
  float la1, lb0, lb1, ldrive, ldrive2, lgain, lgain2, lres, lcomp, lA[5];
  const float* lut;          // kLut + 1 (guard)
  // phaser (one instance)
  const float* pG;           // G per 4-sample update step
  int64_t pG_len;
  float pfeedback, pdry, pwet;
  // chorus (first effect of the chain, feedback 0): delay in samples per t
  const float* cD;
  float cdry, cwet;
  // reverb (juce::Reverb, mono): 8 combs + 4 allpasses, buffers in the caller's workspace,
  // interleaved by clip ([offset + index][clip]) so the lanes of a wave touch consecutive words
  int rsize[12], roff[12];
  int rstride;               // floats of buffer per clip
  float rgain, rdamp, rfb, rdry, rwet;
};

__device__ __forceinline__ float sat_lut(const float* __restrict__ lut, float x) {
  // juce::dsp::LookupTableTransform::processSample: clamp, scale, truncate, lerp
  const float xc = fminf(fmaxf(x, -5.0f), 5.0f);
  const float idx = 12.7f * xc + 63.5f;
  const unsigned i = (unsigned)idx;
  const float f = idx - (float)i;
  const float x0 = lut[i], x1 = lut[i + 1];
  return x0 + f * (x1 - x0);
}

struct Chain {
  float ls[5];
  float ps[6];
  float plast;
  float rlast[8];
  int ridx[12];
  const float* x;  // the clip (chorus reads its history)
  float* rbuf;     // workspace + clip (reverb buffers, stride = batch_pad)
  int64_t rpitch;
};

// (x + 0.1f) - 0.1f: JUCE_UNDENORMALISE on x86 builds (juce::Reverb's comb / allpass state);
// volatile-free, but written so the compiler may not fold it away (no fast-math)
__device__ __forceinline__ float undenorm(float v) {
  v = __fadd_rn(v, 0.1f);
  return __fsub_rn(v, 0.1f);
}

// effects [0, e) applied to one sample; only Gain / Distortion may precede a Chorus
__device__ __forceinline__ float memoryless_prefix(const FxDev& d, int e, float x) {
  for (int q = 0; q < e; ++q) x = d.kind[q] == ABD_FX_DISTORTION ? tanhf(x * d.gain[q]) : x * d.gain[q];
  return x;
}

__device__ __forceinline__ float run_chain(const FxDev& d, Chain& c, float x, int64_t t) {
  for (int e = 0; e < d.n; ++e) {
    switch (d.kind[e]) {
      case ABD_FX_GAIN:
        x = x * d.gain[e];
        break;
      case ABD_FX_DISTORTION:
        x = tanhf(x * d.gain[e]);
        break;
      case ABD_FX_LADDER: {
        const float dx = d.lgain * sat_lut(d.lut, d.ldrive * x);
        const float a = dx + d.lres * -4.0f * (d.lgain2 * sat_lut(d.lut, d.ldrive2 * c.ls[4]) - dx * d.lcomp);
        const float b = d.lb1 * c.ls[0] + d.la1 * c.ls[1] + d.lb0 * a;
        const float cc = d.lb1 * c.ls[1] + d.la1 * c.ls[2] + d.lb0 * b;
        const float dd = d.lb1 * c.ls[2] + d.la1 * c.ls[3] + d.lb0 * cc;
        const float ee = d.lb1 * c.ls[3] + d.la1 * c.ls[4] + d.lb0 * dd;
        c.ls[0] = a;
        c.ls[1] = b;
        c.ls[2] = cc;
        c.ls[3] = dd;
        c.ls[4] = ee;
        x = a * d.lA[0] + b * d.lA[1] + cc * d.lA[2] + dd * d.lA[3] + ee * d.lA[4];
        break;
      }
      case ABD_FX_CHORUS: {  // juce::dsp::Chorus, feedback 0: linear-interpolated delay of the input
        const float dl = d.cD[t];
        const int di = (int)floorf(dl);
        const float fr = dl - (float)di;
        const int64_t s1 = t - di, s2 = t - di - 1;
        // the delay line holds the chorus's own input: the clip through the (memoryless) effects
        // before it -- Gain / Distortion, checked at board creation; zeros before t = 0
        const float v1 = s1 >= 0 ? memoryless_prefix(d, e, c.x[s1]) : 0.0f;
        const float v2 = s2 >= 0 ? memoryless_prefix(d, e, c.x[s2]) : 0.0f;
        const float wet = __fadd_rn(v1, __fmul_rn(fr, __fsub_rn(v2, v1)));
        x = __fadd_rn(__fmul_rn(wet, d.cwet), __fmul_rn(x, d.cdry));
        break;
      }
      case ABD_FX_REVERB: {  // juce::Reverb::processMono, float ops in JUCE's order (no contraction)
        const float in = __fmul_rn(x, d.rgain);
        float out = 0.0f;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float* b = c.rbuf + (int64_t)(d.roff[j] + c.ridx[j]) * c.rpitch;
          const float o = *b;
          float l = __fadd_rn(__fmul_rn(o, __fsub_rn(1.0f, d.rdamp)), __fmul_rn(c.rlast[j], d.rdamp));
          l = undenorm(l);
          c.rlast[j] = l;
          *b = undenorm(__fadd_rn(in, __fmul_rn(l, d.rfb)));
          c.ridx[j] = c.ridx[j] + 1 == d.rsize[j] ? 0 : c.ridx[j] + 1;
          out = __fadd_rn(out, o);
        }
#pragma unroll
        for (int j = 8; j < 12; ++j) {
          float* b = c.rbuf + (int64_t)(d.roff[j] + c.ridx[j]) * c.rpitch;
          const float bv = *b;
          *b = undenorm(__fadd_rn(out, __fmul_rn(bv, 0.5f)));
          c.ridx[j] = c.ridx[j] + 1 == d.rsize[j] ? 0 : c.ridx[j] + 1;
          out = __fsub_rn(bv, out);
        }
        x = __fadd_rn(__fmul_rn(out, d.rwet), __fmul_rn(x, d.rdry));
        break;
      }
      case ABD_FX_PHASER: {
        const float G = d.pG[t >> 2];
        float o = x - c.plast;
#pragma unroll
        for (int n = 0; n < 6; ++n) {  // FirstOrderTPTFilter allpass
          const float v = G * (o - c.ps[n]);
          const float y = v + c.ps[n];
          c.ps[n] = y + v;
          o = 2.0f * y - o;
        }
        c.plast = o * d.pfeedback;
        x = o * d.pwet + x * d.pdry;  // DryWetMixer (linear rule): wet * w + dry * (1 - w)
        break;
      }
      default:
        break;
    }
  }
  return x;
}

constexpr int kThreads = 64;

__global__ void __launch_bounds__(kThreads) board_kernel(FxDev d, const float* __restrict__ in, int64_t in_stride,
                                                        const int32_t* __restrict__ rows, int64_t batch,
                                                        int64_t length, float* __restrict__ out,
                                                        int64_t out_stride, float* __restrict__ ws,
                                                        int64_t ws_pitch) {
  const int64_t u = blockIdx.x * (int64_t)kThreads + threadIdx.x;
  if (u >= batch) return;
  const int64_t row = rows ? rows[u] : u;
  const float* x = in + row * in_stride;
  float* y = out + u * out_stride;
  Chain c{};
  c.x = x;
  c.rpitch = ws_pitch;
  c.rbuf = ws ? ws + u : nullptr;
  if (ws)  // reset=True: zeroed reverb buffers for every clip
    for (int64_t i = 0; i < d.rstride; ++i) c.rbuf[i * ws_pitch] = 0.0f;
  const bool vec = ((in_stride | out_stride) & 3) == 0;
  int64_t t = 0;
  if (vec) {
    for (; t + 4 <= length; t += 4) {
      const float4 v = *reinterpret_cast<const float4*>(x + t);
      float4 r;
      r.x = run_chain(d, c, v.x, t);
      r.y = run_chain(d, c, v.y, t + 1);
      r.z = run_chain(d, c, v.z, t + 2);
      r.w = run_chain(d, c, v.w, t + 3);
      *reinterpret_cast<float4*>(y + t) = r;
    }
  }
  for (; t < length; ++t) y[t] = run_chain(d, c, x[t], t);
}

// Fast path for chains in canonical order (Gain? -> Distortion? -> LadderFilter? -> Phaser?,
// each at most once: every board get_boards() can run).  The chain is a compile-time
// signature, the saturation table sits in LDS (the ladder's feedback lookup is on the
// recursion's critical path) and the phaser runs one sample behind the ladder, so the two
// recursions are independent within an iteration and their latencies overlap.
template <bool GAIN, bool DIST, bool LADDER, bool PHASER>
__global__ void __launch_bounds__(kThreads) board_fast_kernel(FxDev d, int gi, int di,
                                                             const float* __restrict__ in, int64_t in_stride,
                                                             const int32_t* __restrict__ rows, int64_t batch,
                                                             int64_t length, float* __restrict__ out,
                                                             int64_t out_stride) {
  __shared__ float lut[kLut + 1];
  if (LADDER)
    for (int i = threadIdx.x; i <= kLut; i += kThreads) lut[i] = d.lut[i];
  __syncthreads();
  const int64_t u = blockIdx.x * (int64_t)kThreads + threadIdx.x;
  if (u >= batch) return;
  const int64_t row = rows ? rows[u] : u;
  const float* x = in + row * in_stride;
  float* y = out + u * out_stride;
  const float g = GAIN ? d.gain[gi] : 1.0f, gd = DIST ? d.gain[di] : 1.0f;
  float ls0 = 0.f, ls1 = 0.f, ls2 = 0.f, ls3 = 0.f, ls4 = 0.f;
  float ps[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float plast = 0.0f, pend = 0.0f;
  for (int64_t t = 0; t <= length; ++t) {
    float v = 0.0f;
    if (t < length) {  // stage A: gain / distortion / ladder of sample t
      v = x[t];
      if (GAIN) v = v * g;
      if (DIST) v = tanhf(v * gd);
      if (LADDER) {
        const float dx = d.lgain * sat_lut(lut, d.ldrive * v);
        const float a = dx + d.lres * -4.0f * (d.lgain2 * sat_lut(lut, d.ldrive2 * ls4) - dx * d.lcomp);
        const float b = d.lb1 * ls0 + d.la1 * ls1 + d.lb0 * a;
        const float c = d.lb1 * ls1 + d.la1 * ls2 + d.lb0 * b;
        const float e3 = d.lb1 * ls2 + d.la1 * ls3 + d.lb0 * c;
        const float e4 = d.lb1 * ls3 + d.la1 * ls4 + d.lb0 * e3;
        ls0 = a;
        ls1 = b;
        ls2 = c;
        ls3 = e3;
        ls4 = e4;
        v = a * d.lA[0] + b * d.lA[1] + c * d.lA[2] + e3 * d.lA[3] + e4 * d.lA[4];
      }
    }
    if (PHASER) {  // stage B: phaser of sample t - 1 (independent of stage A above)
      if (t > 0) {
        const int64_t tp = t - 1;
        const float G = d.pG[tp >> 2];
        float o = pend - plast;
#pragma unroll
        for (int n = 0; n < 6; ++n) {
          const float vv = G * (o - ps[n]);
          const float yy = vv + ps[n];
          ps[n] = yy + vv;
          o = 2.0f * yy - o;
        }
        plast = o * d.pfeedback;
        y[tp] = o * d.pwet + pend * d.pdry;
      }
      pend = v;
    } else if (t < length) {
      y[t] = v;
    }
  }
}

// ---- PitchShift stage (styles 0 and 3) -------------------------------------------------------
// pedalboard.PitchShift is Rubber Band R2 in real-time mode: a phase-vocoder time stretch by
// r = 2^(semitones/12) followed by a resample by 1/r.  Rubber Band publishes no bit-level spec, so
// the stage is a phase vocoder of that structure whose every constant is defined in
// oracle/effects.py (pitch_shift) -- parity unpinned against pedalboard, 1e-4 against the oracle.
// Five launches per board application, each over the whole batch:
//   analysis   grid (frame pairs, clips): two windowed real frames packed into one complex
//              N-point FFT (Stockham radix-4 [+2] in LDS), split into the two half spectra,
//              stored as (|X|, arg X) per bin; an all-zero frame stores exact zeros (the oracle's
//              rfft of a zero frame), not the packing's rounding cross-talk
//   phase      thread per (clip, bin): the phase-vocoder recursion over the frames, in place
//              -> Y = |X| e^{i phi_s}; every phase increment reduced mod 2 pi with the k h mod N
//              terms formed in integers, so the fp32 accumulator stays within [-pi, pi]
//   synthesis  grid (frame pairs, clips): two Hermitian spectra packed into one inverse FFT,
//              real / imaginary parts = the two frames, times the window
//   ola        thread per stretched sample: the <= 4 overlapping frames summed in frame order,
//              divided by sum w^2
//   resample   thread per output sample: windowed-sinc interpolation at n r (position in double)
// Work per 1 s clip at 16 kHz: 117 frames of N = 1024 each way -- HBM / latency-bound, off the
// training step (jingleback poisons once, jingleback.py:69-78).
struct PitchDev {
  int N, K, Hs, Tmax;
  double r;
  float fc, W;
  const int* ia;       // analysis centres, Tmax
  const float* win;    // periodic Hann, N
  const float2* tw;    // exp(-2 pi i e / N), e < N
};

constexpr int kPitchThreads = 256;
constexpr float kTwoPi = 6.283185307179586f;

__device__ __forceinline__ float2 cmulf(float2 a, float2 b) {
  return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ float princargf(float x) { return x - kTwoPi * rintf(x * (1.0f / kTwoPi)); }

// forward FFT of a[0..N) (LDS), b scratch; returns the buffer holding the result
template <int N>
__device__ float2* fft_lds(float2* a, float2* b, const float2* __restrict__ tw) {
  float2* src = a;
  float2* dst = b;
  int ns = 1;
  for (; ns * 4 <= N; ns *= 4) {
    const int tstep = N / (4 * ns);
    for (int j = threadIdx.x; j < N / 4; j += kPitchThreads) {
      const int k = j & (ns - 1);
      float2 v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[r] = src[j + r * (N / 4)];
        if (r > 0) v[r] = cmulf(v[r], tw[k * r * tstep]);
      }
      const float2 t0 = make_float2(v[0].x + v[2].x, v[0].y + v[2].y);
      const float2 t1 = make_float2(v[0].x - v[2].x, v[0].y - v[2].y);
      const float2 t2 = make_float2(v[1].x + v[3].x, v[1].y + v[3].y);
      const float2 t3 = make_float2(v[1].x - v[3].x, v[1].y - v[3].y);
      const int d = (j - k) * 4 + k;
      dst[d] = make_float2(t0.x + t2.x, t0.y + t2.y);
      dst[d + ns] = make_float2(t1.x + t3.y, t1.y - t3.x);       // t1 - i t3
      dst[d + 2 * ns] = make_float2(t0.x - t2.x, t0.y - t2.y);
      dst[d + 3 * ns] = make_float2(t1.x - t3.y, t1.y + t3.x);   // t1 + i t3
    }
    __syncthreads();
    float2* tmp = src;
    src = dst;
    dst = tmp;
  }
  if (ns < N) {  // one radix-2 pass (N = 2 * 4^m)
    const int tstep = N / (2 * ns);
    for (int j = threadIdx.x; j < N / 2; j += kPitchThreads) {
      const int k = j & (ns - 1);
      const float2 v0 = src[j], v1 = cmulf(src[j + N / 2], tw[k * tstep]);
      const int d = (j - k) * 2 + k;
      dst[d] = make_float2(v0.x + v1.x, v0.y + v1.y);
      dst[d + ns] = make_float2(v0.x - v1.x, v0.y - v1.y);
    }
    __syncthreads();
    src = dst;
  }
  return src;
}

template <int N>
__global__ void __launch_bounds__(kPitchThreads) pitch_analysis_kernel(PitchDev p, const float* __restrict__ in,
                                                                      int64_t in_stride, const int32_t* __restrict__ rows,
                                                                      int L, int T, float2* __restrict__ spec) {
  __shared__ float2 bufa[N], bufb[N];
  const int64_t u = blockIdx.y;
  const int t0 = 2 * blockIdx.x, t1 = t0 + 1;
  const float* x = in + (rows ? (int64_t)rows[u] : u) * in_stride;
  const int c0 = p.ia[t0] - N / 2, c1 = t1 < T ? p.ia[t1] - N / 2 : 0;
  bool nz0 = false, nz1 = false;
  for (int n = threadIdx.x; n < N; n += kPitchThreads) {
    const int s0 = c0 + n, s1 = c1 + n;
    const float a = (s0 >= 0 && s0 < L) ? x[s0] : 0.0f;
    const float b = (t1 < T && s1 >= 0 && s1 < L) ? x[s1] : 0.0f;
    nz0 |= a != 0.0f;
    nz1 |= b != 0.0f;
    const float w = p.win[n];
    bufa[n] = make_float2(a * w, b * w);
  }
  nz0 = __syncthreads_or(nz0);
  nz1 = __syncthreads_or(nz1);
  const float2* Z = fft_lds<N>(bufa, bufb, p.tw);
  constexpr int K = N / 2 + 1;
  float2* s0 = spec + ((int64_t)u * T + t0) * K;
  float2* s1 = spec + ((int64_t)u * T + t1) * K;
  for (int k = threadIdx.x; k < K; k += kPitchThreads) {
    const float2 zk = Z[k], zn = Z[(N - k) & (N - 1)];
    // A = (Z[k] + conj Z[N-k]) / 2, B = (Z[k] - conj Z[N-k]) / 2i
    const float ar = 0.5f * (zk.x + zn.x), ai = 0.5f * (zk.y - zn.y);
    const float br = 0.5f * (zk.y + zn.y), bi = -0.5f * (zk.x - zn.x);
    const float ma = sqrtf(ar * ar + ai * ai), mb = sqrtf(br * br + bi * bi);
    s0[k] = nz0 ? make_float2(ma, ma == 0.0f ? 0.0f : atan2f(ai, ar)) : make_float2(0.0f, 0.0f);
    if (t1 < T) s1[k] = nz1 ? make_float2(mb, mb == 0.0f ? 0.0f : atan2f(bi, br)) : make_float2(0.0f, 0.0f);
  }
}

__global__ void __launch_bounds__(kPitchThreads) pitch_phase_kernel(PitchDev p, int T, float2* __restrict__ spec) {
  const int k = blockIdx.x * kPitchThreads + threadIdx.x;
  if (k >= p.K) return;
  float2* s = spec + (int64_t)blockIdx.y * T * p.K + k;
  const int N = p.N;
  const float adv = kTwoPi * (float)((k * p.Hs) % N) / (float)N;  // 2 pi (k Hs mod N) / N
  float pa_prev = 0.0f, ps = 0.0f;
  for (int t = 0; t < T; ++t) {
    const float2 mp = s[(int64_t)t * p.K];
    if (t == 0) {
      ps = mp.y;
    } else {
      const int h = p.ia[t] - p.ia[t - 1];
      const float omh = kTwoPi * (float)((int)(((int64_t)k * h) % N)) / (float)N;
      const float dphi = princargf(mp.y - pa_prev - omh);
      ps = princargf(ps + adv + ((float)p.Hs / (float)h) * dphi);
    }
    pa_prev = mp.y;
    float sn, cs;
    sincosf(ps, &sn, &cs);
    s[(int64_t)t * p.K] = make_float2(mp.x * cs, mp.x * sn);
  }
}

template <int N>
__global__ void __launch_bounds__(kPitchThreads) pitch_synthesis_kernel(PitchDev p, int T, const float2* __restrict__ spec,
                                                                       float* __restrict__ frames) {
  __shared__ float2 bufa[N], bufb[N];
  constexpr int K = N / 2 + 1;
  const int64_t u = blockIdx.y;
  const int t0 = 2 * blockIdx.x, t1 = t0 + 1;
  const float2* s0 = spec + ((int64_t)u * T + t0) * K;
  const float2* s1 = spec + ((int64_t)u * T + t1) * K;
  for (int k = threadIdx.x; k < N; k += kPitchThreads) {
    const int kk = k <= N / 2 ? k : N - k;
    float2 y0 = s0[kk], y1 = t1 < T ? s1[kk] : make_float2(0.0f, 0.0f);
    if (kk == 0 || kk == N / 2) {  // irfft: the imaginary parts of DC and Nyquist are dropped
      y0.y = 0.0f;
      y1.y = 0.0f;
    }
    if (k > N / 2) {  // Hermitian extension
      y0.y = -y0.y;
      y1.y = -y1.y;
    }
    // Z = Y0 + i Y1; inverse FFT as conj(FFT(conj Z)) / N
    bufa[k] = make_float2(y0.x - y1.y, -(y0.y + y1.x));
  }
  __syncthreads();
  const float2* R = fft_lds<N>(bufa, bufb, p.tw);
  float* f0 = frames + ((int64_t)u * T + t0) * N;
  float* f1 = frames + ((int64_t)u * T + t1) * N;
  const float inv = 1.0f / (float)N;
  for (int n = threadIdx.x; n < N; n += kPitchThreads) {
    const float w = p.win[n];
    f0[n] = (R[n].x * inv) * w;
    if (t1 < T) f1[n] = (-R[n].y * inv) * w;
  }
}

__global__ void __launch_bounds__(kPitchThreads) pitch_ola_kernel(PitchDev p, int T, int Ls, const float* __restrict__ frames,
                                                                 float* __restrict__ ys) {
  const int j = blockIdx.x * kPitchThreads + threadIdx.x;
  if (j >= Ls) return;
  const int64_t u = blockIdx.y;
  const int N = p.N, H = p.Hs;
  // frames t with 0 <= j - t H + N/2 < N
  const int tlo = max(0, (j + N / 2 - N + 1 + H - 1) / H), thi = min(T - 1, (j + N / 2) / H);
  float acc = 0.0f, ws = 0.0f;
  for (int t = tlo; t <= thi; ++t) {
    const int i = j - t * H + N / 2;
    acc += frames[((int64_t)u * T + t) * N + i];
    const float w = p.win[i];
    ws += w * w;
  }
  ys[u * Ls + j] = ws > 1e-6f ? acc / ws : 0.0f;
}

__global__ void __launch_bounds__(kPitchThreads) pitch_resample_kernel(PitchDev p, int Ls, const float* __restrict__ ys,
                                                                      int L, float* __restrict__ out, int64_t out_stride) {
  const int n = blockIdx.x * kPitchThreads + threadIdx.x;
  if (n >= L) return;
  const int64_t u = blockIdx.y;
  const double pos = (double)n * p.r;
  const int jlo = max(0, (int)ceil(pos - (double)p.W)), jhi = min(Ls - 1, (int)floor(pos + (double)p.W));
  const float* y = ys + u * Ls;
  const float f2 = 2.0f * p.fc;
  float acc = 0.0f;
  for (int j = jlo; j <= jhi; ++j) {
    const float d = (float)(pos - (double)j);
    if (fabsf(d) < p.W) {
      const float z = f2 * d;
      const float sc = z == 0.0f ? 1.0f : sinpif(z) / (3.14159265358979f * z);
      acc += y[j] * (f2 * sc * 0.5f * (1.0f + cospif(d / p.W)));
    }
  }
  out[u * out_stride + n] = acc;
}

// workspace regions of the pitch stage for `batch` clips of `length` samples (256-B aligned)
struct PitchWs {
  size_t spec, frames, ys, pout, total;
};
inline size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }
PitchWs pitch_ws(const PitchDev& p, int64_t batch, int64_t length, bool need_out) {
  const double r = p.r;
  const int64_t Ls = (int64_t)std::ceil((double)length * r);
  const int64_t T = (Ls + p.Hs - 1) / p.Hs + 1;
  PitchWs w{};
  w.spec = 0;
  w.frames = w.spec + align256((size_t)batch * T * p.K * sizeof(float2));
  w.ys = w.frames + align256((size_t)batch * T * p.N * sizeof(float));
  w.pout = w.ys + align256((size_t)batch * Ls * sizeof(float));
  w.total = w.pout + (need_out ? align256((size_t)batch * length * sizeof(float)) : 0);
  return w;
}

// ---- host-side JUCE restatements (float, like the plugins) --------------------------------
float decibels_to_gain(float db) { return db > -100.0f ? std::pow(10.0f, db * 0.05f) : 0.0f; }

}  // namespace

struct abd_style_board {
  FxDev dev;
  float* block = nullptr;
  int sample_rate;
  int64_t max_length;
  bool reverb = false;
  bool pitch = false;  // a PitchShift opens the board: run as the pitch stage, then dev's chain
  PitchDev pd{};
  void* pblock = nullptr;  // pitch tables: ia, window, twiddles
};

extern "C" {

int abd_style_board_create(const abd_effect* fx, int n, int sample_rate, int64_t max_length,
                           abd_style_board** board) {
  ABD_CHECK(board && (fx || n == 0), ABD_E_INVALID, "NULL argument");
  ABD_CHECK(n >= 0 && n <= kMaxFx && sample_rate > 0 && max_length >= 0, ABD_E_INVALID, "bad board parameters");
  // PitchShift: the board's pitch stage (first effect only); the rest is the sample chain
  PitchDev pd{};
  const bool pitch = n > 0 && fx[0].kind == ABD_FX_PITCHSHIFT;
  std::vector<int> ia;
  std::vector<float> win;
  std::vector<float2> tw;
  if (pitch) {
    const double st = fx[0].p[0];
    ABD_CHECK(std::isfinite(st) && std::fabs(st) <= 24.0, ABD_E_INVALID, "PitchShift semitones %g outside [-24, 24]", st);
    pd.r = std::pow(2.0, st / 12.0);
    pd.N = sample_rate < 32000 ? 1024 : 2048;
    pd.K = pd.N / 2 + 1;
    pd.Hs = pd.N / 4;
    pd.fc = (float)(0.475 / std::max(pd.r, 1.0));
    pd.W = (float)(8.0 / (2.0 * (0.475 / std::max(pd.r, 1.0))));
    const int64_t Ls = (int64_t)std::ceil((double)max_length * pd.r);
    pd.Tmax = (int)((Ls + pd.Hs - 1) / pd.Hs + 1);
    ia.resize(pd.Tmax);
    for (int t = 0; t < pd.Tmax; ++t) ia[t] = (int)std::floor((double)t * pd.Hs / pd.r + 0.5);
    win.resize(pd.N);
    tw.resize(pd.N);
    for (int i = 0; i < pd.N; ++i) {
      win[i] = (float)(0.5 - 0.5 * std::cos(2.0 * M_PI * i / pd.N));
      tw[i] = make_float2((float)std::cos(-2.0 * M_PI * i / pd.N), (float)std::sin(-2.0 * M_PI * i / pd.N));
    }
    ++fx;
    --n;
  }
  for (int e = 0; e < n; ++e)
    ABD_CHECK(fx[e].kind != ABD_FX_PITCHSHIFT, ABD_E_UNSUPPORTED, "PitchShift is accelerated as the first effect of a board only");
  FxDev d{};
  d.n = n;
  int nlad = 0, nph = 0, nrv = 0;
  std::vector<float> lut(kLut + 1), G, CD;
  for (int e = 0; e < n; ++e) {
    const abd_effect& f = fx[e];
    d.kind[e] = f.kind;
    switch (f.kind) {
      case ABD_FX_GAIN:
      case ABD_FX_DISTORTION:
        d.gain[e] = decibels_to_gain(f.p[0]);
        break;
      case ABD_FX_LADDER: {
        ABD_CHECK(++nlad == 1, ABD_E_UNSUPPORTED, "one LadderFilter per board");
        const int mode = (int)f.p[0];
        ABD_CHECK(mode >= 0 && mode <= 5, ABD_E_INVALID, "LadderFilter mode %d", mode);
        // juce::dsp::LadderFilter::setMode (LPF12, HPF12, BPF12, LPF24, HPF24, BPF24), x 1.2
        static const float A[6][5] = {{0, 0, 1, 0, 0}, {1, -2, 1, 0, 0}, {0, 0, -1, 1, 0},
                                      {0, 0, 0, 0, 1}, {1, -4, 6, -4, 1}, {0, 0, 1, -2, 1}};
        static const float comp[6] = {0.5f, 0.0f, 0.5f, 0.5f, 0.0f, 0.5f};
        for (int i = 0; i < 5; ++i) d.lA[i] = A[mode][i] * 1.2f;
        d.lcomp = comp[mode];
        const float cutoff = f.p[1], resonance = f.p[2], drive = f.p[3];
        const float scaler = (float)(-2.0 * M_PI) / (float)sample_rate;  // setSampleRate
        d.la1 = std::exp(cutoff * scaler);                               // cutoffTransformValue
        const float g = d.la1 * -1.0f + 1.0f;
        d.lb0 = g * 0.76923076923f;
        d.lb1 = g * 0.23076923076f;
        d.lres = 0.1f + resonance * (1.0f - 0.1f);                       // jmap(res, 0.1, 1.0)
        d.ldrive = drive;
        d.lgain = std::pow(drive, -2.642f) * 0.6103f + 0.3903f;
        d.ldrive2 = drive * 0.04f + 0.96f;
        d.lgain2 = std::pow(d.ldrive2, -2.642f) * 0.6103f + 0.3903f;
        for (int i = 0; i < kLut; ++i) {
          const float v = -5.0f + (10.0f * (float)i) / (float)(kLut - 1);  // jmap(i, 0, 127, -5, 5)
          lut[i] = std::tanh(std::min(5.0f, std::max(-5.0f, v)));
        }
        lut[kLut] = lut[kLut - 1];  // LookupTable guard point
        break;
      }
      case ABD_FX_PHASER: {
        ABD_CHECK(++nph == 1, ABD_E_UNSUPPORTED, "one Phaser per board");
        const float rate = f.p[0], depth = f.p[1], centre = f.p[2], feedback = f.p[3], mix = f.p[4];
        // setCentreFrequency runs before prepare(): JUCE's default 44.1 kHz sets the log range
        const float lo = 20.0f;
        const float hi_set = (float)std::min(20000.0, 0.49 * 44100.0);
        const float norm = (std::log10(centre) - std::log10(lo)) / (std::log10(hi_set) - std::log10(lo));
        const float hi = (float)std::min(20000.0, 0.49 * (double)sample_rate);
        const float osc_sr = (float)((double)sample_rate / 4.0);
        const float inc = ((float)(2.0 * M_PI) / osc_sr) * rate;  // Oscillator baseIncrement * freq
        const float two_pi = (float)(2.0 * M_PI), pi = (float)M_PI;
        const float vol = depth * 0.5f;
        const int64_t steps = (max_length + 3) / 4;
        G.resize((size_t)std::max<int64_t>(steps, 1));
        float phase = 0.0f;
        for (int64_t k = 0; k < steps; ++k) {
          const float last = phase;  // Phase::advance returns the pre-increment phase
          float next = last + inc;
          while (next >= two_pi) next -= two_pi;
          phase = next;
          const float lfo = std::min(1.0f, std::max(0.0f, std::sin(last - pi) * vol + norm));
          const float cut = std::pow(10.0f, lfo * (std::log10(hi) - std::log10(lo)) + std::log10(lo));
          const float gg = (float)std::tan(M_PI * (double)cut / (double)sample_rate);  // FirstOrderTPTFilter
          G[k] = gg / (1.0f + gg);
        }
        d.pfeedback = feedback;
        d.pwet = mix;
        d.pdry = 1.0f - mix;
        break;
      }
      case ABD_FX_CHORUS: {
        for (int q = 0; q < e; ++q)
          ABD_CHECK(fx[q].kind == ABD_FX_GAIN || fx[q].kind == ABD_FX_DISTORTION, ABD_E_UNSUPPORTED,
                    "only Gain / Distortion may precede a Chorus (its delay line re-applies them to the history)");
        const float rate = f.p[0], depth = f.p[1], centre = f.p[2], feedback = f.p[3], mix = f.p[4];
        ABD_CHECK(feedback == 0.0f, ABD_E_UNSUPPORTED, "Chorus feedback != 0 is not accelerated");
        // juce::dsp::Chorus: sine LFO at the sample rate (float phase), x depth * 0.5, delay
        // max(1, 20 * lfo + centre) ms -> samples, clamped to the delay line's maximum
        const float two_pi = (float)(2.0 * M_PI), pi = (float)M_PI;
        const float inc = (two_pi / (float)sample_rate) * rate;
        const float vol = depth * 0.5f;
        const float cdelay = std::min(100.0f, std::max(1.0f, centre));  // setCentreDelay jlimit(1, 100)
        const double max_delay = std::ceil((20.0 * 1.0 * 0.5 + 100.0) * (double)sample_rate / 1000.0);
        CD.resize((size_t)std::max<int64_t>(max_length, 1));
        float phase = 0.0f;
        for (int64_t k = 0; k < max_length; ++k) {
          const float last = phase;
          float next = last + inc;
          while (next >= two_pi) next -= two_pi;
          phase = next;
          const float lfo = std::max(1.0f, 20.0f * (std::sin(last - pi) * vol) + cdelay);
          const float ds = (float)((double)lfo * (double)sample_rate / 1000.0);
          CD[k] = std::min((float)max_delay, std::max(0.0f, ds));
        }
        d.cwet = mix;
        d.cdry = 1.0f - mix;
        break;
      }
      case ABD_FX_REVERB: {
        ABD_CHECK(++nrv == 1, ABD_E_UNSUPPORTED, "one Reverb per board");
        const float room = f.p[0], damping = f.p[1], wet_level = f.p[2], dry_level = f.p[3], width = f.p[4],
                    freeze = f.p[5];
        // juce::Reverb::setSampleRate / setParameters / updateDamping (smoothers snap in prepare)
        static const int comb[8] = {1116, 1188, 1277, 1356, 1422, 1491, 1557, 1617};
        static const int ap[4] = {556, 441, 341, 225};
        int off = 0;
        for (int j = 0; j < 12; ++j) {
          const int tuning = j < 8 ? comb[j] : ap[j - 8];
          d.rsize[j] = std::max(1, (sample_rate * tuning) / 44100);
          d.roff[j] = off;
          off += d.rsize[j];
        }
        d.rstride = off;
        const bool frozen = freeze >= 0.5f;
        const float wet = wet_level * 3.0f;
        d.rdry = dry_level * 2.0f;
        d.rwet = 0.5f * wet * (1.0f + width);
        d.rgain = frozen ? 0.0f : 0.015f;
        d.rdamp = frozen ? 0.0f : damping * 0.4f;
        d.rfb = frozen ? 1.0f : room * 0.28f + 0.7f;
        break;
      }
      default:
        ABD_CHECK(false, ABD_E_UNSUPPORTED, "effect kind %d is not accelerated", f.kind);
    }
  }
  auto* b = new abd_style_board{};
  const size_t nfl = (size_t)(kLut + 1) + G.size() + CD.size();
  hipError_t e = hipMalloc(&b->block, std::max<size_t>(nfl, 1) * sizeof(float));
  if (e == hipSuccess) e = hipMemcpy(b->block, lut.data(), (kLut + 1) * sizeof(float), hipMemcpyHostToDevice);
  if (e == hipSuccess && !G.empty())
    e = hipMemcpy(b->block + kLut + 1, G.data(), G.size() * sizeof(float), hipMemcpyHostToDevice);
  if (e == hipSuccess && !CD.empty())
    e = hipMemcpy(b->block + kLut + 1 + G.size(), CD.data(), CD.size() * sizeof(float), hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    if (b->block) (void)hipFree(b->block);
    delete b;
    abd::set_last_error("style board table upload: %s", hipGetErrorString(e));
    return (int)e;
  }
  if (pitch) {
    const size_t nb = ia.size() * sizeof(int) + win.size() * sizeof(float) + tw.size() * sizeof(float2);
    e = hipMalloc(&b->pblock, nb);
    char* pb = static_cast<char*>(b->pblock);
    if (e == hipSuccess) e = hipMemcpy(pb, tw.data(), tw.size() * sizeof(float2), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(pb + tw.size() * sizeof(float2), win.data(), win.size() * sizeof(float), hipMemcpyHostToDevice);
    if (e == hipSuccess)
      e = hipMemcpy(pb + tw.size() * sizeof(float2) + win.size() * sizeof(float), ia.data(), ia.size() * sizeof(int),
                    hipMemcpyHostToDevice);
    if (e != hipSuccess) {
      if (b->pblock) (void)hipFree(b->pblock);
      (void)hipFree(b->block);
      delete b;
      abd::set_last_error("pitch table upload: %s", hipGetErrorString(e));
      return (int)e;
    }
    pd.tw = reinterpret_cast<const float2*>(pb);
    pd.win = reinterpret_cast<const float*>(pb + tw.size() * sizeof(float2));
    pd.ia = reinterpret_cast<const int*>(pb + tw.size() * sizeof(float2) + win.size() * sizeof(float));
    b->pitch = true;
    b->pd = pd;
  }
  d.lut = b->block;
  d.pG = b->block + kLut + 1;
  d.pG_len = (int64_t)G.size();
  d.cD = b->block + kLut + 1 + G.size();
  b->reverb = nrv > 0;
  b->dev = d;
  b->sample_rate = sample_rate;
  b->max_length = max_length;
  *board = b;
  return ABD_OK;
}

void abd_style_board_destroy(abd_style_board* board) {
  if (!board) return;
  if (board->block) (void)hipFree(board->block);
  if (board->pblock) (void)hipFree(board->pblock);
  delete board;
}

// workspace: [pitch stage regions (pitch_ws)][reverb buffers]
static size_t pitch_bytes(const abd_style_board* b, int64_t batch, int64_t length) {
  return b->pitch ? pitch_ws(b->pd, batch, length, b->dev.n > 0).total : 0;
}
size_t abd_style_board_workspace_bytes(const abd_style_board* board, int64_t batch) {
  if (!board || batch <= 0) return 0;
  const size_t pb = pitch_bytes(board, batch, board->max_length);
  if (!board->reverb) return pb;
  const int64_t pitch = (batch + 63) / 64 * 64;
  return pb + (size_t)board->dev.rstride * (size_t)pitch * sizeof(float);
}

int abd_style_board_apply(const abd_style_board* board, const float* in, int64_t in_stride, const int32_t* rows,
                          int64_t batch, int64_t length, float* out, int64_t out_stride, void* workspace,
                          size_t workspace_bytes, abd_stream_t stream) {
  ABD_CHECK(board && in && out, ABD_E_INVALID, "NULL argument");
  const size_t need = abd_style_board_workspace_bytes(board, batch);
  ABD_CHECK(workspace_bytes >= need && (need == 0 || workspace), ABD_E_WORKSPACE, "workspace too small (%zu < %zu)",
            workspace_bytes, need);
  ABD_CHECK(batch >= 0 && length >= 0 && in_stride >= length && out_stride >= length, ABD_E_INVALID, "bad sizes");
  ABD_CHECK(length <= board->max_length, ABD_E_INVALID, "length %lld exceeds the board's max_length %lld",
            (long long)length, (long long)board->max_length);
  if (batch == 0 || length == 0) return ABD_OK;
  const unsigned grid = (unsigned)((batch + kThreads - 1) / kThreads);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const FxDev& d = board->dev;
  // reverb buffers sit past the pitch regions (sized for max_length, like workspace_bytes)
  char* rws = static_cast<char*>(workspace) + pitch_bytes(board, batch, board->max_length);
  if (board->pitch) {
    const PitchDev& p = board->pd;
    ABD_CHECK(length <= INT32_MAX / 4 && batch <= 65535, ABD_E_INVALID, "pitch stage: batch %lld / length %lld too large",
              (long long)batch, (long long)length);
    const PitchWs w = pitch_ws(p, batch, length, d.n > 0);
    const int Ls = (int)std::ceil((double)length * p.r);
    const int T = (Ls + p.Hs - 1) / p.Hs + 1;
    ABD_CHECK(T <= p.Tmax, ABD_E_INVALID, "pitch stage: %d frames > %d", T, p.Tmax);
    char* base = static_cast<char*>(workspace);
    float2* spec = reinterpret_cast<float2*>(base + w.spec);
    float* frames = reinterpret_cast<float*>(base + w.frames);
    float* ys = reinterpret_cast<float*>(base + w.ys);
    float* pout = d.n > 0 ? reinterpret_cast<float*>(base + w.pout) : out;
    const int64_t pstride = d.n > 0 ? length : out_stride;
    const dim3 gpair((unsigned)((T + 1) / 2), (unsigned)batch);
    if (p.N == 1024) pitch_analysis_kernel<1024><<<gpair, kPitchThreads, 0, s>>>(p, in, in_stride, rows, (int)length, T, spec);
    else pitch_analysis_kernel<2048><<<gpair, kPitchThreads, 0, s>>>(p, in, in_stride, rows, (int)length, T, spec);
    pitch_phase_kernel<<<dim3((unsigned)((p.K + kPitchThreads - 1) / kPitchThreads), (unsigned)batch), kPitchThreads, 0, s>>>(
        p, T, spec);
    if (p.N == 1024) pitch_synthesis_kernel<1024><<<gpair, kPitchThreads, 0, s>>>(p, T, spec, frames);
    else pitch_synthesis_kernel<2048><<<gpair, kPitchThreads, 0, s>>>(p, T, spec, frames);
    pitch_ola_kernel<<<dim3((unsigned)((Ls + kPitchThreads - 1) / kPitchThreads), (unsigned)batch), kPitchThreads, 0, s>>>(
        p, T, Ls, frames, ys);
    pitch_resample_kernel<<<dim3((unsigned)((length + kPitchThreads - 1) / kPitchThreads), (unsigned)batch), kPitchThreads,
                            0, s>>>(p, Ls, ys, (int)length, pout, pstride);
    ABD_LAUNCH_CHECK();
    if (d.n == 0) return ABD_OK;
    in = pout;  // the sample chain reads the shifted clips in batch order
    in_stride = length;
    rows = nullptr;
  }
  // canonical order Gain < Distortion < Ladder < Phaser (kinds 0..3), each at most once -> fast path
  int mask = 0, last = -1, gi = 0, di = 0;
  bool canon = getenv("ABD_FX_GENERIC") == nullptr;
  for (int e = 0; e < d.n && canon; ++e) {
    const int k = d.kind[e];
    canon = k > last && k <= ABD_FX_PHASER;
    last = k;
    mask |= 1 << k;
    if (k == ABD_FX_GAIN) gi = e;
    if (k == ABD_FX_DISTORTION) di = e;
  }
  if (!canon) {
    board_kernel<<<grid, kThreads, 0, s>>>(d, in, in_stride, rows, batch, length, out, out_stride,
                                           board->reverb ? reinterpret_cast<float*>(rws) : nullptr,
                                           (batch + 63) / 64 * 64);
  } else {
    switch (mask) {
#define ABD_FX_CASE(M)                                                                                        \
  case M:                                                                                                     \
    board_fast_kernel<(M & 1) != 0, (M & 2) != 0, (M & 4) != 0, (M & 8) != 0><<<grid, kThreads, 0, s>>>(     \
        d, gi, di, in, in_stride, rows, batch, length, out, out_stride);                                      \
    break;
      ABD_FX_CASE(0) ABD_FX_CASE(1) ABD_FX_CASE(2) ABD_FX_CASE(3) ABD_FX_CASE(4) ABD_FX_CASE(5) ABD_FX_CASE(6)
      ABD_FX_CASE(7) ABD_FX_CASE(8) ABD_FX_CASE(9) ABD_FX_CASE(10) ABD_FX_CASE(11) ABD_FX_CASE(12)
      ABD_FX_CASE(13) ABD_FX_CASE(14) ABD_FX_CASE(15)
#undef ABD_FX_CASE
    }
  }
  ABD_LAUNCH_CHECK();
  return ABD_OK;
}

}  // extern "C"
