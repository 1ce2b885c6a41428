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
        const float v1 = s1 >= 0 ? c.x[s1] : 0.0f, v2 = s2 >= 0 ? c.x[s2] : 0.0f;
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

// ---- host-side JUCE restatements (float, like the plugins) --------------------------------
float decibels_to_gain(float db) { return db > -100.0f ? std::pow(10.0f, db * 0.05f) : 0.0f; }

}  // namespace

struct abd_style_board {
  FxDev dev;
  float* block = nullptr;
  int sample_rate;
  int64_t max_length;
  bool reverb = false;
};

extern "C" {

int abd_style_board_create(const abd_effect* fx, int n, int sample_rate, int64_t max_length,
                           abd_style_board** board) {
  ABD_CHECK(board && (fx || n == 0), ABD_E_INVALID, "NULL argument");
  ABD_CHECK(n >= 0 && n <= kMaxFx && sample_rate > 0 && max_length >= 0, ABD_E_INVALID, "bad board parameters");
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
        ABD_CHECK(e == 0, ABD_E_UNSUPPORTED, "Chorus must be the first effect of a board (it reads the clip's history)");
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
  delete board;
}

size_t abd_style_board_workspace_bytes(const abd_style_board* board, int64_t batch) {
  if (!board || !board->reverb || batch <= 0) return 0;
  const int64_t pitch = (batch + 63) / 64 * 64;
  return (size_t)board->dev.rstride * (size_t)pitch * sizeof(float);
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
                                           board->reverb ? static_cast<float*>(workspace) : nullptr,
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
