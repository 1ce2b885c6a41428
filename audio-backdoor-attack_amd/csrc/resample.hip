// Band-limited resampling: torchaudio.functional.resample (sinc_interp_hann) as called by
// prepare_dataset.py:60 (16 kHz Speech Commands -> 44.1 kHz for the ultrasonic attack).
//
// torchaudio's algorithm (reduce by gcd: 16000/44100 -> orig 160, new 441):
//   base = min(orig, new) * rolloff, width = ceil(lpw * orig / base)
//   kernel[p][k] = sinc(pi * t) * cos(pi t / (2 lpw))^2 * base / orig,
//       t = clamp(base * (-p / new + (k - width) / orig), -lpw, lpw),  k < 2 width + orig
//   out[i * new + p] = sum_k kernel[p][k] * x[i * orig + k - width]   (zero outside x)
//   keep the first ceil(new * length / orig) outputs.
// A polyphase FIR: 2 width + orig taps (174 for 16k -> 44.1k) per output sample, ~15 MFLOP
// and 236 KB of HBM traffic per 1 s clip -- VALU-bound (fp32 MFMA has the same 157 TF peak
// as the vector ALUs on gfx950, so there is nothing to gain from a GEMM reshape).
//
// Kernel: persistent blocks, one thread per output phase p (new <= kMaxNew); each thread
// keeps its phase's taps in registers (loaded once per block, reused for every clip and
// frame the block handles); the input span of kFB frames is staged in LDS and read as
// float4 broadcasts (all lanes of a wave read the same address).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <numeric>
#include <vector>

#include "abd_common.h"

namespace {

constexpr int kMaxTaps = 176;   // taps padded to a multiple of 4 (174 for 16k -> 44.1k)
constexpr int kMaxNew = 448;    // threads per block: one per phase
constexpr int kFB = 16;         // frames per work item

struct ResDev {
  const float* taps;  // [new][ntap4] (zero-padded)
  int orig, nw, width, ntap4;
};

template <int NT4, bool VEC>
__global__ void __launch_bounds__(kMaxNew) resample_kernel(ResDev r, const float* __restrict__ in, int64_t in_stride,
                                                          int64_t batch, int64_t length, float* __restrict__ out,
                                                          int64_t out_stride, int64_t out_len) {
  extern __shared__ __attribute__((aligned(16))) float xs[];  // kFB * orig + 4 * NT4 floats
  const int p = threadIdx.x;
  const bool live = p < r.nw;
  float4 k4[NT4];
#pragma unroll
  for (int j = 0; j < NT4; ++j)
    k4[j] = live ? reinterpret_cast<const float4*>(r.taps)[(int64_t)p * NT4 + j] : make_float4(0.f, 0.f, 0.f, 0.f);
  const int64_t frames = (out_len + r.nw - 1) / r.nw;
  const int64_t chunks = (frames + kFB - 1) / kFB;
  const int span = kFB * r.orig + 4 * NT4;
  for (int64_t item = blockIdx.x; item < batch * chunks; item += gridDim.x) {
    const int64_t u = item / chunks;
    const int64_t i0 = (item - u * chunks) * kFB;
    const float* x = in + u * in_stride;
    const int64_t s0 = i0 * r.orig - r.width;  // first input sample of the span
    __syncthreads();                           // previous item's reads are done
    for (int j = threadIdx.x; j < span; j += blockDim.x) {
      const int64_t s = s0 + j;
      xs[j] = (s >= 0 && s < length) ? x[s] : 0.0f;
    }
    __syncthreads();
    if (!live) continue;
    const int nf = frames - i0 < kFB ? (int)(frames - i0) : kFB;
    for (int f = 0; f < nf; ++f) {
      const float* xf = xs + f * r.orig;
      float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
#pragma unroll
      for (int j = 0; j < NT4; ++j) {
        // VEC (orig % 4 == 0): one ds_read_b128 broadcast per 4 taps
        const float4 v = VEC ? reinterpret_cast<const float4*>(xf)[j]
                             : make_float4(xf[4 * j], xf[4 * j + 1], xf[4 * j + 2], xf[4 * j + 3]);
        a0 = fmaf(v.x, k4[j].x, a0);
        a1 = fmaf(v.y, k4[j].y, a1);
        a2 = fmaf(v.z, k4[j].z, a2);
        a3 = fmaf(v.w, k4[j].w, a3);
      }
      const int64_t o = (i0 + f) * r.nw + p;
      if (o < out_len) out[u * out_stride + o] = (a0 + a1) + (a2 + a3);
    }
  }
}

}  // namespace

struct abd_resample_plan {
  ResDev dev;
  int orig_freq, new_freq;
  float* block = nullptr;
};

extern "C" {

int abd_resample_plan_create(int orig_freq, int new_freq, int lowpass_filter_width, double rolloff,
                             abd_resample_plan** plan) {
  ABD_CHECK(plan != nullptr, ABD_E_INVALID, "NULL out pointer");
  ABD_CHECK(orig_freq > 0 && new_freq > 0 && lowpass_filter_width > 0 && rolloff > 0.0, ABD_E_INVALID,
            "bad resample parameters");
  const int g = std::gcd(orig_freq, new_freq);
  const int orig = orig_freq / g, nw = new_freq / g;
  const double base = std::min(orig, nw) * rolloff;
  const int width = (int)std::ceil(lowpass_filter_width * (double)orig / base);
  const int ntaps = 2 * width + orig;
  // taps padded with zeros up to an instantiated register count
  int ntap4 = 0;
  for (int c : {4, 8, 16, 32, 44})
    if (!ntap4 && c * 4 >= ntaps) ntap4 = c;
  ABD_CHECK(ntap4 > 0 && nw <= kMaxNew, ABD_E_UNSUPPORTED,
            "resample %d -> %d needs %d taps x %d phases (supported: <= %d x %d)", orig_freq, new_freq, ntaps, nw,
            kMaxTaps, kMaxNew);
  std::vector<float> h((size_t)nw * ntap4 * 4, 0.0f);
  const double lpw = lowpass_filter_width;
  for (int p = 0; p < nw; ++p)
    for (int k = 0; k < ntaps; ++k) {
      double t = (-(double)p / nw + (double)(k - width) / orig) * base;
      t = std::max(-lpw, std::min(lpw, t));
      const double w = std::cos(t * M_PI / lpw / 2.0);
      const double tp = t * M_PI;
      const double s = tp == 0.0 ? 1.0 : std::sin(tp) / tp;
      h[(size_t)p * ntap4 * 4 + k] = (float)(s * w * w * base / orig);
    }
  auto* pl = new abd_resample_plan{};
  hipError_t e = hipMalloc(&pl->block, h.size() * sizeof(float));
  if (e == hipSuccess) e = hipMemcpy(pl->block, h.data(), h.size() * sizeof(float), hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    if (pl->block) (void)hipFree(pl->block);
    delete pl;
    abd::set_last_error("resample table upload: %s", hipGetErrorString(e));
    return (int)e;
  }
  pl->dev = ResDev{pl->block, orig, nw, width, ntap4};
  pl->orig_freq = orig_freq;
  pl->new_freq = new_freq;
  *plan = pl;
  return ABD_OK;
}

void abd_resample_plan_destroy(abd_resample_plan* plan) {
  if (!plan) return;
  if (plan->block) (void)hipFree(plan->block);
  delete plan;
}

int64_t abd_resample_output_length(const abd_resample_plan* plan, int64_t length) {
  if (!plan || length < 0) return -1;
  // ceil(new * length / orig) on the gcd-reduced rates (torchaudio's target_length)
  return (plan->dev.nw * length + plan->dev.orig - 1) / plan->dev.orig;
}

int abd_resample_f32(const abd_resample_plan* plan, const float* in, int64_t in_stride, int64_t batch,
                     int64_t length, float* out, int64_t out_stride, abd_stream_t stream) {
  ABD_CHECK(plan && in && out, ABD_E_INVALID, "NULL argument");
  ABD_CHECK(batch >= 0 && length >= 0 && in_stride >= length, ABD_E_INVALID, "bad sizes");
  const int64_t out_len = abd_resample_output_length(plan, length);
  ABD_CHECK(out_stride >= out_len, ABD_E_INVALID, "out_stride %lld < output length %lld", (long long)out_stride,
            (long long)out_len);
  if (batch == 0 || out_len == 0) return ABD_OK;
  const ResDev& d = plan->dev;
  const int threads = (d.nw + 63) / 64 * 64;
  const size_t lds = ((size_t)kFB * d.orig + 4 * (size_t)d.ntap4) * sizeof(float);
  ABD_CHECK(lds <= 64 * 1024, ABD_E_UNSUPPORTED, "resample span too large for LDS");
  const int64_t frames = (out_len + d.nw - 1) / d.nw;
  const int64_t items = batch * ((frames + kFB - 1) / kFB);
  const unsigned grid = (unsigned)std::min<int64_t>(items, 256 * 4);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const bool vec = d.orig % 4 == 0;
  switch (d.ntap4) {
#define ABD_RS_CASE(N)                                                                                          \
  case N:                                                                                                       \
    if (vec)                                                                                                    \
      resample_kernel<N, true><<<grid, threads, lds, s>>>(d, in, in_stride, batch, length, out, out_stride, out_len); \
    else                                                                                                        \
      resample_kernel<N, false><<<grid, threads, lds, s>>>(d, in, in_stride, batch, length, out, out_stride, out_len); \
    break;
    ABD_RS_CASE(4)
    ABD_RS_CASE(8)
    ABD_RS_CASE(16)
    ABD_RS_CASE(32)
    ABD_RS_CASE(44)
#undef ABD_RS_CASE
    default:
      ABD_CHECK(false, ABD_E_UNSUPPORTED, "no resample kernel instantiated for %d taps", d.ntap4 * 4);
  }
  ABD_LAUNCH_CHECK();
  return ABD_OK;
}

}  // extern "C"
