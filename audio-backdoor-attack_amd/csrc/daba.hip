// DABA trigger / host selection (utils/daba_selection_tools.py:24-160) as batched device work.
//
// The reference scores every candidate with a batch-1 forward of the untrained, train-mode
// model, one wav file round trip at a time: 60 pool triggers for certainty (:68-96) and,
// for each of 3000 hosts, the trigger and the pydub-poisoned host for influence (:115-139).
// Here those become one per-utterance-BatchNorm forward over all rows
// (abd_smallcnn_forward_per_utterance) fed by:
//   ragged_overlay_kernel  pydub gain + overlay (audioop.mul then audioop.add, bit-exact: the
//                          linear gain comes from the caller as the same double pydub uses)
//                          on int16 hosts of their own lengths, with the
//                          int16 -> float (soundfile.read) conversion fused, zero past the end
//   softmax_entropy_kernel F.softmax of the log-probs and calc_ent (:55-65, log2, double sum)
//   pair_ce_kernel         cross_entropy(a, y) = sum nan_to_num(-y log a - (1-y) log(1-a)) in
//                          float32 like numpy on the float32 softmax rows (:67-68)
// One thread per row for the K <= 64 class reductions: rows are independent and K is tiny.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>

#include "abd_common.h"

namespace {

constexpr int kThreads = 256;

__global__ void __launch_bounds__(kThreads) ragged_overlay_kernel(
    const int16_t* __restrict__ host, int64_t host_stride, const int32_t* __restrict__ host_len,
    const int16_t* __restrict__ trig, int64_t trig_stride, int64_t trig_len, const double* __restrict__ gain,
    int64_t L, int16_t* __restrict__ out_i16, float* __restrict__ out_f32) {
  const int64_t u = blockIdx.y;
  const int64_t n_host = host_len ? (int64_t)host_len[u] : L;
  const int64_t n = n_host < trig_len ? n_host : trig_len;
  const double factor = gain[u];  // pydub db_to_float(dB), evaluated by the caller in double like pydub
  const int16_t* h = host + u * host_stride;
  const int16_t* t = trig + u * trig_stride;
  for (int64_t s = blockIdx.x * (int64_t)kThreads + threadIdx.x; s < L; s += (int64_t)gridDim.x * kThreads) {
    int v = 0;
    if (s < n_host) {
      v = h[s];
      if (s < n) {
        // audioop.mul: scale, clamp to the int16 range, floor; audioop.add: saturate
        double g = (double)t[s] * factor;
        if (g > 32767.0) g = 32767.0;
        else if (g < -32767.0) g = -32768.0;
        v += (int)floor(g);
        v = v > 32767 ? 32767 : (v < -32768 ? -32768 : v);
      }
    }
    if (out_i16) out_i16[u * L + s] = (int16_t)v;
    if (out_f32) out_f32[u * L + s] = (float)v * (1.0f / 32768.0f);  // soundfile int16 -> float
  }
}

__global__ void __launch_bounds__(kThreads) softmax_entropy_kernel(const float* __restrict__ logp, int64_t n, int K,
                                                                   float* __restrict__ probs,
                                                                   double* __restrict__ entropy) {
  const int64_t r = blockIdx.x * (int64_t)kThreads + threadIdx.x;
  if (r >= n) return;
  const float* x = logp + r * K;
  float mx = -INFINITY;
  for (int k = 0; k < K; ++k) mx = fmaxf(mx, x[k]);
  float sum = 0.0f;
  for (int k = 0; k < K; ++k) sum += expf(x[k] - mx);
  double h = 0.0;
  for (int k = 0; k < K; ++k) {
    const float p = expf(x[k] - mx) / sum;
    if (probs) probs[r * K + k] = p;
    const double pd = (double)p;
    h += pd * log2(pd);  // math.log2 of the float32 probability (p == 0 -> nan, as math.log2 raises)
  }
  entropy[r] = -h;
}

__device__ __forceinline__ float nan_to_num(float v) {
  if (isnan(v)) return 0.0f;
  if (isinf(v)) return v > 0.0f ? FLT_MAX : -FLT_MAX;
  return v;
}

__global__ void __launch_bounds__(kThreads) pair_ce_kernel(const float* __restrict__ pa, const float* __restrict__ py,
                                                           int64_t n, int K, float* __restrict__ out) {
  const int64_t r = blockIdx.x * (int64_t)kThreads + threadIdx.x;
  if (r >= n) return;
  const float* a = pa + r * K;
  const float* y = py + r * K;
  float acc = 0.0f;
  for (int k = 0; k < K; ++k) {
    const float t = -y[k] * logf(a[k]) - (1.0f - y[k]) * logf(1.0f - a[k]);
    acc += nan_to_num(t);
  }
  out[r] = acc;
}

unsigned blocks_for(int64_t n) { return (unsigned)((n + kThreads - 1) / kThreads); }

}  // namespace

extern "C" {

int abd_pydub_overlay_i16(const int16_t* host, int64_t host_len, const int16_t* trig, int64_t trig_len,
                          const double* gain, int64_t batch, int16_t* out, abd_stream_t stream) {
  ABD_CHECK(host && trig && gain && out, ABD_E_INVALID, "NULL argument");
  ABD_CHECK(host_len > 0 && trig_len >= 0 && batch >= 0, ABD_E_INVALID, "bad sizes");
  if (batch == 0) return ABD_OK;
  ABD_CHECK(batch < 65536, ABD_E_INVALID, "batch %lld exceeds the grid's y extent (split it)", (long long)batch);
  const unsigned gx = (unsigned)std::min<int64_t>((host_len + kThreads - 1) / kThreads, 64);
  ragged_overlay_kernel<<<dim3(gx, (unsigned)batch), dim3(kThreads), 0, static_cast<hipStream_t>(stream)>>>(
      host, host_len, nullptr, trig, trig_len, trig_len, gain, host_len, out, nullptr);
  ABD_LAUNCH_CHECK();
  return ABD_OK;
}

int abd_pydub_overlay_ragged_i16(const int16_t* host, int64_t host_stride, const int32_t* host_len,
                                 const int16_t* trig, int64_t trig_stride, int64_t trig_len, const double* gain,
                                 int64_t batch, int64_t length, int16_t* out_i16, float* out_f32,
                                 abd_stream_t stream) {
  ABD_CHECK(host && trig && gain && (out_i16 || out_f32), ABD_E_INVALID, "NULL argument");
  ABD_CHECK(batch >= 0 && length > 0 && trig_len >= 0 && host_stride >= 0 && trig_stride >= 0, ABD_E_INVALID,
            "bad sizes");
  if (batch == 0) return ABD_OK;
  ABD_CHECK(batch < 65536, ABD_E_INVALID, "batch %lld exceeds the grid's y extent (split it)", (long long)batch);
  const unsigned gx = (unsigned)std::min<int64_t>((length + kThreads - 1) / kThreads, 64);
  ragged_overlay_kernel<<<dim3(gx, (unsigned)batch), dim3(kThreads), 0, static_cast<hipStream_t>(stream)>>>(
      host, host_stride, host_len, trig, trig_stride, trig_len, gain, length, out_i16, out_f32);
  ABD_LAUNCH_CHECK();
  return ABD_OK;
}

int abd_softmax_entropy(const float* logprobs, int64_t n, int num_classes, float* probs, double* entropy,
                        abd_stream_t stream) {
  ABD_CHECK(logprobs && entropy, ABD_E_INVALID, "NULL argument");
  ABD_CHECK(num_classes >= 1 && num_classes <= 64 && n >= 0, ABD_E_INVALID, "bad sizes");
  if (n == 0) return ABD_OK;
  softmax_entropy_kernel<<<blocks_for(n), kThreads, 0, static_cast<hipStream_t>(stream)>>>(logprobs, n, num_classes,
                                                                                            probs, entropy);
  ABD_LAUNCH_CHECK();
  return ABD_OK;
}

int abd_pair_cross_entropy(const float* probs_a, const float* probs_y, int64_t n, int num_classes, float* out,
                           abd_stream_t stream) {
  ABD_CHECK(probs_a && probs_y && out, ABD_E_INVALID, "NULL argument");
  ABD_CHECK(num_classes >= 1 && num_classes <= 64 && n >= 0, ABD_E_INVALID, "bad sizes");
  if (n == 0) return ABD_OK;
  pair_ce_kernel<<<blocks_for(n), kThreads, 0, static_cast<hipStream_t>(stream)>>>(probs_a, probs_y, n, num_classes,
                                                                                    out);
  ABD_LAUNCH_CHECK();
  return ABD_OK;
}

}  // extern "C"
