// Packed-FP32 operand selection under GPU sharing.  The kernels that
// went nondeterministic with two processes on one GPU (conv1_stats_fold_kernel, conv1_wgrad_kernel;
// wrong LOW-lane results) broadcast one half of a ds_read2_b32 register pair into both lanes of
// v_pk_fma_f32: `op_sel:[0,1,0]` makes the LOW lane read the HIGH dword of src1.  scripts/pk_probe.hip
// (clean in round 4) never emitted that form -- its broadcasts were op_sel_hi only.  This probe runs
// the same FMA chain with src1's selection fixed by inline asm:
//   V=0  op_sel:[0,1,0]     low lane <- src1.hi, high lane <- src1.hi   (the failing kernels' form)
//   V=1  op_sel_hi:[1,0,1]  low lane <- src1.lo, high lane <- src1.lo   (pk_probe's form)
//   V=2  no selection       low lane <- src1.lo, high lane <- src1.hi
// Every launch's output must equal the first launch's bit for bit; run several processes at once.
//   hipcc --offload-arch=gfx950 -O3 scripts/pk_opsel_probe.hip -o scripts/pk_opsel_probe
//   ./scripts/pk_opsel_probe VARIANT LAUNCHES
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int kIters = 16384;
constexpr int kLds = 2048;  // floats of staged input per block

template <int V>
__device__ __forceinline__ f2 pk_fma_sel(f2 a, f2 b, f2 c) {
  f2 r;
  if constexpr (V == 0)
    asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[0,1,0]" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  else if constexpr (V == 1)
    asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[1,0,1]" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  else
    asm volatile("v_pk_fma_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

template <int V>
__global__ void __launch_bounds__(256) probe_kernel(const float* __restrict__ x, const f2* __restrict__ w,
                                                    f2* __restrict__ out, int n) {
  __shared__ __attribute__((aligned(16))) float xs[kLds];
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  for (int j = threadIdx.x; j < kLds; j += 256) xs[j] = x[(blockIdx.x * kLds + j) % n];
  __syncthreads();
  f2 k0 = w[(i & 31) * 4 + 0], k1 = w[(i & 31) * 4 + 1], k2 = w[(i & 31) * 4 + 2], k3 = w[(i & 31) * 4 + 3];
  f2 acc = f2{0.0f, 0.0f}, sq = f2{0.0f, 0.0f};
  int p = (threadIdx.x * 6) & (kLds - 1);
  for (int it = 0; it < kIters; ++it) {
    // two adjacent samples as one register pair (ds_read2_b32 / ds_read_b64), like c1_at_ptr's taps
    const f2 xa = *reinterpret_cast<const f2*>(xs + p);
    const f2 xb = *reinterpret_cast<const f2*>(xs + p + 40);
    f2 r = pk_fma_sel<V>(k0, xa, k3);
    r = pk_fma_sel<V>(k1, xb, r);
    r = pk_fma_sel<V>(k2, xa, r);
    r = f2{fmaxf(r.x, 0.0f), fmaxf(r.y, 0.0f)};
    acc += r;
    sq = __builtin_elementwise_fma(r, r, sq);
    p = (p + 2 * (1 + (it & 3))) & (kLds - 64);
  }
  if (i < n) out[i] = acc + sq;
}

int main(int argc, char** argv) {
  const int variant = argc > 1 ? atoi(argv[1]) : 0;
  const int launches = argc > 2 ? atoi(argv[2]) : 500;
  const int n = 256 * 2048;
  std::vector<float> hx(n);
  std::vector<f2> hw(128);
  for (int i = 0; i < n; ++i) hx[i] = (float)((i * 2654435761u) % 1000) / 500.0f - 1.0f;
  for (int i = 0; i < 128; ++i) hw[i] = f2{0.01f * (float)(i % 17) - 0.08f, 0.013f * (float)(i % 11) - 0.06f};
  float* dx = nullptr;
  f2 *dw = nullptr, *dout = nullptr;
  if (hipMalloc(&dx, n * sizeof(float)) != hipSuccess || hipMalloc(&dw, 128 * sizeof(f2)) != hipSuccess ||
      hipMalloc(&dout, n * sizeof(f2)) != hipSuccess)
    return 2;
  (void)hipMemcpy(dx, hx.data(), n * sizeof(float), hipMemcpyHostToDevice);
  (void)hipMemcpy(dw, hw.data(), 128 * sizeof(f2), hipMemcpyHostToDevice);
  std::vector<f2> ref(n), cur(n);
  long bad_launches = 0, bad_lo = 0, bad_hi = 0;
  for (int l = 0; l < launches; ++l) {
    if (variant == 0) probe_kernel<0><<<n / 256, 256>>>(dx, dw, dout, n);
    else if (variant == 1) probe_kernel<1><<<n / 256, 256>>>(dx, dw, dout, n);
    else probe_kernel<2><<<n / 256, 256>>>(dx, dw, dout, n);
    if (hipDeviceSynchronize() != hipSuccess) return 3;
    (void)hipMemcpy(l == 0 ? ref.data() : cur.data(), dout, n * sizeof(f2), hipMemcpyDeviceToHost);
    if (l == 0) continue;
    long lo = 0, hi = 0;
    for (int i = 0; i < n; ++i) {
      const float cx = cur[i].x, cy = cur[i].y, rx = ref[i].x, ry = ref[i].y;
      lo += memcmp(&cx, &rx, 4) != 0;
      hi += memcmp(&cy, &ry, 4) != 0;
    }
    if (lo || hi) ++bad_launches;
    bad_lo += lo;
    bad_hi += hi;
  }
  printf("pk_opsel_probe V=%d: %d launches, %ld differing launches, %ld low-half and %ld high-half differing values\n",
         variant, launches, bad_launches, bad_lo, bad_hi);
  return 0;
}
