// MFMA issue-rate probe for the conv2 GEMM's inner loop shape (v_mfma_f32_32x32x16_bf16, NJ = 2
// accumulator chains, 6 split terms per 16-deep K step, 8 waves per CU = 2 per SIMD).
// Variants (argv[1]):
//   0  MFMAs only (operands in registers)
//   1  + the B-fragment LDS reads of the weight-stationary kernel (6 ds_read_b128 per step, one
//      step ahead)
//   2  + the A split VALU of split3_x8 (one 8-element split per tap = per step)
//   3  1 + 2 with the split written as scalar v_sub_f32 (no v_pk_add_f32)
//   4  variant 0 on v_mfma_f32_16x16x32_bf16 (same FLOPs: 4 16x16 tiles per 32x32 tile)
// Build: hipcc --offload-arch=gfx950 -O3 -o /tmp/mfma_probe scripts/mfma_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

constexpr int NJ = 2, NP = 3, K = 256, LD = K + 8, STEPS = 16;
__device__ __forceinline__ void split3(const float4& lo, const float4& hi, bf16x8* pl, bool scalar_sub) {
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
        const float b0 = __builtin_bit_cast(float, u[q][h] << 16), b1 = __builtin_bit_cast(float, u[q][h] & 0xffff0000u);
        if (scalar_sub) {
          float x0 = x[0], x1 = x[1];
          asm volatile("v_sub_f32 %0, %0, %1" : "+v"(x0) : "v"(b0));
          asm volatile("v_sub_f32 %0, %0, %1" : "+v"(x1) : "v"(b1));
          x = f32x2{x0, x1};
        } else {
          x -= f32x2{b0, b1};
        }
      }
    }
  }
#pragma unroll
  for (int q = 0; q < 3; ++q) pl[q] = __builtin_bit_cast(bf16x8, make_uint4(u[q][0], u[q][1], u[q][2], u[q][3]));
}

template <int V>
__global__ void __launch_bounds__(512, 1) probe(int iters, float* out, const float* src) {
  __shared__ __attribute__((aligned(16))) __bf16 Bs[NP][64 * LD];
  const int tid = threadIdx.x, lane = tid & 63;
  for (int i = tid; i < NP * 64 * LD; i += 512) (&Bs[0][0])[i] = (__bf16)(0.001f * (i % 97));
  __syncthreads();
  f32x16 acc[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.0f;
  f32x4 acc4[NJ][4];
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int q = 0; q < 4; ++q) acc4[j][q] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 av[NP], bv[2][NJ][NP];
  float4 lo = *reinterpret_cast<const float4*>(src + 8 * lane), hi = *reinterpret_cast<const float4*>(src + 8 * lane + 4);
#pragma unroll
  for (int q = 0; q < NP; ++q) {
    av[q] = __builtin_bit_cast(bf16x8, make_uint4(lane, lane + 1, lane + 2, q));
#pragma unroll
    for (int j = 0; j < NJ; ++j) bv[0][j][q] = bv[1][j][q] = av[q];
  }
  const int kq = 8 * (lane >> 5);
  constexpr int TA[6] = {2, 0, 1, 1, 0, 0}, TB[6] = {0, 2, 1, 0, 1, 0};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int ks = 0; ks < STEPS; ++ks) {
      if constexpr (V == 1 || V == 3) {
        const int kb = ((ks + 1) % STEPS) * 16 + kq;
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
          for (int q = 0; q < NP; ++q)
            bv[(ks + 1) & 1][j][q] = *reinterpret_cast<const bf16x8*>(&Bs[q][(32 * j + (lane & 31)) * LD + kb]);
      }
      if constexpr (V == 2 || V == 3) {
        split3(lo, hi, av, V == 3);
        lo.x += 1.0f;  // a fresh operand every step
      }
      if constexpr (V == 4) {
#pragma unroll
        for (int term = 0; term < 6; ++term)
#pragma unroll
          for (int j = 0; j < NJ; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q)
              acc4[j][q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[TA[term]], bv[0][j][TB[term]], acc4[j][q], 0, 0, 0);
      } else {
#pragma unroll
        for (int term = 0; term < 6; ++term)
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[TA[term]], bv[ks & 1][j][TB[term]], acc[j], 0, 0, 0);
      }
    }
  }
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
#pragma unroll
    for (int r = 0; r < 16; ++r) s += acc[j][r];
#pragma unroll
    for (int q = 0; q < 4; ++q) s += acc4[j][q][0] + acc4[j][q][1] + acc4[j][q][2] + acc4[j][q][3];
  }
  out[blockIdx.x * 512 + tid] = s;
}

int main(int argc, char** argv) {
  const int v = argc > 1 ? atoi(argv[1]) : 0;
  const int iters = argc > 2 ? atoi(argv[2]) : 2000;
  int cu = 256;
  (void)hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, 0);
  float *out, *src;
  (void)hipMalloc(&out, (size_t)cu * 512 * 4);
  (void)hipMalloc(&src, 64 * 8 * 4);
  (void)hipMemset(src, 0, 64 * 8 * 4);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  auto run = [&]() {
    switch (v) {
      case 0: probe<0><<<cu, 512>>>(iters, out, src); break;
      case 1: probe<1><<<cu, 512>>>(iters, out, src); break;
      case 2: probe<2><<<cu, 512>>>(iters, out, src); break;
      case 3: probe<3><<<cu, 512>>>(iters, out, src); break;
      default: probe<4><<<cu, 512>>>(iters, out, src); break;
    }
  };
  run();
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) run();
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  ms /= 5;
  const double mfma = (double)cu * 8 * iters * STEPS * 6 * NJ;  // 32x32x16 equivalents
  const double flop = mfma * 2.0 * 32 * 32 * 16;
  printf("variant %d: %.3f ms per launch, %.1f TFLOP/s bf16, %.2f ns per 32x32x16-equivalent per SIMD\n", v, ms,
         flop / (ms * 1e-3) / 1e12, ms * 1e6 / (mfma / (cu * 4.0)));
  return 0;
}
