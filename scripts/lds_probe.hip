// LDS integrity under GPU sharing: every block fills its LDS with a pattern of its own, then for
// `rounds` rounds re-reads and checks it (mismatches counted with a vector atomic), does some VALU
// work and rewrites it with the next round's pattern.  Two processes running this at once share
// the CUs (and the hardware queues): a nonzero count means a block's LDS changed under it.
//   hipcc --offload-arch=gfx950 -O3 scripts/lds_probe.hip -o scripts/lds_probe
//   ./scripts/lds_probe KB LAUNCHES ROUNDS
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

template <int WORDS>
__global__ void __launch_bounds__(512, 1) lds_kernel(unsigned* bad, int rounds, unsigned salt) {
  __shared__ unsigned buf[WORDS];
  const unsigned key = (blockIdx.x * 2654435761u) ^ salt;
  for (int i = threadIdx.x; i < WORDS; i += blockDim.x) buf[i] = key ^ (unsigned)i * 40503u;
  __syncthreads();
  unsigned nbad = 0;
  float f = (float)threadIdx.x;
  for (int r = 0; r < rounds; ++r) {
    const unsigned k0 = key + (unsigned)r * 97u, k1 = key + (unsigned)(r + 1) * 97u;
    for (int i = threadIdx.x; i < WORDS; i += blockDim.x) nbad += buf[i] != (k0 ^ (unsigned)i * 40503u);
#pragma unroll 1
    for (int j = 0; j < 64; ++j) f = fmaf(f, 1.0000001f, 0.5f);
    __syncthreads();
    for (int i = threadIdx.x; i < WORDS; i += blockDim.x) buf[i] = k1 ^ (unsigned)i * 40503u;
    __syncthreads();
  }
  if (f == 12345.0f) nbad += 1000000;  // keep the VALU work
  if (nbad) atomicAdd(bad, nbad);
}

template <int WORDS>
int run(int launches, int rounds) {
  unsigned* d = nullptr;
  if (hipMalloc(&d, sizeof(unsigned)) != hipSuccess) return 2;
  (void)hipMemset(d, 0, sizeof(unsigned));
  int cu = 256;
  (void)hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, 0);
  for (int l = 0; l < launches; ++l) lds_kernel<WORDS><<<cu * 2, 512>>>(d, rounds, 0x9e3779b9u * (unsigned)l);
  if (hipDeviceSynchronize() != hipSuccess) return 3;
  unsigned h = 0;
  (void)hipMemcpy(&h, d, sizeof(unsigned), hipMemcpyDeviceToHost);
  printf("lds_probe %d KB: %d launches x %d rounds x %d blocks: %u mismatching words\n", (int)(WORDS * 4 / 1024),
         launches, rounds, cu * 2, h);
  (void)hipFree(d);
  return 0;
}

int main(int argc, char** argv) {
  const int kb = argc > 1 ? atoi(argv[1]) : 128;
  const int launches = argc > 2 ? atoi(argv[2]) : 20;
  const int rounds = argc > 3 ? atoi(argv[3]) : 200;
  if (kb >= 128) return run<128 * 256>(launches, rounds);
  if (kb >= 96) return run<96 * 256>(launches, rounds);
  if (kb >= 64) return run<64 * 256>(launches, rounds);
  return run<32 * 256>(launches, rounds);
}
