// Microbenchmark: dependent LDS round trips (pointer chase through a 128 KB table) on gfx950, with
// 1..16 waves per CU; reports the latency of one round trip in shader cycles (s_memtime) and ns.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int MODE>
__global__ void k(uint64_t *out, int iters) {
  extern __shared__ __align__(16) uint32_t t[];
  const int n = 32768;
  for (int i = threadIdx.x; i < n; i += blockDim.x) t[i] = (i * 2654435761u + 12345u) & (n - 1);
  __syncthreads();
  uint32_t x = (threadIdx.x * 977u) & (n - 1);
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; it++) {
    if (MODE == 0) x = t[x];                                  // ds_read_b32 chase
    else if (MODE == 1) x = atomicAdd(&t[x], 0u) & (n - 1);  // ds_add_rtn chase
    else { const uint4 v = *(const uint4 *)&t[x & ~3u]; x = (v.x ^ v.y ^ v.z ^ v.w) & (n - 1); }  // b128 chase
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
  if (x == 0xffffffffu) out[0] = x;
}

template <int MODE>
void run(const char *name, int threads) {
  uint64_t *d;
  (void)hipMalloc(&d, 256 * 8);
  const int iters = 2000;
  (void)hipFuncSetAttribute((const void *)k<MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072);
  k<MODE><<<256, threads, 131072>>>(d, iters);
  (void)hipDeviceSynchronize();
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  (void)hipEventRecord(a);
  k<MODE><<<256, threads, 131072>>>(d, iters);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  uint64_t h[256];
  (void)hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  double avg = 0;
  for (int i = 0; i < 256; i++) avg += h[i];
  avg /= 256;
  printf("%-10s waves/CU %2d: %7.1f memtime-ticks/RT  %7.1f ns/RT (wall)\n", name, threads / 64, avg / iters,
         ms * 1e6 / iters);
  (void)hipFree(d);
}

int main() {
  for (int th : {64, 256, 512, 1024}) run<0>("b32 chase", th);
  for (int th : {64, 256, 1024}) run<1>("rtn chase", th);
  for (int th : {64, 256, 1024}) run<2>("b128 chase", th);
  return 0;
}
