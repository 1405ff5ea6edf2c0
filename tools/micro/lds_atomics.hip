// Microbenchmark: LDS random-access throughput on gfx950 (ds_add rtn / no-rtn, ds_read_b128, ds_read_b64).
// One 1024-thread workgroup per CU, 128 KB LDS table, 4096 ops per thread; reports cycles per wave-op.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int MODE>
__global__ __launch_bounds__(1024) void k(uint64_t *out, int iters) {
  extern __shared__ __align__(16) uint32_t t[];
  const int n = 32768;  // u32 words (128 KB)
  for (int i = threadIdx.x; i < n; i += 1024) t[i] = i;
  __syncthreads();
  uint32_t x = threadIdx.x * 0x9E3779B9u + blockIdx.x;
  uint32_t acc = 0;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; it++) {
    x = x * 1664525u + 1013904223u;
    const uint32_t a = (x >> 8) & (n - 1);
    if (MODE == 0) atomicAdd(&t[a], 1u);                       // no return
    else if (MODE == 1) acc += atomicAdd(&t[a], 1u);           // return, used
    else if (MODE == 2) { const uint4 v = *(const uint4 *)&t[a & ~3u]; acc += v.x ^ v.w; }
    else if (MODE == 3) { const uint2 v = *(const uint2 *)&t[a & ~1u]; acc += v.x ^ v.y; }
    else if (MODE == 4) { acc += atomicCAS(&t[a], acc, acc + 1); }
    else if (MODE == 5) { atomicAdd((unsigned long long *)&t[a & ~1u], 1ull); }
    else if (MODE == 6) { t[a] = acc; }
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
  if (acc == 0xdeadbeef) out[0] = acc;
}

template <int MODE>
void run(const char *name) {
  uint64_t *d;
  hipMalloc(&d, 256 * 8);
  const int iters = 4096;
  hipFuncSetAttribute((const void *)k<MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072);
  k<MODE><<<256, 1024, 131072>>>(d, iters);
  hipDeviceSynchronize();
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  hipEventRecord(a);
  k<MODE><<<256, 1024, 131072>>>(d, iters);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  uint64_t h[256]; hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  double avg = 0; for (int i = 0; i < 256; i++) avg += h[i]; avg /= 256;
  const double ops = 256.0 * 1024 * iters;
  // cycles per CU per wave-op: 16 waves per CU, iters ops each
  printf("%-24s %8.3f ms  %7.2f G lane-ops/s  %6.2f CU-cycles/wave-op (memtime)\n", name, ms, ops / ms / 1e6,
         avg / (16.0 * iters));
  hipFree(d);
}

int main() {
  run<0>("ds_add_u32 (no rtn)");
  run<1>("ds_add_rtn_u32");
  run<2>("ds_read_b128");
  run<3>("ds_read_b64");
  run<4>("ds_cmpst_rtn_b32");
  run<5>("ds_add_u64 (no rtn)");
  run<6>("ds_write_b32");
  return 0;
}
