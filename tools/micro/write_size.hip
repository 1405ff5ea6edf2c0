// Calibration of rocprofv3's write counters (TCC_EA0_WRREQ, TCC_EA0_WRREQ_64B) on gfx950 for the store shapes of
// k_extract_scatter at k = 21: coalesced u32 and u8 streams, and the extraction's run pattern (every workgroup writes a
// run of R records into each of 256 bins; a bin's runs from the workgroups of one XCD are consecutive in its segment,
// consecutive lanes store consecutive records of a run). Each kernel writes a known byte count; the PMC pass over
// this program gives the counters per dispatch. Test infrastructure, not part of the library.
//   hipcc --offload-arch=gfx950 -O3 tools/micro/write_size.hip -o tools/micro/write_size
//   rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum -- tools/micro/write_size
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <algorithm>

#define CHECK(x)                                                                        \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));         \
      return 1;                                                                         \
    }                                                                                   \
  } while (0)

__global__ void k_stream_u32(uint32_t *out, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    out[i] = (uint32_t)i;
}
__global__ void k_stream_u8(uint8_t *out, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    out[i] = (uint8_t)i;
}

// NB bins, R records per bin per workgroup, 8 segments per bin (workgroup b writes segment b % 8, the XCD it runs on)
constexpr int NB = 256, NT = 256;
template <int R, bool U8PLANE>
__global__ __launch_bounds__(NT) void k_runs(uint32_t *w, uint8_t *x, unsigned long long *cursor) {
  __shared__ unsigned long long goff[NB];
  const uint32_t sub = blockIdx.x % 8;
  for (int d = threadIdx.x; d < NB; d += NT) goff[d] = atomicAdd(&cursor[sub * NB + d], (unsigned long long)R);
  __syncthreads();
  for (int p = threadIdx.x; p < NB * R; p += NT) {
    const int d = p / R, r = p - d * R;
    const unsigned long long dst = goff[d] + r;
    w[dst] = (uint32_t)(dst * 2654435761u);
    if (U8PLANE) x[dst] = (uint8_t)dst;
  }
}

template <int R, bool U8PLANE>
static int run_runs(uint32_t *w, uint8_t *x, unsigned long long *cur, uint32_t grid) {
  const uint64_t cap = (uint64_t)(grid / 8) * R;  // records of one (bin, segment)
  unsigned long long h[8 * NB];
  for (int s = 0; s < 8; s++)
    for (int d = 0; d < NB; d++) h[s * NB + d] = ((uint64_t)d * 8 + s) * cap;
  CHECK(hipMemcpy(cur, h, sizeof(h), hipMemcpyHostToDevice));
  k_runs<R, U8PLANE><<<grid, NT>>>(w, x, cur);
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  const double recs = (double)grid * NB * R;
  printf("runs R=%d%s: %.0f records, %.3f GB written (u32%s)\n", R, U8PLANE ? " +u8" : "", recs,
         recs * (U8PLANE ? 5 : 4) / 1e9, U8PLANE ? " + u8 planes" : " plane");
  return 0;
}

int main() {
  const uint64_t n32 = 256ull << 20, n8 = 1ull << 30;  // 1 GiB each
  const uint32_t grid = 8 * 2048;                        // workgroups of the run kernels (a multiple of 8)
  const uint64_t rmax = (uint64_t)grid * NB * 28;
  uint32_t *w;
  uint8_t *x;
  unsigned long long *cur;
  CHECK(hipMalloc(&w, std::max(n32 * 4, rmax * 4)));
  CHECK(hipMalloc(&x, std::max(n8, rmax)));
  CHECK(hipMalloc(&cur, 8 * NB * 8));
  k_stream_u32<<<4096, 256>>>(w, n32);
  CHECK(hipDeviceSynchronize());
  printf("stream u32: %.3f GB written\n", n32 * 4 / 1e9);
  k_stream_u8<<<4096, 256>>>(x, n8);
  CHECK(hipDeviceSynchronize());
  printf("stream u8: %.3f GB written\n", n8 / 1e9);
  if (run_runs<14, false>(w, x, cur, grid) || run_runs<14, true>(w, x, cur, grid) ||
      run_runs<28, false>(w, x, cur, grid) || run_runs<28, true>(w, x, cur, grid))
    return 1;
  CHECK(hipFree(w));
  CHECK(hipFree(x));
  CHECK(hipFree(cur));
  return 0;
}
