// Where the KmerMap hand-off's host time goes: on this host, with T threads,
//   fault   first touch of fresh 2 MB-aligned anonymous memory advised for huge pages (one store per 4 KB page),
//   write   a parallel sequential write of the same bytes once they are mapped,
//   memcpy  a parallel copy of half the bytes into the other half (read + write),
// for `bytes` (default 1.5 GB, the C2 KmerMap<32>'s slot array). Prints one JSON line.
//   fill_probe [bytes] [threads]
#include <sys/mman.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <thread>
#include <vector>

static double ms_since(std::chrono::steady_clock::time_point t) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

template <typename F>
static double par(int T, F f) {
  auto t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> th;
  for (int t = 0; t < T; t++) th.emplace_back(f, t);
  for (auto &x : th) x.join();
  return ms_since(t0);
}

int main(int argc, char **argv) {
  const size_t bytes = argc > 1 ? strtoull(argv[1], nullptr, 10) : (size_t)1536 << 20;
  const int T = argc > 2 ? atoi(argv[2]) : 16;
  const size_t sz = (bytes + (2u << 20) - 1) & ~(size_t)((2u << 20) - 1);
  std::string thp = "?";
  {
    std::ifstream f("/sys/kernel/mm/transparent_hugepage/enabled");
    if (f) std::getline(f, thp);
  }
  auto map = [&]() {
    void *p = mmap(nullptr, sz, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (p == MAP_FAILED) exit(2);
    (void)madvise(p, sz, MADV_HUGEPAGE);
    return (char *)p;
  };
  char *a = map();
  const size_t per = sz / T;
  const double fault = par(T, [&](int t) {
    for (size_t i = t * per; i < (t + 1) * per; i += 4096) a[i] = 1;
  });
  const double write = par(T, [&](int t) { memset(a + t * per, 7, per); });
  const size_t half = sz / 2, ph = half / T;
  const double cpy = par(T, [&](int t) { memcpy(a + half + t * ph, a + t * ph, ph); });
  munmap(a, sz);
  char *b = map();
  const double fault_write = par(T, [&](int t) { memset(b + t * per, 7, per); });
  munmap(b, sz);
  printf("{\"bytes\": %zu, \"threads\": %d, \"thp\": \"%s\", \"fault_ms\": %.2f, \"write_ms\": %.2f, \"write_GBps\": %.1f, "
         "\"memcpy_half_ms\": %.2f, \"fresh_write_ms\": %.2f}\n",
         sz, T, thp.c_str(), fault, write, sz / (write * 1e-3) / 1e9, cpy, fault_write);
  return 0;
}
