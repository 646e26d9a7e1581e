// Host memcpy bandwidth between malloc'd and hipHostMalloc'd buffers, 1 and N threads
// (how the engine's PXRB pass should read fetched columns).  tools/, GPU box.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

static double Copy(uint8_t* dst, const uint8_t* src, size_t n, int th) {
  auto t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> v;
  for (int k = 0; k < th; ++k)
    v.emplace_back([=] { std::memcpy(dst + n / th * k, src + n / th * k, n / th); });
  for (auto& t : v) t.join();
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

int main() {
  const size_t n = size_t(192) << 20;
  uint8_t *m1 = static_cast<uint8_t*>(malloc(n)), *m2 = static_cast<uint8_t*>(malloc(n));
  uint8_t *p1 = nullptr, *p2 = nullptr, *p3 = nullptr;
  if (hipHostMalloc(&p1, n, hipHostMallocDefault) != hipSuccess || hipHostMalloc(&p2, n, hipHostMallocDefault) != hipSuccess ||
      hipHostMalloc(&p3, n, hipHostMallocNonCoherent) != hipSuccess)
    return 1;
  memset(m1, 1, n); memset(m2, 2, n); memset(p1, 3, n); memset(p2, 4, n); memset(p3, 5, n);
  struct C { const char* name; uint8_t* d; const uint8_t* s; } cases[] = {
      {"malloc->malloc", m2, m1}, {"pinned->malloc", m2, p1}, {"malloc->pinned", p2, m1}, {"pinned->pinned", p2, p1},
      {"pinnedNC->pinned", p2, p3}, {"pinned->pinnedNC", p3, p1}};
  for (auto& c : cases)
    for (int th : {1, 4, 8, 16}) {
      double best = 1e9;
      for (int r = 0; r < 3; ++r) best = std::min(best, Copy(c.d, c.s, n, th));
      std::printf("%-18s threads %2d  %6.1f GB/s\n", c.name, th, n / best / 1e9);
    }
  return 0;
}
