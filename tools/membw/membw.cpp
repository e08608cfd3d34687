// Host memory-bandwidth probe: read / write / copy GB/s
// of this process's CPU share with 1..N threads over buffers far beyond the
// caches, so the end-to-end path's "host stages are DRAM-bound" reading can
// be checked against a measured ceiling. Build: g++ -O3 -march=native
// -pthread tools/membw/membw.cpp -o tools/membw/membw
//   ./membw [threads...]   (one JSON line per thread count)
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <thread>
#include <vector>

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const size_t bytes = (size_t)1 << 31;  // 2 GiB per buffer
  const size_t n = bytes / 8;
  uint64_t* a = (uint64_t*)aligned_alloc(4096, bytes);
  uint64_t* b = (uint64_t*)aligned_alloc(4096, bytes);
  if (!a || !b) return 1;
  std::vector<int> ths;
  for (int i = 1; i < argc; ++i) ths.push_back(atoi(argv[i]));
  if (ths.empty()) ths = {1, 4, 8, 16};
  // first touch by the widest thread count (pages spread like the workload's)
  {
    const int T = *std::max_element(ths.begin(), ths.end());
    std::vector<std::thread> w;
    for (int t = 0; t < T; ++t)
      w.emplace_back([=] {
        const size_t lo = n * t / T, hi = n * (t + 1) / T;
        for (size_t i = lo; i < hi; ++i) { a[i] = i; b[i] = 0; }
      });
    for (auto& x : w) x.join();
  }
  volatile uint64_t sink = 0;
  for (int T : ths) {
    double best[3] = {0, 0, 0};
    for (int rep = 0; rep < 3; ++rep) {
      for (int k = 0; k < 3; ++k) {
        std::vector<std::thread> w;
        std::vector<uint64_t> part(T, 0);
        const double t0 = now();
        for (int t = 0; t < T; ++t)
          w.emplace_back([&, t] {
            const size_t lo = n * t / T, hi = n * (t + 1) / T;
            if (k == 0) {  // read
              uint64_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;
              for (size_t i = lo; i + 3 < hi; i += 4) { s0 += a[i]; s1 += a[i + 1]; s2 += a[i + 2]; s3 += a[i + 3]; }
              part[t] = s0 + s1 + s2 + s3;
            } else if (k == 1) {  // write
              memset(b + lo, (int)t, (hi - lo) * 8);
            } else {  // copy
              memcpy(b + lo, a + lo, (hi - lo) * 8);
            }
          });
        for (auto& x : w) x.join();
        const double dt = now() - t0;
        for (uint64_t v : part) sink += v;
        const double moved = (k == 2 ? 2.0 : 1.0) * (double)bytes;
        best[k] = std::max(best[k], moved / dt / 1e9);
      }
    }
    printf("{\"threads\": %d, \"read_gbs\": %.1f, \"write_gbs\": %.1f, \"copy_gbs\": %.1f, \"buffer_gib\": 2}\n", T,
           best[0], best[1], best[2]);
    fflush(stdout);
  }
  return (int)(sink & 0);
}
