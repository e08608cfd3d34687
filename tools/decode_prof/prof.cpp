// Host decode anatomy (no GPU): single-thread time of load_jsonl (the JSONL
// scan into events + pool) and History::finalize (renumber, chains, records),
// and of load_jsonl_finalized (the direct decode into the finalized form)
// over C4-shaped histories written by tools/decode_prof/gen.py:
//   make -C tools/decode_prof && python3 tools/decode_prof/gen.py /tmp/c4.bin 500 &&
//   tools/decode_prof/prof /tmp/c4.bin [reps]
#include <chrono>
#include <stdio.h>
#include <stdlib.h>
#include <string>
#include <vector>

#include "history.h"

using namespace s2lc;
using Clk = std::chrono::steady_clock;

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  std::vector<std::vector<uint8_t>> blobs;
  for (;;) {
    uint64_t n;
    if (fread(&n, 8, 1, f) != 1) break;
    blobs.emplace_back(n);
    if (fread(blobs.back().data(), 1, n, f) != n) return 2;
  }
  fclose(f);
  const int reps = argc > 2 ? atoi(argv[2]) : 5;
  size_t bytes = 0;
  for (auto& b : blobs) bytes += b.size();
  std::vector<History> hs(blobs.size());
  double best_scan = 1e9, best_fin = 1e9, best_dir = 1e9;
  for (int r = 0; r < reps; ++r) {
    double scan = 0, fin = 0;
    for (size_t i = 0; i < blobs.size(); ++i) {
      hs[i].recycle();
      std::string err;
      const auto t0 = Clk::now();
      if (load_jsonl(blobs[i].data(), blobs[i].size(), hs[i], err)) { fprintf(stderr, "%s\n", err.c_str()); return 1; }
      const auto t1 = Clk::now();
      if (hs[i].finalize()) return 1;
      const auto t2 = Clk::now();
      scan += std::chrono::duration<double>(t1 - t0).count();
      fin += std::chrono::duration<double>(t2 - t1).count();
    }
    best_scan = std::min(best_scan, scan);
    best_fin = std::min(best_fin, fin);
    double dir = 0;
    for (size_t i = 0; i < blobs.size(); ++i) {
      hs[i].recycle();
      std::string err;
      const auto t0 = Clk::now();
      if (load_jsonl_finalized(blobs[i].data(), blobs[i].size(), hs[i], err)) return 1;
      dir += std::chrono::duration<double>(Clk::now() - t0).count();
    }
    best_dir = std::min(best_dir, dir);
  }
  const double n = (double)blobs.size();
  printf("{\"histories\": %zu, \"bytes_per_history\": %.0f, \"scan_us\": %.2f, \"finalize_us\": %.2f, "
         "\"scan_GBps\": %.3f, \"histories_per_s_thread\": %.0f, \"finalized_us\": %.2f}\n",
         blobs.size(), bytes / n, 1e6 * best_scan / n, 1e6 * best_fin / n, bytes / best_scan / 1e9,
         n / (best_scan + best_fin), 1e6 * best_dir / n);
  return 0;
}
