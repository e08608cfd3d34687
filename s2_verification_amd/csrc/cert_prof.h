// cert_prof.h — certification phase counters for profiling builds only
// (make EXTRA=-DS2LC_CERT_PROF; tools/cert_probe.py reads what
// collect_results prints). Without the define every macro is empty.
#pragma once
#include <stdint.h>
#ifdef S2LC_CERT_PROF
#include <x86intrin.h>
#include <atomic>
namespace s2lc {
extern std::atomic<uint64_t> g_cert_prof[16];
}
#define CP_DECL(t) uint64_t t = __rdtsc()
#define CP_LAP(i, t) do { const uint64_t _n = __rdtsc(); s2lc::g_cert_prof[i].fetch_add(_n - (t), std::memory_order_relaxed); (t) = _n; } while (0)
#define CP_CNT(i, v) s2lc::g_cert_prof[i].fetch_add(v, std::memory_order_relaxed)
#else
#define CP_CNT(i, v) do {} while (0)
#define CP_DECL(t) do {} while (0)
#define CP_LAP(i, t) do {} while (0)
#endif
