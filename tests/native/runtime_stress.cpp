// Host-side sanitizer harness for csrc/runtime.cpp (race detection / sanitizers).
// Built twice by tests/test_native_sanitizers.py: -fsanitize=thread (the lock-free trace ring under
// 8 concurrent writer threads) and -fsanitize=address,undefined (scheduler + arena layout).
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <thread>
#include <vector>

extern "C" {
void fr_trace_init(int64_t capacity);
void fr_trace_event(int32_t id, int32_t phase);
int64_t fr_trace_count();
int64_t fr_trace_copy(int64_t* ts, int32_t* ids, int32_t* phase, int64_t* tid, int64_t max_n);
double fr_schedule(int32_t n, const double* workloads, const double* mem_per_wl, int32_t m, const double* speed,
                   const double* memory, int32_t mode, int64_t node_budget, int32_t* out_assign);
int64_t fr_layout(int32_t n, const int64_t* numel, int32_t elem_bytes, int32_t align, int64_t* out_offsets);
void fr_sc_reset();
void fr_sc_access(int64_t addr, int64_t nbytes, int32_t stream, int32_t write, int32_t tag);
void fr_sc_wait(int32_t dst, int32_t src);
void fr_sc_sync(int32_t stream);
int64_t fr_sc_hazard_count();
int64_t fr_sc_access_count();
}

#define CHECK(c)                                              \
  do {                                                        \
    if (!(c)) {                                               \
      std::fprintf(stderr, "CHECK failed: %s (line %d)\n", #c, __LINE__); \
      return 1;                                               \
    }                                                         \
  } while (0)

int main() {
  // 1. concurrent trace writers (no wrap-around: every event gets its own slot)
  const int T = 8, E = 20000;
  fr_trace_init((int64_t)T * E * 2);
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t)
    th.emplace_back([t] {
      for (int i = 0; i < E; ++i) fr_trace_event(t * E + i, i & 1);
    });
  for (auto& x : th) x.join();
  const int64_t n = fr_trace_count();
  CHECK(n == (int64_t)T * E);
  std::vector<int64_t> ts(n), tid(n);
  std::vector<int32_t> ids(n), ph(n);
  CHECK(fr_trace_copy(ts.data(), ids.data(), ph.data(), tid.data(), n) == n);
  std::vector<int> seen((size_t)T * E, 0);
  for (int64_t i = 0; i < n; ++i) {
    CHECK(ids[i] >= 0 && ids[i] < T * E);
    seen[ids[i]]++;
  }
  for (int v : seen) CHECK(v == 1);

  // 2. scheduler: random heterogeneous instances, every workload assigned within memory
  std::mt19937 rng(1234);
  std::uniform_real_distribution<double> U(0.5, 2.0);
  for (int trial = 0; trial < 50; ++trial) {
    const int nw = 1 + trial % 40, m = 1 + trial % 8;
    std::vector<double> w(nw), mem(nw), sp(m), cap(m);
    double tot = 0;
    for (int i = 0; i < nw; ++i) {
      w[i] = U(rng);
      mem[i] = U(rng);
      tot += mem[i];
    }
    for (int j = 0; j < m; ++j) {
      sp[j] = U(rng);
      cap[j] = tot;  // feasible
    }
    std::vector<int32_t> a(nw, -1);
    const double mk = fr_schedule(nw, w.data(), mem.data(), m, sp.data(), cap.data(), trial & 1, 20000, a.data());
    CHECK(mk > 0);
    for (int i = 0; i < nw; ++i) CHECK(a[i] >= 0 && a[i] < m);
  }

  // 3. arena layout: aligned, non-overlapping
  std::vector<int64_t> numel = {7, 1, 4096, 3, 100000, 0, 5};
  std::vector<int64_t> off(numel.size());
  const int64_t total = fr_layout((int32_t)numel.size(), numel.data(), 4, 256, off.data());
  int64_t end = 0;
  for (size_t i = 0; i < numel.size(); ++i) {
    CHECK((off[i] * 4) % 256 == 0);
    CHECK(off[i] >= end);
    end = off[i] + numel[i];
  }
  CHECK(total >= end);
  // 4. stream checker fed from 8 host threads (each its own stream and buffers; a final unordered
  //    cross-stream write per thread must be reported exactly once per thread)
  fr_sc_reset();
  {
    std::vector<std::thread> sc;
    for (int t = 0; t < 8; ++t)
      sc.emplace_back([t] {
        for (int i = 0; i < 2000; ++i) fr_sc_access(0x100000 * (t + 1) + 64 * (i % 50), 64, t, i & 1, 0);
      });
    for (auto& x : sc) x.join();
  }
  CHECK(fr_sc_hazard_count() == 0);
  CHECK(fr_sc_access_count() == 8 * 2000);
  for (int t = 0; t < 8; ++t) fr_sc_access(0x100000 * (t + 1), 64, 100 + t, 1, 1);
  CHECK(fr_sc_hazard_count() == 8);
  std::printf("runtime stress ok: %lld trace events, 50 schedules, layout total %lld\n", (long long)n,
              (long long)total);
  return 0;
}
