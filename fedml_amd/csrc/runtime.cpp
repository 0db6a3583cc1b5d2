// libfedml_runtime.so — host-side native runtime for fedml_amd.
//
//  * fr_trace_*  : fixed-capacity, lock-free (single atomic cursor) ring buffer of
//                  begin/end events with steady-clock ns timestamps.
//  * fr_schedule : best-first branch-and-bound assignment of client workloads to
//                  heterogeneous GPUs under per-GPU memory budgets, minimising the
//                  makespan (the intent of the reference's unused
//                  `core/schedule/scheduler.py:4-172`, here with a priority queue,
//                  a node budget and an LPT fallback so 100+ clients stay tractable).
//  * fr_layout   : 256-byte aligned flat-arena offsets for an ordered tensor list.
//
// Plain C ABI, loaded with ctypes (no torch headers → compiles in ~1 s).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <numeric>
#include <pthread.h>
#include <queue>
#include <vector>

namespace {

struct TraceEv {
  int64_t ts;
  int64_t tid;
  int32_t id;
  int32_t phase;
};

std::vector<TraceEv> g_ring;
std::atomic<uint64_t> g_cursor{0};
std::mutex g_init_mu;

inline int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

}  // namespace

extern "C" {

int fr_version() { return 1; }

void fr_trace_init(int64_t capacity) {
  std::lock_guard<std::mutex> lk(g_init_mu);
  if (capacity < 16) capacity = 16;
  if ((int64_t)g_ring.size() != capacity) g_ring.assign((size_t)capacity, TraceEv{0, 0, 0, 0});
  g_cursor.store(0);
}

void fr_trace_event(int32_t id, int32_t phase) {
  if (g_ring.empty()) return;
  uint64_t slot = g_cursor.fetch_add(1, std::memory_order_relaxed);
  TraceEv& e = g_ring[slot % g_ring.size()];
  e.ts = now_ns();
  e.tid = (int64_t)pthread_self();
  e.id = id;
  e.phase = phase;
}

int64_t fr_trace_count() {
  uint64_t c = g_cursor.load();
  return (int64_t)std::min<uint64_t>(c, g_ring.size());
}

// copy events oldest→newest
int64_t fr_trace_copy(int64_t* ts, int32_t* ids, int32_t* phase, int64_t* tid, int64_t max_n) {
  uint64_t c = g_cursor.load();
  uint64_t n = std::min<uint64_t>(c, g_ring.size());
  n = std::min<uint64_t>(n, (uint64_t)max_n);
  uint64_t start = c - n;
  for (uint64_t i = 0; i < n; ++i) {
    const TraceEv& e = g_ring[(start + i) % g_ring.size()];
    ts[i] = e.ts;
    ids[i] = e.id;
    phase[i] = e.phase;
    tid[i] = e.tid;
  }
  return (int64_t)n;
}

void fr_trace_clear() { g_cursor.store(0); }

int64_t fr_now_ns() { return now_ns(); }

// ---------------------------------------------------------------------------------
// Scheduler.
//   workloads[n]  : work units per client (e.g. samples × FLOP/sample)
//   speed[m]      : time per work unit on resource j (reference "constraints")
//   memory[m]     : memory budget of resource j (same unit as mem_per_wl)
//   mem_per_wl[n] : memory footprint of each client when resident
//   mode 0 = serial (clients on one GPU run back-to-back: cost adds)
//   mode 1 = packed (resident clients run concurrently: memory adds, cost = makespan)
// out_assign[n] ← resource index per client (original order). Returns the makespan,
// or -1 if infeasible.
// ---------------------------------------------------------------------------------
double fr_schedule(int32_t n, const double* workloads, const double* mem_per_wl, int32_t m,
                   const double* speed, const double* memory, int32_t mode, int64_t node_budget,
                   int32_t* out_assign) {
  if (n <= 0 || m <= 0) return 0.0;
  std::vector<int32_t> order(n);
  std::iota(order.begin(), order.end(), 0);
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return workloads[a] > workloads[b]; });

  struct Node {
    double bound;               // max cost over resources (monotone → admissible)
    int32_t depth;              // number of assigned (sorted) workloads
    std::vector<double> cost;   // per-resource time
    std::vector<double> mem;    // per-resource resident memory
    std::vector<int32_t> assign;
  };
  auto cmp = [](const Node& a, const Node& b) {
    if (a.bound != b.bound) return a.bound > b.bound;
    return a.depth < b.depth;  // prefer deeper on ties → reaches leaves quickly
  };
  std::priority_queue<Node, std::vector<Node>, decltype(cmp)> pq(cmp);
  Node root{0.0, 0, std::vector<double>(m, 0.0), std::vector<double>(m, 0.0), std::vector<int32_t>(n, -1)};
  pq.push(root);
  int64_t expanded = 0;
  bool found = false;
  Node best;
  while (!pq.empty()) {
    Node cur = pq.top();
    pq.pop();
    if (cur.depth == n) {
      best = cur;
      found = true;
      break;
    }
    if (++expanded > node_budget) {
      // budget exhausted: finish this node greedily (LPT: least loaded feasible resource)
      for (int d = cur.depth; d < n; ++d) {
        int w = order[d];
        int pick = -1;
        double pick_cost = 0;
        for (int j = 0; j < m; ++j) {
          double nm = (mode == 1) ? cur.mem[j] + mem_per_wl[w] : std::max(cur.mem[j], mem_per_wl[w]);
          if (nm > memory[j]) continue;
          double c = cur.cost[j] + speed[j] * workloads[w];
          if (pick < 0 || c < pick_cost) { pick = j; pick_cost = c; }
        }
        if (pick < 0) return -1.0;
        cur.cost[pick] = pick_cost;
        cur.mem[pick] = (mode == 1) ? cur.mem[pick] + mem_per_wl[w] : std::max(cur.mem[pick], mem_per_wl[w]);
        cur.assign[w] = pick;
      }
      cur.depth = n;
      cur.bound = *std::max_element(cur.cost.begin(), cur.cost.end());
      best = cur;
      found = true;
      break;
    }
    int w = order[cur.depth];
    for (int j = 0; j < m; ++j) {
      // mode 1: clients stay resident together → memory accumulates;
      // mode 0: clients run one after another → only one footprint at a time.
      double nm = (mode == 1) ? cur.mem[j] + mem_per_wl[w] : std::max(cur.mem[j], mem_per_wl[w]);
      if (nm > memory[j]) continue;
      Node nx = cur;
      nx.depth = cur.depth + 1;
      nx.mem[j] = nm;
      nx.cost[j] = cur.cost[j] + speed[j] * workloads[w];  // a GPU's throughput is shared either way
      nx.assign[w] = j;
      nx.bound = *std::max_element(nx.cost.begin(), nx.cost.end());
      pq.push(std::move(nx));
    }
  }
  if (!found) return -1.0;
  for (int i = 0; i < n; ++i) out_assign[i] = best.assign[i];
  return best.bound;
}

// Flat-arena layout: offsets (in elements) for tensors of numel[i] elements of
// elem_bytes each, every tensor starting on an `align`-byte boundary. Returns total elements.
int64_t fr_layout(int32_t n, const int64_t* numel, int32_t elem_bytes, int32_t align, int64_t* out_offsets) {
  int64_t align_el = std::max<int64_t>(1, align / std::max(1, elem_bytes));
  int64_t off = 0;
  for (int i = 0; i < n; ++i) {
    off = (off + align_el - 1) / align_el * align_el;
    out_offsets[i] = off;
    off += numel[i];
  }
  return (off + align_el - 1) / align_el * align_el;
}

}  // extern "C"
