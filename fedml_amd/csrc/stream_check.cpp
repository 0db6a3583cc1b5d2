// Stream-ordering checker ("HIP stream-ordering assertions — an event-dependency checker in
// debug builds"). The reference has no GPU concurrency to check; this engine overlaps RCCL collectives
// (comm stream) with compute (compute stream) and captures graphs on side streams, so a missing
// event wait is a silent data race on HBM buffers. The checker is a vector-clock race detector over
// HIP streams (the FastTrack idea applied to streams instead of threads):
//
//   * every stream s has a logical clock E[s], advanced by each access it issues;
//   * VC[s][t] = the newest epoch of stream t that s is ordered after (set by an event wait
//     s ← t, transitively merged; a device/host synchronise orders every stream after everything);
//   * every buffer (address range) remembers its last write (stream, epoch) and the last read epoch
//     of every stream since that write;
//   * an access of stream s conflicts if the buffer's last write — or, for a write, any read since —
//     came from another stream t at an epoch VC[s][t] has not reached: RAW / WAW / WAR hazard.
//
// Host-side only (it sees the launch order, not the GPU): the ops layer reports each kernel's tensors
// and stream, the comm layer reports event waits. Off by default; FEDML_AMD_STREAM_CHECK=1 enables it.
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <unordered_map>
#include <vector>

namespace {

struct Access {
  int32_t stream = -1;
  int64_t epoch = 0;
};

struct Buffer {
  int64_t end = 0;                              // [begin, end)
  Access write;                                 // last write
  std::unordered_map<int32_t, int64_t> reads;   // stream → last read epoch since the last write
};

struct Hazard {
  int32_t kind;       // 0 RAW, 1 WAW, 2 WAR
  int32_t stream;     // accessing stream
  int32_t other;      // stream of the unordered earlier access
  int64_t addr;
  int32_t tag;        // caller-supplied op id
};

struct Checker {
  std::mutex mu;
  std::unordered_map<int32_t, int64_t> epoch;                               // E[s]
  std::unordered_map<int32_t, std::unordered_map<int32_t, int64_t>> vc;     // VC[s][t]
  std::map<int64_t, Buffer> bufs;                                           // begin → buffer
  std::vector<Hazard> hazards;
  int64_t n_access = 0;

  std::unordered_map<int32_t, int64_t> floor_;   // host-synchronised epoch of each stream (orders everyone)

  int64_t ordered(int32_t s, int32_t t) {   // newest epoch of t that s is ordered after
    if (s == t) return INT64_MAX;
    auto ft = floor_.find(t);
    const int64_t fl = ft == floor_.end() ? 0 : ft->second;
    auto it = vc.find(s);
    if (it == vc.end()) return fl;
    auto jt = it->second.find(t);
    return std::max(fl, jt == it->second.end() ? (int64_t)0 : jt->second);
  }

  void report(int32_t kind, int32_t s, int32_t t, int64_t addr, int32_t tag) {
    if (hazards.size() < 4096) hazards.push_back({kind, s, t, addr, tag});
  }

  // overlapping buffers of [b, e): exact-range entries are reused, partial overlaps are checked too
  void access(int64_t b, int64_t e, int32_t s, int write, int32_t tag) {
    const int64_t ep = ++epoch[s];
    ++n_access;
    bool exact = false;
    // linear scan of the ranges that start before e (nested views — an arena and its slices — overlap
    // arbitrarily; a debug tool can afford O(#buffers) per launch)
    for (auto it = bufs.begin(); it != bufs.end() && it->first < e; ++it) {
      Buffer& buf = it->second;
      if (buf.end <= b) continue;
      const Access& w = buf.write;
      if (w.stream >= 0 && w.stream != s && ordered(s, w.stream) < w.epoch) report(write ? 1 : 0, s, w.stream, b, tag);
      if (write) {
        for (auto& r : buf.reads)
          if (r.first != s && ordered(s, r.first) < r.second) report(2, s, r.first, b, tag);
      }
      if (it->first == b && buf.end == e) exact = true;
    }
    if (!exact) {
      Buffer nb;
      nb.end = e;
      bufs[b] = nb;
    }
    Buffer& buf = bufs[b];
    if (write) {
      buf.write = {s, ep};
      buf.reads.clear();
    } else {
      buf.reads[s] = ep;
    }
  }

  // stream `dst` waits for everything `src` has issued so far (hipStreamWaitEvent on an event recorded
  // on src now); ordering is transitive: dst also inherits what src was ordered after
  void wait(int32_t dst, int32_t src, int64_t upto = -1) {
    if (dst == src) return;
    auto& d = vc[dst];
    const int64_t cur = upto >= 0 ? std::min(upto, epoch[src]) : epoch[src];
    d[src] = std::max(d[src], cur);
    auto it = vc.find(src);
    if (it != vc.end())
      for (auto& kv : it->second)
        if (kv.first != dst) d[kv.first] = std::max(d[kv.first], kv.second);
  }

  // host synchronisation of `s` (hipStreamSynchronize) followed by work on any stream: everything s
  // issued is ordered before all later accesses; s = -1 → device-wide synchronise
  void sync(int32_t s) {
    for (auto& et : epoch)
      if (s < 0 || et.first == s) floor_[et.first] = std::max(floor_[et.first], et.second);
  }
};

Checker* g_chk = nullptr;
std::mutex g_init;

Checker& chk() {
  std::lock_guard<std::mutex> lk(g_init);
  if (!g_chk) g_chk = new Checker();
  return *g_chk;
}

}  // namespace

extern "C" {

void fr_sc_reset() {
  Checker& c = chk();
  std::lock_guard<std::mutex> lk(c.mu);
  c.epoch.clear();
  c.vc.clear();
  c.bufs.clear();
  c.hazards.clear();
  c.floor_.clear();
  c.n_access = 0;
}

void fr_sc_access(int64_t addr, int64_t nbytes, int32_t stream, int32_t write, int32_t tag) {
  if (nbytes <= 0) return;
  Checker& c = chk();
  std::lock_guard<std::mutex> lk(c.mu);
  c.access(addr, addr + nbytes, stream, write, tag);
}

void fr_sc_wait(int32_t dst, int32_t src) {
  Checker& c = chk();
  std::lock_guard<std::mutex> lk(c.mu);
  c.wait(dst, src);
}

// event form: dst waits for an event recorded on src when src's clock read `epoch` (fr_sc_epoch)
void fr_sc_wait_epoch(int32_t dst, int32_t src, int64_t epoch) {
  Checker& c = chk();
  std::lock_guard<std::mutex> lk(c.mu);
  c.wait(dst, src, epoch);
}

int64_t fr_sc_epoch(int32_t stream) {
  Checker& c = chk();
  std::lock_guard<std::mutex> lk(c.mu);
  return c.epoch[stream];
}

void fr_sc_sync(int32_t stream) {
  Checker& c = chk();
  std::lock_guard<std::mutex> lk(c.mu);
  c.sync(stream);
}

// forget a freed allocation (the caching allocator hands the range to a new tensor)
void fr_sc_release(int64_t addr, int64_t nbytes) {
  Checker& c = chk();
  std::lock_guard<std::mutex> lk(c.mu);
  auto it = c.bufs.lower_bound(addr);
  while (it != c.bufs.end() && it->first < addr + nbytes) it = c.bufs.erase(it);
}

int64_t fr_sc_hazard_count() {
  Checker& c = chk();
  std::lock_guard<std::mutex> lk(c.mu);
  return (int64_t)c.hazards.size();
}

int64_t fr_sc_access_count() {
  Checker& c = chk();
  std::lock_guard<std::mutex> lk(c.mu);
  return c.n_access;
}

// copy up to max_n hazards as rows of (kind, stream, other, tag) + addresses
int64_t fr_sc_hazards(int32_t* kind_stream_other_tag, int64_t* addr, int64_t max_n) {
  Checker& c = chk();
  std::lock_guard<std::mutex> lk(c.mu);
  const int64_t n = std::min<int64_t>(max_n, (int64_t)c.hazards.size());
  for (int64_t i = 0; i < n; ++i) {
    const Hazard& h = c.hazards[i];
    kind_stream_other_tag[4 * i + 0] = h.kind;
    kind_stream_other_tag[4 * i + 1] = h.stream;
    kind_stream_other_tag[4 * i + 2] = h.other;
    kind_stream_other_tag[4 * i + 3] = h.tag;
    addr[i] = h.addr;
  }
  return n;
}

}  // extern "C"
