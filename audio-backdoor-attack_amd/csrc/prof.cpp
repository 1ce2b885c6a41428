// Per-phase HIP-event timing (see prof.h).  Events are recorded on the stream each
// kernel is launched on, so a bracket measures exactly that launch.
#include "prof.h"

#include <mutex>
#include <vector>

#include "../../include/abd.h"

namespace abd {
unsigned long long g_prof_mask = 0;
namespace {
struct Rec {
  int phase;
  hipEvent_t b, e;
};
std::mutex g_mu;
std::vector<hipEvent_t> g_pool;
std::vector<Rec> g_recs;
size_t g_next = 0;
int g_open[64];
long long g_seen[64];  // begins per phase since start (sampling: every g_every-th is bracketed)
int g_every = 1;
// Step-sampled mode (abd_profile_step called at least once since start): a begin is bracketed iff
// the current step index is a multiple of g_every, so EVERY launch of a phase in a sampled step is
// timed.  Counting launches instead aliases with the step's launch pattern: a phase launched k
// times per step with gcd(k, every) > 1 would always bracket the same call site.
long long g_step = 0;
bool g_by_step = false;
}  // namespace

void prof_record(int phase, bool begin, hipStream_t s) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (begin) {
    const long long k = g_by_step ? g_step : g_seen[phase]++;
    if (k % g_every != 0) {  // not sampled: the matching end records nothing
      g_open[phase] = -1;
      return;
    }
    if (g_next + 2 > g_pool.size()) return;  // pool exhausted: stop recording
    Rec r{phase, g_pool[g_next], g_pool[g_next + 1]};
    g_next += 2;
    (void)hipEventRecord(r.b, s);
    g_open[phase] = (int)g_recs.size();
    g_recs.push_back(r);
  } else {
    const int i = g_open[phase];
    if (i >= 0 && i < (int)g_recs.size() && g_recs[i].phase == phase) (void)hipEventRecord(g_recs[i].e, s);
    g_open[phase] = -1;
  }
}
}  // namespace abd

extern "C" {
int abd_profile_start(unsigned long long phase_mask, int max_records) {
  return abd_profile_start_every(phase_mask, max_records, 1);
}

int abd_profile_start_every(unsigned long long phase_mask, int max_records, int every) {
  if (every < 1 || max_records < 0) return ABD_E_INVALID;
  std::lock_guard<std::mutex> lk(abd::g_mu);
  abd::g_every = every;
  abd::g_step = 0;
  abd::g_by_step = false;
  for (int i = 0; i < 64; ++i) abd::g_seen[i] = 0;
  for (auto e : abd::g_pool) (void)hipEventDestroy(e);
  abd::g_pool.clear();
  abd::g_recs.clear();
  abd::g_next = 0;
  for (int i = 0; i < 64; ++i) abd::g_open[i] = -1;
  abd::g_pool.resize(2 * (size_t)max_records);
  // timing-only events: no system-scope release / acquire at record (hipEventDisableSystemFence).
  // With the default fence every bracket wrote the L2's dirty lines back: 6-10 us of idle GPU
  // around each bracketed launch (rocprofv3 traces of the bench, round 5), inside the timed steps
  for (auto& e : abd::g_pool) {
    hipError_t rc = hipEventCreateWithFlags(&e, hipEventDisableSystemFence);
    if (rc != hipSuccess) return (int)rc;
  }
  abd::g_prof_mask = phase_mask;
  return 0;
}

int abd_profile_step(void) {
  std::lock_guard<std::mutex> lk(abd::g_mu);
  if (abd::g_by_step) ++abd::g_step;
  abd::g_by_step = true;  // the first call marks step 0's start
  return 0;
}

int abd_profile_stop(double* total_ms, int* counts, int n_phases) {
  std::lock_guard<std::mutex> lk(abd::g_mu);
  abd::g_prof_mask = 0;
  for (int i = 0; i < n_phases; ++i) {
    total_ms[i] = 0.0;
    counts[i] = 0;
  }
  int rc = 0;
  for (auto& r : abd::g_recs) {
    if (hipEventSynchronize(r.e) != hipSuccess) {
      rc = 1;
      continue;
    }
    float ms = 0.0f;
    if (hipEventElapsedTime(&ms, r.b, r.e) == hipSuccess && r.phase < n_phases) {
      total_ms[r.phase] += ms;
      counts[r.phase] += 1;
    }
  }
  for (auto e : abd::g_pool) (void)hipEventDestroy(e);
  abd::g_pool.clear();
  abd::g_recs.clear();
  abd::g_next = 0;
  return rc;
}
}
