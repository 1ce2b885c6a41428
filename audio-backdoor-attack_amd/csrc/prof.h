// Optional per-phase HIP-event timing of libabd launches (bench.py roofline).
#pragma once
#include <hip/hip_runtime.h>

namespace abd {
enum Phase {
  PH_STFT_MEL = 0, PH_DB_DCT, PH_ROW_SCALE, PH_PREP_W, PH_CONV1_STATS, PH_CONV1_POOL, PH_CONV2_FWD,
  PH_BN2_POOL, PH_CONV3_FWD, PH_BN3_POOL, PH_FC1_FWD, PH_FC2_LOSS, PH_METRICS, PH_FC2_BWD, PH_FC1_WGRAD,
  PH_FC1_DGRAD, PH_BN3_BWD, PH_CONV3_WGRAD, PH_CONV3_DGRAD, PH_BN2_BWD, PH_CONV2_WGRAD, PH_CONV2_DGRAD,
  PH_CONV1_BWD, PH_ADAM, PH_FINALIZE, PH_HEAD_FWD, PH_HEAD_MID, PH_HEAD_BWD, PH_HEAD_DGRAD, PH_COUNT
};
extern unsigned long long g_prof_mask;
void prof_record(int phase, bool begin, hipStream_t s);
inline void prof_begin(int phase, hipStream_t s) {
  if (g_prof_mask & (1ull << phase)) prof_record(phase, true, s);
}
inline void prof_end(int phase, hipStream_t s) {
  if (g_prof_mask & (1ull << phase)) prof_record(phase, false, s);
}
}  // namespace abd
