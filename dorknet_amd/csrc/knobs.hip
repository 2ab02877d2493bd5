// Path selectors and tuning knobs of the library, in one registry.
//
// the entry points are reentrant and keep no unsynchronised global mutable state.
// Every knob the dispatch code reads lives here as a std::atomic<int> (relaxed loads and stores: a
// reader racing a setter sees the old or the new value, never a torn one) holding its built-in
// default.  dk_debug_set_gemm_config(kind, v) (kind = the KnobId) overrides a knob for tests and A/B
// runs; v = -1 puts the default back.  Nothing on the training path writes a knob, and no environment
// variable reaches one (the run-time switches are the Python layer's).
#include <atomic>

#include "dk_common.h"

namespace dk {
namespace {

// Built-in defaults, indexed by KnobId (dk_common.h); the retired numbers hold 0.
constexpr int kDefaults[kNumKnobs] = {
    -1,          // kKnobRowCfg: forward / dgrad GEMM tile (-1 = heuristic)
    -1,          // kKnobSplitCfg: split-K weight-gradient tile (-1 = heuristic)
    1,           // kKnobFillSplits: split-K grids sized to one round of resident blocks
    1,           // kKnobPwStream: streaming K = C = 64 / 128 pointwise kernels (0: the tiled engine)
    kNtDefault,  // kKnobNtStores: nontemporal output stores, a bitmask of NtFam
    0,           // 5: retired (the streaming fused backward's prefetch switch, neutral)
    0,           // 6: unused
    768,         // kKnobDwbBlocks: blocks the fused depthwise backward aims for
    -1,          // kKnobDwSeg: depthwise-forward output rows per thread (-1 = rule)
    1,           // kKnobPwsh: bf16 streaming pointwise kernels
    0,           // 10: unused
    1,           // kKnobPwDeep: fp32 weight-stationary deep pointwise kernels
    0,           // 12: retired (deep pointwise walkers per resident slot: more than one round was slower)
    1,           // kKnobPwDeep16: bf16 weight-stationary deep pointwise kernels
    1,           // kKnobPwDeepBwd: fused deep pointwise backward (dgrad + wgrad)
    0,           // 15-17: retired (K = C = 128 streaming-forward switch; tiled fused backward prefetch and
    0,           //        occupancy overrides)
    0,           //
    1024,        // kKnobWgradBlocks: blocks a split-K weight gradient aims for
    22,          // kKnobEwVariant: launch variant of dk_bn_bwd_apply_f32
    0,           // 20: retired (fused bf16 pointwise backward selector)
    2,           // kKnobDwbCols: columns per thread of the fused depthwise backward
    0,           // 22: retired (one launch per deferred reduce)
};

struct Table {
  std::atomic<int> v[kNumKnobs];
  int dflt[kNumKnobs];
  Table() {
    for (int i = 0; i < kNumKnobs; ++i) {
      dflt[i] = kDefaults[i];
      v[i].store(dflt[i], std::memory_order_relaxed);
    }
  }
};

Table& table() {
  static Table t;  // initialised once, thread-safe
  return t;
}

}  // namespace

int knob(int id) { return table().v[id].load(std::memory_order_relaxed); }

void knob_set(int id, int v) {
  Table& t = table();
  t.v[id].store(v < 0 ? t.dflt[id] : v, std::memory_order_relaxed);
}

int nt_stores(int fam) { return (knob(kKnobNtStores) >> fam) & 1; }

}  // namespace dk
