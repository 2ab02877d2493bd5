// Run-time switches and tuning knobs of the library, in one registry.
//
// the entry points are reentrant and keep no unsynchronised global mutable state.
// Every switch the dispatch code reads lives here as a std::atomic<int> (relaxed loads and stores:
// a reader racing a setter sees the old or the new value, never a torn one), initialised once --
// thread-safe static initialisation -- from its DORKNET_* environment variable, else the built-in
// default.  dk_debug_set_gemm_config(kind, v) (kind = the KnobId) overrides a knob for A/B runs;
// v = -1 puts the default back.  Nothing on the training path writes a knob.
#include <stdlib.h>

#include <atomic>

#include "dk_common.h"

namespace dk {
namespace {

struct KnobDef {
  const char* env;  // environment variable giving the default (nullptr: none)
  int dflt;         // built-in default
};

// Indexed by KnobId (dk_common.h).
constexpr KnobDef kDefs[kNumKnobs] = {
    {nullptr, -1},                       // kKnobRowCfg: forward / dgrad GEMM tile (-1 = heuristic)
    {nullptr, -1},                       // kKnobSplitCfg: split-K weight-gradient tile (-1 = heuristic)
    {nullptr, 1},                        // kKnobFillSplits: split-K grids sized to one round of resident blocks
    {"DORKNET_PW_STREAM", 1},            // kKnobPwStream: streaming K = C = 64 pointwise kernels
    {"DORKNET_NT_STORES", kNtDefault},   // kKnobNtStores: nontemporal output stores, a bitmask of NtFam
    {"DORKNET_PWS_BWD_PF", 0},           // kKnobPwsBwdPf: the streaming fused backward's operand prefetch
    {nullptr, 0},                        // 6: unused
    {"DORKNET_DWB_BLOCKS", 768},         // kKnobDwbBlocks: blocks the fused depthwise backward aims for
    {nullptr, -1},                       // kKnobDwSeg: depthwise-forward output rows per thread (-1 = rule)
    {"DORKNET_PW_STREAM_BF16", 1},       // kKnobPwsh: bf16 streaming pointwise kernels
    {nullptr, 0},                        // 10: unused (the round-3 column-sliced bf16 kernels, deleted)
    {"DORKNET_PW_DEEP", 1},              // kKnobPwDeep: fp32 weight-stationary deep pointwise kernels
    {nullptr, 0},                        // 12: unused (the output-stationary deep weight gradient, deleted)
    {"DORKNET_PW_DEEP_BF16", 1},         // kKnobPwDeep16: bf16 weight-stationary deep pointwise kernels
    {"DORKNET_PW_DEEP_BWD", 1},          // kKnobPwDeepBwd: fused deep pointwise backward (dgrad + wgrad)
    {"DORKNET_PW_STREAM128", 1},         // kKnobPwStream128: streaming forward at K = C = 128
    {"DORKNET_PWF_PREFETCH", -1},        // kKnobPwfPrefetch: tiled fused backward prefetch (-1 = per shape)
    {"DORKNET_PWF_BLOCKS_PER_CU", 0},    // kKnobPwfBlocksPerCu: its resident blocks per CU (0 = occupancy)
    {"DORKNET_WGRAD_BLOCKS", 1024},      // kKnobWgradBlocks: blocks a split-K weight gradient aims for
    {nullptr, 22},                       // kKnobEwVariant: launch variant of dk_bn_bwd_apply_f32
    {"DORKNET_PW_BF16_BWD", 1},          // kKnobPwsh16Bwd: fused bf16 pointwise backward (1: K = C = 64 and
                                          // K in {128, 256}; 2: K = C = 64 only; 0: off)
    {"DORKNET_DWB_COLS", 2},             // kKnobDwbCols: columns per thread of the fused depthwise backward
    {"DORKNET_MULTI_REDUCE", 1},         // kKnobMultiReduce: a flush's reduces in one launch (0: one each)
};

struct Table {
  std::atomic<int> v[kNumKnobs];
  int dflt[kNumKnobs];
  Table() {
    for (int i = 0; i < kNumKnobs; ++i) {
      const char* e = kDefs[i].env ? getenv(kDefs[i].env) : nullptr;
      dflt[i] = (e && *e) ? atoi(e) : kDefs[i].dflt;
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
