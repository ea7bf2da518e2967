// The dispatch-switch table of libmde_hip (tuning.h) and its C ABI.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>

#include "../../include/mde.h"
#include "tuning.h"

namespace mde {

namespace {

struct KnobDef {
  const char* name;  // ABI name; environment variable MDE_<NAME upper-case>
  const char* env;
  int def;
  int lo, hi;  // accepted range
};

constexpr KnobDef kKnobs[KNOB_COUNT] = {
    {"splitk", "MDE_SPLITK", 1, 0, 1},
    {"lnfold", "MDE_LNFOLD", 1, 0, 1},
    {"conv_narrow", "MDE_CONV_NARROW", 1, 0, 1},
    {"upconv", "MDE_UPCONV", 1, 0, 1},
    {"gemm256", "MDE_GEMM256", 1, 0, 2},
    {"deep64", "MDE_DEEP64", 1, 0, 1},
    {"w8small", "MDE_W8SMALL", 1, 0, 1},
    {"conv_persist", "MDE_CONV_PERSIST", 1, 0, 2},
    {"panel", "MDE_PANEL", 1, 0, 2},
    {"panel32", "MDE_PANEL32", 0, 0, 1},
    {"narrow_resid", "MDE_NARROW_RESID", 1, 0, 1},
    {"attn16", "MDE_ATTN16", 1, 0, 1},
    {"splitk_fused", "MDE_SPLITK_FUSED", 0, 0, 1},
    {"attn_tail", "MDE_ATTN_TAIL", 2, 0, 2},
    {"resize_fold", "MDE_RESIZE_FOLD", 1, 0, 1},
};

std::atomic<int> g_val[KNOB_COUNT];
std::once_flag g_once;

void init_once() {
  std::call_once(g_once, [] {
    for (int i = 0; i < KNOB_COUNT; ++i) {
      int v = kKnobs[i].def;
      if (const char* e = std::getenv(kKnobs[i].env)) {  // the library's only environment read
        char* end = nullptr;
        const long x = std::strtol(e, &end, 10);
        if (end != e && *end == '\0' && x >= kKnobs[i].lo && x <= kKnobs[i].hi)
          v = (int)x;
        else  // a rejected value is reported, never silently dropped
          std::fprintf(stderr, "[mde] %s=%s ignored (accepted: integer %d..%d); using %d\n", kKnobs[i].env, e,
                       kKnobs[i].lo, kKnobs[i].hi, v);
      }
      g_val[i].store(v, std::memory_order_relaxed);
    }
  });
}

int find(const char* name) {
  if (!name) return -1;
  for (int i = 0; i < KNOB_COUNT; ++i)
    if (std::strcmp(kKnobs[i].name, name) == 0) return i;
  return -1;
}

}  // namespace

int knob(Knob k) {
  init_once();
  return g_val[k].load(std::memory_order_relaxed);
}

}  // namespace mde

extern "C" {

int mde_tuning_set(const char* name, int value) {
  mde::init_once();
  const int i = mde::find(name);
  if (i < 0) return MDE_ERR_NAME;
  if (value < mde::kKnobs[i].lo || value > mde::kKnobs[i].hi) return MDE_ERR_ARG;
  mde::g_val[i].store(value, std::memory_order_relaxed);
  return MDE_OK;
}

int mde_tuning_get(const char* name, int* value) {
  mde::init_once();
  const int i = mde::find(name);
  if (i < 0) return MDE_ERR_NAME;
  if (!value) return MDE_ERR_ARG;
  *value = mde::g_val[i].load(std::memory_order_relaxed);
  return MDE_OK;
}

}  // extern "C"
