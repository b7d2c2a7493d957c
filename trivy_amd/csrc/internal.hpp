// Shared internals of the C ABI (capi.cpp, gpu.hip).
#pragma once
#include <atomic>
#include <cstdint>
#include <memory>
#include <mutex>
#include <string>

#include "../../include/trivy_secret.h"
#include "plan.hpp"
#include "scanner.hpp"

struct tsg_ruleset {
  tsg::Ruleset rs;
  std::unique_ptr<tsg::Plan> plan;
};

struct tsg_result {
  std::string buf;
};

namespace tsg {
void set_error(const std::string& msg);
int fail(int code, const std::string& msg);
// the rule set a context was created with (pipeline.cpp)
const tsg_ruleset* ctx_ruleset(const tsg_ctx* c);
// bytes of a default pinned slot (tsg_ctx_options.slot_mib)
uint64_t ctx_slot_bytes(const tsg_ctx* c);

// test and measurement knobs (knobs.cpp, tsg_test_knob); 0 = default
struct Knobs {
  std::atomic<int64_t> tar_range_kib{0}, piece_mib{0}, pike_only{0}, no_k1x{0}, emu_wordrec{0},
      x_step{0}, k1_automaton{0}, group_states{0}, group_table_kib{0}, k1f_grid{0},
      k1f_list{0};
  std::mutex m;
  std::string emu_kw_unknown;
};
Knobs& knobs();
std::string knob_kw_unknown();
}  // namespace tsg
