// Test and measurement knobs (tsg_test_knob, include/trivy_secret.h): process-wide
// switches that change how the library computes, never what.  They are set through the C
// API only; nothing here reads the environment, so a process that loads the library (a Go
// binary over cgo) cannot have its plans or kernels changed by stray environment variables.
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>

#include "internal.hpp"

namespace tsg {

Knobs& knobs() {
  static Knobs k;
  return k;
}

std::string knob_kw_unknown() {
  Knobs& k = knobs();
  std::lock_guard<std::mutex> g(k.m);
  return k.emu_kw_unknown;
}

}  // namespace tsg

extern "C" int tsg_test_knob(const char* name, const char* value) {
  using namespace tsg;
  if (!name) return fail(TSG_ERR_ARG, "bad argument");
  const std::string v = value ? value : "";
  const long long x = v.empty() ? 0 : strtoll(v.c_str(), nullptr, 10);
  Knobs& k = knobs();
  if (!strcmp(name, "tar_range_kib")) k.tar_range_kib = x;
  else if (!strcmp(name, "piece_mib")) k.piece_mib = x;
  else if (!strcmp(name, "pike_only")) k.pike_only = x;
  else if (!strcmp(name, "no_k1x")) k.no_k1x = x;
  else if (!strcmp(name, "emu_wordrec")) k.emu_wordrec = x;
  else if (!strcmp(name, "k1_automaton")) k.k1_automaton = x;
  else if (!strcmp(name, "group_states")) k.group_states = x;
  else if (!strcmp(name, "k1f_list")) k.k1f_list = x;  // K1F lists the event chunks (no gates pass)
  else if (!strcmp(name, "k1f_grid")) {  // cap on K1F's blocks: many tiles per wave in small tests
    if (x < 0) return fail(TSG_ERR_ARG, "k1f_grid must be >= 0");
    k.k1f_grid = x;
  }
  else if (!strcmp(name, "group_table_kib")) {
    if (x < 0 || x > 64) return fail(TSG_ERR_ARG, "group_table_kib must be 0..64");
    k.group_table_kib = x;
  }
  else if (!strcmp(name, "x_step")) {
    if (x != 0 && x != 1 && x != 2 && x != 4) return fail(TSG_ERR_ARG, "x_step must be 0, 1, 2 or 4");
    k.x_step = x;
  }
  else if (!strcmp(name, "emu_kw_unknown")) {
    std::lock_guard<std::mutex> g(k.m);
    k.emu_kw_unknown = v;
  } else {
    return fail(TSG_ERR_ARG, std::string("unknown knob: ") + name);
  }
  return TSG_OK;
}
