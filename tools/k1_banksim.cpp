// K1 LDS bank-conflict simulator (measurement tool, not product code).
//
// Replays K1's lane -> byte-stream mapping (quad lanes on consecutive 4 KiB items, two
// chains per lane on the item's 2 KiB segments) over a batch with the rule set's literal
// automaton, and counts for every wave instruction the extra LDS cycles of the class read
// and the transition read under the current table layout and under candidate layouts.
// ds_read_b32 / ds_read_u16 banks are (byte address / 4) mod 32, serviced per 32-lane half;
// an instruction costs one cycle per half plus (max distinct dwords on one bank - 1).
//
// Built by tools/k1_banksim.py into /tmp and loaded next to libtrivy_secret.so.
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <vector>

#include "../trivy_amd/csrc/internal.hpp"

namespace {

struct Half {
  // distinct dwords per bank in one 32-lane half
  uint32_t seen[32][32];
  uint32_t cnt[32];
  void reset() { std::memset(cnt, 0, sizeof(cnt)); }
  void add(uint32_t dword) {
    const uint32_t b = dword & 31;
    for (uint32_t k = 0; k < cnt[b]; k++)
      if (seen[b][k] == dword) return;
    if (cnt[b] < 32) seen[b][cnt[b]++] = dword;
  }
  uint32_t extra() const {
    uint32_t m = 0;
    for (int b = 0; b < 32; b++) m = std::max(m, cnt[b]);
    return m ? m - 1 : 0;
  }
};

}  // namespace

extern "C" int k1_banksim(const tsg_ruleset* rs, const uint8_t* data, uint64_t n, uint32_t waves,
                          double* out, uint32_t nout) {
  const tsg::Plan& p = *rs->plan;
  const tsg::DFA& d = *p.kw_dfa;
  const uint32_t nc = (uint32_t)d.nclasses, ns = (uint32_t)d.nstates;
  uint32_t stride = nc;
  while (stride % 4 != 2) stride++;
  // device numbering: reporting states (they end a literal) last
  std::vector<uint32_t> id(ns);
  uint32_t k = 0;
  for (int pass = 0; pass < 2; pass++)
    for (uint32_t s = 0; s < ns; s++)
      if ((d.eot_acc[s] != 0) == (pass == 1)) id[s] = k++;
  const uint32_t start = d.start[0];
  const uint32_t seg = 8 * 256, item = 2 * seg;
  // per-state visit counts (hot rows) and the statistics below
  std::vector<uint64_t> visits(ns, 0);
  double cls_extra = 0, tab_extra = 0, tab_extra_nostart = 0, tab_extra_hot8 = 0, steps = 0;
  double lanes_start = 0, lane_steps = 0, distinct_states = 0, distinct_dw = 0;
  double cls_extra_u8x4 = 0;
  Half h;
  // pass 1: visit counts for the hot-row variant; pass 2: conflicts
  std::vector<uint8_t> hot(ns, 0);
  for (int pass = 0; pass < 2; pass++) {
    if (pass == 1) {
      std::vector<uint32_t> order(ns);
      for (uint32_t s = 0; s < ns; s++) order[s] = s;
      std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return visits[a] > visits[b]; });
      for (uint32_t i = 0; i < 8 && i < ns; i++) hot[order[i]] = 1;
    }
    for (uint32_t w = 0; w < waves; w++) {
      const uint64_t base = (uint64_t)w * 64 * item;
      if (base + 64 * item > n) break;
      uint32_t st[64][2];
      for (int l = 0; l < 64; l++) st[l][0] = st[l][1] = start;
      for (uint32_t j = 0; j < seg; j++) {
        for (int c = 0; c < 2; c++) {
          uint8_t by[64];
          for (int l = 0; l < 64; l++) by[l] = data[base + (uint64_t)l * item + (uint64_t)c * seg + j];
          if (pass == 1) {
            for (int half = 0; half < 2; half++) {
              // class read: u32 table at 0, byte * 4
              h.reset();
              for (int l = half * 32; l < half * 32 + 32; l++) h.add(by[l]);
              cls_extra += h.extra();
              // u8 class table, 4 bytes per dword
              h.reset();
              for (int l = half * 32; l < half * 32 + 32; l++) h.add(by[l] >> 2);
              cls_extra_u8x4 += h.extra();
              // transition read: u16 at 1024 + 2 * (row + class)
              h.reset();
              uint32_t nd = 0;
              std::map<uint32_t, int> sset;
              for (int l = half * 32; l < half * 32 + 32; l++) {
                const uint32_t s = st[l][c];
                h.add((1024 + 2 * (id[s] * stride + d.cls[by[l]])) / 4);
                sset[s]++;
              }
              for (int b = 0; b < 32; b++) nd += h.cnt[b];
              tab_extra += h.extra();
              distinct_states += sset.size();
              distinct_dw += nd;
              // lanes in the start state take their next state from the class word instead
              h.reset();
              for (int l = half * 32; l < half * 32 + 32; l++) {
                const uint32_t s = st[l][c];
                h.add(s == start ? 256 : (1024 + 2 * (id[s] * stride + d.cls[by[l]])) / 4);
              }
              tab_extra_nostart += h.extra();
              // ... and lanes in the 8 hottest rows from a replicated image (no conflict)
              h.reset();
              for (int l = half * 32; l < half * 32 + 32; l++) {
                const uint32_t s = st[l][c];
                h.add(hot[s] ? 256 : (1024 + 2 * (id[s] * stride + d.cls[by[l]])) / 4);
              }
              tab_extra_hot8 += h.extra();
              steps += 1;
              for (int l = half * 32; l < half * 32 + 32; l++) lanes_start += st[l][c] == start;
              lane_steps += 32;
            }
          }
          for (int l = 0; l < 64; l++) {
            const uint32_t s = d.next[(size_t)st[l][c] * nc + d.cls[by[l]]];
            st[l][c] = s;
            if (pass == 0) visits[s]++;
          }
        }
      }
    }
  }
  const double v[] = {steps,
                      cls_extra / steps * 2,          // per wave instruction (2 halves)
                      cls_extra_u8x4 / steps * 2,
                      tab_extra / steps * 2,
                      tab_extra_nostart / steps * 2,
                      tab_extra_hot8 / steps * 2,
                      lanes_start / lane_steps,
                      distinct_states / steps,
                      distinct_dw / steps,
                      (double)ns,
                      (double)nc};
  for (uint32_t i = 0; i < nout && i < sizeof(v) / sizeof(v[0]); i++) out[i] = v[i];
  return 0;
}
