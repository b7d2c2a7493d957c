// Host interface of the gfx950 kernels (kernels.hip) for the batch pipeline (pipeline.cpp).
//
// One DeviceRules per device holds the compiled rule set's tables in HBM (K1 literal
// automaton, K2 rule-group DFAs, the Global.AllowPath DFA, gates).  A batch runs on one
// DeviceLane (its own HIP stream and HBM buffers); enqueue_scan puts the whole device part
// of a batch on that stream with no host round trip:
//
//   H2D (pinned slot -> HBM) and one H2D of the file offsets  prep (zero fills, coarse file
//   map)  K1  keyword gates  event-chunk compaction  item counts  item layout
//   (device-side)  item lists  K2  outputs (candidates, keyword bits, overflow / skip
//   flags, counters: written straight into pinned, host-mapped memory)
//
// and records the batch's completion event.  Two lanes per device let the H2D of one batch
// overlap the kernels of the other.
#pragma once
#include <hip/hip_runtime_api.h>

#include <cstdint>
#include <memory>
#include <vector>

#include "plan.hpp"

namespace tsg {

struct DeviceRules;

// Pinned host memory of one batch's device outputs, which the outputs kernel writes straight
// into host-mapped memory (no runtime D2H copy).
struct HostOut {
  uint8_t* blk = nullptr;       // host-mapped block: counts | gskip | ovf | kw
  uint8_t* blk_dev = nullptr;   // its device address
  uint32_t* kw = nullptr;       // [files_cap * kw_words]
  uint8_t* ovf = nullptr;       // [files_cap] 1 = resolve the file whole
  uint8_t* gskip = nullptr;     // [groups] 1 = K2 skipped the group (item capacity)
  Candidate* cand = nullptr;    // [cand_cap] host-mapped: K2 candidates copied out
  Candidate* cand_dev = nullptr;  // device address of `cand`
  uint32_t* counts = nullptr;   // [48] 0 candidates, 1 event chunks, 2 K2 list entries,
                                // 3 dense entries, 5 items, 6 entries, 7 skipped groups,
                                // 8-11 K2 diagnostics (TSG_K2_DIAG), 14-15 K1X, 16-17 K1F,
                                // 32-39 kernel clock stamps (u64)
  uint32_t files_cap = 0, cand_cap = 0, groups = 0, kw_words = 0;
  uint32_t wall_khz = 0;        // the device wall clock's rate (hipDeviceAttributeWallClockRate)
  // stage boundaries of the batch on its lane's stream: data H2D | offsets H2D | prep |
  // wait for the previous batch's kernels | K1 | gates | K2 | outputs; ev[kEvDone]
  // completes the batch
  hipEvent_t ev[9] = {};
};

constexpr int kEvDone = 8;
// per-batch K2 diagnostics (K2 work that is not the chunks themselves)
struct K2Diag {
  unsigned long long tail_bytes, tail_max, long_tails, replays;
};

struct ScanInput {
  const uint8_t* data;       // pinned host, `total` bytes
  const uint64_t* off;       // [nfiles + 1]
  uint32_t nfiles;
  uint64_t total;
  const char* paths;         // pinned host
  const uint64_t* poff;      // [nfiles + 1]
  // the slot's whole pinned data buffer (data == room): enqueue_scan writes the zero tail
  // and a copy of the offsets behind the batch there, so one H2D carries all three
  uint8_t* room = nullptr;
  uint64_t room_bytes = 0;
};

// pinned bytes a slot's data buffer keeps past its capacity for that tail and the offsets
inline uint64_t slot_room_bytes(uint32_t files_cap) { return (128u << 10) + 8ull * ((uint64_t)files_cap + 1) + 64; }

struct ScanTimes {  // HIP-event milliseconds of one batch on its lane
  float h2d = 0, meta = 0, wait = 0, prep = 0, k1 = 0, gates = 0, k2 = 0, out = 0;
  // device wall clock (stamped inside the kernels): K1F's first block start to last block
  // end; K1F start to K2's last block end; the gates pass's start to K2's end
  float k1_clk = 0, chain_clk = 0, post_k1_clk = 0;
};

struct LaneState;  // HBM buffers + stream + events of one lane

int device_rules_create(int device, const Plan& plan, uint32_t chunk, uint32_t ext_cap,
                        uint32_t adapt_mib, DeviceRules** out);
void device_rules_destroy(DeviceRules* d);
// keyword bits K1 no longer reports after its adaptation (null before / without it)
std::shared_ptr<const std::vector<uint8_t>> device_rules_kw_unknown(const DeviceRules* d);
uint32_t device_rules_hot_states(const DeviceRules* d);
// true: K1 runs as K1F (k1f_kernel, batches under 4 GiB); false: the automaton (k1_kernel)
bool device_rules_k1_filter(const DeviceRules* d);

int lane_create(DeviceRules* d, LaneState** out);
void lane_destroy(LaneState* l);
hipStream_t lane_stream(LaneState* l);

int host_out_alloc(const DeviceRules* d, uint32_t files_cap, HostOut* out);
void host_out_free(HostOut* o);

// The device part of one batch on lane `l`, asynchronously; out->ev[kEvDone] completes it.
int enqueue_scan(DeviceRules* d, LaneState* l, const ScanInput& in, HostOut* out);
// after out->ev[kEvDone]: the HIP-event times of that batch's stages
int batch_times(const HostOut* out, ScanTimes* t);
// keyword bits of the lane's last batch, as K1 / K1X left them on the device (test hook)
int lane_kw(LaneState* l, uint32_t* kw, size_t n);
// K1 output of the lane's last batch (test hook): chunk events [nchunks]
int lane_events(LaneState* l, uint32_t* ev, size_t n);
// K2 per-entry trace of the lane's last batch (TSG_K2_TRACE; empty otherwise): per entry
// {start, end, group << 32 | items, XCC_ID << 32 | HW_ID}
int lane_k2_trace(LaneState* l, std::vector<unsigned long long>* out);
int lane_k1f_trace(LaneState* l, std::vector<unsigned long long>* out);  // TSG_K1F_TRACE

}  // namespace tsg
