// Host pipeline of the GPU path (include/trivy_secret.h): pinned slots, device lanes,
// batch submission / collection, and the queue that coalesces concurrent per-file callers.
//
// A batch = the files of one pinned slot.  Submitting it puts its whole device part on one
// lane's stream (device.hpp enqueue_scan: H2D, K1, gates, device-side layout, K2, outputs
// back to pinned host buffers) and starts its host job, which waits for the lane's
// completion event and resolves the candidates exactly (plan.cpp resolve_batch).  With
// two lanes, the H2D of batch i+1 overlaps the kernels of batch i, and the host
// resolution of earlier batches runs on the resolver pool meanwhile.  Nothing here waits
// for the device except the jobs (and tsg_batch_kernels, a synchronous test hook).
//
// Replaces, on the reference side, the per-file io.ReadAll + Scan of
// SecretAnalyzer.Analyze (pkg/fanal/analyzer/secret/secret.go:85-101) run from the
// analyzer's per-file goroutines (pkg/fanal/analyzer/analyzer.go:419-443).
#include <hip/hip_runtime_api.h>
#include <malloc.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <set>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "device.hpp"
#include "internal.hpp"

namespace tsg {

#define HIP_TRY(x)                                                                    \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess)                                                             \
      return fail(TSG_ERR_GPU, std::string(#x) + ": " + hipGetErrorString(e_));       \
  } while (0)

namespace {

enum SlotOwner : int { kFree = 0, kCaller = 1, kUpload = 2, kQueue = 3 };

// Pinned host staging of one batch (context-owned; the caller writes into it directly
// with the slot API, or the context copies into it).
struct Slot {
  uint8_t* data = nullptr;
  uint64_t data_cap = 0;
  uint64_t* off = nullptr;
  uint32_t files_cap = 0;
  char* paths = nullptr;
  uint64_t paths_cap = 0;
  uint64_t* poff = nullptr;
  bool pinned = false;
  int inflight = 0;  // submissions whose host job has not finished
  int owner = kFree;
  std::thread::id holder;  // thread that took it (kCaller / kUpload)
  // files the library itself wrote into the slot (upload, queue); kUnknownFill when the
  // caller writes it (tsg_slot_acquire).  Only a submission of exactly those files, with no
  // other submission of the slot in flight, may use the slot's bytes past its batch for the
  // zero tail and the offsets (enqueue_scan's single H2D): nothing the caller owns is there.
  uint32_t filled = 0;
};
constexpr uint32_t kUnknownFill = 0xFFFFFFFFu;

// ScanInput of a submission of the slot's first nfiles files (lock held)
ScanInput slot_input(const Slot& s, uint32_t nfiles) {
  const bool room = s.inflight == 0 && s.filled == nfiles;
  return ScanInput{s.data, s.off, nfiles, s.off[nfiles], s.paths, s.poff, room ? s.data : nullptr,
                   room ? s.data_cap + slot_room_bytes(s.files_cap) : 0};
}

// One submission of a slot.
struct Batch {
  uint32_t slot = 0;
  uint32_t nfiles = 0;
  uint64_t bytes = 0;
  int out = -1;          // HostOut index (device mode)
  bool keep_result = false;  // queue: keep the BatchResult instead of serializing
  uint64_t ticket = 0;
  // completion: set by the batch's job thread once its results (or error) are final
  std::mutex dm;
  std::condition_variable dcv;
  bool done = false;
  std::function<void(const std::shared_ptr<Batch>&)> on_done;  // called after `done`
  int rc = TSG_OK;
  std::string err;
  std::unique_ptr<tsg_result> res;
  BatchResult br;
  ScanTimes t;
  uint32_t counts[48] = {};
  double resolve_ms = 0;
  uint64_t files_found = 0;
};

uint64_t round_up(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }

}  // namespace
}  // namespace tsg

using namespace tsg;

struct tsg_ctx {
  mutable std::mutex m;
  std::condition_variable cv;
  int device = 0;
  bool emulate = false;
  const tsg_ruleset* rs = nullptr;
  tsg_ctx_options opt{};
  int nt = 16;
  DeviceRules* dr = nullptr;
  std::vector<LaneState*> lanes;
  uint64_t seq = 0;
  std::vector<std::unique_ptr<Slot>> slots;
  std::vector<HostOut> outs;
  std::vector<char> out_busy;
  std::map<uint64_t, std::shared_ptr<Batch>> pending;  // submitted, uncollected, by ticket
  uint64_t next_ticket = 1;
  int jobs = 0;                                // host jobs submitted and not finished (any API)
  tsg_stats stats{};
  // completion threads: a fixed set (one per device lane; 4 for an emulated context) takes
  // the submitted host jobs in order; each job waits for its batch's device completion,
  // then resolves it on the process-wide pool
  std::deque<std::function<void()>> jq;
  std::vector<std::thread> workers;
  bool stopping = false;
  std::multiset<std::thread::id> slot_waiters;  // threads waiting in slot_take

  ~tsg_ctx() {
    {
      std::unique_lock<std::mutex> lk(m);
      cv.wait(lk, [&] { return jobs == 0; });
      stopping = true;
    }
    cv.notify_all();
    for (auto& t : workers) t.join();
    if (!emulate) (void)hipSetDevice(device);
    for (auto* l : lanes) lane_destroy(l);
    for (auto& o : outs) host_out_free(&o);
    for (auto& s : slots) {
      void* ps[] = {s->data, s->off, s->paths, s->poff};
      for (void* p : ps)
        if (p) {
          if (s->pinned) (void)hipHostFree(p);
          else free(p);
        }
    }
    if (dr) device_rules_destroy(dr);
  }
};

namespace tsg {
namespace {

void* host_alloc(bool pinned, size_t bytes) {
  if (!pinned) return malloc(std::max<size_t>(bytes, 16));
  void* p = nullptr;
  if (hipHostMalloc(&p, std::max<size_t>(bytes, 16), hipHostMallocDefault) != hipSuccess) return nullptr;
  return p;
}

void host_free(bool pinned, void* p) {
  if (!p) return;
  if (pinned) (void)hipHostFree(p);
  else free(p);
}

// (re)allocate a slot for at least these capacities
int slot_reserve(tsg_ctx* c, Slot* s, uint64_t bytes, uint32_t files, uint64_t pbytes) {
  const bool pinned = !c->emulate;
  if (s->data && (s->data_cap < bytes || s->files_cap < files || s->paths_cap < pbytes)) {
    void* ps[] = {s->data, s->off, s->paths, s->poff};
    for (void* p : ps) host_free(s->pinned, p);
    *s = Slot{};
  }
  if (s->data) return TSG_OK;
  s->pinned = pinned;
  s->data_cap = round_up(std::max<uint64_t>(bytes, 1), 1 << 20);
  s->files_cap = (uint32_t)std::min<uint64_t>(round_up(std::max<uint32_t>(files, 1), 4096), 0xFFFFFFF0u);
  s->paths_cap = round_up(std::max<uint64_t>(pbytes, 1), 1 << 16);
  s->data = (uint8_t*)host_alloc(pinned, s->data_cap + slot_room_bytes(s->files_cap));
  s->off = (uint64_t*)host_alloc(pinned, sizeof(uint64_t) * ((size_t)s->files_cap + 1));
  s->paths = (char*)host_alloc(pinned, s->paths_cap + 16);
  s->poff = (uint64_t*)host_alloc(pinned, sizeof(uint64_t) * ((size_t)s->files_cap + 1));
  if (!s->data || !s->off || !s->paths || !s->poff) {
    void* ps[] = {s->data, s->off, s->paths, s->poff};
    for (void* p : ps) host_free(pinned, p);
    *s = Slot{};
    return fail(TSG_ERR_NOMEM, "cannot allocate a pinned slot");
  }
  s->off[0] = 0;
  s->poff[0] = 0;
  return TSG_OK;
}

// a free slot (no owner, nothing in flight) with these capacities, grown or created if
// needed; waits while every slot is busy and the context is at max_slots (lock held)
int slot_take(tsg_ctx* c, std::unique_lock<std::mutex>& lk, int owner, uint64_t bytes, uint32_t files,
              uint64_t pbytes, uint32_t* id) {
  const size_t max_slots = c->opt.max_slots ? c->opt.max_slots : 16;
  for (;;) {
    int fit = -1, any = -1;
    for (size_t i = 0; i < c->slots.size(); i++) {
      const Slot& s = *c->slots[i];
      if (s.owner != kFree || s.inflight) continue;
      if (any < 0) any = (int)i;
      if (s.data_cap >= bytes && s.files_cap >= files && s.paths_cap >= pbytes) {
        fit = (int)i;
        break;
      }
    }
    int pick = fit >= 0 ? fit : any;
    if (pick < 0 && c->slots.size() < max_slots) {
      c->slots.push_back(std::make_unique<Slot>());
      pick = (int)c->slots.size() - 1;
    }
    if (pick >= 0) {
      int rc = slot_reserve(c, c->slots[pick].get(), bytes, files, pbytes);
      if (rc) return rc;
      c->slots[pick]->owner = owner;
      c->slots[pick]->filled = kUnknownFill;
      c->slots[pick]->holder = std::this_thread::get_id();
      *id = (uint32_t)pick;
      return TSG_OK;
    }
    // Nothing will free a slot if no job is running and every held slot's holder is this
    // thread or another thread that is itself waiting here (two callers that each hold a
    // slot and ask for another): fail instead of waiting forever.  (A queue batch's slot is
    // submitted as soon as its last writer is done; an upload's holder is copying.)
    const auto me = std::this_thread::get_id();
    bool progress = c->jobs != 0;
    for (const auto& sl : c->slots) {
      if (sl->owner == kFree) continue;
      progress |= sl->owner == kQueue || sl->owner == kUpload ||
                  (sl->holder != me && !c->slot_waiters.count(sl->holder));
    }
    if (!progress)
      return fail(TSG_ERR_ARG, "every pinned slot is held by a caller that is waiting for another slot");
    c->slot_waiters.insert(me);
    c->cv.wait(lk);
    c->slot_waiters.erase(c->slot_waiters.find(me));
  }
}

int out_take(tsg_ctx* c, uint32_t nfiles, int* idx) {
  for (size_t i = 0; i < c->outs.size(); i++)
    if (!c->out_busy[i] && c->outs[i].files_cap >= nfiles) {
      c->out_busy[i] = 1;
      *idx = (int)i;
      return TSG_OK;
    }
  for (size_t i = 0; i < c->outs.size(); i++)  // grow a free one
    if (!c->out_busy[i]) {
      host_out_free(&c->outs[i]);
      int rc = host_out_alloc(c->dr, (uint32_t)std::min<uint64_t>(round_up(nfiles, 65536), 0xFFFFFFF0u), &c->outs[i]);
      if (rc) return rc;
      c->out_busy[i] = 1;
      *idx = (int)i;
      return TSG_OK;
    }
  HostOut h;
  int rc = host_out_alloc(c->dr, (uint32_t)std::min<uint64_t>(round_up(std::max<uint32_t>(nfiles, 1), 65536), 0xFFFFFFF0u), &h);
  if (rc) return rc;
  c->outs.push_back(h);
  c->out_busy.push_back(1);
  *idx = (int)c->outs.size() - 1;
  return TSG_OK;
}

int check_layout(const Slot& s, uint32_t nfiles) {
  if (nfiles > s.files_cap) return fail(TSG_ERR_ARG, "more files than the slot holds");
  if (s.off[0] != 0 || s.poff[0] != 0) return fail(TSG_ERR_ARG, "offsets[0] must be 0");
  for (uint32_t i = 0; i < nfiles; i++)
    if (s.off[i + 1] < s.off[i] || s.poff[i + 1] < s.poff[i])
      return fail(TSG_ERR_ARG, "offsets must be non-decreasing");
  if (s.off[nfiles] > s.data_cap || s.poff[nfiles] > s.paths_cap) return fail(TSG_ERR_ARG, "offsets exceed the slot");
  // candidate ends are 32-bit offsets in a file: a file of 4 GiB or more is resolved whole
  return TSG_OK;
}

void update_stats(tsg_ctx* c, const Batch& b) {
  tsg_stats& s = c->stats;
  s.k1_ms = b.t.k1;
  s.k2_ms = b.t.k2;
  s.gate_ms = b.t.gates;
  s.h2d_ms = b.t.h2d;
  s.aux_ms = b.t.out;
  s.prep_ms = b.t.prep;
  s.meta_ms = b.t.meta;
  s.resolve_ms = b.resolve_ms;
  s.bytes = b.bytes;
  s.candidates = b.counts[0];
  s.overflow = b.counts[0] > (c->opt.cand_capacity ? c->opt.cand_capacity : (1u << 22)) ? 1 : 0;
  s.k2_items = b.counts[5];
  s.k2_bytes = (uint64_t)b.counts[5] * c->opt.chunk_bytes;
  s.k2_launches = b.counts[6];
  s.groups_skipped = b.counts[7];
  s.files_resolved = b.files_found;
  s.wait_ms = b.t.wait;
  s.k2_tail_bytes = b.counts[8];
  s.k2_tail_max = b.counts[9];
  s.k2_long_tails = b.counts[10];
  s.k2_replays = b.counts[11];
  s.k1x_records = b.counts[14];
  s.k1x_inline = b.counts[15];
  s.k1f_listed = b.counts[16];
  s.k1f_arrivals = b.counts[17];
  s.k1_clock_ms = b.t.k1_clk;
  s.chain_clock_ms = b.t.chain_clk;
  s.post_k1_clock_ms = b.t.post_k1_clk;
  s.sum_k1_clock_ms += b.t.k1_clk;
  s.sum_chain_clock_ms += b.t.chain_clk;
  s.sum_post_k1_clock_ms += b.t.post_k1_clk;
  s.event_chunks = b.counts[1];
  s.k1_filter = c->dr && device_rules_k1_filter(c->dr) && b.bytes + (1u << 16) < (1ull << 32) ? 1u : 0u;
  s.k1_hot_states = c->dr ? device_rules_hot_states(c->dr) : 0;
  s.batches++;
  s.sum_bytes += b.bytes;
  s.sum_k1_ms += b.t.k1;
  s.sum_gate_ms += b.t.gates;
  s.sum_k2_ms += b.t.k2;
  s.sum_h2d_ms += b.t.h2d;
  s.sum_d2h_ms += b.t.out;
  s.sum_prep_ms += b.t.prep;
  s.sum_meta_ms += b.t.meta;
  s.sum_resolve_ms += b.resolve_ms;
}

// the host job of one submission: wait for the device, resolve, serialize
void run_job(tsg_ctx* c, std::shared_ptr<Batch> b, BatchView view, HostOut ho,
             std::shared_ptr<const std::vector<uint8_t>> kwu) {
  const tsg_ruleset* rs = c->rs;
  try {
    KernelOutput emu;
    KernelOutputView kv;
    if (c->emulate) {
      emulate_kernels(*rs->plan, view, c->opt.chunk_bytes, c->opt.ext_cap, &emu);
      kv = emu.view();
      b->counts[0] = (uint32_t)std::min<size_t>(emu.cand.size(), 0xFFFFFFFFu);
    } else {
      if (hipEventSynchronize(ho.ev[kEvDone]) != hipSuccess) throw std::runtime_error("device batch failed");
      (void)batch_times(&ho, &b->t);
      std::memcpy(b->counts, ho.counts, sizeof(b->counts));
      // counts from the device: 0 candidates, 1 event chunks, 2 K2 entries; layout stats
      // 4+1 items, 4+2 entries, 4+3 skipped groups
      const uint32_t items = ho.counts[5], entries = ho.counts[6], skipped = ho.counts[7];
      b->counts[5] = items;
      b->counts[6] = entries;
      b->counts[7] = skipped;
      kv.kw = ho.kw;
      kv.cand = ho.cand;
      kv.ncand = std::min<uint32_t>(ho.counts[0], ho.cand_cap);
      kv.overflow = ho.ovf;
      kv.sparse_kw = true;  // outputs_kernel: flags and the keyword rows the host reads
      kv.kw_unknown = kwu ? kwu->data() : nullptr;
      kv.path_ok = nullptr;  // Global.AllowPath on the host (plan.cpp path_allowed)
      kv.group_skipped = skipped ? ho.gskip : nullptr;
    }
    const auto t0 = std::chrono::steady_clock::now();
    resolve_batch(rs->rs, *rs->plan, view, kv, c->nt, &b->br);
    for (uint8_t st : b->br.status) b->files_found += st == kHasFindings;
    if (!b->keep_result) {
      b->res = std::make_unique<tsg_result>();
      serialize_batch(b->br, &b->res->buf, c->nt);
      b->br = BatchResult{};
    }
    b->resolve_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  } catch (const std::bad_alloc&) {
    b->rc = TSG_ERR_NOMEM;
    b->err = "out of memory";
  } catch (const std::exception& ex) {
    b->rc = c->emulate ? TSG_ERR_INTERNAL : TSG_ERR_GPU;
    b->err = ex.what();
  }
  {  // the slot may be reused and the pinned outputs retaken from here on
    std::lock_guard<std::mutex> g(c->m);
    c->slots[b->slot]->inflight--;
    if (b->out >= 0) c->out_busy[b->out] = 0;
    if (b->rc == TSG_OK) update_stats(c, *b);
    c->cv.notify_all();
  }
  {
    std::lock_guard<std::mutex> g(b->dm);
    b->done = true;
  }
  b->dcv.notify_all();
  if (b->on_done) {  // moved out first: a callback holding the batch's owner is no cycle
    auto cb = std::move(b->on_done);
    b->on_done = nullptr;
    cb(b);
  }
  b.reset();  // (the last reference may be this thread's)
  std::lock_guard<std::mutex> g(c->m);
  c->jobs--;  // after this the context may be destroyed: only its completion thread (joined
              // by the destructor) touches it again
  c->cv.notify_all();
}

// a completion thread of the context: takes queued host jobs until the context stops
void job_worker(tsg_ctx* c) {
  std::unique_lock<std::mutex> lk(c->m);
  for (;;) {
    c->cv.wait(lk, [&] { return c->stopping || !c->jq.empty(); });
    if (c->jq.empty()) return;  // stopping, nothing left
    auto job = std::move(c->jq.front());
    c->jq.pop_front();
    lk.unlock();
    job();
    lk.lock();
  }
}

// submit nfiles files of slot `sid` (lock held); the job is queued for the context's
// completion threads, where it mostly waits for the lane's completion event (the
// resolution itself fans out on the process-wide pool)
int submit_locked(tsg_ctx* c, uint32_t sid, uint32_t nfiles, bool keep_result,
                  std::function<void(const std::shared_ptr<Batch>&)> on_done, std::shared_ptr<Batch>* out) {
  Slot& s = *c->slots[sid];
  int rc = check_layout(s, nfiles);
  if (rc) return rc;
  auto b = std::make_shared<Batch>();
  b->slot = sid;
  b->nfiles = nfiles;
  b->bytes = s.off[nfiles];
  b->keep_result = keep_result;
  b->on_done = std::move(on_done);
  BatchView view{s.data, s.off, nfiles, s.paths, s.poff};
  HostOut ho;
  std::shared_ptr<const std::vector<uint8_t>> kwu;
  if (!c->emulate) {
    if ((rc = out_take(c, nfiles, &b->out))) return rc;
    LaneState* l = c->lanes[c->seq++ % c->lanes.size()];
    const ScanInput in = slot_input(s, nfiles);
    if ((rc = enqueue_scan(c->dr, l, in, &c->outs[b->out]))) {
      c->out_busy[b->out] = 0;
      return rc;
    }
    ho = c->outs[b->out];
    kwu = device_rules_kw_unknown(c->dr);
  }
  s.inflight++;
  c->jobs++;
  try {
    c->jq.push_back([c, b, view, ho, kwu] { run_job(c, b, view, ho, kwu); });
  } catch (const std::exception& ex) {  // no room: the enqueued device work is waited for here
    s.inflight--;
    c->jobs--;
    if (b->out >= 0) {
      (void)hipEventSynchronize(ho.ev[kEvDone]);
      c->out_busy[b->out] = 0;
    }
    return fail(TSG_ERR_INTERNAL, std::string("cannot queue a batch job: ") + ex.what());
  }
  c->cv.notify_all();
  b->ticket = c->next_ticket++;
  *out = b;
  return TSG_OK;
}

// wait for a submission's job; its result
int finish(const std::shared_ptr<Batch>& b) {
  std::unique_lock<std::mutex> lk(b->dm);
  b->dcv.wait(lk, [&] { return b->done; });
  if (b->rc) return fail(b->rc, b->err);
  return TSG_OK;
}

void parallel_copy(void* dst, const void* src, size_t n, int nt) {
  const size_t blk = 8 << 20;
  const size_t nb = (n + blk - 1) / blk;
  pool_for(nb, nb > 1 ? nt : 1, [&](size_t i) {
    const size_t a = i * blk, e = std::min(n, a + blk);
    std::memcpy((uint8_t*)dst + a, (const uint8_t*)src + a, e - a);
  }, 1);
}

template <class F>
int guard(F f) {
  try {
    return f();
  } catch (const std::bad_alloc&) {
    return fail(TSG_ERR_NOMEM, "out of memory");
  } catch (const std::exception& ex) {
    return fail(TSG_ERR_INTERNAL, ex.what());
  }
}

}  // namespace
}  // namespace tsg

// ---------------------------------------------------------------- tsg_queue
struct QBatch;

// A batch being filled by concurrent callers: its files are appended to one slot.
struct OpenBatch {
  uint32_t slot = 0;
  Slot* sp = nullptr;  // the slot (stable: slots are never moved)
  uint32_t nfiles = 0;
  uint64_t bytes = 0, pbytes = 0;
  int writers = 0;  // callers copying into the slot right now
  bool sealed = false;
  std::chrono::steady_clock::time_point first;
  std::shared_ptr<QBatch> qb;
};

// Completion of a submitted queue batch: wakes its callers.
struct QBatch {
  std::mutex m;
  std::condition_variable cv;
  bool ready = false;
  int rc = TSG_OK;
  std::string err;
  std::shared_ptr<Batch> b;
};

struct tsg_queue {
  tsg_ctx* c = nullptr;
  uint32_t flush_us = 2000;
  uint64_t slot_bytes = 0, paths_cap = 0;
  uint32_t files_cap = 0;
  std::mutex m;
  std::condition_variable cv;
  std::shared_ptr<OpenBatch> open;     // accepting files
  std::thread flusher;
  bool stop = false;
  int calls = 0;                       // tsg_queue_scan calls in progress
};

namespace tsg {
namespace {

// submit a sealed batch whose writers are done (q->m held); its job marks the QBatch
// ready, which wakes the batch's callers
void q_submit(tsg_queue* q, std::shared_ptr<OpenBatch> ob) {
  auto qb = ob->qb;
  std::shared_ptr<Batch> b;
  int rc;
  auto ready = [qb](const std::shared_ptr<Batch>& done) {
    std::lock_guard<std::mutex> g(qb->m);
    qb->b = done;
    qb->rc = done->rc;
    qb->err = done->err;
    qb->ready = true;
    qb->cv.notify_all();
  };
  {
    std::lock_guard<std::mutex> g(q->c->m);
    q->c->slots[ob->slot]->filled = ob->nfiles;  // the queue wrote exactly these files
    rc = submit_locked(q->c, ob->slot, ob->nfiles, true, ready, &b);
    q->c->slots[ob->slot]->owner = kFree;  // free once its job is done
    q->c->cv.notify_all();
  }
  if (rc) {
    std::lock_guard<std::mutex> g(qb->m);
    qb->rc = rc;
    qb->err = tsg_last_error();
    qb->ready = true;
    qb->cv.notify_all();
  }
}

// no more files for this batch; submitted as soon as its last writer is done (q->m held)
void q_seal(tsg_queue* q, std::shared_ptr<OpenBatch> ob) {  // (by value: may be q->open)
  if (ob->sealed) return;
  ob->sealed = true;
  if (q->open == ob) q->open.reset();
  if (ob->writers == 0) q_submit(q, ob);
}

void q_flusher(tsg_queue* q) {
  std::unique_lock<std::mutex> lk(q->m);
  while (!q->stop) {
    auto ob = q->open;
    if (ob && ob->nfiles) {
      const auto due = ob->first + std::chrono::microseconds(q->flush_us);
      if (std::chrono::steady_clock::now() >= due) {
        q_seal(q, ob);
        continue;
      }
      q->cv.wait_until(lk, due);
    } else {
      q->cv.wait(lk);
    }
  }
}

}  // namespace

const tsg_ruleset* ctx_ruleset(const tsg_ctx* c) { return c ? c->rs : nullptr; }
uint64_t ctx_slot_bytes(const tsg_ctx* c) { return (uint64_t)(c && c->opt.slot_mib ? c->opt.slot_mib : 256) << 20; }
}  // namespace tsg

extern "C" {

int tsg_ctx_create(int device, const tsg_ruleset* rs, const tsg_ctx_options* opt, tsg_ctx** out) {
  if (!rs || !out) return fail(TSG_ERR_ARG, "bad argument");
  return guard([&]() -> int {
    auto c = std::make_unique<tsg_ctx>();
    c->device = device;
    c->rs = rs;
    if (opt) c->opt = *opt;
    if (c->opt.chunk_bytes == 0) c->opt.chunk_bytes = 256;
    if (c->opt.chunk_bytes % 16) return fail(TSG_ERR_ARG, "chunk_bytes must be a multiple of 16");
    if (c->opt.ext_cap == 0) c->opt.ext_cap = 1u << 16;
    if (c->opt.cand_capacity == 0) c->opt.cand_capacity = 1u << 22;
    c->nt = c->opt.host_threads > 0 ? c->opt.host_threads : 16;
    c->emulate = (c->opt.flags & TSG_CTX_EMULATE) != 0;
    // The per-batch host buffers (keyword bits, result vectors, serialized results) are
    // tens of MB: keep such blocks on the heap (reused, already faulted in) instead of
    // fresh mmap'ed pages for every batch.
    static std::once_flag heap_once;
    std::call_once(heap_once, [] {
      mallopt(M_MMAP_THRESHOLD, 32 << 20);
      mallopt(M_TRIM_THRESHOLD, 1 << 30);
    });
    if (!c->emulate) {
      int rc = device_rules_create(device, *rs->plan, c->opt.chunk_bytes, c->opt.ext_cap, c->opt.adapt_mib, &c->dr);
      if (rc) return rc;
      for (int i = 0; i < 2; i++) {
        LaneState* l = nullptr;
        if ((rc = lane_create(c->dr, &l))) return rc;
        c->lanes.push_back(l);
      }
    }
    const size_t nw = c->emulate ? 4 : c->lanes.size();
    for (size_t i = 0; i < nw; i++) c->workers.emplace_back(job_worker, c.get());
    *out = c.release();
    return TSG_OK;
  });
}

void tsg_ctx_destroy(tsg_ctx* ctx) { delete ctx; }

int tsg_slot_acquire(tsg_ctx* c, uint64_t data_bytes, uint32_t nfiles, uint64_t path_bytes, tsg_slot_view* out) {
  if (!c || !out) return fail(TSG_ERR_ARG, "bad argument");
  return guard([&]() -> int {
    std::unique_lock<std::mutex> lk(c->m);
    uint32_t id;
    int rc = slot_take(c, lk, kCaller, data_bytes, nfiles, path_bytes, &id);
    if (rc) return rc;
    const Slot& s = *c->slots[id];
    *out = tsg_slot_view{id, s.data, s.data_cap, s.off, s.files_cap, s.paths, s.paths_cap, s.poff};
    return TSG_OK;
  });
}

int tsg_slot_submit(tsg_ctx* c, uint32_t slot_id, uint32_t nfiles, uint64_t* ticket) {
  if (!c || !ticket) return fail(TSG_ERR_ARG, "bad argument");
  return guard([&]() -> int {
    std::lock_guard<std::mutex> g(c->m);
    if (slot_id >= c->slots.size() || c->slots[slot_id]->owner != kCaller) return fail(TSG_ERR_ARG, "not an acquired slot");
    std::shared_ptr<Batch> b;
    int rc = submit_locked(c, slot_id, nfiles, false, nullptr, &b);
    if (rc) return rc;
    c->pending.emplace(b->ticket, b);
    *ticket = b->ticket;
    return TSG_OK;
  });
}

int tsg_slot_release(tsg_ctx* c, uint32_t slot_id) {
  if (!c) return fail(TSG_ERR_ARG, "bad argument");
  std::lock_guard<std::mutex> g(c->m);
  if (slot_id >= c->slots.size() || c->slots[slot_id]->owner != kCaller) return fail(TSG_ERR_ARG, "not an acquired slot");
  c->slots[slot_id]->owner = kFree;
  c->cv.notify_all();
  return TSG_OK;
}

namespace tsg {
namespace {
// a free slot owned by `owner` holding a copy of the caller's batch
int upload_into_slot(tsg_ctx* c, int owner, const uint8_t* data, const uint64_t* offsets, uint32_t nfiles,
                     const char* paths, const uint64_t* path_offsets, uint32_t* id) {
  if (!offsets || !path_offsets) return fail(TSG_ERR_ARG, "bad argument");
  if (offsets[0] != 0 || path_offsets[0] != 0) return fail(TSG_ERR_ARG, "offsets[0] must be 0");
  for (uint32_t i = 0; i < nfiles; i++)
    if (offsets[i + 1] < offsets[i] || path_offsets[i + 1] < path_offsets[i])
      return fail(TSG_ERR_ARG, "offsets must be non-decreasing");
  const uint64_t total = offsets[nfiles], pbytes = path_offsets[nfiles];
  if ((total && !data) || (pbytes && !paths)) return fail(TSG_ERR_ARG, "bad argument");
  Slot* sp;
  {
    std::unique_lock<std::mutex> lk(c->m);
    int rc = slot_take(c, lk, owner, total, nfiles, pbytes, id);
    if (rc) return rc;
    sp = c->slots[*id].get();
  }
  Slot& s = *sp;  // ours alone until it is submitted
  parallel_copy(s.data, data, total, c->nt);
  std::memcpy(s.off, offsets, sizeof(uint64_t) * ((size_t)nfiles + 1));
  if (pbytes) std::memcpy(s.paths, paths, pbytes);
  std::memcpy(s.poff, path_offsets, sizeof(uint64_t) * ((size_t)nfiles + 1));
  s.filled = nfiles;
  return TSG_OK;
}
}  // namespace
}  // namespace tsg

int tsg_batch_upload(tsg_ctx* c, const uint8_t* data, const uint64_t* offsets, uint32_t nfiles, const char* paths,
                     const uint64_t* path_offsets, uint32_t* slot_id) {
  if (!c || !slot_id) return fail(TSG_ERR_ARG, "bad argument");
  return guard([&]() -> int { return upload_into_slot(c, kCaller, data, offsets, nfiles, paths, path_offsets, slot_id); });
}

int tsg_batch_collect(tsg_ctx* c, uint64_t ticket, tsg_result** out) {
  if (!c || !out) return fail(TSG_ERR_ARG, "bad argument");
  return guard([&]() -> int {
    std::shared_ptr<Batch> b;
    {
      std::lock_guard<std::mutex> g(c->m);
      auto it = c->pending.find(ticket);
      if (it == c->pending.end()) return fail(TSG_ERR_ARG, "no such submitted batch (unknown or already collected ticket)");
      b = it->second;
      c->pending.erase(it);
    }
    int rc = finish(b);
    if (rc) return rc;
    *out = b->res.release();
    return TSG_OK;
  });
}

int tsg_batch_pending(const tsg_ctx* c) {
  if (!c) return TSG_ERR_ARG;
  std::lock_guard<std::mutex> g(c->m);
  return (int)c->pending.size();
}

int tsg_scan_batch(tsg_ctx* c, const uint8_t* data, const uint64_t* offsets, uint32_t nfiles, const char* paths,
                   const uint64_t* path_offsets, tsg_result** out) {
  if (!c || !out) return fail(TSG_ERR_ARG, "bad argument");
  return guard([&]() -> int {
    uint32_t id;
    int rc = upload_into_slot(c, kUpload, data, offsets, nfiles, paths, path_offsets, &id);
    if (rc) return rc;
    std::shared_ptr<Batch> b;
    {
      std::lock_guard<std::mutex> g(c->m);
      rc = submit_locked(c, id, nfiles, false, nullptr, &b);
      c->slots[id]->owner = kFree;  // reusable once its submission is done
      c->cv.notify_all();
    }
    if (rc) return rc;
    if ((rc = finish(b))) return rc;
    *out = b->res.release();
    return TSG_OK;
  });
}

int tsg_batch_kernels(tsg_ctx* c, uint32_t slot_id, uint32_t nfiles, uint32_t* kw, size_t kw_len, uint32_t* ev,
                      size_t ev_len) {
  if (!c) return fail(TSG_ERR_ARG, "bad argument");
  return guard([&]() -> int {
    // the whole call holds the context lock: no other batch can be enqueued on the lane
    // before its event buffer is read back
    std::lock_guard<std::mutex> g(c->m);
    if (slot_id >= c->slots.size() || c->slots[slot_id]->owner != kCaller) return fail(TSG_ERR_ARG, "not an acquired slot");
    Slot& s = *c->slots[slot_id];
    int rc = check_layout(s, nfiles);
    if (rc) return rc;
    const size_t W = (size_t)c->rs->plan->kw_words;
    BatchView view{s.data, s.off, nfiles, s.paths, s.poff};
    if (c->emulate) {
      std::vector<uint32_t> kwv, evv;
      k1_reference(*c->rs->plan, view, c->opt.chunk_bytes, &kwv, &evv);
      if (kw) std::memcpy(kw, kwv.data(), sizeof(uint32_t) * std::min(kw_len, kwv.size()));
      if (ev) std::memcpy(ev, evv.data(), sizeof(uint32_t) * std::min(ev_len, evv.size()));
      return TSG_OK;
    }
    int oi;
    if ((rc = out_take(c, nfiles, &oi))) return rc;
    LaneState* l = c->lanes[c->seq++ % c->lanes.size()];
    const ScanInput in = slot_input(s, nfiles);
    if ((rc = enqueue_scan(c->dr, l, in, &c->outs[oi]))) {
      c->out_busy[oi] = 0;
      return rc;
    }
    HostOut ho = c->outs[oi];
    hipError_t e = hipEventSynchronize(ho.ev[kEvDone]);
    if (e == hipSuccess) {
      Batch b;
      (void)batch_times(&ho, &b.t);
      std::memcpy(b.counts, ho.counts, sizeof(b.counts));
      b.bytes = s.off[nfiles];
      update_stats(c, b);
      if (kw) rc = lane_kw(l, kw, std::min(kw_len, W * nfiles));
      if (ev && !rc) rc = lane_events(l, ev, ev_len);
      if (const char* tp = getenv("TSG_K1F_TRACE")) {  // append K1F's per-wave trace (measurements)
        std::vector<unsigned long long> tr;
        if (!rc) rc = lane_k1f_trace(l, &tr);
        if (FILE* f = tr.empty() ? nullptr : fopen(tp, "ab")) {
          fwrite(tr.data(), sizeof(unsigned long long), tr.size(), f);
          fclose(f);
        }
      }
      if (const char* tp = getenv("TSG_K2_TRACE")) {  // append the K2 entry trace (measurements)
        std::vector<unsigned long long> tr;
        if (!rc) rc = lane_k2_trace(l, &tr);
        if (FILE* f = tr.empty() ? nullptr : fopen(tp, "ab")) {
          fwrite(tr.data(), sizeof(unsigned long long), tr.size(), f);
          fclose(f);
        }
      }
    }
    c->out_busy[oi] = 0;
    if (e != hipSuccess) return fail(TSG_ERR_GPU, std::string("tsg_batch_kernels: ") + hipGetErrorString(e));
    return rc;
  });
}

int tsg_ctx_get_stats(const tsg_ctx* c, tsg_stats* out) {
  if (!c || !out) return fail(TSG_ERR_ARG, "bad argument");
  std::lock_guard<std::mutex> g(c->m);
  *out = c->stats;
  return TSG_OK;
}

int tsg_queue_create(tsg_ctx* c, uint32_t flush_us, tsg_queue** out) {
  if (!c || !out) return fail(TSG_ERR_ARG, "bad argument");
  return guard([&]() -> int {
    auto q = std::make_unique<tsg_queue>();
    q->c = c;
    q->flush_us = flush_us ? flush_us : 2000;
    q->slot_bytes = (uint64_t)(c->opt.slot_mib ? c->opt.slot_mib : 256) << 20;
    q->files_cap = (uint32_t)std::max<uint64_t>(q->slot_bytes / 512, 4096);
    q->paths_cap = std::max<uint64_t>(q->slot_bytes / 16, 1 << 20);
    q->flusher = std::thread(q_flusher, q.get());
    *out = q.release();
    return TSG_OK;
  });
}

int tsg_queue_scan(tsg_queue* q, const char* path, size_t path_len, const uint8_t* content, size_t len,
                   tsg_result** out) {
  if (!q || !out || (!content && len) || (!path && path_len)) return fail(TSG_ERR_ARG, "bad argument");
  tsg_ctx* c = q->c;
  if (len > q->slot_bytes / 2 || path_len > q->paths_cap / 2)  // too large to share a slot: exact CPU path
    return tsg_scan_cpu(c->rs, path, path_len, content, len, out);
  return guard([&]() -> int {
    std::shared_ptr<OpenBatch> ob;
    uint32_t idx = 0;
    uint64_t at = 0, pat = 0;
    {
      std::unique_lock<std::mutex> lk(q->m);
      q->calls++;
      for (;;) {
        ob = q->open;
        if (ob && (ob->bytes + len > q->slot_bytes || ob->nfiles + 1 > q->files_cap ||
                   ob->pbytes + path_len > q->paths_cap)) {
          q_seal(q, ob);
          ob.reset();
        }
        if (ob) break;
        // open a new batch: take a free slot (may wait for a batch in flight to finish)
        uint32_t id;
        lk.unlock();
        int rc;
        Slot* sp = nullptr;
        {
          std::unique_lock<std::mutex> lc(c->m);
          rc = slot_take(c, lc, kQueue, q->slot_bytes, q->files_cap, q->paths_cap, &id);
          if (!rc) sp = c->slots[id].get();
        }
        lk.lock();
        if (rc) {
          q->calls--;
          q->cv.notify_all();
          return rc;
        }
        if (q->open) {  // another caller opened one meanwhile: give ours back, use theirs
          std::lock_guard<std::mutex> lc(c->m);
          c->slots[id]->owner = kFree;
          c->cv.notify_all();
          continue;
        }
        auto nb = std::make_shared<OpenBatch>();
        nb->slot = id;
        nb->sp = sp;
        nb->first = std::chrono::steady_clock::now();
        nb->qb = std::make_shared<QBatch>();
        q->open = nb;
        q->cv.notify_all();  // the flusher times it
      }
      Slot& s = *ob->sp;
      idx = ob->nfiles++;
      at = ob->bytes;
      pat = ob->pbytes;
      ob->bytes += len;
      ob->pbytes += path_len;
      s.off[idx + 1] = ob->bytes;
      s.poff[idx + 1] = ob->pbytes;
      ob->writers++;
      if (ob->bytes >= q->slot_bytes - q->slot_bytes / 8 || ob->nfiles == q->files_cap) q_seal(q, ob);
    }
    Slot& s = *ob->sp;
    if (len) std::memcpy(s.data + at, content, len);
    if (path_len) std::memcpy(s.paths + pat, path, path_len);
    {
      std::lock_guard<std::mutex> lk(q->m);
      if (--ob->writers == 0 && ob->sealed) q_submit(q, ob);
    }
    auto qb = ob->qb;
    std::unique_lock<std::mutex> wl(qb->m);
    qb->cv.wait(wl, [&] { return qb->ready; });
    const int rc = qb->rc;
    const std::string err = qb->err;
    std::shared_ptr<Batch> b = qb->b;
    wl.unlock();
    {
      std::lock_guard<std::mutex> lk(q->m);
      q->calls--;
      q->cv.notify_all();
    }
    if (rc) return fail(rc, err);
    FileResult fr;
    const BatchResult& br = b->br;
    if (br.slot[idx] != UINT32_MAX) fr = br.res[br.slot[idx]];
    else fr.status = br.status[idx];
    auto r = std::make_unique<tsg_result>();
    serialize_results({fr}, &r->buf);
    *out = r.release();
    return TSG_OK;
  });
}

int tsg_queue_flush(tsg_queue* q) {
  if (!q) return fail(TSG_ERR_ARG, "bad argument");
  return guard([&]() -> int {
    std::lock_guard<std::mutex> lk(q->m);
    if (q->open && q->open->nfiles) q_seal(q, q->open);
    return TSG_OK;
  });
}

void tsg_queue_destroy(tsg_queue* q) {
  if (!q) return;
  {
    std::unique_lock<std::mutex> lk(q->m);
    q->cv.wait(lk, [&] { return q->calls == 0; });
    q->stop = true;
    q->cv.notify_all();
  }
  q->flusher.join();
  if (q->open) {  // opened, never filled
    std::lock_guard<std::mutex> g(q->c->m);
    q->c->slots[q->open->slot]->owner = kFree;
    q->c->cv.notify_all();
  }
  delete q;
}

}  // extern "C"
