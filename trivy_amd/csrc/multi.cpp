// One process, several GPUs: the in-process multi-device dispatcher (tsg_multi_*).
//
// trivy is one Go process.  An image scan analyzes every missing layer in its own
// goroutine (pkg/fanal/artifact/image/image.go:210-234) and every file of a layer in a
// per-file goroutine (pkg/fanal/analyzer/analyzer.go:419-443), so a node's GPUs are
// driven from one address space: this file binds one tsg_ctx per device and shards each
// batch's files over them, largest first onto the least-loaded device (LPT by bytes,
// SURVEY.md §8e).  Each device's share is copied straight from the caller's buffers into
// that device's pinned slots, submitted on the context's own lanes, and the serialized
// per-file results are gathered back in input order on the host.  There is no collective:
// files are independent (scanner.go:341).  The resolver pool is process-wide
// (plan.cpp Pool), so N contexts share its threads instead of multiplying them.
#include <algorithm>
#include <cstring>
#include <memory>
#include <mutex>
#include <numeric>
#include <queue>
#include <thread>
#include <vector>

#include "internal.hpp"

struct tsg_multi {
  std::vector<tsg_ctx*> ctx;
  uint64_t piece_bytes = 0;  // bytes per submitted slot
};

namespace tsg {
namespace {

// LPT: files largest first, each onto the device with the fewest bytes so far (ties: the
// lower device).  Returns each device's files in input order.
std::vector<std::vector<uint32_t>> lpt_shards(const uint64_t* off, uint32_t nfiles, uint32_t ndev) {
  std::vector<uint32_t> order(nfiles);
  std::iota(order.begin(), order.end(), 0u);
  std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
    return off[a + 1] - off[a] > off[b + 1] - off[b];
  });
  using Load = std::pair<uint64_t, uint32_t>;  // (bytes, device)
  std::priority_queue<Load, std::vector<Load>, std::greater<Load>> heap;
  for (uint32_t d = 0; d < ndev; d++) heap.push({0, d});
  std::vector<uint32_t> dev_of(nfiles);
  for (uint32_t f : order) {
    Load l = heap.top();
    heap.pop();
    dev_of[f] = l.second;
    l.first += off[f + 1] - off[f];
    heap.push(l);
  }
  std::vector<std::vector<uint32_t>> shard(ndev);
  for (uint32_t f = 0; f < nfiles; f++) shard[dev_of[f]].push_back(f);
  return shard;
}

struct Piece {
  uint64_t ticket = 0;
  uint32_t first = 0, count = 0;  // range of the device's shard list
  std::string buf;
  std::vector<size_t> rec;
};

// one device's share: pieces of at most piece_bytes, each copied into a pinned slot of the
// device's context, submitted, then collected
int run_shard(tsg_ctx* c, uint64_t piece_bytes, const std::vector<uint32_t>& files, const uint8_t* data,
              const uint64_t* off, const char* paths, const uint64_t* poff, std::vector<Piece>* pieces) {
  size_t i = 0;
  int rc = TSG_OK;
  while (i < files.size() && rc == TSG_OK) {
    Piece pc;
    pc.first = (uint32_t)i;
    uint64_t bytes = 0, pbytes = 0;
    while (i < files.size()) {
      const uint32_t f = files[i];
      const uint64_t len = off[f + 1] - off[f];
      if (pc.count && bytes + len > piece_bytes) break;
      bytes += len;
      pbytes += poff[f + 1] - poff[f];
      pc.count++;
      i++;
    }
    tsg_slot_view v;
    if ((rc = tsg_slot_acquire(c, bytes, pc.count, pbytes, &v))) break;
    v.offsets[0] = 0;
    v.path_offsets[0] = 0;
    for (uint32_t k = 0; k < pc.count; k++) {
      const uint32_t f = files[pc.first + k];
      v.offsets[k + 1] = v.offsets[k] + (off[f + 1] - off[f]);
      v.path_offsets[k + 1] = v.path_offsets[k] + (poff[f + 1] - poff[f]);
    }
    pool_for(pc.count, 16, [&](size_t k) {
      const uint32_t f = files[pc.first + k];
      if (off[f + 1] > off[f]) std::memcpy(v.data + v.offsets[k], data + off[f], off[f + 1] - off[f]);
      if (poff[f + 1] > poff[f]) std::memcpy(v.paths + v.path_offsets[k], paths + poff[f], poff[f + 1] - poff[f]);
    }, 256);
    rc = tsg_slot_submit(c, v.id, pc.count, &pc.ticket);
    const int rr = tsg_slot_release(c, v.id);  // free again once the submission is done
    if (!rc) rc = rr;
    if (!rc) pieces->push_back(std::move(pc));
  }
  // collect every submitted piece, also after a failure (nothing stays pending)
  int crc = TSG_OK;
  for (auto& pc : *pieces) {
    tsg_result* r = nullptr;
    int e = tsg_batch_collect(c, pc.ticket, &r);
    if (e) {
      if (!crc) crc = e;
      continue;
    }
    pc.buf = std::move(r->buf);
    tsg_result_free(r);
  }
  return rc ? rc : crc;
}

}  // namespace
}  // namespace tsg

using namespace tsg;

extern "C" {

int tsg_multi_create(const int* devices, uint32_t n, const tsg_ruleset* rs, const tsg_ctx_options* opt,
                     tsg_multi** out) {
  if (!devices || !n || !rs || !out) return fail(TSG_ERR_ARG, "bad argument");
  try {
    auto m = std::make_unique<tsg_multi>();
    for (uint32_t i = 0; i < n; i++) {
      tsg_ctx* c = nullptr;
      int rc = tsg_ctx_create(devices[i], rs, opt, &c);
      if (rc) {
        for (auto* x : m->ctx) tsg_ctx_destroy(x);
        return rc;
      }
      m->ctx.push_back(c);
    }
    m->piece_bytes = (uint64_t)(opt && opt->slot_mib ? opt->slot_mib : 256) << 20;
    // one context's resolution fans out over 16 threads; N devices in one process get up to
    // 16 per device (as many as the machine has), so their batches resolve side by side
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    const int per = opt && opt->host_threads > 0 ? opt->host_threads : 16;
    pool_reserve((int)std::min<unsigned>(hw, (unsigned)per * n) - 1);
    *out = m.release();
    return TSG_OK;
  } catch (const std::bad_alloc&) {
    return fail(TSG_ERR_NOMEM, "out of memory");
  }
}

int tsg_multi_size(const tsg_multi* m) { return m ? (int)m->ctx.size() : TSG_ERR_ARG; }

int tsg_multi_ctx(tsg_multi* m, uint32_t i, tsg_ctx** out) {
  if (!m || !out || i >= m->ctx.size()) return fail(TSG_ERR_ARG, "bad argument");
  *out = m->ctx[i];
  return TSG_OK;
}

int tsg_multi_scan_batch(tsg_multi* m, const uint8_t* data, const uint64_t* offsets, uint32_t nfiles,
                         const char* paths, const uint64_t* path_offsets, tsg_result** out) {
  if (!m || !out || !offsets || !path_offsets) return fail(TSG_ERR_ARG, "bad argument");
  if (offsets[0] != 0 || path_offsets[0] != 0) return fail(TSG_ERR_ARG, "offsets[0] must be 0");
  for (uint32_t i = 0; i < nfiles; i++)
    if (offsets[i + 1] < offsets[i] || path_offsets[i + 1] < path_offsets[i])
      return fail(TSG_ERR_ARG, "offsets must be non-decreasing");
  if ((offsets[nfiles] && !data) || (path_offsets[nfiles] && !paths)) return fail(TSG_ERR_ARG, "bad argument");
  try {
    const uint32_t D = (uint32_t)m->ctx.size();
    const auto shard = lpt_shards(offsets, nfiles, D);
    std::vector<std::vector<Piece>> pieces(D);
    std::vector<int> rcs(D, TSG_OK);
    std::vector<std::string> errs(D);
    {
      std::vector<std::thread> th;  // one host thread per device: its copies and submissions
      for (uint32_t d = 0; d < D; d++)
        th.emplace_back([&, d] {
          try {
            rcs[d] = run_shard(m->ctx[d], m->piece_bytes, shard[d], data, offsets, paths, path_offsets, &pieces[d]);
          } catch (const std::bad_alloc&) {
            rcs[d] = fail(TSG_ERR_NOMEM, "out of memory");
          } catch (const std::exception& ex) {
            rcs[d] = fail(TSG_ERR_INTERNAL, ex.what());
          }
          if (rcs[d]) errs[d] = tsg_last_error();
        });
      for (auto& t : th) t.join();
    }
    for (uint32_t d = 0; d < D; d++)
      if (rcs[d]) return fail(rcs[d], "device " + std::to_string(d) + ": " + errs[d]);
    // gather: file i is record (i's position in its device's list) of that device's pieces
    struct Loc {
      uint32_t dev, piece, rec;
    };
    std::vector<Loc> loc(nfiles);
    size_t total = 8;
    for (uint32_t d = 0; d < D; d++)
      for (uint32_t p = 0; p < pieces[d].size(); p++) {
        Piece& pc = pieces[d][p];
        result_record_spans(pc.buf, &pc.rec);
        if (pc.rec.size() != (size_t)pc.count + 1) throw std::runtime_error("result file count mismatch");
        for (uint32_t k = 0; k < pc.count; k++) loc[shard[d][pc.first + k]] = Loc{d, p, k};
        total += pc.rec[pc.count] - pc.rec[0];
      }
    auto r = std::make_unique<tsg_result>();
    r->buf.resize(total);
    char* w = &r->buf[0];
    const uint32_t hdr[2] = {0x31475354u, nfiles};
    std::memcpy(w, hdr, 8);
    w += 8;
    for (uint32_t i = 0; i < nfiles; i++) {
      const Piece& pc = pieces[loc[i].dev][loc[i].piece];
      const size_t a = pc.rec[loc[i].rec], e = pc.rec[loc[i].rec + 1];
      std::memcpy(w, pc.buf.data() + a, e - a);
      w += e - a;
    }
    *out = r.release();
    return TSG_OK;
  } catch (const std::bad_alloc&) {
    return fail(TSG_ERR_NOMEM, "out of memory");
  } catch (const std::exception& ex) {
    return fail(TSG_ERR_INTERNAL, ex.what());
  }
}

int tsg_multi_get_stats(const tsg_multi* m, uint32_t i, tsg_stats* out) {
  if (!m || i >= m->ctx.size()) return fail(TSG_ERR_ARG, "bad argument");
  return tsg_ctx_get_stats(m->ctx[i], out);
}

void tsg_multi_destroy(tsg_multi* m) {
  if (!m) return;
  for (auto* c : m->ctx) tsg_ctx_destroy(c);
  delete m;
}

}  // extern "C"
