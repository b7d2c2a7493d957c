// Native layer-tar ingest: one pass over an uncompressed image-layer tar
// that walks it like walker.LayerTar (pkg/fanal/walker/tar.go:33-111, walk.go:25-76),
// gates every regular file like SecretAnalyzer.Required (analyzer/secret/secret.go:112-150)
// and utils.IsBinary (utils.go:71-89), and packs the kept files back to back into one
// batch (the layout tsg_batch_upload / tsg_scan_batch take), with the "/" prefix of image
// files on their scan paths (secret.go:90-96).  The Python mirror is trivy_amd/walker.py.
//
// Tar decoding follows Go 1.19 archive/tar: ustar/PAX/GNU headers, PAX 'x' records
// (path, linkpath, size), GNU 'L'/'K' long names, TypeRegA -> TypeReg (TypeDir with a
// trailing "/"), header-only types carry no data, end = a zero block or end of input.
#include <cstdint>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <string_view>
#include <functional>
#include <memory>
#include <vector>
#include <thread>
#include <atomic>
#include <mutex>

#include <cerrno>
#include <dirent.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>

#include "internal.hpp"

namespace tsg {
namespace {
// open / openat that waits out a full descriptor table (EMFILE / ENFILE: concurrent walks
// of wide trees, each holding directory and file descriptors) instead of treating it as an
// unreadable file, which the walk would skip; another error is returned as it is
int open_at_retry(int dfd, const char* path, int flags) {
  for (int tries = 0;; tries++) {
    const int fd = dfd >= 0 ? openat(dfd, path, flags) : open(path, flags);
    if (fd >= 0 || (errno != EMFILE && errno != ENFILE) || tries >= 5000) return fd;
    std::this_thread::sleep_for(std::chrono::microseconds(500));
  }
}

// A failed open of a file the walk listed (analyzer.go:411-416): a permission error skips the
// file; any other error -- a file gone since the listing, or a descriptor table still full
// after open_at_retry's wait -- fails the scan ("unable to open"), as os.Open's error does
// there.  Files are opened following symlinks, as os.Open does (fs.go:66-70).
// Thread-safe: the parallel readers record the first such error.
struct OpenErr {
  std::mutex m;
  std::atomic<bool> set{false};
  std::string msg;
  void add(int e, const std::string& path) {
    if (e == EACCES || e == EPERM) return;  // fs.ErrPermission
    std::lock_guard<std::mutex> g(m);
    if (!set) msg = "unable to open " + path + ": " + strerror(e);
    set = true;
  }
};
}  // namespace
}  // namespace tsg

struct tsg_layer {
  std::unique_ptr<uint8_t[]> data;  // not zero-filled: every byte is copied in
  const uint8_t* ext = nullptr;     // the kept files in a context's pinned slot (*_pack_slot)
  std::vector<uint64_t> offsets{0};
  std::string paths;
  std::vector<uint64_t> path_offsets{0};
  std::string opq, wh;  // NUL-terminated lists
  uint32_t walked = 0;  // files handed to the analyzer (before Required / IsBinary)
};

namespace tsg {
namespace {

// Go path.Clean
// true when p is what clean(p) returns (no empty, "." or ".." element, no trailing "/"):
// most archive names are, and the general path below allocates per element
bool is_clean(const std::string& p) {
  if (p.empty()) return false;
  if (p == "/") return true;
  if (p.back() == '/') return false;
  size_t start = p[0] == '/' ? 1 : 0;
  for (size_t k = start; k <= p.size(); k++) {
    if (k < p.size() && p[k] != '/') continue;
    const size_t len = k - start;
    if (len == 0 || (len == 1 && p[start] == '.') || (len == 2 && p[start] == '.' && p[start + 1] == '.'))
      return false;
    start = k + 1;
  }
  return true;
}

std::string clean(const std::string& p) {
  if (is_clean(p)) return p;
  if (p.empty()) return ".";
  const bool rooted = p[0] == '/';
  std::vector<std::string> out;
  size_t i = 0;
  while (i <= p.size()) {
    size_t j = p.find('/', i);
    if (j == std::string::npos) j = p.size();
    std::string part = p.substr(i, j - i);
    i = j + 1;
    if (part.empty() || part == ".") continue;
    if (part == "..") {
      if (!out.empty() && out.back() != "..") out.pop_back();
      else if (!rooted) out.push_back("..");
      continue;
    }
    out.push_back(part);
  }
  std::string s;
  for (size_t k = 0; k < out.size(); k++) {
    if (k) s += '/';
    s += out[k];
  }
  if (rooted) return "/" + s;
  return s.empty() ? "." : s;
}

std::string trim_left_slash(const std::string& s) {
  size_t i = 0;
  while (i < s.size() && s[i] == '/') i++;
  return s.substr(i);
}

std::string base(std::string p) {  // Go filepath.Base
  if (p.empty()) return ".";
  while (!p.empty() && p.back() == '/') p.pop_back();
  if (p.empty()) return "/";
  size_t k = p.rfind('/');
  return k == std::string::npos ? p : p.substr(k + 1);
}

// Go filepath.Rel on "/" paths; false where Go returns an error
bool rel(const std::string& basepath, const std::string& targpath, std::string* out) {
  std::string b = clean(basepath), t = clean(targpath);
  if (t == b) {
    *out = ".";
    return true;
  }
  if (b == ".") b.clear();
  if ((!b.empty() && b[0] == '/') != (!t.empty() && t[0] == '/')) return false;
  const size_t bl = b.size(), tl = t.size();
  size_t b0 = 0, bi = 0, t0 = 0, ti = 0;
  for (;;) {
    while (bi < bl && b[bi] != '/') bi++;
    while (ti < tl && t[ti] != '/') ti++;
    if (t.compare(t0, ti - t0, b, b0, bi - b0) != 0) break;
    if (bi < bl) bi++;
    if (ti < tl) ti++;
    b0 = bi;
    t0 = ti;
  }
  if (b.compare(b0, bi - b0, "..") == 0) return false;
  if (b0 != bl) {
    size_t seps = 0;
    for (size_t k = b0; k < bl; k++) seps += b[k] == '/';
    std::string s = "..";
    for (size_t k = 0; k < seps; k++) s += "/..";
    if (t0 != tl) s += "/" + t.substr(t0);
    *out = s;
    return true;
  }
  *out = t.substr(t0);
  return true;
}

bool starts_with(const std::string& s, const char* p) { return s.rfind(p, 0) == 0; }

bool contains(const std::vector<std::string>& v, const std::string& s) {
  for (const auto& x : v)
    if (x == s) return true;
  return false;
}

// tar numeric field: octal (spaces / NULs trimmed) or GNU base-256
bool parse_num(const uint8_t* f, size_t n, int64_t* out) {
  if (n && (f[0] & 0x80)) {
    if (f[0] & 0x40) return false;  // negative
    uint64_t v = f[0] & 0x7f;
    for (size_t i = 1; i < n; i++) {
      if (v >> 55) return false;
      v = (v << 8) | f[i];
    }
    *out = (int64_t)v;
    return true;
  }
  size_t a = 0, b = n;
  while (a < b && (f[a] == ' ' || f[a] == 0)) a++;
  while (b > a && (f[b - 1] == ' ' || f[b - 1] == 0)) b--;
  uint64_t v = 0;
  for (size_t i = a; i < b; i++) {
    if (f[i] < '0' || f[i] > '7') return false;
    v = v * 8 + (f[i] - '0');
  }
  *out = (int64_t)v;
  return true;
}

std::string cstr(const uint8_t* f, size_t n) {
  size_t k = 0;
  while (k < n && f[k]) k++;
  return std::string((const char*)f, k);
}

bool checksum_ok(const uint8_t* h) {
  int64_t want;
  if (!parse_num(h + 148, 8, &want)) return false;
  int64_t u = 0, s = 0;
  for (int i = 0; i < 512; i++) {
    const uint8_t c = (i >= 148 && i < 156) ? ' ' : h[i];
    u += c;
    s += (int8_t)c;
  }
  return want == u || want == s;
}

bool header_only(char t) {  // archive/tar isHeaderOnlyType
  return t == '1' || t == '2' || t == '3' || t == '4' || t == '5' || t == '6';
}

// PAX records "len key=value\n"
bool parse_pax(const uint8_t* p, size_t n, std::vector<std::pair<std::string, std::string>>* recs) {
  size_t i = 0;
  while (i < n) {
    size_t sp = i;
    uint64_t len = 0;
    while (sp < n && p[sp] >= '0' && p[sp] <= '9') {
      if (len > (n - i) / 10) return false;  // longer than the rest of the block (or overflow)
      len = len * 10 + (p[sp++] - '0');
    }
    if (sp >= n || p[sp] != ' ' || len == 0 || len > n - i || p[i + len - 1] != '\n' || sp + 1 > i + len - 1)
      return false;
    std::string rec((const char*)p + sp + 1, i + len - 1 - (sp + 1));
    size_t eq = rec.find('=');
    if (eq == std::string::npos) return false;
    recs->emplace_back(rec.substr(0, eq), rec.substr(eq + 1));
    i += len;
  }
  return true;
}

struct Gate {  // SecretAnalyzer.Required (secret.go:112-150) + walker skip lists
  const Ruleset& rs;
  const Plan* plan;
  std::string config_base;
  std::vector<std::string> skip_files, skip_dirs;

  bool required(const std::string& fp, int64_t size) const {
    static const std::vector<std::string> kSkipFiles = {
        "go.mod", "go.sum", "package-lock.json", "yarn.lock", "pnpm-lock.yaml", "Pipfile.lock",
        "Gemfile.lock"};  // secret.go:27-35
    static const std::vector<std::string> kSkipDirs = {".git", "node_modules"};  // :36
    static const std::vector<std::string> kSkipExts = {
        ".jpg", ".png", ".gif", ".doc", ".pdf", ".bin", ".svg", ".socket", ".deb", ".rpm",
        ".zip", ".gz", ".gzip", ".tar", ".pyc"};  // :37-40
    if (size < 10) return false;
    const size_t k = fp.rfind('/');
    const std::string dir = k == std::string::npos ? "" : fp.substr(0, k + 1);
    const std::string name = k == std::string::npos ? fp : fp.substr(k + 1);
    size_t i = 0;
    for (;;) {  // strings.Split(dir, "/")
      size_t j = dir.find('/', i);
      const std::string part = dir.substr(i, j == std::string::npos ? std::string::npos : j - i);
      if (contains(kSkipDirs, part)) return false;
      if (j == std::string::npos) break;
      i = j + 1;
    }
    if (contains(kSkipFiles, name)) return false;
    if (config_base == fp) return false;
    std::string ext;
    for (size_t e = name.size(); e-- > 0;)
      if (name[e] == '.') {
        ext = name.substr(e);
        break;
      }
    if (contains(kSkipExts, ext)) return false;
    return !path_allowed(rs, plan, fp.data(), fp.size());
  }
};

bool is_binary(const uint8_t* p, int64_t n) {  // utils.go:71-89
  const int64_t h = n < 300 ? n : 300;
  for (int64_t i = 0; i < h; i++) {
    const uint8_t b = p[i];
    if (b < 7 || b == 11 || (13 < b && b < 27) || (27 < b && b < 0x20) || b == 0x7f) return true;
  }
  return false;
}

// One member of a tar stream after archive/tar's header processing: extended headers
// ('x' PAX records, 'L' GNU long names, 'K' long link names) are applied to the entry
// they precede.  type is the header's typeflag ('\0' kept as is).
struct TarEntry {
  uint64_t hdr;   // position of the entry's own header
  uint64_t dpos;  // its data
  uint64_t size;  // data bytes (0 for header-only types)
  char type;
  std::string name;
};

bool zero_block(const uint8_t* tar, uint64_t p) {
  for (int i = 0; i < 512; i++)
    if (tar[p + i]) return false;
  return true;
}

// archive/tar Reader.Next from header position `pos`: appends entries while the position
// of the next entry group (its first extended header, or its header) is < stop.  Returns
// the position of the first group at or past stop (its headers unread), tar_len when the
// archive ended, or (uint64_t)-1 with *err on a malformed archive.  `groups` (optional)
// receives the position at which each appended entry's group starts.
uint64_t walk_tar(const uint8_t* tar, uint64_t tar_len, uint64_t pos, uint64_t stop, std::vector<TarEntry>* out,
                  std::vector<uint64_t>* groups, std::string* err) {
  std::string long_name;
  bool have_long = false;
  std::vector<std::pair<std::string, std::string>> pax;
  uint64_t group = pos;
  auto bad = [&](const char* what) {
    *err = what;
    return ~0ull;
  };
  for (;;) {  // archive/tar Reader.readHeader
    if (!have_long && pax.empty()) {
      group = pos;
      if (pos >= stop) return pos;
    }
    if (pos == tar_len) return have_long || !pax.empty() ? bad("unexpected EOF") : tar_len;
    if (tar_len - pos < 512) return bad("unexpected EOF");
    const uint8_t* h = tar + pos;
    if (zero_block(tar, pos)) {  // end: two zero blocks (or one, then end of input)
      const uint64_t p2 = pos + 512;
      if (p2 == tar_len) return tar_len;
      if (tar_len - p2 < 512) return bad("unexpected EOF");
      if (zero_block(tar, p2)) return tar_len;
      return bad("invalid header");
    }
    if (!checksum_ok(h)) return bad("invalid header");
    int64_t size;
    if (!parse_num(h + 124, 12, &size) || size < 0) return bad("invalid size");
    char type = (char)h[156];
    const bool ustar = std::memcmp(h + 257, "ustar\0" "00", 8) == 0;
    std::string name = cstr(h, 100);
    if (ustar) {
      const std::string prefix = cstr(h + 345, 155);
      if (!prefix.empty()) name = prefix + "/" + name;
    }
    const uint64_t dpos = pos + 512;
    if (dpos > tar_len) return bad("unexpected EOF");
    if (type == 'x' || type == 'L' || type == 'K') {
      if ((uint64_t)size > tar_len - dpos) return bad("unexpected EOF");
      if (type == 'x') {
        if (!parse_pax(tar + dpos, (size_t)size, &pax)) return bad("invalid PAX record");
        if (pax.empty()) pax.emplace_back("", "");  // (an empty record set still binds)
      } else if (type == 'L') {
        long_name = cstr(tar + dpos, (size_t)size);
        have_long = true;
      }
      pos = dpos + (((uint64_t)size + 511) & ~511ull);
      continue;
    }
    if (have_long) name = long_name;
    for (const auto& kv : pax) {
      if (kv.first == "path") name = kv.second;
      else if (kv.first == "size") {
        // strconv.ParseInt(v, 10, 64) in archive/tar: digits only, no overflow
        int64_t v = 0;
        if (kv.second.empty()) return bad("invalid PAX size");
        for (char c : kv.second) {
          if (c < '0' || c > '9' || v > (INT64_MAX - (c - '0')) / 10) return bad("invalid PAX size");
          v = v * 10 + (c - '0');
        }
        size = v;
      }
    }
    pax.clear();
    have_long = false;
    const uint64_t dlen = header_only(type == 0 && !name.empty() && name.back() == '/' ? '5' : type) ? 0 : (uint64_t)size;
    if (dlen > tar_len - dpos) return bad("unexpected EOF");
    out->push_back({pos, dpos, dlen, type, std::move(name)});
    if (groups) groups->push_back(group);
    pos = dpos + ((dlen + 511) & ~511ull);  // > the header's position: the walk always advances
  }
}

// The index of a whole tar stream.  The header chain is inherently sequential (each size
// gives the next header), so large archives are walked speculatively in parallel: range
// k starts at the first block past its start that checksums as a ustar header and walks
// to the end of its range; the true chain, from 0, then continues into range k exactly
// where range k-1's walk left it.  If range k's walk passed that position at the start
// of an entry group, its entries from there on ARE the true chain's (a tar walk from a
// given group position is deterministic); otherwise range k is walked again from the true
// position.  Errors count only on the true chain, so the result (entries or the first
// error) is that of one sequential walk.
// walk_tar(pos, stop) with the speculative parallel walk above, same contract (entries,
// groups, return value); index_tar is walk_par(0, tar_len).
uint64_t walk_par(const uint8_t* tar, uint64_t tar_len, uint64_t pos0, uint64_t stop, std::vector<TarEntry>* out,
                  std::vector<uint64_t>* groups, std::string* err) {
  // ranges of at least 64 MiB (the "tar_range_kib" knob lowers it: tests of the stitching)
  const int64_t kib = knobs().tar_range_kib.load();
  const uint64_t kMinRange = kib > 0 ? (uint64_t)kib << 10 : 64ull << 20;
  const uint64_t span = stop > pos0 ? stop - pos0 : 0;
  const int T = (int)std::min<uint64_t>(16, std::max<uint64_t>(1, span / kMinRange));
  if (T == 1) return walk_tar(tar, tar_len, pos0, stop, out, groups, err);
  struct Part {
    uint64_t lo = 0, hi = 0, start = 0, end = 0;
    std::vector<TarEntry> e;
    std::vector<uint64_t> groups;
    std::string err;
  };
  std::vector<Part> parts(T);
  for (int k = 0; k < T; k++) {
    parts[k].lo = k == 0 ? pos0 : ((pos0 + span * k / T) & ~511ull);
    parts[k].hi = k + 1 == T ? stop : ((pos0 + span * (k + 1) / T) & ~511ull);
  }
  pool_for((size_t)T, T, [&](size_t k) {
    Part& P = parts[k];
    uint64_t c = P.lo;
    if (k > 0) {  // first plausible header of the range
      while (c + 512 <= P.hi &&
             !(std::memcmp(tar + c + 257, "ustar", 5) == 0 && checksum_ok(tar + c)))
        c += 512;
      if (c + 512 > P.hi) {
        P.start = ~0ull;  // none: the true chain crosses the range inside one member
        return;
      }
    }
    P.start = c;
    P.end = walk_tar(tar, tar_len, c, P.hi, &P.e, &P.groups, &P.err);
  }, 1);
  uint64_t pos = pos0;
  for (int k = 0; k < T; k++) {
    Part& P = parts[k];
    if (pos >= P.hi && k + 1 < T) continue;  // the previous member spans this range
    size_t first = 0;
    bool synced = false;
    if (k == 0) {
      synced = true;
    } else if (P.start != ~0ull) {
      auto it = std::lower_bound(P.groups.begin(), P.groups.end(), pos);
      if (it != P.groups.end() && *it == pos) {
        synced = true;
        first = (size_t)(it - P.groups.begin());
      } else if (P.end == pos && P.end != ~0ull) {
        synced = true;  // the walk reached the true position exactly at its stop
        first = P.e.size();
      }
    }
    if (!synced) {  // walk the range again from the true position
      P.e.clear();
      P.groups.clear();
      P.err.clear();
      P.end = walk_tar(tar, tar_len, pos, P.hi, &P.e, &P.groups, &P.err);
      first = 0;
    }
    for (size_t i = first; i < P.e.size(); i++) {
      out->push_back(std::move(P.e[i]));
      if (groups) groups->push_back(P.groups[i]);
    }
    if (P.end == ~0ull) {
      *err = P.err;
      return ~0ull;
    }
    if (P.end == tar_len) return tar_len;  // the archive ended
    pos = P.end;
  }
  return pos;
}

bool index_tar(const uint8_t* tar, uint64_t tar_len, std::vector<TarEntry>* out, std::string* err) {
  return walk_par(tar, tar_len, 0, tar_len, out, nullptr, err) != ~0ull;
}

}  // namespace
}  // namespace tsg

using namespace tsg;

extern "C" int tsg_layer_pack(const tsg_ruleset* rs, const uint8_t* tar, uint64_t tar_len,
                              const char* const* skip_files, uint32_t n_skip_files,
                              const char* const* skip_dirs, uint32_t n_skip_dirs,
                              const char* config_path, tsg_layer** out) {
  return tsg_layer_pack_shard(rs, tar, tar_len, skip_files, n_skip_files, skip_dirs, n_skip_dirs,
                              config_path, 0, 1, out);
}

namespace tsg {
namespace {

struct Walked {
  uint64_t dpos, size;
  std::string fp;
};

Gate make_gate(const tsg_ruleset* rs, const char* const* skip_files, uint32_t n_skip_files,
               const char* const* skip_dirs, uint32_t n_skip_dirs, const char* config_path) {
  Gate g{rs->rs, rs->plan.get(), base(config_path ? config_path : ""), {}, {}};
  for (uint32_t i = 0; i < n_skip_files; i++)  // walk.go:25-33
    g.skip_files.push_back(trim_left_slash(clean(skip_files[i])));
  std::vector<std::string> sd;
  for (uint32_t i = 0; i < n_skip_dirs; i++) sd.push_back(skip_dirs[i]);
  for (const char* s : {"proc", "sys", "dev"}) sd.push_back(s);  // walk.go:15
  for (const auto& s : sd) g.skip_dirs.push_back(trim_left_slash(clean(s)));
  return g;
}

// LayerTar.Walk's per-entry logic (tar.go:45-84) over entries [first, end) in walk order.
// `skipped` is tar.go:35's skipDirs: it enters with the directories earlier entries added
// (another rank's, for a range of the layer) and leaves with this run's appended.
// a clean relative path without "." / ".." elements: Rel against another such path is
// decided by prefix tests (under_skipped)
bool simple_rel_path(const std::string& p) { return is_clean(p) && p[0] != '/'; }

// tar.go:100-111 underSkippedDir: filepath.Rel(skipDir, filePath) does not start with
// "../" for some skip dir (an error ends the search: false).  For simple paths Rel is a
// prefix question: fp is the dir, below it, or its parent (Rel = "..", which Go also
// counts); other paths take the general Rel.
bool under_skipped(const std::vector<std::string>& skipped, const std::vector<uint8_t>& simple, const std::string& fp) {
  const bool fsimple = simple_rel_path(fp);
  for (size_t i = 0; i < skipped.size(); i++) {
    const std::string& s = skipped[i];
    if (fsimple && simple[i]) {
      const size_t ns = s.size(), nf = fp.size();
      if (nf == ns ? fp == s
                   : nf > ns ? fp[ns] == '/' && fp.compare(0, ns, s) == 0
                             : s[nf] == '/' && s.compare(0, nf, fp) == 0 && s.find('/', nf + 1) == std::string::npos)
        return true;
      continue;
    }
    std::string r;
    if (!rel(s, fp, &r)) return false;
    if (!starts_with(r, "../")) return true;
  }
  return false;
}

// LayerTar.Walk's per-entry logic (tar.go:45-84) over entries [first, end) in walk order.
// `skipped` is tar.go:35's skipDirs: it enters with the directories earlier entries added
// (another rank's, for a range of the layer) and leaves with this run's appended.
void classify(const std::vector<TarEntry>& entries, size_t first, const Gate& g,
              std::vector<std::string>* skipped, tsg_layer* L, std::vector<Walked>* walked) {
  // the per-entry path work (Clean) in parallel; the walk's order-dependent logic (skip
  // dirs accumulate in archive order) sequentially below
  const size_t n = entries.size() > first ? entries.size() - first : 0;
  std::vector<std::string> fps(n);
  pool_for(n, 16, [&](size_t j) { fps[j] = trim_left_slash(clean(entries[first + j].name)); }, 256);
  std::vector<uint8_t> simple;
  for (const auto& x : *skipped) simple.push_back(simple_rel_path(x));
  for (size_t i = first; i < entries.size(); i++) {
    const TarEntry& te = entries[i];
    char type = te.type;
    const std::string& name = te.name;
    if (type == 0) type = (!name.empty() && name.back() == '/') ? '5' : '0';
    std::string& fp = fps[i - first];  // (already without leading "/")
    const std::string_view fv(fp);
    const size_t k = fv.rfind('/');
    const std::string_view fdir = k == std::string_view::npos ? std::string_view() : fv.substr(0, k + 1);
    const std::string_view fname = k == std::string_view::npos ? fv : fv.substr(k + 1);
    if (fname == ".wh..wh..opq") {
      L->opq.append(fdir);
      L->opq += '\0';
      continue;
    }
    if (fname.substr(0, 4) == ".wh.") {
      std::string j(fdir);
      j.append(fname.substr(4));
      L->wh += j.empty() ? j : clean(j);
      L->wh += '\0';
      continue;
    }
    if (type == '5') {
      // walk.go:56-71 (base(fp) is fname for a non-empty clean path)
      if ((!fp.empty() && fname == ".git") || contains(g.skip_dirs, fp)) {
        skipped->push_back(fp);
        simple.push_back(simple_rel_path(fp));
      }
      continue;  // directories carry no content
    }
    if (type != '0') continue;  // links, devices, fifos, sparse, contiguous: no content
    if (contains(g.skip_files, fp)) continue;
    if (under_skipped(*skipped, simple, fp)) continue;
    L->walked++;
    walked->push_back({te.dpos, te.size, std::move(fp)});
  }
}

}  // namespace
}  // namespace tsg

namespace tsg {

struct SinkError {
  int rc;
  std::string msg;
};

// Where a pack's kept files go: the layer's own pageable buffer (tsg_layer_pack /
// tsg_fs_pack), or a pinned slot of a context (the *_pack_slot entry points: the bytes are
// written once, straight into the memory the device uploads from).
struct Sink {
  tsg_ctx* ctx = nullptr;
  tsg_slot_view v{};
  bool held = false;
  // room for `total` bytes of nfiles files and pbytes of paths; the data pointer
  uint8_t* reserve(tsg_layer* L, uint64_t total, uint32_t nfiles, uint64_t pbytes) {
    if (!ctx) {
      L->data.reset(new uint8_t[total ? total : 1]);
      return L->data.get();
    }
    const int rc = tsg_slot_acquire(ctx, total, nfiles, pbytes, &v);
    if (rc != TSG_OK) throw SinkError{rc, tsg_last_error()};
    held = true;
    L->ext = v.data;
    return v.data;
  }
  // the batch's offsets and paths into the slot
  void finish(const tsg_layer* L) {
    if (!ctx) return;
    std::memcpy(v.offsets, L->offsets.data(), L->offsets.size() * sizeof(uint64_t));
    if (!L->paths.empty()) std::memcpy(v.paths, L->paths.data(), L->paths.size());
    std::memcpy(v.path_offsets, L->path_offsets.data(), L->path_offsets.size() * sizeof(uint64_t));
  }
  uint32_t take() {
    held = false;
    return v.id;
  }
  ~Sink() {
    if (held) (void)tsg_slot_release(ctx, v.id);
  }
};

// The kept files of L (offsets / paths already laid out) scanned in pieces of about the
// context's slot size, in order: each piece is written straight into a pinned slot by
// fill(i, dst) (file i's bytes; returns how many it wrote, <= its size: a file that shrank
// since the walk), submitted, and released (free again once its job is done), while the
// next piece is being written, so ingest, upload, kernels and host resolution of successive
// pieces overlap.  The pieces' results are joined in file order into *out; L's offsets
// become the files' actual sizes.
int scan_in_pieces(tsg_ctx* ctx, tsg_layer* L, const std::function<uint64_t(size_t, uint8_t*)>& fill,
                   tsg_result** out, const std::vector<uint8_t>* drop) {
  const size_t n = L->offsets.size() - 1;
  // about 8 pieces of at least 16 MiB (a batch has ~0.5 ms of fixed cost, tools/batch_sizes.py)
  // and at most a slot: with one piece nothing overlaps -- a 200 MiB tree in 9 pieces
  // collects 1.3 ms after its last submit against 5.8 ms in one (profiles/r04/fs_pieces)
  // (the "piece_mib" knob overrides the floor: measurements)
  const uint64_t floor_mib = knobs().piece_mib.load() > 0 ? (uint64_t)knobs().piece_mib.load() : 16;
  const uint64_t piece_bytes =
      std::min(ctx_slot_bytes(ctx), std::max<uint64_t>(floor_mib << 20, L->offsets.back() / 8));
  std::vector<uint64_t> tickets, got(n, 0);
  int rc = TSG_OK;
  size_t i = 0;
  // TSG_LAYER_PROF: time waiting for a free slot, writing pieces, submitting, collecting
  const bool prof = getenv("TSG_LAYER_PROF") != nullptr;
  double t_acq = 0, t_fill = 0, t_sub = 0;
  auto now = [] { return std::chrono::steady_clock::now(); };
  auto ms = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
    return std::chrono::duration<double, std::milli>(b - a).count();
  };
  while (i < n && rc == TSG_OK) {
    const size_t a = i;
    while (i < n && (i == a || L->offsets[i + 1] - L->offsets[a] <= piece_bytes)) i++;
    const uint64_t bytes = L->offsets[i] - L->offsets[a];
    const uint64_t pbytes = L->path_offsets[i] - L->path_offsets[a];
    tsg_slot_view v;
    const auto p0 = now();
    if ((rc = tsg_slot_acquire(ctx, bytes, (uint32_t)(i - a), pbytes, &v))) break;
    const auto p1 = now();
    pool_for(i - a, 16, [&](size_t k) {
      got[a + k] = fill(a + k, v.data + (L->offsets[a + k] - L->offsets[a]));
    }, 1);
    const auto p2 = now();
    t_acq += ms(p0, p1);
    t_fill += ms(p1, p2);
    uint64_t o = 0;
    v.offsets[0] = 0;
    v.path_offsets[0] = 0;
    for (size_t k = 0; k < i - a; k++) {  // (a short file moves the rest of the piece down)
      const uint64_t at = L->offsets[a + k] - L->offsets[a];
      if (o != at && got[a + k]) std::memmove(v.data + o, v.data + at, got[a + k]);
      o += got[a + k];
      v.offsets[k + 1] = o;
      v.path_offsets[k + 1] = L->path_offsets[a + k + 1] - L->path_offsets[a];
    }
    if (pbytes) std::memcpy(v.paths, L->paths.data() + L->path_offsets[a], pbytes);
    uint64_t t = 0;
    const auto p3 = now();
    rc = tsg_slot_submit(ctx, v.id, (uint32_t)(i - a), &t);
    const int rr = tsg_slot_release(ctx, v.id);
    t_sub += ms(p3, now());
    if (!rc) {
      tickets.push_back(t);
      rc = rr;
    }
  }
  const auto c0 = now();
  // every submitted piece is collected, also after a failure (nothing stays pending)
  auto res = std::make_unique<tsg_result>();
  res->buf.assign(8, '\0');
  int crc = TSG_OK;
  for (uint64_t t : tickets) {
    tsg_result* r = nullptr;
    const int e = tsg_batch_collect(ctx, t, &r);
    if (e) {
      if (!crc) crc = e;
      continue;
    }
    res->buf.append(r->buf, 8, std::string::npos);  // the piece's records (after its header)
    tsg_result_free(r);
  }
  if (prof)
    fprintf(stderr, "pieces: %zu pieces, %zu files: slot waits %.1f ms, writes %.1f ms, submits %.1f ms, "
            "collect after the last submit %.1f ms\n", tickets.size(), n, t_acq, t_fill, t_sub, ms(c0, now()));
  if (rc || crc) return rc ? rc : crc;
  const uint32_t hdr[2] = {0x31475354u, (uint32_t)n};
  std::memcpy(&res->buf[0], hdr, 8);
  if (drop) {  // the files fill() dropped leave the result and L
    std::vector<size_t> rec;
    result_record_spans(res->buf, &rec);
    auto kept = std::make_unique<tsg_result>();
    kept->buf.assign(8, '\0');
    std::string paths;
    std::vector<uint64_t> offs{0}, poffs{0};
    for (size_t k = 0; k < n; k++) {
      if ((*drop)[k]) continue;
      kept->buf.append(res->buf, rec[k], rec[k + 1] - rec[k]);
      offs.push_back(offs.back() + got[k]);
      paths.append(L->paths, L->path_offsets[k], L->path_offsets[k + 1] - L->path_offsets[k]);
      poffs.push_back(paths.size());
    }
    const uint32_t h2[2] = {0x31475354u, (uint32_t)(offs.size() - 1)};
    std::memcpy(&kept->buf[0], h2, 8);
    L->offsets.swap(offs);
    L->path_offsets.swap(poffs);
    L->paths.swap(paths);
    *out = kept.release();
    return TSG_OK;
  }
  for (size_t k = 0; k < n; k++) L->offsets[k + 1] = L->offsets[k] + got[k];
  *out = res.release();
  return TSG_OK;
}

namespace {

// AnalyzerGroup.AnalyzeFile (analyzer.go:399-409) + SecretAnalyzer.Analyze: the gates of the
// walked files in parallel (Required's AllowPath is the costly part), then the kept files
// copied into the batch (the sink) in parallel
// the gates of the walked files in parallel; the kept ones (in walk order) get their
// offsets and "/"-prefixed paths in L; returns their indices into walked
std::vector<size_t> gate_kept(const uint8_t* tar, const Gate& g, const std::vector<Walked>& walked, tsg_layer* L) {
  const size_t n = walked.size();
  std::vector<uint8_t> keep(n);
  pool_for(n, 16, [&](size_t i) {
    const Walked& w = walked[i];
    keep[i] = g.required(w.fp, (int64_t)w.size) && !is_binary(tar + w.dpos, (int64_t)w.size);
  }, 64);
  std::vector<size_t> kept;
  uint64_t total = 0;
  for (size_t i = 0; i < n; i++)
    if (keep[i]) {
      kept.push_back(i);
      total += walked[i].size;
      L->offsets.push_back(total);
      L->paths += '/';
      L->paths += walked[i].fp;
      L->path_offsets.push_back(L->paths.size());
    }
  return kept;
}

void gate_and_pack(const uint8_t* tar, const Gate& g, const std::vector<Walked>& walked, tsg_layer* L,
                   std::chrono::steady_clock::time_point t0, Sink& sink) {
  auto now = [] { return std::chrono::steady_clock::now(); };
  const bool prof = getenv("TSG_LAYER_PROF") != nullptr;
  auto t1 = now();
  const size_t n = walked.size();
  const int T = 16;  // the process-wide host pool (plan.cpp)
  const std::vector<size_t> kept = gate_kept(tar, g, walked, L);
  auto t2 = now();
  std::vector<uint64_t> dst(n);
  std::vector<uint8_t> keep(n, 0);
  for (size_t k = 0; k < kept.size(); k++) {
    dst[kept[k]] = L->offsets[k];
    keep[kept[k]] = 1;
  }
  const uint64_t total = L->offsets.back();
  uint8_t* const out = sink.reserve(L, total, (uint32_t)(L->offsets.size() - 1), L->paths.size());
  // the copies in pieces of at most 4 MiB, so one large file does not serialize the pack
  constexpr uint64_t kPiece = 4ull << 20;
  std::vector<std::pair<size_t, uint64_t>> pieces;  // (file, offset in it)
  for (size_t i = 0; i < n; i++)
    if (keep[i])
      for (uint64_t o = 0; o < walked[i].size; o += kPiece) pieces.push_back({i, o});
  pool_for(pieces.size(), T, [&](size_t k) {
    const size_t i = pieces[k].first;
    const uint64_t o = pieces[k].second, len = std::min(kPiece, walked[i].size - o);
    std::memcpy(out + dst[i] + o, tar + walked[i].dpos + o, len);
  }, 16);
  sink.finish(L);
  if (prof)
    fprintf(stderr, "layer: walk %.1f ms, gates %.1f ms, pack %.1f ms (%d threads)\n",
            std::chrono::duration<double, std::milli>(t1 - t0).count(),
            std::chrono::duration<double, std::milli>(t2 - t1).count(),
            std::chrono::duration<double, std::milli>(now() - t2).count(), T);
}

}  // namespace
}  // namespace tsg

// One rank's share of a layer (SURVEY.md §8e, configs[2]): every rank indexes the header
// chain (headers only, parallel), and applies the walker's whiteout / skip-dir logic, which
// needs the whole chain; the walked files are then cut into `world` contiguous runs of
// about equal bytes, and only this rank's run is gated (Required, IsBinary) and packed.
// (tsg_layer_range_* below splits the index itself over the ranks.)
static int layer_pack(const tsg_ruleset* rs, const uint8_t* tar, uint64_t tar_len,
                      const char* const* skip_files, uint32_t n_skip_files,
                      const char* const* skip_dirs, uint32_t n_skip_dirs,
                      const char* config_path, uint32_t rank, uint32_t world, Sink& sink,
                      tsg_layer** out) {
  if (!rs || !out || (!tar && tar_len) || world == 0 || rank >= world)
    return fail(TSG_ERR_ARG, "bad argument");
  *out = nullptr;
  try {
    const Gate g = make_gate(rs, skip_files, n_skip_files, skip_dirs, n_skip_dirs, config_path);
    const auto t0 = std::chrono::steady_clock::now();
    auto L = std::make_unique<tsg_layer>();
    std::vector<Walked> walked;
    std::vector<std::string> skipped;  // tar.go:35 skipDirs
    std::vector<TarEntry> entries;
    {
      std::string err;
      if (!index_tar(tar, tar_len, &entries, &err))
        return fail(TSG_ERR_ARG, std::string("failed to extract the archive: ") + err);
    }
    classify(entries, 0, g, &skipped, L.get(), &walked);
    if (world > 1) {  // this rank's contiguous run of the walked files, by bytes
      uint64_t all = 0;
      for (const Walked& w : walked) all += w.size;
      std::vector<Walked> mine;
      uint64_t p = 0;
      for (size_t i = 0; i < walked.size(); i++) {
        // owner of the file's first byte (zero-length files: of their position)
        const uint64_t r = all ? (uint64_t)((unsigned __int128)p * world / all) : i * world / walked.size();
        if (r == rank) mine.push_back(std::move(walked[i]));
        p += walked[i].size;
      }
      walked.swap(mine);
    }
    gate_and_pack(tar, g, walked, L.get(), t0, sink);
    *out = L.release();
    return TSG_OK;
  } catch (const SinkError& e) {
    return fail(e.rc, e.msg);
  } catch (const std::bad_alloc&) {
    return fail(TSG_ERR_NOMEM, "out of memory");
  } catch (const std::exception& e) {
    return fail(TSG_ERR_INTERNAL, e.what());
  }
}

extern "C" int tsg_layer_pack_shard(const tsg_ruleset* rs, const uint8_t* tar, uint64_t tar_len,
                                    const char* const* skip_files, uint32_t n_skip_files,
                                    const char* const* skip_dirs, uint32_t n_skip_dirs,
                                    const char* config_path, uint32_t rank, uint32_t world,
                                    tsg_layer** out) {
  Sink sink;
  return layer_pack(rs, tar, tar_len, skip_files, n_skip_files, skip_dirs, n_skip_dirs, config_path, rank,
                    world, sink, out);
}

// tsg_layer_pack with the kept files copied once, tar -> a pinned slot of ctx
extern "C" int tsg_layer_pack_slot(tsg_ctx* ctx, const uint8_t* tar, uint64_t tar_len,
                                   const char* const* skip_files, uint32_t n_skip_files,
                                   const char* const* skip_dirs, uint32_t n_skip_dirs,
                                   const char* config_path, uint32_t* slot_id, tsg_layer** out) {
  if (!ctx || !slot_id) return fail(TSG_ERR_ARG, "bad argument");
  Sink sink;
  sink.ctx = ctx;
  const int rc = layer_pack(ctx_ruleset(ctx), tar, tar_len, skip_files, n_skip_files, skip_dirs, n_skip_dirs,
                            config_path, 0, 1, sink, out);
  if (rc == TSG_OK) *slot_id = sink.take();
  return rc;
}

// One call: walk, gate and scan a layer, pipelined in pieces (scan_in_pieces)
extern "C" int tsg_layer_scan(tsg_ctx* ctx, const uint8_t* tar, uint64_t tar_len,
                              const char* const* skip_files, uint32_t n_skip_files,
                              const char* const* skip_dirs, uint32_t n_skip_dirs, const char* config_path,
                              tsg_layer** layer, tsg_result** out) {
  if (!ctx || !layer || !out || (!tar && tar_len)) return fail(TSG_ERR_ARG, "bad argument");
  *layer = nullptr;
  *out = nullptr;
  try {
    const auto t0 = std::chrono::steady_clock::now();
    const Gate g = make_gate(ctx_ruleset(ctx), skip_files, n_skip_files, skip_dirs, n_skip_dirs, config_path);
    auto L = std::make_unique<tsg_layer>();
    std::vector<TarEntry> entries;
    {
      std::string err;
      if (!index_tar(tar, tar_len, &entries, &err))
        return fail(TSG_ERR_ARG, std::string("failed to extract the archive: ") + err);
    }
    const auto t1 = std::chrono::steady_clock::now();
    std::vector<std::string> skipped;
    std::vector<Walked> walked;
    classify(entries, 0, g, &skipped, L.get(), &walked);
    const auto t2 = std::chrono::steady_clock::now();
    const std::vector<size_t> kept = gate_kept(tar, g, walked, L.get());
    if (getenv("TSG_LAYER_PROF"))
      fprintf(stderr, "layer scan: index %.1f ms, classify %.1f ms, gates %.1f ms\n",
              std::chrono::duration<double, std::milli>(t1 - t0).count(),
              std::chrono::duration<double, std::milli>(t2 - t1).count(),
              std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t2).count());
    constexpr uint64_t kPart = 4ull << 20;  // (a large file is copied by several threads)
    const int rc = scan_in_pieces(ctx, L.get(), [&](size_t k, uint8_t* dst) {
      const Walked& w = walked[kept[k]];
      if (w.size <= kPart) {
        std::memcpy(dst, tar + w.dpos, w.size);
      } else {
        pool_for((w.size + kPart - 1) / kPart, 16, [&](size_t j) {
          std::memcpy(dst + j * kPart, tar + w.dpos + j * kPart, std::min(kPart, w.size - j * kPart));
        }, 1);
      }
      return w.size;
    }, out, nullptr);
    if (rc) return rc;
    *layer = L.release();
    return TSG_OK;
  } catch (const std::bad_alloc&) {
    return fail(TSG_ERR_NOMEM, "out of memory");
  } catch (const std::exception& e) {
    return fail(TSG_ERR_INTERNAL, e.what());
  }
}

// ---------------------------------------------------------------- distributed index
// The header index split over the ranks (configs[2] at N GPUs): rank r owns the entry groups
// that start in its byte range [lo, hi) of the tar.  The speculative walk of index_tar runs
// per rank (tsg_layer_range_walk); the ranks exchange {lo, hi, start, end} and fix the true
// chain in rank order (trivy_amd/shard.py:layer_chain); a rank whose speculative start was
// not on the chain is re-synced with tsg_layer_range_sync.  The skip dirs each range adds
// (tsg_layer_range_dirs) go to the later ranks, which apply them before their own (tar.go:35
// accumulates them in walk order); then every rank classifies, gates and packs its range.
struct tsg_layer_range {
  const uint8_t* tar;
  uint64_t tar_len, lo, hi, start, end;
  std::vector<tsg::TarEntry> e;
  std::vector<uint64_t> groups;
  std::string err;
  size_t first = 0;      // first entry on the true chain (after a sync)
  bool synced = false;
  bool empty = false;    // no group starts in the range
};

extern "C" int tsg_layer_range_walk(const uint8_t* tar, uint64_t tar_len, uint32_t rank, uint32_t world,
                                    tsg_layer_range** out, uint64_t info[4]) {
  if (!out || !info || (!tar && tar_len) || world == 0 || rank >= world) return fail(TSG_ERR_ARG, "bad argument");
  *out = nullptr;
  try {
    auto R = std::make_unique<tsg_layer_range>();
    R->tar = tar;
    R->tar_len = tar_len;
    R->lo = (uint64_t)((unsigned __int128)tar_len * rank / world) & ~511ull;
    R->hi = rank + 1 == world ? tar_len : ((uint64_t)((unsigned __int128)tar_len * (rank + 1) / world) & ~511ull);
    uint64_t c = R->lo;
    if (rank > 0) {  // first plausible header of the range
      while (c + 512 <= R->hi && !(std::memcmp(tar + c + 257, "ustar", 5) == 0 && tsg::checksum_ok(tar + c)))
        c += 512;
    }
    if (rank > 0 && c + 512 > R->hi) {
      R->start = R->end = ~0ull;  // none: the chain crosses the range inside one member
    } else {
      R->start = c;
      R->end = tsg::walk_par(tar, tar_len, c, R->hi, &R->e, &R->groups, &R->err);
    }
    info[0] = R->lo;
    info[1] = R->hi;
    info[2] = R->start;
    info[3] = R->end;
    *out = R.release();
    return TSG_OK;
  } catch (const std::bad_alloc&) {
    return fail(TSG_ERR_NOMEM, "out of memory");
  } catch (const std::exception& e) {
    return fail(TSG_ERR_INTERNAL, e.what());
  }
}

// The true chain enters the range at `pos` (the previous range's true end; 0 for rank 0).
// Keeps the walk's entries from there, or walks the range again from pos.  *end = the true
// end of this range (the next range's pos).  A malformed archive on the true chain fails
// with the walker's error, as one sequential walk would.
extern "C" int tsg_layer_range_sync(tsg_layer_range* R, uint64_t pos, uint64_t* end) {
  if (!R || !end) return fail(TSG_ERR_ARG, "bad argument");
  try {
    R->synced = true;
    if (pos >= R->hi) {  // the previous member spans this range, or the archive ended
      R->empty = true;
      R->first = R->e.size();
      *end = pos;
      return TSG_OK;
    }
    bool ok = false;
    if (R->start == pos) {
      ok = true;
      R->first = 0;
    } else if (R->start != ~0ull) {
      auto it = std::lower_bound(R->groups.begin(), R->groups.end(), pos);
      if (it != R->groups.end() && *it == pos) {
        ok = true;
        R->first = (size_t)(it - R->groups.begin());
      } else if (R->end == pos) {
        ok = true;  // the walk reached the true position exactly at its stop
        R->first = R->e.size();
      }
    }
    if (!ok) {
      R->e.clear();
      R->groups.clear();
      R->err.clear();
      R->first = 0;
      R->start = pos;
      R->end = tsg::walk_par(R->tar, R->tar_len, pos, R->hi, &R->e, &R->groups, &R->err);
    }
    if (R->end == ~0ull) return fail(TSG_ERR_ARG, std::string("failed to extract the archive: ") + R->err);
    *end = R->end;
    return TSG_OK;
  } catch (const std::bad_alloc&) {
    return fail(TSG_ERR_NOMEM, "out of memory");
  } catch (const std::exception& e) {
    return fail(TSG_ERR_INTERNAL, e.what());
  }
}

// The directories this range's entries add to the walker's skipDirs (tar.go:62-66), as
// NUL-terminated strings in walk order (*out valid until the range is freed).
extern "C" int tsg_layer_range_dirs(tsg_layer_range* R, const char* const* skip_dirs, uint32_t n_skip_dirs,
                                    const char** out, uint64_t* out_len) {
  if (!R || !out || !out_len || !R->synced) return fail(TSG_ERR_ARG, "bad argument");
  try {
    std::vector<std::string> sd;
    for (uint32_t i = 0; i < n_skip_dirs; i++) sd.push_back(skip_dirs[i]);
    for (const char* s : {"proc", "sys", "dev"}) sd.push_back(s);
    for (auto& s : sd) s = tsg::trim_left_slash(tsg::clean(s));
    R->err.clear();
    for (size_t i = R->first; i < R->e.size(); i++) {
      const tsg::TarEntry& te = R->e[i];
      const bool dir = te.type == '5' || (te.type == 0 && !te.name.empty() && te.name.back() == '/');
      if (!dir) continue;
      const std::string fp = tsg::trim_left_slash(tsg::clean(te.name));
      const size_t k = fp.rfind('/');
      const std::string fname = k == std::string::npos ? fp : fp.substr(k + 1);
      if (fname == ".wh..wh..opq" || tsg::starts_with(fname, ".wh.")) continue;
      if (tsg::base(fp) == ".git" || tsg::contains(sd, fp)) {
        R->err += fp;
        R->err += '\0';
      }
    }
    *out = R->err.data();
    *out_len = R->err.size();
    return TSG_OK;
  } catch (const std::exception& e) {
    return fail(TSG_ERR_INTERNAL, e.what());
  }
}

// Classify, gate and pack the range's entries (tsg_layer_pack's batch for them); `prior`
// holds the skip dirs of the ranks before this one, in rank order.
static int range_pack(const tsg_ruleset* rs, const tsg_layer_range* R, const char* const* skip_files,
                      uint32_t n_skip_files, const char* const* skip_dirs, uint32_t n_skip_dirs,
                      const char* const* prior, uint32_t n_prior, const char* config_path, tsg::Sink& sink,
                      tsg_layer** out) {
  if (!rs || !R || !out || !R->synced) return fail(TSG_ERR_ARG, "bad argument");
  *out = nullptr;
  try {
    const auto t0 = std::chrono::steady_clock::now();
    const tsg::Gate g = tsg::make_gate(rs, skip_files, n_skip_files, skip_dirs, n_skip_dirs, config_path);
    auto L = std::make_unique<tsg_layer>();
    std::vector<std::string> skipped;
    for (uint32_t i = 0; i < n_prior; i++) skipped.push_back(prior[i]);
    std::vector<tsg::Walked> walked;
    tsg::classify(R->e, R->first, g, &skipped, L.get(), &walked);
    tsg::gate_and_pack(R->tar, g, walked, L.get(), t0, sink);
    *out = L.release();
    return TSG_OK;
  } catch (const tsg::SinkError& e) {
    return fail(e.rc, e.msg);
  } catch (const std::bad_alloc&) {
    return fail(TSG_ERR_NOMEM, "out of memory");
  } catch (const std::exception& e) {
    return fail(TSG_ERR_INTERNAL, e.what());
  }
}

extern "C" int tsg_layer_range_pack(const tsg_ruleset* rs, const tsg_layer_range* R,
                                    const char* const* skip_files, uint32_t n_skip_files,
                                    const char* const* skip_dirs, uint32_t n_skip_dirs,
                                    const char* const* prior, uint32_t n_prior,
                                    const char* config_path, tsg_layer** out) {
  tsg::Sink sink;
  return range_pack(rs, R, skip_files, n_skip_files, skip_dirs, n_skip_dirs, prior, n_prior, config_path, sink,
                    out);
}

// tsg_layer_range_pack with the range's kept files copied once, tar -> a pinned slot of ctx
extern "C" int tsg_layer_range_pack_slot(tsg_ctx* ctx, const tsg_layer_range* R,
                                         const char* const* skip_files, uint32_t n_skip_files,
                                         const char* const* skip_dirs, uint32_t n_skip_dirs,
                                         const char* const* prior, uint32_t n_prior,
                                         const char* config_path, uint32_t* slot_id, tsg_layer** out) {
  if (!ctx || !slot_id) return fail(TSG_ERR_ARG, "bad argument");
  tsg::Sink sink;
  sink.ctx = ctx;
  const int rc = range_pack(tsg::ctx_ruleset(ctx), R, skip_files, n_skip_files, skip_dirs, n_skip_dirs, prior,
                            n_prior, config_path, sink, out);
  if (rc == TSG_OK) *slot_id = sink.take();
  return rc;
}

extern "C" void tsg_layer_range_free(tsg_layer_range* R) { delete R; }

extern "C" int tsg_layer_get(const tsg_layer* L, tsg_layer_view* v) {
  if (!L || !v) return fail(TSG_ERR_ARG, "bad argument");
  v->data = L->ext ? L->ext : (L->offsets.back() && L->data) ? L->data.get() : nullptr;
  v->offsets = L->offsets.data();
  v->nfiles = (uint32_t)(L->offsets.size() - 1);
  v->paths = (const uint8_t*)L->paths.data();
  v->path_offsets = L->path_offsets.data();
  v->opq = L->opq.data();
  v->opq_len = L->opq.size();
  v->wh = L->wh.data();
  v->wh_len = L->wh.size();
  v->walked = L->walked;
  return TSG_OK;
}

extern "C" void tsg_layer_free(tsg_layer* L) { delete L; }

// ---------------------------------------------------------------- filesystem ingest
// walker.FS.Walk (pkg/fanal/walker/fs.go:25-63) + the fs artifact's callback
// (pkg/fanal/artifact/local/fs.go:83-100) + AnalyzerGroup.AnalyzeFile's Required gate
// (analyzer.go:399-409) + SecretAnalyzer.Analyze's IsBinary (secret.go:78-84): walks a
// directory tree and packs every file the secret analyzer would scan into one batch.
// The reference walks with concurrent goroutines (order unspecified); here the tree is
// walked level by level on the host pool and files are packed in path order.
//   1. walk: each level's directories listed in parallel; lstat per entry (regular files
//      only, fs.go:37-38), skip dirs / files, Required on the walk-time size;
//   2. heads: every kept file opened once in parallel; a file up to kSmall bytes is read
//      whole, a larger one only for IsBinary's 300 bytes (utils.go:74-77);
//   3. pack: the non-binary files in path order into the sink (a pinned slot for
//      tsg_fs_pack_slot): small files copied from their head, large files read straight
//      into place with pread.
namespace tsg {
namespace {

constexpr uint64_t kSmall = 64 << 10;

struct FsFile {
  std::string full, fp;
  uint64_t size = 0;                // at the walk
  std::vector<uint8_t> head;        // whole content (size <= kSmall) or the first 300 bytes
  uint64_t got = 0;                 // bytes of the file as read
  bool keep = false;
};

// up to n bytes of the file at fd from offset 0 into p; the bytes read (a file that shrank
// since the walk is read as it is now)
uint64_t read_upto(int fd, uint8_t* p, uint64_t n) {
  uint64_t r = 0;
  while (r < n) {
    const ssize_t k = pread(fd, p + r, n - r, (off_t)r);
    if (k <= 0) break;
    r += (uint64_t)k;
  }
  return r;
}

// steps 1-2 (walk, heads) into *files (path order, keep flags) and L's walked count
// 2. io.ReadAll (secret.go:85) of a small file, IsBinary's head of a large one
void read_head(FsFile& f, int fd) {
  const uint64_t want = f.size <= kSmall ? f.size : 300;
  f.head.resize(want);
  const uint64_t r = read_upto(fd, f.head.data(), want);
  f.head.resize(r);
  f.got = f.size <= kSmall ? r : f.size;
  f.keep = !is_binary(f.head.data(), (int64_t)(f.size <= kSmall ? r : std::min<uint64_t>(r, f.size)));
}

// heads = false: no file is opened; every file that passes Required is listed with its
// lstat size (keep, got = size), for a caller that reads files straight into place and
// applies IsBinary there (tsg_fs_scan)
int fs_collect(const tsg_ruleset* rs, const char* root, const char* const* skip_files, uint32_t n_skip_files,
               const char* const* skip_dirs, uint32_t n_skip_dirs, const char* config_path,
               std::vector<std::unique_ptr<FsFile>>* out_files, uint32_t* out_walked, bool heads = true) {
  {
    Gate g{rs->rs, rs->plan.get(), base(config_path ? config_path : ""), {}, {}};
    for (uint32_t i = 0; i < n_skip_files; i++)  // walk.go:25-33
      g.skip_files.push_back(trim_left_slash(clean(skip_files[i])));
    std::vector<std::string> sd;
    for (uint32_t i = 0; i < n_skip_dirs; i++) sd.push_back(skip_dirs[i]);
    for (const char* x : {"proc", "sys", "dev"}) sd.push_back(x);  // walk.go:15
    for (const auto& x : sd) g.skip_dirs.push_back(trim_left_slash(clean(x)));
    auto skip_dir = [&](const std::string& dir) {  // walk.go:58-75
      const std::string d = trim_left_slash(dir);
      return base(d) == ".git" || contains(g.skip_dirs, d);
    };
    const std::string r0 = clean(root);
    struct stat st;
    if (lstat(r0.c_str(), &st) != 0) return fail(TSG_ERR_ARG, "walk error: cannot stat " + r0);
    // local/fs.go:86-90: a file given as the root is analyzed relative to its directory
    std::string directory = r0;
    if (!S_ISDIR(st.st_mode)) {
      const size_t k = r0.rfind('/');
      directory = k == std::string::npos ? "." : (k == 0 ? "/" : r0.substr(0, k));
    }
    const int T = 16;  // the process-wide host pool (plan.cpp)
    const auto t_walk0 = std::chrono::steady_clock::now();
    std::vector<std::unique_ptr<FsFile>> files;
    uint32_t walked = 0;
    // a regular file at `path` (name relative to the open directory dfd, or dfd < 0): the
    // walk's file callback, its Required gate and its head; true if walked
    OpenErr oe;
    auto visit_file = [&](int dfd, const char* name, const std::string& path, std::unique_ptr<FsFile>* keep) {
      if (contains(g.skip_files, trim_left_slash(path))) return false;
      std::string fp;
      if (!rel(directory, path, &fp)) fp = path;
      // Required's path tests first (only its size test needs the file): a file they drop
      // is never opened
      if (!g.required(trim_left_slash(fp), INT64_MAX)) return true;
      if (!heads) {
        struct stat s3;
        if ((dfd >= 0 ? fstatat(dfd, name, &s3, AT_SYMLINK_NOFOLLOW) : lstat(path.c_str(), &s3)) != 0 ||
            !S_ISREG(s3.st_mode))
          return false;  // (gone or replaced since the listing)
        if (s3.st_size >= 10) {  // (secret.go:113-115)
          auto f = std::make_unique<FsFile>();
          f->full = path;
          f->fp = std::move(fp);
          f->size = f->got = (uint64_t)s3.st_size;
          f->keep = true;
          *keep = std::move(f);
        }
        return true;
      }
      const int fd = open_at_retry(dfd, dfd >= 0 ? name : path.c_str(), O_RDONLY | O_CLOEXEC);
      if (fd < 0) {  // analyzer.go:411-416 (OpenErr)
        oe.add(errno, path);
        return true;
      }
      struct stat fs2;
      if (fstat(fd, &fs2) != 0 || !S_ISREG(fs2.st_mode)) {  // (replaced since the listing)
        close(fd);
        return false;
      }
      if (fs2.st_size >= 10) {  // (secret.go:113-115)
        auto f = std::make_unique<FsFile>();
        f->full = path;
        f->fp = std::move(fp);
        f->size = (uint64_t)fs2.st_size;
        read_head(*f, fd);
        *keep = std::move(f);
      }
      close(fd);
      return true;
    };
    std::vector<std::string> level;
    {
      struct stat s0;
      if (lstat(r0.c_str(), &s0) == 0 && S_ISDIR(s0.st_mode)) {
        level.push_back(r0);
      } else if (lstat(r0.c_str(), &s0) == 0 && S_ISREG(s0.st_mode)) {  // fs.go:37-38
        std::unique_ptr<FsFile> f;
        walked += visit_file(-1, nullptr, r0, &f);
        if (oe.set) return fail(TSG_ERR_ARG, oe.msg);
        if (f) files.push_back(std::move(f));
      }
    }
    // 1. the walk, one level of directories at a time (at most kDirs open at once, so that
    // concurrent walks stay well inside a 1024-descriptor limit; a full table is waited out,
    // open_at_retry): the
    // level's directories listed in parallel (d_type; lstat only where the file system
    // does not say), then its regular files opened relative to their directory, in parallel
    constexpr size_t kDirs = 64;
    struct Dir {
      DIR* d = nullptr;
      int err = 0;                                  // open errno (not EACCES)
      std::vector<std::string> subdirs;             // cleaned paths
      std::vector<std::string> names;               // regular files
    };
    struct Entry {
      uint32_t dir;
      const std::string* name;
    };
    while (!level.empty()) {
      std::vector<std::string> next;
      for (size_t l0 = 0; l0 < level.size(); l0 += kDirs) {
        const size_t nd = std::min(kDirs, level.size() - l0);
        std::vector<Dir> dirs(nd);
        pool_for(nd, T, [&](size_t i) {
          const std::string& path = level[l0 + i];
          Dir& v = dirs[i];
          if (skip_dir(path)) return;
          const int fd = open_at_retry(-1, path.c_str(), O_RDONLY | O_DIRECTORY | O_NOFOLLOW | O_CLOEXEC);
          if (fd < 0 || !(v.d = fdopendir(fd))) {
            if (fd >= 0) close(fd);
            // fs.go:48-55: permission errors are ignored; so is a directory gone (or
            // replaced) since its parent was listed
            if (errno != EACCES && errno != ENOENT && errno != ENOTDIR && errno != ELOOP) v.err = errno ? errno : EIO;
            return;
          }
          const int dfd = dirfd(v.d);
          while (dirent* e = readdir(v.d)) {
            const char* nm = e->d_name;
            if (!strcmp(nm, ".") || !strcmp(nm, "..")) continue;
            unsigned char t = e->d_type;
            if (t == DT_UNKNOWN) {
              struct stat s2;
              if (fstatat(dfd, nm, &s2, AT_SYMLINK_NOFOLLOW) != 0) continue;
              t = S_ISDIR(s2.st_mode) ? DT_DIR : S_ISREG(s2.st_mode) ? DT_REG : DT_LNK;
            }
            if (t == DT_DIR) v.subdirs.push_back(clean(path + "/" + nm));
            else if (t == DT_REG) v.names.push_back(nm);
          }
        }, 1);
        std::vector<Entry> ents;
        for (size_t i = 0; i < nd; i++) {
          if (dirs[i].err) {
            for (auto& v : dirs) if (v.d) closedir(v.d);
            return fail(TSG_ERR_ARG, "walk error: cannot read " + level[l0 + i]);
          }
          for (const auto& nm : dirs[i].names) ents.push_back({(uint32_t)i, &nm});
        }
        std::vector<std::unique_ptr<FsFile>> got(ents.size());
        std::vector<uint8_t> wk(ents.size(), 0);
        pool_for(ents.size(), T, [&](size_t k) {
          const Dir& v = dirs[ents[k].dir];
          wk[k] = visit_file(dirfd(v.d), ents[k].name->c_str(), clean(level[l0 + ents[k].dir] + "/" + *ents[k].name),
                             &got[k]);
        }, 8);
        if (oe.set) {
          for (auto& v : dirs) if (v.d) closedir(v.d);
          return fail(TSG_ERR_ARG, oe.msg);
        }
        for (size_t k = 0; k < ents.size(); k++) {
          walked += wk[k];
          if (got[k]) files.push_back(std::move(got[k]));
        }
        for (auto& v : dirs) {
          if (v.d) closedir(v.d);
          for (auto& c : v.subdirs) next.push_back(std::move(c));
        }
      }
      level.swap(next);
    }
    const auto tw = std::chrono::steady_clock::now();
    std::sort(files.begin(), files.end(), [](const std::unique_ptr<FsFile>& a, const std::unique_ptr<FsFile>& b) {
      return a->fp < b->fp;
    });
    const size_t n = files.size();
    if (getenv("TSG_LAYER_PROF"))
      fprintf(stderr, "fs: walk %.1f ms, sort %.1f ms (%zu files)\n",
              std::chrono::duration<double, std::milli>(tw - t_walk0).count(),
              std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tw).count(), n);
    *out_files = std::move(files);
    *out_walked = walked;
    return TSG_OK;
  }
}

// the kept files' offsets and paths in L (fs scans keep the relative path: secret.go:94-96,
// no "/"); returns their indices
std::vector<size_t> fs_layout(const std::vector<std::unique_ptr<FsFile>>& files, tsg_layer* L) {
  std::vector<size_t> kept;
  uint64_t total = 0;
  for (size_t i = 0; i < files.size(); i++) {
    const FsFile& f = *files[i];
    if (!f.keep) continue;
    kept.push_back(i);
    total += f.got;
    L->offsets.push_back(total);
    L->paths += f.fp;
    L->path_offsets.push_back(L->paths.size());
  }
  return kept;
}

// file f's bytes at dst: a small file from its head, a large one read in place
uint64_t fs_fill(FsFile& f, uint8_t* dst, OpenErr* oe) {
  if (f.size <= kSmall) {
    if (f.got) std::memcpy(dst, f.head.data(), f.got);
    return f.got;
  }
  const int fd = open_at_retry(-1, f.full.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) oe->add(errno, f.full);
  const uint64_t r = fd < 0 ? 0 : read_upto(fd, dst, f.got);
  if (fd >= 0) close(fd);
  return r;
}

int fs_pack(const tsg_ruleset* rs, const char* root, const char* const* skip_files, uint32_t n_skip_files,
            const char* const* skip_dirs, uint32_t n_skip_dirs, const char* config_path, Sink& sink,
            tsg_layer** out) {
  if (!rs || !root || !out) return fail(TSG_ERR_ARG, "bad argument");
  *out = nullptr;
  try {
    std::vector<std::unique_ptr<FsFile>> files;
    uint32_t walked = 0;
    int rc = fs_collect(rs, root, skip_files, n_skip_files, skip_dirs, n_skip_dirs, config_path, &files, &walked);
    if (rc) return rc;
    auto L = std::make_unique<tsg_layer>();
    L->walked = walked;
    // 3. the pack, in path order
    const std::vector<size_t> kept = fs_layout(files, L.get());
    uint8_t* const dst = sink.reserve(L.get(), L->offsets.back(), (uint32_t)kept.size(), L->paths.size());
    std::vector<uint64_t> got(kept.size());
    OpenErr oe;
    pool_for(kept.size(), 16, [&](size_t k) { got[k] = fs_fill(*files[kept[k]], dst + L->offsets[k], &oe); }, 4);
    if (oe.set) return fail(TSG_ERR_ARG, oe.msg);
    // a large file that shrank between the walk and its read: close the gaps (rare)
    bool short_read = false;
    for (size_t k = 0; k < kept.size(); k++) short_read |= got[k] != L->offsets[k + 1] - L->offsets[k];
    if (short_read) {
      uint64_t o = 0;
      for (size_t k = 0; k < kept.size(); k++) {
        if (o != L->offsets[k]) std::memmove(dst + o, dst + L->offsets[k], got[k]);
        o += got[k];
      }
      for (size_t k = 0; k < kept.size(); k++) L->offsets[k + 1] = L->offsets[k] + got[k];
    }
    sink.finish(L.get());
    *out = L.release();
    return TSG_OK;
  } catch (const SinkError& e) {
    return fail(e.rc, e.msg);
  } catch (const std::bad_alloc&) {
    return fail(TSG_ERR_NOMEM, "out of memory");
  } catch (const std::exception& e) {
    return fail(TSG_ERR_INTERNAL, e.what());
  }
}

}  // namespace
}  // namespace tsg

// One rank's share of a tree (SURVEY.md §8e, configs[0] over several GPUs): every rank lists
// the tree (no file is opened: Required's path tests and lstat sizes), the listed files in
// path order are cut into `world` contiguous runs of about equal bytes, and only this rank's
// run is read, IsBinary-gated and packed.  The union over the ranks, in rank order, is
// tsg_fs_pack's batch; walked is the whole tree's.
extern "C" int tsg_fs_pack_shard(const tsg_ruleset* rs, const char* root, const char* const* skip_files,
                                 uint32_t n_skip_files, const char* const* skip_dirs, uint32_t n_skip_dirs,
                                 const char* config_path, uint32_t rank, uint32_t world, tsg_layer** out) {
  if (!rs || !root || !out || world == 0 || rank >= world) return fail(TSG_ERR_ARG, "bad argument");
  *out = nullptr;
  try {
    std::vector<std::unique_ptr<tsg::FsFile>> files;
    uint32_t walked = 0;
    int rc = tsg::fs_collect(rs, root, skip_files, n_skip_files, skip_dirs, n_skip_dirs, config_path, &files,
                             &walked, false);
    if (rc) return rc;
    uint64_t all = 0;
    for (const auto& f : files) all += f->size;
    std::vector<size_t> mine;
    uint64_t p = 0;
    for (size_t i = 0; i < files.size(); i++) {  // owner of the file's first byte
      const uint64_t r = all ? (uint64_t)((unsigned __int128)p * world / all) : i * world / files.size();
      if (r == rank) mine.push_back(i);
      p += files[i]->size;
    }
    // read this rank's files whole (in parallel), then IsBinary on what was read
    std::vector<std::vector<uint8_t>> body(mine.size());
    std::vector<uint8_t> keep(mine.size(), 0);
    tsg::OpenErr oe;
    tsg::pool_for(mine.size(), 16, [&](size_t k) {
      const tsg::FsFile& f = *files[mine[k]];
      const int fd = tsg::open_at_retry(-1, f.full.c_str(), O_RDONLY | O_CLOEXEC);
      if (fd < 0) {  // analyzer.go:411-416 (OpenErr)
        oe.add(errno, f.full);
        return;
      }
      body[k].resize(f.size);
      body[k].resize(tsg::read_upto(fd, body[k].data(), f.size));
      close(fd);
      keep[k] = !tsg::is_binary(body[k].data(), (int64_t)body[k].size());
    }, 4);
    if (oe.set) return tsg::fail(TSG_ERR_ARG, oe.msg);
    auto L = std::make_unique<tsg_layer>();
    L->walked = walked;
    uint64_t total = 0;
    for (size_t k = 0; k < mine.size(); k++)
      if (keep[k]) {
        total += body[k].size();
        L->offsets.push_back(total);
        L->paths += files[mine[k]]->fp;
        L->path_offsets.push_back(L->paths.size());
      }
    tsg::Sink sink;
    uint8_t* dst = sink.reserve(L.get(), total, (uint32_t)(L->offsets.size() - 1), L->paths.size());
    std::vector<size_t> kept;
    for (size_t k = 0; k < mine.size(); k++)
      if (keep[k]) kept.push_back(k);
    tsg::pool_for(kept.size(), 16, [&](size_t j) {
      const auto& b = body[kept[j]];
      if (!b.empty()) std::memcpy(dst + L->offsets[j], b.data(), b.size());
    }, 16);
    sink.finish(L.get());
    *out = L.release();
    return TSG_OK;
  } catch (const tsg::SinkError& e) {
    return fail(e.rc, e.msg);
  } catch (const std::bad_alloc&) {
    return fail(TSG_ERR_NOMEM, "out of memory");
  } catch (const std::exception& e) {
    return fail(TSG_ERR_INTERNAL, e.what());
  }
}

extern "C" int tsg_fs_pack(const tsg_ruleset* rs, const char* root, const char* const* skip_files,
                           uint32_t n_skip_files, const char* const* skip_dirs, uint32_t n_skip_dirs,
                           const char* config_path, tsg_layer** out) {
  tsg::Sink sink;
  return tsg::fs_pack(rs, root, skip_files, n_skip_files, skip_dirs, n_skip_dirs, config_path, sink, out);
}

// One call: walk, gate and scan a tree, pipelined in pieces (scan_in_pieces)
extern "C" int tsg_fs_scan(tsg_ctx* ctx, const char* root, const char* const* skip_files, uint32_t n_skip_files,
                           const char* const* skip_dirs, uint32_t n_skip_dirs, const char* config_path,
                           tsg_layer** layer, tsg_result** out) {
  if (!ctx || !root || !layer || !out) return fail(TSG_ERR_ARG, "bad argument");
  *layer = nullptr;
  *out = nullptr;
  try {
    auto now = [] { return std::chrono::steady_clock::now(); };
    auto ms = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
      return std::chrono::duration<double, std::milli>(b - a).count();
    };
    const auto t0 = now();
    std::vector<std::unique_ptr<tsg::FsFile>> files;
    uint32_t walked = 0;
    int rc = tsg::fs_collect(tsg::ctx_ruleset(ctx), root, skip_files, n_skip_files, skip_dirs, n_skip_dirs,
                             config_path, &files, &walked, false);
    if (rc) return rc;
    const auto t1 = now();
    auto L = std::make_unique<tsg_layer>();
    L->walked = walked;
    const std::vector<size_t> kept = tsg::fs_layout(files, L.get());
    const auto t2 = now();
    // every listed file read straight into its place in a piece; an unreadable or binary
    // one is scanned along (its bytes are there already) and dropped from the results
    std::vector<uint8_t> drop(kept.size(), 0);
    tsg::OpenErr oe;
    rc = tsg::scan_in_pieces(ctx, L.get(), [&](size_t k, uint8_t* dst) -> uint64_t {
      const tsg::FsFile& f = *files[kept[k]];
      const int fd = tsg::open_at_retry(-1, f.full.c_str(), O_RDONLY | O_CLOEXEC);
      if (fd < 0) {  // analyzer.go:411-416 (OpenErr)
        oe.add(errno, f.full);
        drop[k] = 1;
        return 0;
      }
      const uint64_t r = tsg::read_upto(fd, dst, f.size);
      close(fd);
      if (tsg::is_binary(dst, (int64_t)r)) drop[k] = 1;  // secret.go:78-84 (its first 300 bytes)
      return r;
    }, out, &drop);
    if (rc) return rc;
    if (oe.set) {
      tsg_result_free(*out);
      *out = nullptr;
      return tsg::fail(TSG_ERR_ARG, oe.msg);
    }
    const auto t3 = now();
    // the listing (one heap block per file) is freed behind the return
    try {
      std::thread([f = std::move(files)]() mutable { f.clear(); }).detach();
    } catch (const std::exception&) {
      files.clear();
    }
    if (getenv("TSG_LAYER_PROF"))
      fprintf(stderr, "fs_scan: %.1f ms (walk+sort %.1f, layout %.1f, pieces %.1f, free %.1f)\n", ms(t0, now()),
              ms(t0, t1), ms(t1, t2), ms(t2, t3), ms(t3, now()));
    *layer = L.release();
    return TSG_OK;
  } catch (const std::bad_alloc&) {
    return fail(TSG_ERR_NOMEM, "out of memory");
  } catch (const std::exception& e) {
    return fail(TSG_ERR_INTERNAL, e.what());
  }
}

// tsg_fs_pack with the kept files read straight into a pinned slot of ctx
extern "C" int tsg_fs_pack_slot(tsg_ctx* ctx, const char* root, const char* const* skip_files,
                                uint32_t n_skip_files, const char* const* skip_dirs, uint32_t n_skip_dirs,
                                const char* config_path, uint32_t* slot_id, tsg_layer** out) {
  if (!ctx || !slot_id) return fail(TSG_ERR_ARG, "bad argument");
  tsg::Sink sink;
  sink.ctx = ctx;
  const int rc = tsg::fs_pack(tsg::ctx_ruleset(ctx), root, skip_files, n_skip_files, skip_dirs, n_skip_dirs,
                              config_path, sink, out);
  if (rc == TSG_OK) *slot_id = sink.take();
  return rc;
}
