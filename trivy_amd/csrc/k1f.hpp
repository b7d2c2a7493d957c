// K1F: the keyword / anchor-literal prefilter and run counters of K1 as a stateless filter
// over 16-byte words plus an exact verification of the rare filter hits (kernels.hip
// k1f_kernel), replacing the LDS-resident automaton's dependent per-byte transition chain.
//
// Semantics are k1_reference's (plan.hpp) bit for bit: keyword bits per file (a literal
// counts for the file holding its last byte when it starts inside that file), chunk events
// of every literal occurrence (its last byte's chunk) and of the two run counters, all
// literals ASCII case folded, the batch one byte stream.  The reference behaviour they
// restate is Rule.MatchKeywords (pkg/fanal/secret/scanner.go:164-176).
//
// The filter ("Teddy" style, 16 buckets): every active literal i is represented by one
// 4-byte window of its bytes, [j0_i, j0_i + 4) (j0_i < 0 for literals shorter than 4: the
// positions before the literal accept any byte), and the literals are grouped into 16
// buckets.  A 16-byte entry per byte value b holds, for window position j = 0..3, the
// dword d_j(b):
//   bits 0..15   bucket k accepts b at window position j (some literal of bucket k has b --
//                case folded -- or "any" there)
//   bits 16..23  run flags laid out so that an AND of four consecutive bytes' dwords gives
//                the flags of all four: bit 16 + j = U(b), bit 20 + j = D(b), every other
//                high bit 1
// so the window ending at byte q gives
//   R(q) = d_0(b[q-3]) & d_1(b[q-2]) & d_2(b[q-1]) & d_3(b[q])
// whose low half names the buckets that may hold a literal whose window ends at q, and
// whose byte 2 holds U and D of bytes q-3..q.  Per byte that is one conflict-free LDS read
// of the entry (replicated per 16 lanes) and two VALU ops; nothing depends on the previous
// byte's result.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "plan.hpp"

#if defined(__HIP__)
#define K1F_HD __host__ __device__
#else
#define K1F_HD
#endif

namespace tsg {

constexpr int kFBuckets = 16;
constexpr uint32_t kFTile = 1024;        // bytes of a wave's tile (64 lanes x 16 B)
constexpr uint32_t kFImgMax = 16 * 1024; // verification image staged in LDS
constexpr int kFRunU = 32, kFRunD = 12;  // run lengths the flags logic is written for

// one verification record per active literal (32 B, kept in bucket order)
struct K1FLit {
  uint32_t wkey;   // the window's bytes (ASCII lowercased; 0 where "any")
  uint32_t wmask;  // 0xFF per window byte inside the literal
  uint16_t wend;   // window end - literal start (j0 + 3)
  uint16_t len;
  uint32_t boff;   // image offset of the lowercased literal bytes (4-aligned, zero padded)
  int32_t kw;      // keyword id, or -1 (anchor literal only)
  uint32_t ev;     // event bits
  uint32_t id;     // plan literal id (sampling counters)
  uint32_t pad;
};
static_assert(sizeof(K1FLit) == 32, "K1FLit is 32 bytes");

// verification image: u16 bstart[kFBuckets + 1] (records of bucket k: [bstart[k],
// bstart[k+1])) padded to kFImgLits, the records, the literal bytes
constexpr uint32_t kFImgLits = 64;

struct K1FTables {
  std::vector<uint32_t> ent;  // [256 * 4]: d_0..d_3 of every byte value
  std::vector<uint8_t> img;   // verification image
  uint32_t nlit = 0;          // records
  std::vector<int> bucket_of; // [n_lit] bucket of each plan literal, -1 = not in the filter
  std::vector<int> j0;        // [n_lit] window offset
};

// Builds the filter for the plan's K1 literals (Plan::k1_lits) except those flagged in
// `quiet` ([n_lit], the adaptation's hot literals; empty = none).  The windows and buckets
// are priced with a Markov model of source text (bigram.inc), or -- given a sample of the
// data (the adaptation's first batch) -- by their exact counts in it.  False (with the
// reason) when K1F does not apply to the plan; the automaton K1 runs then.
bool k1f_build(const Plan& p, const std::vector<uint8_t>& quiet, K1FTables* t, std::string* why,
               const uint8_t* sample = nullptr, size_t sample_len = 0);

// CPU emulation of k1f_kernel's algorithm (filter, run flags, verification) with the same
// tables and bit logic; tests compare it with k1_reference.  hits ([nlit] or null) counts
// verified arrivals per record, stats[0] flagged word groups, stats[1] arrivals.
void k1f_emulate(const Plan& p, const K1FTables& t, const BatchView& b, uint32_t chunk,
                 std::vector<uint32_t>* kw, std::vector<uint32_t>* ev, uint64_t stats[2]);

// ------------------------------------------------------------------ shared bit logic
K1F_HD inline uint32_t k1f_perm(uint32_t s0, uint32_t s1, uint32_t sel) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_perm(s0, s1, sel);
#else
  const uint64_t v = (uint64_t)s0 << 32 | s1;  // bytes 0-3 = s1, 4-7 = s0
  uint32_t r = 0;
  for (int i = 0; i < 4; i++) {
    const uint32_t s = (sel >> (8 * i)) & 0xFF;
    const uint32_t b = s < 8 ? (uint32_t)(v >> (8 * s)) & 0xFF : s == 12 ? 0u : 0xFFu;
    r |= b << (8 * i);
  }
  return r;
#endif
}

K1F_HD inline uint32_t k1f_and3(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x80);
#else
  return a & b & c;
#endif
}
K1F_HD inline uint32_t k1f_or3(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0xFE);
#else
  return a | b | c;
#endif
}

// the run flags of one 16-byte word from the windows ending at its bytes 3, 7, 11, 15:
// bit k = U(byte k), bit 16 + k = D(byte k)
K1F_HD inline uint32_t k1f_flags(uint32_t r3, uint32_t r7, uint32_t r11, uint32_t r15) {
  // byte 2 of the window ending at 4i+3 is [U(4i..4i+3) | D(4i..4i+3) << 4]; gathered in the
  // order i = 0, 2, 1, 3 the nibbles read (low first) u0 d0 u2 d2 u1 d1 u3 d3, and one delta
  // swap at distance 12 (d0 <-> u1, d2 <-> u3) leaves u0 u1 u2 u3 d0 d1 d2 d3
  const uint32_t x = k1f_perm(r11, r3, 0x0C0C0602u) | k1f_perm(r15, r7, 0x06020C0Cu);
  const uint32_t t = ((x >> 12) ^ x) & 0x0000F0F0u;
  return x ^ t ^ (t << 12);
}

K1F_HD inline uint32_t k1f_ctz(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_ctz(x);
#else
  return (uint32_t)__builtin_ctz(x);
#endif
}

// Run events of word l from the flags of words l, l-1, l-2 (k1f_flags): bit 0 (kEvRunU) if
// some byte p of word l ends a run of >= 32 class-U bytes, bit 1 (kEvRunD) >= 12 class-D.
// A U run of 32 ending in word l covers all of word l-1: it needs word l-1 all U, a prefix
// p0 >= 1 of word l and a suffix s2 of word l-2 with s2 + 16 + p0 >= 32.
K1F_HD inline uint32_t k1f_runs(uint32_t m, uint32_t m1, uint32_t m2) {
  uint32_t x = (m1 >> 16) | (m & 0xFFFF0000u);  // D flags of words l-1 | l
  x &= x >> 1;
  x &= x >> 2;
  x &= x >> 4;
  x &= x >> 4;  // bit i: bytes i..i+11 of the pair all D
  const uint32_t evd = (x & 0x001FFFE0u) ? 2u : 0u;  // ends i + 11 in [16, 31]
  const uint32_t p0 = k1f_ctz((~m & 0xFFFFu) | 0x10000u);
  const uint32_t nm2 = ~(m2 << 16);  // leading zeros = the U suffix of word l-2
  const uint32_t s2 = nm2 ? (uint32_t)__builtin_clz(nm2) : 32u;
  const uint32_t evu = ((m1 & 0xFFFFu) == 0xFFFFu && p0 >= 1 && s2 + p0 >= 16) ? 1u : 0u;
  return evu | evd;
}

// ASCII 'A'..'Z' -> +0x20 in each byte, every other byte unchanged
K1F_HD inline uint32_t k1f_lower4(uint32_t x) {
  const uint32_t t = x & 0x7F7F7F7Fu;
  const uint32_t ge_a = t + 0x3F3F3F3Fu;  // bit 7: byte >= 'A'
  const uint32_t gt_z = t + 0x25252525u;  // bit 7: byte > 'Z'
  const uint32_t up = ge_a & ~gt_z & ~x & 0x80808080u;
  return x | (up >> 2);
}

}  // namespace tsg
