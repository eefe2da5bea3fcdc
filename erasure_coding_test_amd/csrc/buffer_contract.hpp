// buffer_contract.hpp -- the buffer contract of every coding call: the
// regions a call touches are either the SAME buffer or disjoint.
//
// The reference runs a call as a sequence of whole-region byte loops
// (galois.cpp:447-465 region multiply, :731-754 region XOR, jerasure.cpp:
// 561-620 dot products), so a destination that partially overlaps another
// region of the call (a shifted alias) gets bytes fixed by the reference's
// loop order.  The GPU kernels read and write every column in parallel across
// many workgroups, so on such input they would return different -- and, from
// launch to launch, different -- bytes.  Every entry point therefore rejects a
// partial overlap that involves a written region (ECGPU_ERR_ARG, with both
// regions named) before anything is launched.  Identical pointers keep their
// meaning: the synchronous calls replay the reference's sequence on them
// (planner.hpp), and the batched plan API allows an output that is also a
// source of its own stripe (one launch reads a column before it writes it).
// Overlapping regions that are only read give the same bytes either way and
// are allowed.
//
// Host-only code (no HIP): also compiled into the CPU tests' harness.
#pragma once
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <string>
#include <utility>
#include <vector>

namespace ecgpu {

struct Span {
  const void* p = nullptr;
  int64_t n = 0;         // bytes; spans of n <= 0 touch nothing
  bool written = false;  // the call writes this region
  int tag = 0;           // the caller's index (names the region in messages)
};

// The first pair (a, b) of spans that break the contract, or (-1, -1).
// same_ok(x, y) decides a pair of IDENTICAL spans (same pointer and length)
// of which at least one is written; any other overlap involving a written
// span is a conflict.
template <class SameOk>
std::pair<int, int> find_conflict(const std::vector<Span>& s, SameOk same_ok) {
  std::vector<int> ix;
  ix.reserve(s.size());
  for (int i = 0; i < int(s.size()); ++i)
    if (s[size_t(i)].n > 0) ix.push_back(i);
  auto addr = [&](int i) { return reinterpret_cast<uintptr_t>(s[size_t(i)].p); };
  auto end = [&](int i) { return addr(i) + uint64_t(s[size_t(i)].n); };
  std::sort(ix.begin(), ix.end(), [&](int a, int b) {
    return addr(a) != addr(b) ? addr(a) < addr(b) : s[size_t(a)].n < s[size_t(b)].n;
  });
  // 1. identical spans: every pair with a written member
  for (size_t a = 0; a < ix.size();) {
    size_t b = a + 1;
    while (b < ix.size() && addr(ix[b]) == addr(ix[a]) && s[size_t(ix[b])].n == s[size_t(ix[a])].n) ++b;
    for (size_t i = a; i < b; ++i) {
      if (!s[size_t(ix[i])].written) continue;
      for (size_t j = a; j < b; ++j)
        if (j != i && !same_ok(s[size_t(ix[i])], s[size_t(ix[j])])) return {ix[std::min(i, j)], ix[std::max(i, j)]};
    }
    a = b;
  }
  // 2. distinct spans, in address order: one sweep keeps the span reaching
  // furthest so far, and the written span reaching furthest.  A span that
  // starts before the furthest written end overlaps that span; a written span
  // that starts before the furthest end overlaps that one.  (Any overlapping
  // pair with a written member is caught at its later member.)
  int far_any = -1, far_w = -1;
  for (size_t a = 0; a < ix.size();) {
    size_t b = a + 1;
    while (b < ix.size() && addr(ix[b]) == addr(ix[a]) && s[size_t(ix[b])].n == s[size_t(ix[a])].n) ++b;
    int rep = ix[a], rep_w = -1;  // the group's representative, and a written member if any
    for (size_t i = a; i < b; ++i)
      if (s[size_t(ix[i])].written) {
        rep_w = ix[i];
        break;
      }
    const uintptr_t p = addr(rep);
    if (far_w >= 0 && p < end(far_w)) return {far_w, rep_w >= 0 ? rep_w : rep};
    if (rep_w >= 0 && far_any >= 0 && p < end(far_any)) return {far_any, rep_w};
    if (far_any < 0 || end(rep) > end(far_any)) far_any = rep_w >= 0 ? rep_w : rep;
    if (rep_w >= 0 && (far_w < 0 || end(rep_w) > end(far_w))) far_w = rep_w;
    a = b;
  }
  return {-1, -1};
}

inline std::pair<int, int> find_conflict(const std::vector<Span>& s) {
  return find_conflict(s, [](const Span&, const Span&) { return false; });
}

// "<name a> [p, p+n) and <name b> [q, q+n) overlap by X bytes": the message
// of a rejected call.  name(tag) names a span by its tag.
template <class Name>
std::string conflict_message(const char* call, const std::vector<Span>& s, std::pair<int, int> c, Name name) {
  const Span& a = s[size_t(c.first)];
  const Span& b = s[size_t(c.second)];
  const uintptr_t pa = reinterpret_cast<uintptr_t>(a.p), pb = reinterpret_cast<uintptr_t>(b.p);
  const uintptr_t lo = std::max(pa, pb), hi = std::min(pa + uint64_t(a.n), pb + uint64_t(b.n));
  char buf[256];
  std::snprintf(buf, sizeof buf, " [%#llx, +%lld) and ", static_cast<unsigned long long>(pa),
                static_cast<long long>(a.n));
  std::string msg = std::string(call) + ": " + name(a.tag) + buf + name(b.tag);
  std::snprintf(buf, sizeof buf,
                " [%#llx, +%lld) overlap by %llu bytes%s; buffers of one call must be identical or disjoint (the "
                "reference's bytes for a shifted alias depend on its loop order)",
                static_cast<unsigned long long>(pb), static_cast<long long>(b.n),
                static_cast<unsigned long long>(hi > lo ? hi - lo : 0),
                pa == pb && a.n == b.n ? " (the same buffer, used in a way this call does not allow)" : "");
  return msg + buf;
}

// The checks at the library's entry points (contract_host.cpp); each returns
// ECGPU_OK or ECGPU_ERR_ARG with the conflicting pair in ecgpu_last_error().
struct FusedOp;
namespace __attribute__((visibility("hidden"))) rt {
int check_op_buffers(const char* call, const FusedOp& op, int64_t size);
int check_stripe_buffers(const char* call, int k, char** data, char** coding, const std::vector<int>& src_ids,
                         const std::vector<int>& out_ids, int64_t size);
int check_slot_buffers(const char* call, const std::vector<char*>& ptrs, const std::vector<int>& slots,
                       const std::vector<int64_t>& extent, const std::vector<char>& is_out);
}  // namespace rt

}  // namespace ecgpu
