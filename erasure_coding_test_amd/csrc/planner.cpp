// planner.cpp -- see planner.hpp.
#include "planner.hpp"

#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <unordered_map>

#include "gf_host.hpp"
#include "matrix_host.hpp"

namespace ecgpu {

int LinearTracker::id(void* p) {
  // a call names a handful of buffers: a scan beats hashing; the map takes
  // over for long schedules
  if (bufs_.size() <= kScanIds) {
    for (size_t i = 0; i < bufs_.size(); ++i)
      if (bufs_[i] == p) return static_cast<int>(i);
  } else {
    if (idx_.empty())
      for (size_t i = 0; i < bufs_.size(); ++i) idx_.emplace(bufs_[i], static_cast<int>(i));
    auto it = idx_.find(p);
    if (it != idx_.end()) return it->second;
  }
  const int b = static_cast<int>(bufs_.size());
  if (!idx_.empty()) idx_.emplace(p, b);
  bufs_.push_back(p);
  Vec v;
  v.reserve(std::max<size_t>(16, bufs_.size()));  // later ids grow it without reallocating
  v.assign(bufs_.size(), 0);
  v[b] = 1;  // untouched buffer = its own original contents
  state_.push_back(std::move(v));
  written_.push_back(0);
  return b;
}

LinearTracker::Vec& LinearTracker::state(int b) {
  Vec& v = state_[b];
  if (v.size() < bufs_.size()) v.resize(bufs_.size(), 0);
  return v;
}

// All ids are registered before any state reference is taken: id() may grow
// state_, which would invalidate the references.  Ops update the destination
// in place (no temporaries): schedules replay thousands of them per call.
void LinearTracker::copy(void* dst, void* src) {
  const int d = id(dst), s = id(src);
  if (d == s) return;
  const Vec& v = state(s);
  state(d) = v;  // copy-assign reuses the destination's capacity
  written_[d] = 1;
}

void LinearTracker::xor3(void* r1, void* r2, void* r3) {
  const int a = id(r1), b = id(r2), c = id(r3);
  const size_t n = bufs_.size();
  Vec& dst = state(c);
  int other = b;  // the operand not already in dst
  if (c == b && c != a) {
    other = a;
  } else if (c != a) {
    dst = state(a);
  }
  const Vec& o = state(other);
  dst.resize(n, 0);
  for (size_t i = 0; i < n && i < o.size(); ++i) dst[i] ^= o[i];
  written_[c] = 1;
}

void LinearTracker::mul(void* src, int c, void* dst, bool add) {
  const int s = id(src), d = id(dst);
  // in place, element by element (no temporary: s == d reads each element
  // before writing it); both states sized to every registered buffer
  const size_t n = bufs_.size();
  const Vec& v = state(s);
  Vec& out = state(d);
  if (w_ == 8) {
    const auto& T = gf8().mul[c & 0xFF];
    for (size_t i = 0; i < n; ++i) {
      const uint32_t x = v[i];
      out[i] = T[x] ^ (add ? out[i] : 0u);
    }
  } else {
    const uint32_t cw = w_ == 32 ? uint32_t(c) : uint32_t(c) & ((1u << w_) - 1u);
    for (size_t i = 0; i < n; ++i) {
      const uint32_t x = v[i];
      out[i] = (x ? gf_mul_poly(x, cw, w_) : 0u) ^ (add ? out[i] : 0u);
    }
  }
  written_[d] = 1;
}

void LinearTracker::dotprod(int k, const int* row, const int* src_ids, int dest_id, char** data, char** coding,
                            int64_t size) {
  auto buf = [&](int i) -> void* {
    if (!src_ids) return data[i];
    return src_ids[i] < k ? static_cast<void*>(data[src_ids[i]]) : static_cast<void*>(coding[src_ids[i] - k]);
  };
  void* dst = dest_id < k ? static_cast<void*>(data[dest_id]) : static_cast<void*>(coding[dest_id - k]);
  bool init = false;
  for (int i = 0; i < k; ++i) {  // unit coefficients: memcpy, then XOR (jerasure.cpp:580-598)
    if (row[i] != 1) continue;
    if (!init) {
      copy(dst, buf(i));
      memcpy_ += double(size);
      init = true;
    } else {
      xor3(buf(i), dst, dst);
      xor_ += double(size);
    }
  }
  for (int i = 0; i < k; ++i) {  // the rest: region multiply (jerasure.cpp:602-619)
    if (row[i] == 0 || row[i] == 1) continue;
    mul(buf(i), row[i], dst, init);
    gf_ += double(size);
    init = true;
  }
}

FusedOp LinearTracker::finish() const {
  FusedOp op;
  const size_t n = bufs_.size();
  // a state shorter than n has zeros past its end (registered after it was last touched)
  auto at = [&](size_t b, size_t i) -> uint32_t { return i < state_[b].size() ? state_[b][i] : 0u; };
  std::vector<int> outs;
  for (size_t b = 0; b < n; ++b) {
    if (!written_[b]) continue;
    bool identity = at(b, b) == 1;
    for (size_t i = 0; identity && i < n; ++i)
      if (i != b && at(b, i)) identity = false;
    if (!identity) outs.push_back(static_cast<int>(b));  // unchanged content needs no write
  }
  std::vector<int> col(n, -1);
  for (int b : outs)
    for (size_t i = 0; i < n; ++i)
      if (at(size_t(b), i) && col[i] < 0) {
        col[i] = static_cast<int>(op.srcs.size());
        op.srcs.push_back(bufs_[i]);
      }
  op.coef.assign(outs.size() * op.srcs.size(), 0);
  for (size_t r = 0; r < outs.size(); ++r) {
    for (size_t i = 0; i < n; ++i)
      if (const uint32_t c = at(size_t(outs[r]), i)) op.coef[r * op.srcs.size() + col[i]] = c;
    op.dsts.push_back(bufs_[outs[r]]);
    if (col[outs[r]] >= 0) op.dst_is_src = true;
  }
  op.touched = bufs_;
  op.touched_written = written_;
  op.w = w_;
  op.xor_bytes = xor_;
  op.gf_bytes = gf_;
  op.memcpy_bytes = memcpy_;
  return op;
}

// ------------------------------------------------------- PacketTracker ----
namespace {
constexpr int kRowBits = 20;
}

void* PacketTracker::packet_key(int slot, int row) {
  return reinterpret_cast<void*>(((uintptr_t(slot) << kRowBits) | uintptr_t(row)) + 1);
}
int PacketTracker::key_slot(const void* key) { return int((reinterpret_cast<uintptr_t>(key) - 1) >> kRowBits); }
int PacketTracker::key_row(const void* key) {
  return int((reinterpret_cast<uintptr_t>(key) - 1) & ((uintptr_t(1) << kRowBits) - 1));
}

PacketTracker::PacketTracker(int nslots, int nrows)
    : nslots_(nslots), nrows_(nrows), n_(nslots * nrows), words_((nslots * nrows + 63) / 64) {
  bits_.assign(size_t(n_) * size_t(words_), 0);
  for (int b = 0; b < n_; ++b) bits_[size_t(b) * words_ + size_t(b / 64)] |= uint64_t(1) << (b % 64);
  written_.assign(size_t(n_), 0);
}

void PacketTracker::copy(int dslot, int drow, int sslot, int srow) {
  const int d = idx(dslot, drow), s = idx(sslot, srow);
  if (d != s)
    for (int i = 0; i < words_; ++i) bits_[size_t(d) * words_ + i] = bits_[size_t(s) * words_ + i];
  written_[size_t(d)] = 1;
}

void PacketTracker::xor_into(int dslot, int drow, int sslot, int srow) {
  const int d = idx(dslot, drow), s = idx(sslot, srow);
  for (int i = 0; i < words_; ++i) bits_[size_t(d) * words_ + i] ^= bits_[size_t(s) * words_ + i];
  written_[size_t(d)] = 1;
}

FusedOp PacketTracker::finish() const {
  FusedOp op;
  op.w = 1;
  auto for_bits = [&](int b, auto&& fn) {  // every set bit of state b, ascending
    const uint64_t* v = &bits_[size_t(b) * words_];
    for (int i = 0; i < words_; ++i)
      for (uint64_t x = v[i]; x; x &= x - 1) fn(i * 64 + __builtin_ctzll(x));
  };
  std::vector<int> outs;
  for (int b = 0; b < n_; ++b) {
    if (!written_[size_t(b)]) continue;
    const uint64_t* v = &bits_[size_t(b) * words_];
    bool identity = true;
    for (int i = 0; identity && i < words_; ++i)
      identity = v[i] == ((b / 64 == i) ? (uint64_t(1) << (b % 64)) : 0);
    if (!identity) outs.push_back(b);  // unchanged content needs no write
  }
  std::vector<int> col(size_t(n_), -1), src_of;
  for (int b : outs)
    for_bits(b, [&](int i) {
      if (col[size_t(i)] < 0) {
        col[size_t(i)] = int(src_of.size());
        src_of.push_back(i);
      }
    });
  for (int i : src_of) op.srcs.push_back(packet_key(i / nrows_, i % nrows_));
  op.coef.assign(outs.size() * src_of.size(), 0);
  for (size_t r = 0; r < outs.size(); ++r) {
    const int b = outs[r];
    for_bits(b, [&](int i) { op.coef[r * src_of.size() + size_t(col[size_t(i)])] = 1; });
    op.dsts.push_back(packet_key(b / nrows_, b % nrows_));
    if (col[size_t(b)] >= 0) op.dst_is_src = true;
  }
  op.xor_bytes = xor_;
  op.gf_bytes = gf_;
  op.memcpy_bytes = memcpy_;
  return op;
}

namespace {
// make_decoding_matrix with a process-wide cache: a read path decodes
// stripe after stripe with one erasure pattern (a lost node), and the k x k
// inversion is most of a small decode's host cost.  Keyed on
// everything the result depends on -- k, m, w, the erased set and the whole
// coding matrix, compared in full -- so a hit is the same inversion.
struct DmEntry {
  int k = 0, m = 0, w = 0, rc = 0;
  std::vector<int> erased, matrix, dm, dm_ids;
};

int cached_decoding_matrix(int k, int m, int w, const int* matrix, const int* erased, int* dm, int* dm_ids) {
  // bounded by entries (every 4-of-14 pattern of RS(10,4) fits: 1,001) and by
  // the ints held (1 Mi = 4 MiB: a k = 255 inversion alone is 65,025), the
  // whole cache cleared when either fills
  constexpr size_t kEntries = 1024, kInts = size_t(1) << 20;
  static std::mutex mu;
  static std::unordered_map<uint64_t, DmEntry> cache;
  static size_t held = 0;
  const size_t n = size_t(k) + size_t(m), km = size_t(k) * size_t(m), kk = size_t(k) * size_t(k);
  uint64_t h = 1469598103934665603ull;  // FNV-1a over the key
  auto mix = [&h](int v) {
    for (int b = 0; b < 4; ++b) h = (h ^ ((uint32_t(v) >> (8 * b)) & 0xFFu)) * 1099511628211ull;
  };
  mix(k);
  mix(m);
  mix(w);
  for (size_t i = 0; i < n; ++i) mix(erased[i]);
  for (size_t i = 0; i < km; ++i) mix(matrix[i]);
  {
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(h);
    if (it != cache.end()) {
      const DmEntry& e = it->second;
      if (e.k == k && e.m == m && e.w == w && std::equal(e.erased.begin(), e.erased.end(), erased) &&
          std::equal(e.matrix.begin(), e.matrix.end(), matrix)) {
        std::copy(e.dm.begin(), e.dm.end(), dm);
        std::copy(e.dm_ids.begin(), e.dm_ids.end(), dm_ids);
        return e.rc;
      }
    }
  }
  DmEntry e;
  e.k = k;
  e.m = m;
  e.w = w;
  e.rc = make_decoding_matrix(k, m, w, matrix, erased, dm, dm_ids);
  e.erased.assign(erased, erased + n);
  e.matrix.assign(matrix, matrix + km);
  e.dm.assign(dm, dm + kk);
  e.dm_ids.assign(dm_ids, dm_ids + size_t(k));
  const int rc = e.rc;
  const size_t ints = e.erased.size() + e.matrix.size() + e.dm.size() + e.dm_ids.size();
  if (ints > kInts / 16) return rc;  // too big to be worth holding
  std::lock_guard<std::mutex> lk(mu);
  if (cache.size() >= kEntries || held + ints > kInts) {
    cache.clear();
    held = 0;
  }
  auto it = cache.find(h);  // a colliding key replaces the entry (checked in full on every hit)
  if (it != cache.end()) held -= it->second.erased.size() + it->second.matrix.size() + it->second.dm.size() +
                                it->second.dm_ids.size();
  held += ints;
  cache[h] = std::move(e);
  return rc;
}
}  // namespace

void plan_encode(LinearTracker& t, int k, int m, const int* matrix, char** data, char** coding, int64_t size) {
  for (int i = 0; i < m; ++i) t.dotprod(k, matrix + i * k, nullptr, k + i, data, coding, size);
}

int plan_decode(LinearTracker& t, int k, int m, const int* matrix, int row_k_ones, const int* erasures, char** data,
                char** coding, int64_t size) {
  int* erased = erasures_to_erased(k, m, erasures);
  if (!erased) return -1;
  int edd = 0, lastdrive = k;
  for (int i = 0; i < k; ++i)
    if (erased[i]) {
      ++edd;
      lastdrive = i;
    }
  if (!row_k_ones || erased[k]) lastdrive = k;

  std::vector<int> dm, dm_ids;
  if (edd > 1 || (edd > 0 && (!row_k_ones || erased[k]))) {
    dm.resize(size_t(k) * k);
    dm_ids.resize(size_t(k));
    if (cached_decoding_matrix(k, m, t.w(), matrix, erased, dm.data(), dm_ids.data()) < 0) {
      std::free(erased);
      return -1;
    }
  }
  // Data drives from the inverted survivor matrix (jerasure.cpp:223-228).
  for (int i = 0; edd > 0 && i < lastdrive; ++i) {
    if (!erased[i]) continue;
    t.dotprod(k, dm.data() + size_t(i) * k, dm_ids.data(), i, data, coding, size);
    --edd;
  }
  // row_k_ones shortcut for the last data drive (jerasure.cpp:232-239).
  if (edd > 0) {
    std::vector<int> ids(static_cast<size_t>(k));
    for (int i = 0; i < k; ++i) ids[i] = (i < lastdrive) ? i : i + 1;
    t.dotprod(k, matrix, ids.data(), lastdrive, data, coding, size);
  }
  // Re-encode erased coding drives from (now complete) data (jerasure.cpp:243-247).
  for (int i = 0; i < m; ++i)
    if (erased[k + i]) t.dotprod(k, matrix + size_t(i) * k, nullptr, k + i, data, coding, size);
  std::free(erased);
  return 0;
}

}  // namespace ecgpu
