// planner.cpp -- see planner.hpp.
#include "planner.hpp"

#include <cstdlib>

#include "gf_host.hpp"
#include "matrix_host.hpp"

namespace ecgpu {

int LinearTracker::id(void* p) {
  auto it = idx_.find(p);
  if (it != idx_.end()) return it->second;
  const int b = static_cast<int>(bufs_.size());
  idx_.emplace(p, b);
  bufs_.push_back(p);
  Vec v(bufs_.size(), 0);
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

void LinearTracker::copy(void* dst, void* src) {
  const int d = id(dst), s = id(src);
  Vec v = state(s);
  state(d) = std::move(v);
  written_[d] = 1;
}

void LinearTracker::xor3(void* r1, void* r2, void* r3) {
  const int a = id(r1), b = id(r2), c = id(r3);
  Vec v = state(a);
  const Vec& w = state(b);
  for (size_t i = 0; i < v.size(); ++i) v[i] ^= w[i];
  state(c) = std::move(v);
  written_[c] = 1;
}

void LinearTracker::mul(void* src, int c, void* dst, bool add) {
  const int s = id(src), d = id(dst);
  Vec v = state(s);
  if (w_ == 8) {
    const auto& T = gf8().mul[c & 0xFF];
    for (auto& x : v) x = T[x];
  } else {
    const uint32_t cw = w_ == 32 ? uint32_t(c) : uint32_t(c) & ((1u << w_) - 1u);
    for (auto& x : v) x = x ? gf_mul_poly(x, cw, w_) : 0u;
  }
  if (add) {
    const Vec& old = state(d);
    for (size_t i = 0; i < v.size(); ++i) v[i] ^= old[i];
  }
  state(d) = std::move(v);
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
  std::vector<int> outs;
  for (size_t b = 0; b < n; ++b) {
    if (!written_[b]) continue;
    Vec v = state_[b];
    v.resize(n, 0);
    bool identity = v[b] == 1;
    for (size_t i = 0; identity && i < n; ++i)
      if (i != b && v[i]) identity = false;
    if (!identity) outs.push_back(static_cast<int>(b));  // unchanged content needs no write
  }
  std::vector<int> col(n, -1);
  for (int b : outs) {
    Vec v = state_[b];
    v.resize(n, 0);
    for (size_t i = 0; i < n; ++i)
      if (v[i] && col[i] < 0) {
        col[i] = static_cast<int>(op.srcs.size());
        op.srcs.push_back(bufs_[i]);
      }
  }
  op.coef.assign(outs.size() * op.srcs.size(), 0);
  for (size_t r = 0; r < outs.size(); ++r) {
    Vec v = state_[outs[r]];
    v.resize(n, 0);
    for (size_t i = 0; i < n; ++i)
      if (v[i]) op.coef[r * op.srcs.size() + col[i]] = v[i];
    op.dsts.push_back(bufs_[outs[r]]);
    if (col[outs[r]] >= 0) op.dst_is_src = true;
  }
  op.w = w_;
  op.xor_bytes = xor_;
  op.gf_bytes = gf_;
  op.memcpy_bytes = memcpy_;
  return op;
}

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
    if (make_decoding_matrix(k, m, t.w(), matrix, erased, dm.data(), dm_ids.data()) < 0) {
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
