// matrix_host.cpp -- coding/decoding matrices on the host; see matrix_host.hpp.
#include "matrix_host.hpp"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <utility>
#include <vector>

#include "gf_host.hpp"

namespace ecgpu {

namespace {
inline int* alloc_ints(size_t n) { return static_cast<int*>(std::malloc(sizeof(int) * (n ? n : 1))); }
inline int mul(int a, int b, int w) { return single_multiply(a, b, w); }
inline int recip(int a, int w) { return single_divide(1, a, w); }
}  // namespace

// Rows: e0, then powers of i for i = 1..rows-2, then e_{cols-1}.
int* extended_vandermonde_matrix(int rows, int cols, int w) {
  if (w < 30 && ((1 << w) < rows || (1 << w) < cols)) return nullptr;
  int* v = alloc_ints(size_t(rows) * cols);
  if (!v) return nullptr;
  std::memset(v, 0, sizeof(int) * size_t(rows) * cols);
  v[0] = 1;
  if (rows == 1) return v;
  v[(rows - 1) * cols + (cols - 1)] = 1;
  if (rows == 2) return v;
  for (int i = 1; i < rows - 1; ++i) {
    int p = 1;
    for (int j = 0; j < cols; ++j) {
      v[i * cols + j] = p;
      p = mul(p, i, w);
    }
  }
  return v;
}

// Column-reduce the top cols x cols block to the identity (a systematic
// code), then normalise: row `cols` all ones, column 0 all ones.
int* big_vandermonde_distribution_matrix(int rows, int cols, int w) {
  if (cols >= rows) return nullptr;
  int* d = extended_vandermonde_matrix(rows, cols, w);
  if (!d) return nullptr;
  auto at = [&](int r, int c) -> int& { return d[r * cols + c]; };
  for (int i = 1; i < cols; ++i) {
    int r = i;
    while (r < rows && at(r, i) == 0) ++r;
    if (r >= rows) {
      std::fprintf(stderr, "reed_sol_big_vandermonde_distribution_matrix(%d,%d,%d) - couldn't make matrix\n", rows,
                   cols, w);
      std::exit(1);
    }
    if (r != i)
      for (int c = 0; c < cols; ++c) std::swap(at(r, c), at(i, c));
    if (at(i, i) != 1) {
      const int s = recip(at(i, i), w);
      for (int rr = 0; rr < rows; ++rr) at(rr, i) = mul(s, at(rr, i), w);
    }
    for (int c = 0; c < cols; ++c) {
      const int e = at(i, c);
      if (c == i || e == 0) continue;
      for (int rr = 0; rr < rows; ++rr) at(rr, c) ^= mul(e, at(rr, i), w);
    }
  }
  for (int c = 0; c < cols; ++c) {
    const int e = at(cols, c);
    if (e == 1) continue;
    const int s = recip(e, w);
    for (int rr = cols; rr < rows; ++rr) at(rr, c) = mul(s, at(rr, c), w);
  }
  for (int rr = cols + 1; rr < rows; ++rr) {
    const int e = at(rr, 0);
    if (e == 1) continue;
    const int s = recip(e, w);
    for (int c = 0; c < cols; ++c) at(rr, c) = mul(at(rr, c), s, w);
  }
  return d;
}

int* vandermonde_coding_matrix(int k, int m, int w) {
  int* d = big_vandermonde_distribution_matrix(k + m, k, w);
  if (!d) return nullptr;
  int* out = alloc_ints(size_t(m) * k);
  if (!out) {
    std::free(d);
    return nullptr;
  }
  std::memcpy(out, d + k * k, sizeof(int) * size_t(m) * k);
  std::free(d);
  return out;
}

int* r6_coding_matrix(int k, int w) {
  if (w != 8 && w != 16 && w != 32) return nullptr;
  int* out = alloc_ints(size_t(2) * k);
  if (!out) return nullptr;
  int p = 1;
  for (int i = 0; i < k; ++i) {
    out[i] = 1;
    out[k + i] = p;
    p = mul(p, 2, w);
  }
  return out;
}

// Gauss-Jordan over GF(2^w).  Pivot = first non-zero at or below the
// diagonal; the final state of `mat` (identity on success) is part of the
// reference's observable behaviour (jerasure.h:233-236), so the elimination
// order is the textbook one: forward sweep, then back substitution.
int invert_matrix(int* mat, int* inv, int n, int w) {
  for (int r = 0; r < n; ++r)
    for (int c = 0; c < n; ++c) inv[r * n + c] = (r == c);
  for (int i = 0; i < n; ++i) {
    int* ri = mat + i * n;
    int* vi = inv + i * n;
    if (ri[i] == 0) {
      int r = i + 1;
      while (r < n && mat[r * n + i] == 0) ++r;
      if (r == n) return -1;
      for (int c = 0; c < n; ++c) {
        std::swap(ri[c], mat[r * n + c]);
        std::swap(vi[c], inv[r * n + c]);
      }
    }
    if (ri[i] != 1) {
      const int s = recip(ri[i], w);
      for (int c = 0; c < n; ++c) {
        ri[c] = mul(ri[c], s, w);
        vi[c] = mul(vi[c], s, w);
      }
    }
    for (int r = i + 1; r < n; ++r) {
      const int e = mat[r * n + i];
      if (e == 0) continue;
      for (int c = 0; c < n; ++c) {
        mat[r * n + c] ^= mul(e, ri[c], w);
        inv[r * n + c] ^= mul(e, vi[c], w);
      }
    }
  }
  for (int i = n - 1; i >= 0; --i)
    for (int r = 0; r < i; ++r) {
      const int e = mat[r * n + i];
      if (e == 0) continue;
      mat[r * n + i] = 0;
      for (int c = 0; c < n; ++c) inv[r * n + c] ^= mul(e, inv[i * n + c], w);
    }
  return 0;
}

int invertible_matrix(int* mat, int n, int w) {
  for (int i = 0; i < n; ++i) {
    int* ri = mat + i * n;
    if (ri[i] == 0) {
      int r = i + 1;
      while (r < n && mat[r * n + i] == 0) ++r;
      if (r == n) return 0;
      for (int c = 0; c < n; ++c) std::swap(ri[c], mat[r * n + c]);
    }
    if (ri[i] != 1) {
      const int s = recip(ri[i], w);
      for (int c = 0; c < n; ++c) ri[c] = mul(ri[c], s, w);
    }
    for (int r = i + 1; r < n; ++r) {
      const int e = mat[r * n + i];
      if (e == 0) continue;
      for (int c = 0; c < n; ++c) mat[r * n + c] ^= mul(e, ri[c], w);
    }
  }
  return 1;
}

int* matrix_multiply(const int* m1, const int* m2, int r1, int c1, int r2, int c2, int w) {
  int* p = alloc_ints(size_t(r1) * c2);
  if (!p) return nullptr;
  for (int i = 0; i < r1; ++i)
    for (int j = 0; j < c2; ++j) {
      int acc = 0;
      for (int t = 0; t < r2; ++t) acc ^= mul(m1[i * c1 + t], m2[t * c2 + j], w);
      p[i * c2 + j] = acc;
    }
  return p;
}

int* erasures_to_erased(int k, int m, const int* erasures) {
  const int n = k + m;
  int* e = alloc_ints(size_t(n));
  if (!e) return nullptr;
  std::memset(e, 0, sizeof(int) * size_t(n));
  int alive = n;
  for (int i = 0; erasures[i] != -1; ++i) {
    if (e[erasures[i]]) continue;
    e[erasures[i]] = 1;
    if (--alive < k) {
      std::free(e);
      return nullptr;
    }
  }
  return e;
}

// Survivors = the first k non-erased ids in ascending order; their rows of
// the distribution matrix [I; C] form the k x k system to invert.
int make_decoding_matrix(int k, int m, int w, const int* matrix, const int* erased, int* dm, int* dm_ids) {
  (void)m;
  for (int id = 0, n = 0; n < k; ++id)
    if (!erased[id]) dm_ids[n++] = id;
  std::vector<int> sys(size_t(k) * k, 0);
  for (int r = 0; r < k; ++r) {
    if (dm_ids[r] < k)
      sys[size_t(r) * k + dm_ids[r]] = 1;
    else
      std::memcpy(&sys[size_t(r) * k], matrix + size_t(dm_ids[r] - k) * k, sizeof(int) * size_t(k));
  }
  return invert_matrix(sys.data(), dm, k, w);
}

// Element (i,j) of the m x k matrix becomes a w x w block whose column x
// holds the bits of elt * 2^x.
int* matrix_to_bitmatrix(int k, int m, int w, const int* matrix) {
  if (!matrix) return nullptr;
  int* b = alloc_ints(size_t(k) * m * w * w);
  if (!b) return nullptr;
  const int row_len = k * w;
  for (int i = 0; i < m; ++i)
    for (int j = 0; j < k; ++j) {
      int elt = matrix[i * k + j];
      for (int x = 0; x < w; ++x) {
        for (int bit = 0; bit < w; ++bit)
          b[(i * w + bit) * row_len + j * w + x] = (elt >> bit) & 1;
        elt = mul(elt, 2, w);
      }
    }
  return b;
}

int invert_bitmatrix(int* mat, int* inv, int n) {
  for (int r = 0; r < n; ++r)
    for (int c = 0; c < n; ++c) inv[r * n + c] = (r == c);
  for (int i = 0; i < n; ++i) {
    if (mat[i * n + i] == 0) {
      int r = i + 1;
      while (r < n && mat[r * n + i] == 0) ++r;
      if (r == n) return -1;
      for (int c = 0; c < n; ++c) {
        std::swap(mat[i * n + c], mat[r * n + c]);
        std::swap(inv[i * n + c], inv[r * n + c]);
      }
    }
    for (int r = i + 1; r < n; ++r) {
      if (mat[r * n + i] == 0) continue;
      for (int c = 0; c < n; ++c) {
        mat[r * n + c] ^= mat[i * n + c];
        inv[r * n + c] ^= inv[i * n + c];
      }
    }
  }
  for (int i = n - 1; i >= 0; --i)
    for (int r = 0; r < i; ++r) {
      if (!mat[r * n + i]) continue;
      for (int c = 0; c < n; ++c) {
        mat[r * n + c] ^= mat[i * n + c];
        inv[r * n + c] ^= inv[i * n + c];
      }
    }
  return 0;
}

int invertible_bitmatrix(int* mat, int n) {
  for (int i = 0; i < n; ++i) {
    if (mat[i * n + i] == 0) {
      int r = i + 1;
      while (r < n && mat[r * n + i] == 0) ++r;
      if (r == n) return 0;
      for (int c = 0; c < n; ++c) std::swap(mat[i * n + c], mat[r * n + c]);
    }
    for (int r = i + 1; r < n; ++r) {
      if (mat[r * n + i] == 0) continue;
      for (int c = 0; c < n; ++c) mat[r * n + c] ^= mat[i * n + c];
    }
  }
  return 1;
}

int make_decoding_bitmatrix(int k, int m, int w, const int* matrix, const int* erased, int* dm, int* dm_ids) {
  (void)m;
  for (int id = 0, n = 0; n < k; ++id)
    if (!erased[id]) dm_ids[n++] = id;
  const size_t blk = size_t(k) * w * w;  // one block-row of the k*w x k*w system
  std::vector<int> sys(blk * k, 0);
  for (int r = 0; r < k; ++r) {
    int* dst = &sys[r * blk];
    if (dm_ids[r] < k) {
      for (int x = 0; x < w; ++x) dst[x * (k * w) + dm_ids[r] * w + x] = 1;
    } else {
      std::memcpy(dst, matrix + size_t(dm_ids[r] - k) * blk, sizeof(int) * blk);
    }
  }
  return invert_bitmatrix(sys.data(), dm, k * w);
}

}  // namespace ecgpu
