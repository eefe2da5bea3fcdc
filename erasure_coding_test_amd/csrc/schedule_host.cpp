// schedule_host.cpp -- see schedule_host.hpp.
#include "schedule_host.hpp"

#include <cstdlib>
#include <cstring>

#include "matrix_host.hpp"

namespace ecgpu {

namespace {
int* make_op(int sd, int sp, int dd, int dp, int x) {
  int* o = static_cast<int*>(std::malloc(5 * sizeof(int)));
  o[0] = sd;
  o[1] = sp;
  o[2] = dd;
  o[3] = dp;
  o[4] = x;
  return o;
}
int* end_op() {
  int* o = static_cast<int*>(std::malloc(5 * sizeof(int)));
  o[0] = -1;
  return o;
}
}  // namespace

int** dumb_bitmatrix_to_schedule(int k, int m, int w, const int* bitmatrix) {
  int** ops = static_cast<int**>(std::malloc(sizeof(int*) * (size_t(k) * m * w * w + 1)));
  int n = 0;
  const int cols = k * w;
  for (int r = 0; r < m * w; ++r) {
    int xor_flag = 0;
    for (int c = 0; c < cols; ++c)
      if (bitmatrix[r * cols + c]) {
        ops[n++] = make_op(c / w, c % w, k + r / w, r % w, xor_flag);
        xor_flag = 1;
      }
  }
  ops[n] = end_op();
  return ops;
}

// Greedy reuse: repeatedly emit the pending row that is cheapest to build,
// either from scratch (popcount) or as a copy of an already-built row plus
// the XOR of the differing bits (1 + Hamming distance).
int** smart_bitmatrix_to_schedule(int k, int m, int w, const int* bitmatrix) {
  const int rows = m * w, cols = k * w;
  int** ops = static_cast<int**>(std::malloc(sizeof(int*) * (size_t(k) * m * w * w + 1)));
  int n = 0;
  std::vector<int> cost(static_cast<size_t>(rows)), from(static_cast<size_t>(rows), -1),
      next(static_cast<size_t>(rows)), prev(static_cast<size_t>(rows));
  int best = 0, best_cost = cols + 1;
  for (int r = 0; r < rows; ++r) {
    int pop = 0;
    for (int c = 0; c < cols; ++c) pop += bitmatrix[r * cols + c];
    cost[r] = pop;
    next[r] = r + 1;
    prev[r] = r - 1;
    if (pop < best_cost) {
      best_cost = pop;
      best = r;
    }
  }
  next[rows - 1] = -1;
  int head = 0;
  while (head != -1) {
    const int row = best;
    if (prev[row] == -1) {  // unlink row from the pending list
      head = next[row];
      if (head != -1) prev[head] = -1;
    } else {
      next[prev[row]] = next[row];
      if (next[row] != -1) prev[next[row]] = prev[row];
    }
    const int* bits = bitmatrix + row * cols;
    if (from[row] == -1) {
      int xor_flag = 0;
      for (int c = 0; c < cols; ++c)
        if (bits[c]) {
          ops[n++] = make_op(c / w, c % w, k + row / w, row % w, xor_flag);
          xor_flag = 1;
        }
    } else {
      ops[n++] = make_op(k + from[row] / w, from[row] % w, k + row / w, row % w, 0);
      const int* base = bitmatrix + from[row] * cols;
      for (int c = 0; c < cols; ++c)
        if (bits[c] ^ base[c]) ops[n++] = make_op(c / w, c % w, k + row / w, row % w, 1);
    }
    best_cost = cols + 1;
    for (int r = head; r != -1; r = next[r]) {
      int d = 1;
      const int* other = bitmatrix + r * cols;
      for (int c = 0; c < cols; ++c) d += bits[c] ^ other[c];
      if (d < cost[r]) {
        from[r] = row;
        cost[r] = d;
      }
      if (cost[r] < best_cost) {
        best_cost = cost[r];
        best = r;
      }
    }
  }
  ops[n] = end_op();
  return ops;
}

void free_schedule(int** schedule) {
  int i = 0;
  for (; schedule[i][0] >= 0; ++i) std::free(schedule[i]);
  std::free(schedule[i]);
  std::free(schedule);
}

// Survivor/erased layout for scheduled decoding (jerasure.cpp:705-803):
// slot i < k holds data i, or -- if data i is erased -- the lowest unused
// surviving coding device; slots k.. hold the erased data then the erased
// coding devices.  row_ids[slot] = device id, ind_to_row[device] = slot.
bool schedule_layout(int k, int m, const int* erasures, std::vector<int>& row_ids, std::vector<int>& ind_to_row) {
  int* erased = erasures_to_erased(k, m, erasures);
  if (!erased) return false;
  row_ids.assign(size_t(k + m), 0);
  ind_to_row.assign(size_t(k + m), 0);
  int j = k, x = k;
  for (int i = 0; i < k; ++i) {
    if (!erased[i]) {
      row_ids[i] = i;
      ind_to_row[i] = i;
    } else {
      while (erased[j]) ++j;
      row_ids[i] = j;
      ind_to_row[j] = i;
      ++j;
      row_ids[x] = i;
      ind_to_row[i] = x;
      ++x;
    }
  }
  for (int i = k; i < k + m; ++i)
    if (erased[i]) {
      row_ids[x] = i;
      ind_to_row[i] = x;
      ++x;
    }
  std::free(erased);
  return true;
}

char** schedule_ptrs(int k, int m, const int* erasures, char** data, char** coding) {
  std::vector<int> row_ids, ind;
  if (!schedule_layout(k, m, erasures, row_ids, ind)) return nullptr;
  char** p = static_cast<char**>(std::malloc(sizeof(char*) * size_t(k + m)));
  int nerased = 0;
  for (int i = 0; erasures[i] != -1; ++i) ++nerased;
  for (int s = 0; s < k + m; ++s) {
    if (s >= k && s - k >= nerased) {
      p[s] = nullptr;
      continue;
    }
    const int id = row_ids[s];
    p[s] = id < k ? data[id] : coding[id - k];
  }
  return p;
}

// One bit-matrix that rebuilds every erased device in one schedule.
int** decoding_schedule(int k, int m, int w, const int* bitmatrix, const int* erasures, int smart) {
  int ddf = 0, cdf = 0;
  for (int i = 0; erasures[i] != -1; ++i) (erasures[i] < k ? ddf : cdf)++;
  std::vector<int> row_ids, ind;
  if (!schedule_layout(k, m, erasures, row_ids, ind)) return nullptr;
  const int kw = k * w;
  const size_t blk = size_t(kw) * w;
  std::vector<int> real(blk * size_t(ddf + cdf), 0);
  if (ddf > 0) {
    std::vector<int> sys(blk * k, 0), inv(blk * k, 0);
    for (int i = 0; i < k; ++i) {
      int* b = &sys[i * blk];
      if (row_ids[i] == i)
        for (int x = 0; x < w; ++x) b[x * kw + i * w + x] = 1;
      else
        std::memcpy(b, bitmatrix + blk * (row_ids[i] - k), sizeof(int) * blk);
    }
    invert_bitmatrix(sys.data(), inv.data(), kw);
    for (int i = 0; i < ddf; ++i) std::memcpy(&real[i * blk], &inv[blk * row_ids[k + i]], sizeof(int) * blk);
  }
  for (int x = 0; x < cdf; ++x) {
    const int drive = row_ids[x + ddf + k] - k;
    int* out = &real[blk * (ddf + x)];
    const int* coding_blk = bitmatrix + blk * drive;
    std::memcpy(out, coding_blk, sizeof(int) * blk);
    for (int i = 0; i < k; ++i)  // erased data columns are re-expressed ...
      if (row_ids[i] != i)
        for (int j = 0; j < w; ++j) std::memset(out + j * kw + i * w, 0, sizeof(int) * w);
    for (int i = 0; i < k; ++i) {  // ... through the decoding rows of that data device
      if (row_ids[i] == i) continue;
      const int* dec = &real[blk * (ind[i] - k)];
      for (int j = 0; j < w; ++j)
        for (int y = 0; y < w; ++y)
          if (coding_blk[j * kw + i * w + y])
            for (int z = 0; z < kw; ++z) out[j * kw + z] ^= dec[z + y * kw];
    }
  }
  return smart ? smart_bitmatrix_to_schedule(k, ddf + cdf, w, real.data())
               : dumb_bitmatrix_to_schedule(k, ddf + cdf, w, real.data());
}

int*** generate_schedule_cache(int k, int m, int w, const int* bitmatrix, int smart) {
  if (m != 2) return nullptr;
  const int n = k + m;
  int*** cache = static_cast<int***>(std::calloc(size_t(n) * (n + 1), sizeof(int**)));
  if (!cache) return nullptr;
  for (int e1 = 0; e1 < n; ++e1) {
    for (int e2 = 0; e2 < e1; ++e2) {
      const int er[3] = {e1, e2, -1};
      cache[e1 * n + e2] = decoding_schedule(k, m, w, bitmatrix, er, smart);
      cache[e2 * n + e1] = cache[e1 * n + e2];
    }
    const int er[2] = {e1, -1};
    cache[e1 * n + e1] = decoding_schedule(k, m, w, bitmatrix, er, smart);
  }
  return cache;
}

int free_schedule_cache(int k, int m, int*** cache) {
  if (m != 2 || !cache) return -1;
  const int n = k + m;
  for (int e1 = 0; e1 < n; ++e1) {
    for (int e2 = 0; e2 < e1; ++e2) free_schedule(cache[e1 * n + e2]);
    free_schedule(cache[e1 * n + e1]);
  }
  std::free(cache);
  return 0;
}

}  // namespace ecgpu
