// schedule_host.cpp -- see schedule_host.hpp.
#include "schedule_host.hpp"

#include <cstddef>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <vector>

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

// Greedy reuse (jerasure.cpp:1226-1344, the op list is caller-visible so the
// choices must be the reference's): each output row is built either from
// scratch (a copy then XORs: popcount ops) or as a copy of an already-built
// output row plus the XOR of the bits where the two differ (1 + Hamming
// distance).  Rows are held as 64-bit bitsets, so a distance is a few
// popcounts; each step takes the FIRST pending row (in row order) of least
// cost, then lowers the costs of the rows still pending against the row
// just built.
int** smart_bitmatrix_to_schedule(int k, int m, int w, const int* bitmatrix) {
  const int rows = m * w, cols = k * w, words = (cols + 63) / 64;
  std::vector<uint64_t> set(size_t(rows) * size_t(words), 0);
  for (int r = 0; r < rows; ++r)
    for (int c = 0; c < cols; ++c)
      if (bitmatrix[r * cols + c]) set[size_t(r) * words + size_t(c / 64)] |= uint64_t(1) << (c % 64);
  auto row_bits = [&](int r) { return set.data() + size_t(r) * size_t(words); };
  auto distance = [&](int a, int b) {
    int d = 0;
    for (int i = 0; i < words; ++i) d += __builtin_popcountll(row_bits(a)[i] ^ row_bits(b)[i]);
    return d;
  };
  std::vector<int> cost(static_cast<size_t>(rows)), base(static_cast<size_t>(rows), -1),
      pending(static_cast<size_t>(rows));
  for (int r = 0; r < rows; ++r) {
    int pop = 0;
    for (int i = 0; i < words; ++i) pop += __builtin_popcountll(row_bits(r)[i]);
    cost[size_t(r)] = pop;
    pending[size_t(r)] = r;
  }
  int** ops = static_cast<int**>(std::malloc(sizeof(int*) * (size_t(k) * m * w * w + 1)));
  int n = 0;
  // the ops that build output row `row` from the sources where `bits` is set
  auto emit_bits = [&](int row, const uint64_t* bits, int first_xor) {
    int xor_flag = first_xor;
    for (int c = 0; c < cols; ++c)
      if (bits[c / 64] >> (c % 64) & 1u) {
        ops[n++] = make_op(c / w, c % w, k + row / w, row % w, xor_flag);
        xor_flag = 1;
      }
  };
  std::vector<uint64_t> diff(static_cast<size_t>(words));
  while (!pending.empty()) {
    size_t at = 0;
    for (size_t i = 1; i < pending.size(); ++i)
      if (cost[size_t(pending[i])] < cost[size_t(pending[at])]) at = i;
    const int row = pending[at];
    pending.erase(pending.begin() + std::ptrdiff_t(at));
    const int from = base[size_t(row)];
    if (from < 0) {
      emit_bits(row, row_bits(row), 0);
    } else {
      ops[n++] = make_op(k + from / w, from % w, k + row / w, row % w, 0);
      for (int i = 0; i < words; ++i) diff[size_t(i)] = row_bits(row)[i] ^ row_bits(from)[i];
      emit_bits(row, diff.data(), 1);
    }
    for (int r : pending) {
      const int d = 1 + distance(row, r);
      if (d < cost[size_t(r)]) {
        cost[size_t(r)] = d;
        base[size_t(r)] = row;
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
