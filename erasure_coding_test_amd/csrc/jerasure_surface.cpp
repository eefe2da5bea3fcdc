// jerasure_surface.cpp -- the reference surface outside the north-star
// GF(2^8) path: w = 16 / 32 region math and matrix coding (CPU restatement,
// used for ragged sizes only -- whole-word sizes run on the MI355X, see
// jerasure_dropin.cpp), GF(2) bit-matrix coding and XOR schedules
// (jerasure.cpp:257-345, :623-1032, :1153-1344) and matrix printing.  The
// bit-matrix / schedule EXECUTION runs on the MI355X (ecgpu_jerasure_bitmatrix_*,
// ecgpu_schedule_run: one fused GF(2) packet map per call) whenever size is a
// whole number of super-packets; matrix / schedule CONSTRUCTION is host code
// here.  None of the reference's callers uses this surface.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "ecgpu.h"
#include "gf_host.hpp"
// The reference surface is this library's export list (default visibility);
// everything else is built -fvisibility=hidden.
#pragma GCC visibility push(default)
#include "jerasure.h"
#pragma GCC visibility pop
#include "matrix_host.hpp"
#include "schedule_host.hpp"
#include "surface_cpu.hpp"

namespace ecgpu_cpu {

namespace {
std::mutex g_mu;
double g_stats[3] = {0, 0, 0};

inline char* dev_ptr(int id, int k, char** data, char** coding) { return id < k ? data[id] : coding[id - k]; }
}  // namespace

// GPU packet-coding calls: a failure libecgpu could not complete on the CPU
// (cpu_fallback.hpp: fallback off, device memory, or caller memory already
// written) is a message + exit(1), the reference's convention for
// unrecoverable conditions.
void gpu_check(const char* fn, int rc) {
  if (rc == ECGPU_OK) return;
  std::fprintf(stderr, "%s: MI355X path failed (%d): %s\n", fn, rc, ecgpu_last_error());
  std::exit(1);
}

int create_log_tables(int w) { return ecgpu::create_log_tables(w); }
int create_mult_tables(int w) { return ecgpu::create_mult_tables(w); }
int* mult_table(int w) { return ecgpu::mult_table(w); }
int* div_table(int w) { return ecgpu::div_table(w); }
int* log_table(int w) { return ecgpu::log_table(w); }
int* ilog_table(int w) { return ecgpu::ilog_table(w); }
int shift_multiply(int a, int b, int w) { return ecgpu::shift_multiply(a, b, w); }
int shift_inverse(int a, int w) { return ecgpu::shift_inverse(a, w); }

void count(double x, double g, double m) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_stats[0] += x;
  g_stats[1] += g;
  g_stats[2] += m;
}

void take_stats(double out[3]) {
  std::lock_guard<std::mutex> lk(g_mu);
  for (int i = 0; i < 3; ++i) {
    out[i] = g_stats[i];
    g_stats[i] = 0;
  }
}

void region_xor(const char* r1, const char* r2, char* r3, long n) {
  for (long i = 0; i < n; ++i) r3[i] = char(r1[i] ^ r2[i]);
}

void region_multiply_w16(char* region, int multby, int nbytes, char* r2, int add) {
  uint16_t* src = reinterpret_cast<uint16_t*>(region);
  uint16_t* dst = reinterpret_cast<uint16_t*>(r2 ? r2 : region);
  const int n = nbytes / 2;
  if (multby == 0) {  // galois.cpp:499-507
    if (!add) std::memset(dst, 0, size_t(n) * 2);
    return;
  }
  const bool acc = r2 != nullptr && add;
  for (int i = 0; i < n; ++i) {
    const uint16_t p = uint16_t(ecgpu::single_multiply(src[i], multby, 16));
    dst[i] = acc ? uint16_t(dst[i] ^ p) : p;
  }
}

void region_multiply_w32(char* region, int multby, int nbytes, char* r2, int add) {
  uint32_t* src = reinterpret_cast<uint32_t*>(region);
  uint32_t* dst = reinterpret_cast<uint32_t*>(r2 ? r2 : region);
  const int n = nbytes / 4;
  for (int i = 0; i < n; ++i) {  // galois.cpp:698-726: add applies even in place
    const uint32_t p = ecgpu::gf_mul_poly(src[i], uint32_t(multby), 32);
    dst[i] = add ? (dst[i] ^ p) : p;
  }
}

void matrix_dotprod(int k, int w, const int* row, const int* src_ids, int dest_id, char** data, char** coding,
                    int size) {
  char* dst = dev_ptr(dest_id, k, data, coding);
  auto src = [&](int i) { return src_ids ? dev_ptr(src_ids[i], k, data, coding) : data[i]; };
  bool init = false;
  for (int i = 0; i < k; ++i) {
    if (row[i] != 1) continue;
    if (!init) {
      std::memcpy(dst, src(i), size_t(size));
      count(0, 0, size);
      init = true;
    } else {
      region_xor(src(i), dst, dst, size);
      count(size, 0, 0);
    }
  }
  for (int i = 0; i < k; ++i) {
    if (row[i] == 0 || row[i] == 1) continue;
    if (w == 16) region_multiply_w16(src(i), row[i], size, dst, init);
    if (w == 32) region_multiply_w32(src(i), row[i], size, dst, init);
    count(0, size, 0);
    init = true;
  }
}

int matrix_decode(int k, int m, int w, int* matrix, int row_k_ones, int* erasures, char** data, char** coding,
                  int size) {
  int* erased = ecgpu::erasures_to_erased(k, m, erasures);
  if (!erased) return -1;
  int edd = 0, lastdrive = k;
  for (int i = 0; i < k; ++i)
    if (erased[i]) {
      ++edd;
      lastdrive = i;
    }
  if (!row_k_ones || erased[k]) lastdrive = k;
  std::vector<int> dm, ids;
  if (edd > 1 || (edd > 0 && (!row_k_ones || erased[k]))) {
    dm.resize(size_t(k) * k);
    ids.resize(size_t(k));
    if (ecgpu::make_decoding_matrix(k, m, w, matrix, erased, dm.data(), ids.data()) < 0) {
      std::free(erased);
      return -1;
    }
  }
  for (int i = 0; edd > 0 && i < lastdrive; ++i)
    if (erased[i]) {
      matrix_dotprod(k, w, dm.data() + size_t(i) * k, ids.data(), i, data, coding, size);
      --edd;
    }
  if (edd > 0) {
    std::vector<int> t(static_cast<size_t>(k));
    for (int i = 0; i < k; ++i) t[i] = i < lastdrive ? i : i + 1;
    matrix_dotprod(k, w, matrix, t.data(), lastdrive, data, coding, size);
  }
  for (int i = 0; i < m; ++i)
    if (erased[k + i]) matrix_dotprod(k, w, matrix + size_t(i) * k, nullptr, k + i, data, coding, size);
  std::free(erased);
  return 0;
}

int r6_encode(int k, int w, char** data, char** coding, int size) {
  if (w != 16 && w != 32) return 0;
  std::memcpy(coding[0], data[0], size_t(size));
  for (int i = 1; i < k; ++i) region_xor(coding[0], data[i], coding[0], size);
  std::memcpy(coding[1], data[k - 1], size_t(size));
  for (int i = k - 2; i >= 0; --i) {
    if (w == 16) region_multiply_w16(coding[1], 2, size, nullptr, 0);
    else region_multiply_w32(coding[1], 2, size, nullptr, 0);
    region_xor(coding[1], data[i], coding[1], size);
  }
  return 1;
}

}  // namespace ecgpu_cpu

using ecgpu_cpu::count;
using ecgpu_cpu::region_xor;

// ===================================================== bit-matrices ====
int* jerasure_matrix_to_bitmatrix(int k, int m, int w, int* matrix) {
  return ecgpu::matrix_to_bitmatrix(k, m, w, matrix);
}
int jerasure_invert_bitmatrix(int* mat, int* inv, int rows) { return ecgpu::invert_bitmatrix(mat, inv, rows); }
int jerasure_invertible_bitmatrix(int* mat, int rows) { return ecgpu::invertible_bitmatrix(mat, rows); }
int jerasure_make_decoding_bitmatrix(int k, int m, int w, int* matrix, int* erased, int* dm, int* dm_ids) {
  return ecgpu::make_decoding_bitmatrix(k, m, w, matrix, erased, dm, dm_ids);
}

// One output device = w packets; packet j of the output is the XOR of the
// source packets whose bit is set in row j of the device's w x k*w block.
void jerasure_bitmatrix_dotprod(int k, int w, int* bm_row, int* src_ids, int dest_id, char** data, char** coding,
                                int size, int packetsize) {
  const int chunk = w * packetsize;
  if (size % chunk != 0) {
    std::fprintf(stderr, "jerasure_bitmatrix_dotprod - size%%(w*packetsize)) must = 0\n");
    std::exit(1);
  }
  ecgpu_cpu::gpu_check("jerasure_bitmatrix_dotprod", ecgpu_jerasure_bitmatrix_dotprod(
                                                         k, w, bm_row, src_ids, dest_id, data, coding, size, packetsize));
}

namespace {
// The CPU form of jerasure_bitmatrix_dotprod, kept for bitmatrix_decode with a
// size that is not whole super-packets (the reference exits there, from here).
void cpu_bitmatrix_dotprod(int k, int w, int* bm_row, int* src_ids, int dest_id, char** data, char** coding,
                           int size, int packetsize) {
  const int chunk = w * packetsize;
  if (size % chunk != 0) {
    std::fprintf(stderr, "jerasure_bitmatrix_dotprod - size%%(w*packetsize)) must = 0\n");
    std::exit(1);
  }
  char* out = dest_id < k ? data[dest_id] : coding[dest_id - k];
  for (int off = 0; off < size; off += chunk) {
    const int* bit = bm_row;
    for (int j = 0; j < w; ++j) {
      char* dst = out + off + j * packetsize;
      bool started = false;
      for (int x = 0; x < k; ++x) {
        char* base = !src_ids ? data[x] : (src_ids[x] < k ? data[src_ids[x]] : coding[src_ids[x] - k]);
        for (int y = 0; y < w; ++y, ++bit) {
          if (!*bit) continue;
          const char* s = base + off + y * packetsize;
          if (!started) {
            std::memcpy(dst, s, size_t(packetsize));
            count(0, 0, packetsize);
            started = true;
          } else {
            region_xor(dst, s, dst, packetsize);
            count(packetsize, 0, 0);
          }
        }
      }
    }
  }
}

}  // namespace

void jerasure_bitmatrix_encode(int k, int m, int w, int* bitmatrix, char** data, char** coding, int size,
                               int packetsize) {
  if (packetsize % int(sizeof(long)) != 0) {
    std::fprintf(stderr, "jerasure_bitmatrix_encode - packetsize(%d) %% sizeof(long) != 0\n", packetsize);
    std::exit(1);
  }
  if (size % (packetsize * w) != 0) {
    std::fprintf(stderr, "jerasure_bitmatrix_encode - size(%d) %% (packetsize(%d)*w(%d))) != 0\n", size,
                 packetsize, w);
    std::exit(1);
  }
  ecgpu_cpu::gpu_check("jerasure_bitmatrix_encode",
                       ecgpu_jerasure_bitmatrix_encode(k, m, w, bitmatrix, data, coding, size, packetsize));
}

int jerasure_bitmatrix_decode(int k, int m, int w, int* bitmatrix, int row_k_ones, int* erasures, char** data,
                              char** coding, int size, int packetsize) {
  if (w > 0 && packetsize > 0 && size % (w * packetsize) == 0) {
    const int rc = ecgpu_jerasure_bitmatrix_decode(k, m, w, bitmatrix, row_k_ones, erasures, data, coding, size,
                                                   packetsize);
    if (rc == ECGPU_ERR) return -1;
    ecgpu_cpu::gpu_check("jerasure_bitmatrix_decode", rc);
    return 0;
  }
  int* erased = ecgpu::erasures_to_erased(k, m, erasures);
  if (!erased) return -1;
  int edd = 0, lastdrive = k;
  for (int i = 0; i < k; ++i)
    if (erased[i]) {
      ++edd;
      lastdrive = i;
    }
  if (row_k_ones != 1 || erased[k]) lastdrive = k;
  const size_t blk = size_t(k) * w * w;
  std::vector<int> dm, ids;
  if (edd > 1 || (edd > 0 && (row_k_ones != 1 || erased[k]))) {
    dm.resize(blk * k);
    ids.resize(size_t(k));
    if (ecgpu::make_decoding_bitmatrix(k, m, w, bitmatrix, erased, dm.data(), ids.data()) < 0) {
      std::free(erased);
      return -1;
    }
  }
  for (int i = 0; edd > 0 && i < lastdrive; ++i)
    if (erased[i]) {
      cpu_bitmatrix_dotprod(k, w, dm.data() + i * blk, ids.data(), i, data, coding, size, packetsize);
      --edd;
    }
  if (edd > 0) {
    std::vector<int> t(static_cast<size_t>(k));
    for (int i = 0; i < k; ++i) t[i] = i < lastdrive ? i : i + 1;
    cpu_bitmatrix_dotprod(k, w, bitmatrix, t.data(), lastdrive, data, coding, size, packetsize);
  }
  for (int i = 0; i < m; ++i)
    if (erased[k + i])
      cpu_bitmatrix_dotprod(k, w, bitmatrix + i * blk, nullptr, k + i, data, coding, size, packetsize);
  std::free(erased);
  return 0;
}

// ======================================================== schedules ====
// An op is 5 ints {src dev, src packet, dst dev, dst packet, xor?}; a
// schedule is a malloc'd array of malloc'd ops ending with op[0] == -1.
int** jerasure_dumb_bitmatrix_to_schedule(int k, int m, int w, int* bitmatrix) {
  return ecgpu::dumb_bitmatrix_to_schedule(k, m, w, bitmatrix);
}

int** jerasure_smart_bitmatrix_to_schedule(int k, int m, int w, int* bitmatrix) {
  return ecgpu::smart_bitmatrix_to_schedule(k, m, w, bitmatrix);
}

void jerasure_free_schedule(int** schedule) { ecgpu::free_schedule(schedule); }

void jerasure_do_scheduled_operations(char** ptrs, int** ops, int packetsize) {
  ecgpu_cpu::gpu_check("jerasure_do_scheduled_operations",
                       ecgpu_jerasure_do_scheduled_operations(ptrs, ops, packetsize));
}

namespace {
// CPU form, for schedules over a size that is not whole super-packets (the
// reference's loop then runs past the regions).
void cpu_scheduled_operations(char** ptrs, int** ops, int packetsize) {
  for (int i = 0; ops[i][0] >= 0; ++i) {
    const int* o = ops[i];
    char* s = ptrs[o[0]] + o[1] * packetsize;
    char* d = ptrs[o[2]] + o[3] * packetsize;
    if (o[4]) {
      region_xor(s, d, d, packetsize);
      count(packetsize, 0, 0);
    } else {
      std::memcpy(d, s, size_t(packetsize));
      count(0, 0, packetsize);
    }
  }
}

}  // namespace

void jerasure_schedule_encode(int k, int m, int w, int** schedule, char** data, char** coding, int size,
                              int packetsize) {
  if (w > 0 && packetsize > 0 && size % (w * packetsize) == 0) {
    ecgpu_cpu::gpu_check("jerasure_schedule_encode",
                         ecgpu_jerasure_schedule_encode(k, m, w, schedule, data, coding, size, packetsize));
    return;
  }
  std::vector<char*> p(static_cast<size_t>(k + m));
  for (int i = 0; i < k; ++i) p[i] = data[i];
  for (int i = 0; i < m; ++i) p[k + i] = coding[i];
  for (int done = 0; done < size; done += packetsize * w) {
    cpu_scheduled_operations(p.data(), schedule, packetsize);
    for (auto& q : p) q += packetsize * w;
  }
}

namespace {

void run_schedule(int k, int m, int w, int** schedule, char** ptrs, int size, int packetsize) {
  if (w > 0 && packetsize > 0 && size % (w * packetsize) == 0) {
    ecgpu_cpu::gpu_check("jerasure_schedule_decode", ecgpu_schedule_run(k + m, ptrs, schedule, w, size, packetsize));
    return;
  }
  for (int done = 0; done < size; done += packetsize * w) {
    cpu_scheduled_operations(ptrs, schedule, packetsize);
    for (int i = 0; i < k + m; ++i)
      if (ptrs[i]) ptrs[i] += packetsize * w;
  }
}

}  // namespace

int jerasure_schedule_decode_lazy(int k, int m, int w, int* bitmatrix, int* erasures, char** data, char** coding,
                                  int size, int packetsize, int smart) {
  char** ptrs = ecgpu::schedule_ptrs(k, m, erasures, data, coding);
  if (!ptrs) return -1;
  int** sched = ecgpu::decoding_schedule(k, m, w, bitmatrix, erasures, smart);
  if (!sched) {
    std::free(ptrs);
    return -1;
  }
  run_schedule(k, m, w, sched, ptrs, size, packetsize);
  jerasure_free_schedule(sched);
  std::free(ptrs);
  return 0;
}

int jerasure_schedule_decode_cache(int k, int m, int w, int*** scache, int* erasures, char** data, char** coding,
                                   int size, int packetsize) {
  int index;
  if (erasures[1] == -1)
    index = erasures[0] * (k + m) + erasures[0];
  else if (erasures[2] == -1)
    index = erasures[0] * (k + m) + erasures[1];
  else
    return -1;
  char** ptrs = ecgpu::schedule_ptrs(k, m, erasures, data, coding);
  if (!ptrs) return -1;
  run_schedule(k, m, w, scache[index], ptrs, size, packetsize);
  std::free(ptrs);
  return 0;
}

int*** jerasure_generate_schedule_cache(int k, int m, int w, int* bitmatrix, int smart) {
  return ecgpu::generate_schedule_cache(k, m, w, bitmatrix, smart);
}

void jerasure_free_schedule_cache(int k, int m, int*** cache) {
  if (m != 2) {
    std::fprintf(stderr, "jerasure_free_schedule_cache(): m must equal 2\n");
    std::exit(1);
  }
  ecgpu::free_schedule_cache(k, m, cache);
}

// ========================================================= printing ====
void jerasure_print_matrix(int* mtx, int rows, int cols, int w) {
  int width = 10;
  if (w != 32) {
    char buf[32];
    width = std::snprintf(buf, sizeof buf, "%u", (1u << w) - 1u);
  }
  for (int i = 0; i < rows; ++i) {
    for (int j = 0; j < cols; ++j) {
      if (j) std::printf(" ");
      std::printf("%*u", width, unsigned(mtx[i * cols + j]));
    }
    std::printf("\n");
  }
}

void jerasure_print_bitmatrix(int* mtx, int rows, int cols, int w) {
  for (int i = 0; i < rows; ++i) {
    if (i && i % w == 0) std::printf("\n");
    for (int j = 0; j < cols; ++j) {
      if (j && j % w == 0) std::printf(" ");
      std::printf("%d", mtx[i * cols + j]);
    }
    std::printf("\n");
  }
}
