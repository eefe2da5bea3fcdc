// capi_host.cpp -- host-only entry points of include/ecgpu.h (no GPU touched).
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "ecgpu.h"
#include "gf_host.hpp"
#include "knobs.hpp"
#include "shard_stride.hpp"
#include "matrix_host.hpp"
#include "planner.hpp"
#include "schedule_host.hpp"

using namespace ecgpu;

namespace ecgpu {
namespace __attribute__((visibility("hidden"))) rt {
// The thread's last error message (ecgpu_last_error); every translation unit
// of the library reports through fail().
thread_local std::string t_err;

int fail(int code, const std::string& msg) {
  t_err = msg;
  return code;
}
}  // namespace rt
}  // namespace ecgpu

extern "C" {

ECGPU_API const char* ecgpu_version(void) { return "ecgpu 0.1 (gfx950)"; }
ECGPU_API const char* ecgpu_last_error(void) { return rt::t_err.c_str(); }

// Content IDs of this build (erasure_coding_test_amd/build.py): 0 the whole
// library, 1 the w = 8 kernels and their dispatch, 2 the w = 16 / 32 ones,
// 3 the GF(2) packet ones.
#ifndef ECGPU_BUILD_ID
#define ECGPU_BUILD_ID "unknown"
#endif
#ifndef ECGPU_KERNEL_ID
#define ECGPU_KERNEL_ID "unknown"
#endif
#ifndef ECGPU_WIDE_ID
#define ECGPU_WIDE_ID "unknown"
#endif
#ifndef ECGPU_PACKETS_ID
#define ECGPU_PACKETS_ID "unknown"
#endif
ECGPU_API const char* ecgpu_build_id(int what) {
  switch (what) {
    case 1: return ECGPU_KERNEL_ID;
    case 2: return ECGPU_WIDE_ID;
    case 3: return ECGPU_PACKETS_ID;
    default: return ECGPU_BUILD_ID;
  }
}
ECGPU_API void ecgpu_free(void* p) { std::free(p); }

// The shard stride of shard_stride.hpp (the measured per-size skew table,
// and its per-scheme entries when k + m is given).
namespace {
int64_t recommended_stride(int64_t size, int shards) {
  if (size < 0) size = 0;
  const int64_t rounded = (size + 255) & ~int64_t(255);
  // the shard_skew_kib knob (ECGPU_SHARD_SKEW_KIB): one skew for every size
  // (A/B runs of whole workloads); outside 0..1024 the table applies
  const int v = knob(Knob::kShardSkewKib);
  if (v >= 0 && v <= 1024) return rounded + int64_t(v) * 1024;
  return shard_stride(size, shards);
}
}  // namespace

ECGPU_API int64_t ecgpu_recommended_shard_stride(int64_t size) { return recommended_stride(size, 0); }

ECGPU_API int64_t ecgpu_recommended_shard_stride_km(int64_t size, int k, int m) {
  return recommended_stride(size, k > 0 && m >= 0 ? k + m : 0);
}

ECGPU_API int ecgpu_galois_single_multiply(int a, int b, int w) { return single_multiply(a, b, w); }
ECGPU_API int ecgpu_galois_single_divide(int a, int b, int w) { return single_divide(a, b, w); }
ECGPU_API int ecgpu_galois_inverse(int a, int w) { return inverse(a, w); }
// Log / antilog lookups (galois.cpp:269-289).  The reference indexes its
// tables unchecked; here a value outside them -- log: [0, 2^w), ilog:
// [-(2^w - 1), 2(2^w - 1)), the offset table the divide path uses -- or a w
// without tables (w > 30, where the reference exits) returns -1.
ECGPU_API int ecgpu_galois_log(int value, int w) {
  int* t = log_table(w);
  if (!t || value < 0 || int64_t(value) >= (int64_t(1) << w)) return -1;
  return t[value];
}
// Table construction / access and the table-free shift arithmetic
// (galois.cpp:152-267, :292-320, :605-665, galois.h:46-66).  Tables are
// built once per w, thread-safely, and live for the library's lifetime; a
// w the reference cannot build tables for gives -1 / NULL.
ECGPU_API int ecgpu_galois_create_log_tables(int w) { return create_log_tables(w); }
ECGPU_API int ecgpu_galois_create_mult_tables(int w) { return create_mult_tables(w); }
ECGPU_API int* ecgpu_galois_get_mult_table(int w) { return mult_table(w); }
ECGPU_API int* ecgpu_galois_get_div_table(int w) { return div_table(w); }
ECGPU_API int* ecgpu_galois_get_log_table(int w) { return log_table(w); }
ECGPU_API int* ecgpu_galois_get_ilog_table(int w) { return ilog_table(w); }
ECGPU_API int ecgpu_galois_shift_multiply(int a, int b, int w) { return shift_multiply(a, b, w); }
ECGPU_API int ecgpu_galois_shift_inverse(int a, int w) { return shift_inverse(a, w); }
ECGPU_API int ecgpu_galois_create_split_w8_tables(void) { return create_split_w8_tables(); }
ECGPU_API int ecgpu_galois_split_w8_multiply(int x, int y) { return split_w8_multiply(x, y); }

ECGPU_API int ecgpu_galois_ilog(int value, int w) {
  int* t = ilog_table(w);
  if (!t) return -1;
  const int64_t nwm1 = (int64_t(1) << w) - 1;
  if (value < -nwm1 || value >= 2 * nwm1) return -1;
  return t[value];
}

ECGPU_API int* ecgpu_reed_sol_vandermonde_coding_matrix(int k, int m, int w) {
  return vandermonde_coding_matrix(k, m, w);
}
ECGPU_API int* ecgpu_reed_sol_extended_vandermonde_matrix(int rows, int cols, int w) {
  return extended_vandermonde_matrix(rows, cols, w);
}
ECGPU_API int* ecgpu_reed_sol_big_vandermonde_distribution_matrix(int rows, int cols, int w) {
  return big_vandermonde_distribution_matrix(rows, cols, w);
}
ECGPU_API int* ecgpu_reed_sol_r6_coding_matrix(int k, int w) { return r6_coding_matrix(k, w); }
ECGPU_API int ecgpu_jerasure_invert_matrix(int* mat, int* inv, int rows, int w) {
  return invert_matrix(mat, inv, rows, w);
}
ECGPU_API int ecgpu_jerasure_invertible_matrix(int* mat, int rows, int w) { return invertible_matrix(mat, rows, w); }
ECGPU_API int* ecgpu_jerasure_matrix_multiply(int* m1, int* m2, int r1, int c1, int r2, int c2, int w) {
  return matrix_multiply(m1, m2, r1, c1, r2, c2, w);
}
ECGPU_API int* ecgpu_jerasure_erasures_to_erased(int k, int m, int* erasures) {
  return erasures_to_erased(k, m, erasures);
}
ECGPU_API int ecgpu_jerasure_make_decoding_matrix(int k, int m, int w, int* matrix, int* erased, int* dm,
                                                  int* dm_ids) {
  return make_decoding_matrix(k, m, w, matrix, erased, dm, dm_ids);
}

ECGPU_API int* ecgpu_jerasure_matrix_to_bitmatrix(int k, int m, int w, int* matrix) {
  return matrix_to_bitmatrix(k, m, w, matrix);
}
ECGPU_API int ecgpu_jerasure_make_decoding_bitmatrix(int k, int m, int w, int* matrix, int* erased, int* dm,
                                                     int* dm_ids) {
  return make_decoding_bitmatrix(k, m, w, matrix, erased, dm, dm_ids);
}
ECGPU_API int ecgpu_jerasure_invert_bitmatrix(int* mat, int* inv, int rows) { return invert_bitmatrix(mat, inv, rows); }
ECGPU_API int ecgpu_jerasure_invertible_bitmatrix(int* mat, int rows) { return invertible_bitmatrix(mat, rows); }

// ---------------------------------------------------------- schedules ----
ECGPU_API int** ecgpu_jerasure_dumb_bitmatrix_to_schedule(int k, int m, int w, int* bitmatrix) {
  return dumb_bitmatrix_to_schedule(k, m, w, bitmatrix);
}
ECGPU_API int** ecgpu_jerasure_smart_bitmatrix_to_schedule(int k, int m, int w, int* bitmatrix) {
  return smart_bitmatrix_to_schedule(k, m, w, bitmatrix);
}
ECGPU_API void ecgpu_jerasure_free_schedule(int** schedule) { free_schedule(schedule); }
ECGPU_API int*** ecgpu_jerasure_generate_schedule_cache(int k, int m, int w, int* bitmatrix, int smart) {
  return generate_schedule_cache(k, m, w, bitmatrix, smart);
}
ECGPU_API int ecgpu_jerasure_free_schedule_cache(int k, int m, int*** cache) {
  return free_schedule_cache(k, m, cache) == 0 ? ECGPU_OK : ECGPU_ERR_ARG;
}

// jerasure.cpp:935-961: schedule built on the host, executed on the GPU.
ECGPU_API int ecgpu_jerasure_schedule_decode_lazy(int k, int m, int w, int* bitmatrix, int* erasures, char** data_ptrs,
                                                  char** coding_ptrs, int size, int packetsize, int smart) {
  if (k <= 0 || m <= 0 || w <= 0 || packetsize <= 0 || !bitmatrix || !erasures || size % (w * packetsize) != 0)
    return ECGPU_ERR_ARG;
  char** ptrs = schedule_ptrs(k, m, erasures, data_ptrs, coding_ptrs);
  if (!ptrs) return ECGPU_ERR;
  int** sched = decoding_schedule(k, m, w, bitmatrix, erasures, smart);
  if (!sched) {
    std::free(ptrs);
    return ECGPU_ERR;
  }
  const int rc = ecgpu_schedule_run(k + m, ptrs, sched, w, size, packetsize);
  free_schedule(sched);
  std::free(ptrs);
  return rc;
}

// jerasure.cpp:963-995: one or two erasures from a generate_schedule_cache table.
ECGPU_API int ecgpu_jerasure_schedule_decode_cache(int k, int m, int w, int*** scache, int* erasures, char** data_ptrs,
                                                   char** coding_ptrs, int size, int packetsize) {
  if (k <= 0 || m <= 0 || w <= 0 || packetsize <= 0 || !scache || !erasures || size % (w * packetsize) != 0)
    return ECGPU_ERR_ARG;
  int index;
  if (erasures[0] < 0) return ECGPU_ERR;
  if (erasures[1] == -1)
    index = erasures[0] * (k + m) + erasures[0];
  else if (erasures[2] == -1)
    index = erasures[0] * (k + m) + erasures[1];
  else
    return ECGPU_ERR;
  char** ptrs = schedule_ptrs(k, m, erasures, data_ptrs, coding_ptrs);
  if (!ptrs) return ECGPU_ERR;
  const int rc = ecgpu_schedule_run(k + m, ptrs, scache[index], w, size, packetsize);
  std::free(ptrs);
  return rc;
}

// Replays the decode on symbolic buffers whose "pointers" are shard ids + 1,
// then reads the fused map back in terms of ids.
ECGPU_API int ecgpu_decode_plan(int k, int m, int w, const int* matrix, int row_k_ones, const int* erasures,
                                int* out_ids, int* n_out, int* src_ids, int* n_src, int* coefs) {
  if ((w != 8 && w != 16 && w != 32) || k <= 0 || m <= 0 || !matrix || !erasures) return ECGPU_ERR_ARG;
  std::vector<char*> ids(size_t(k + m));
  for (int i = 0; i < k + m; ++i) ids[i] = reinterpret_cast<char*>(uintptr_t(i) + 1);
  LinearTracker t(w);
  for (int i = 0; i < k + m; ++i) t.id(ids[i]);
  if (plan_decode(t, k, m, matrix, row_k_ones, erasures, ids.data(), ids.data() + k, 1) < 0) return ECGPU_ERR;
  const FusedOp op = t.finish();
  *n_out = int(op.dsts.size());
  *n_src = int(op.srcs.size());
  for (size_t r = 0; r < op.dsts.size(); ++r) out_ids[r] = int(reinterpret_cast<uintptr_t>(op.dsts[r]) - 1);
  for (size_t j = 0; j < op.srcs.size(); ++j) src_ids[j] = int(reinterpret_cast<uintptr_t>(op.srcs[j]) - 1);
  for (size_t i = 0; i < op.coef.size(); ++i) coefs[i] = op.coef[i];
  return ECGPU_OK;
}

}  // extern "C"
