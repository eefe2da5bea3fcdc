// jerasure_dropin.cpp -- libjerasure_amd.so: the reference's C++ coding
// surface (include/dropin/*.h == reference include/{galois,jerasure,
// reed_sol}.h signatures, C++ linkage) on top of libecgpu.so.
//
// Callers such as the reference's client (client_main.cpp:1060, :2118) and
// ECX datanode (ecx_datanode_main.cpp:714, :724, :1391) link this library in
// place of src/erasure_coding/*.cpp.  The w = 8 hot path -- matrix encode,
// decode, dot product, region multiply / XOR, parity, RAID-6 -- runs on the
// MI355X through include/ecgpu.h.  A HIP failure before any caller byte was
// written, on host buffers, is completed on the CPU inside libecgpu (SURVEY
// §8b "no new failure modes", cpu_fallback.hpp; counted, logged once); any
// other GPU failure takes the reference's own failure channel (gpu_fatal).
// The w = 16 / 32 region and matrix calls run
// on the MI355X too (wide-word kernels) when the size is a whole number of
// words -- the reference's own precondition (jerasure.h: size a multiple of
// sizeof(long)); a ragged size, where the reference reads and writes past the
// region, takes the exact-word CPU restatement in jerasure_surface.cpp.
// Host-side math (fields, matrices) comes from libecgpu's host C ABI.
// Bit-matrix / schedule coding lives in jerasure_surface.cpp: execution on
// the MI355X (GF(2) packet kernels), matrix / schedule construction on the
// host.
#include <cstdio>
#include <cstdlib>

#include "ecgpu.h"
// The reference surface is this library's export list (default visibility);
// everything else is built -fvisibility=hidden.
#pragma GCC visibility push(default)
#include "galois.h"
#include "jerasure.h"
#include "reed_sol.h"
#pragma GCC visibility pop
#include "surface_cpu.hpp"

namespace {

// A GPU failure libecgpu could not complete on the CPU -- the fallback is off
// (ECGPU_CPU_FALLBACK=0), a buffer is device memory, or the call had already
// written caller memory -- surfaces through the reference's OWN failure
// channels: calls that return a status report it there
// (jerasure_matrix_decode returns -1, which the client already handles,
// client_main.cpp:2118-2124); void calls print a message and exit(1), the
// reference's convention for unrecoverable conditions (galois.cpp:330-334,
// jerasure.cpp:291-294).
// Buffers that break the library's contract (a written region partially
// overlapping another region of the call, buffer_contract.hpp) take the same
// channel: the reference's bytes for them depend on its loop order, and a
// silently different answer would be worse than the reference's own exit.
const char* fallback_note() {
  int on = 1;
  return ecgpu_get_knob("ECGPU_CPU_FALLBACK", &on) == ECGPU_OK && on == 0 ? " [CPU fallback off: ECGPU_CPU_FALLBACK=0]"
                                                                          : "";
}

[[noreturn]] void gpu_fatal(const char* fn, int rc) {
  if (rc == ECGPU_ERR_ARG)
    std::fprintf(stderr, "%s: arguments rejected (%d): %s\n", fn, rc, ecgpu_last_error());
  else
    std::fprintf(stderr, "%s: MI355X path failed (%d): %s%s\n", fn, rc, ecgpu_last_error(), fallback_note());
  std::exit(1);
}

inline void check(const char* fn, int rc) {
  if (rc != ECGPU_OK) gpu_fatal(fn, rc);
}

// w = 8 always runs on the GPU; w = 16 / 32 when size is whole words.
inline bool whole_words(int w, int size) { return w == 8 || ((w == 16 || w == 32) && size % (w / 8) == 0); }

}  // namespace

// ============================================================ galois.h ====
int galois_single_multiply(int a, int b, int w) { return ecgpu_galois_single_multiply(a, b, w); }
int galois_single_divide(int a, int b, int w) { return ecgpu_galois_single_divide(a, b, w); }
int galois_inverse(int x, int w) { return ecgpu_galois_inverse(x, w); }

int galois_log(int value, int w) {
  if (w > 30) {
    std::fprintf(stderr, "Error: galois_log - w is too big.  Sorry\n");
    std::exit(1);
  }
  return ecgpu_galois_log(value, w);
}

int galois_ilog(int value, int w) {
  if (w > 30) {
    std::fprintf(stderr, "Error: galois_ilog - w is too big.  Sorry\n");
    std::exit(1);
  }
  return ecgpu_galois_ilog(value, w);
}

int galois_create_log_tables(int w) { return ecgpu_cpu::create_log_tables(w); }
int galois_create_mult_tables(int w) { return ecgpu_cpu::create_mult_tables(w); }
int galois_create_split_w8_tables() { return ecgpu_galois_create_split_w8_tables(); }

int galois_logtable_multiply(int x, int y, int w) { return (x == 0 || y == 0) ? 0 : ecgpu_galois_single_multiply(x, y, w); }
int galois_logtable_divide(int x, int y, int w) { return ecgpu_galois_single_divide(x, y, w); }
int galois_multtable_multiply(int x, int y, int w) { return ecgpu_galois_single_multiply(x, y, w); }
int galois_multtable_divide(int x, int y, int w) { return ecgpu_galois_single_divide(x, y, w); }
int galois_shift_multiply(int x, int y, int w) { return ecgpu_cpu::shift_multiply(x, y, w); }
int galois_shift_divide(int a, int b, int w) {
  if (b == 0) return -1;
  if (a == 0) return 0;
  return ecgpu_cpu::shift_multiply(a, ecgpu_cpu::shift_inverse(b, w), w);
}
int galois_shift_inverse(int y, int w) { return ecgpu_cpu::shift_inverse(y, w); }
int galois_split_w8_multiply(int x, int y) { return ecgpu_galois_split_w8_multiply(x, y); }

int* galois_get_mult_table(int w) { return ecgpu_cpu::mult_table(w); }
int* galois_get_div_table(int w) { return ecgpu_cpu::div_table(w); }
int* galois_get_log_table(int w) { return ecgpu_cpu::log_table(w); }
int* galois_get_ilog_table(int w) { return ecgpu_cpu::ilog_table(w); }

void galois_region_xor(char* r1, char* r2, char* r3, int nbytes) {
  check("galois_region_xor", ecgpu_galois_region_xor(r1, r2, r3, nbytes));
}

void galois_w08_region_multiply(char* region, int multby, int nbytes, char* r2, int add) {
  check("galois_w08_region_multiply", ecgpu_galois_w08_region_multiply(region, multby, nbytes, r2, add));
}

void galois_w16_region_multiply(char* region, int multby, int nbytes, char* r2, int add) {
  check("galois_w16_region_multiply", ecgpu_galois_w16_region_multiply(region, multby, nbytes, r2, add));
}

void galois_w32_region_multiply(char* region, int multby, int nbytes, char* r2, int add) {
  check("galois_w32_region_multiply", ecgpu_galois_w32_region_multiply(region, multby, nbytes, r2, add));
}

// ========================================================== reed_sol.h ====
int* reed_sol_vandermonde_coding_matrix(int k, int m, int w) { return ecgpu_reed_sol_vandermonde_coding_matrix(k, m, w); }
int* reed_sol_extended_vandermonde_matrix(int rows, int cols, int w) {
  return ecgpu_reed_sol_extended_vandermonde_matrix(rows, cols, w);
}
int* reed_sol_big_vandermonde_distribution_matrix(int rows, int cols, int w) {
  return ecgpu_reed_sol_big_vandermonde_distribution_matrix(rows, cols, w);
}
int* reed_sol_r6_coding_matrix(int k, int w) { return ecgpu_reed_sol_r6_coding_matrix(k, w); }

int reed_sol_r6_encode(int k, int w, char** data_ptrs, char** coding_ptrs, int size) {
  if (w != 8 && w != 16 && w != 32) return 0;
  if (!whole_words(w, size)) return ecgpu_cpu::r6_encode(k, w, data_ptrs, coding_ptrs, size);
  const int rc = ecgpu_reed_sol_r6_encode(k, w, data_ptrs, coding_ptrs, size);
  if (rc < 0) gpu_fatal("reed_sol_r6_encode", rc);
  return rc;
}

void reed_sol_galois_w08_region_multby_2(char* region, int nbytes) {
  check("reed_sol_galois_w08_region_multby_2", ecgpu_reed_sol_galois_w08_region_multby_2(region, nbytes));
}
void reed_sol_galois_w16_region_multby_2(char* region, int nbytes) {
  check("reed_sol_galois_w16_region_multby_2", ecgpu_reed_sol_galois_w16_region_multby_2(region, nbytes));
}
void reed_sol_galois_w32_region_multby_2(char* region, int nbytes) {
  check("reed_sol_galois_w32_region_multby_2", ecgpu_reed_sol_galois_w32_region_multby_2(region, nbytes));
}

// ========================================================== jerasure.h ====
void jerasure_matrix_encode(int k, int m, int w, int* matrix, char** data_ptrs, char** coding_ptrs, int size) {
  if (w != 8 && w != 16 && w != 32) {
    std::fprintf(stderr, "ERROR: jerasure_matrix_encode() and w is not 8, 16 or 32\n");
    std::exit(1);
  }
  if (whole_words(w, size)) {
    check("jerasure_matrix_encode", ecgpu_jerasure_matrix_encode(k, m, w, matrix, data_ptrs, coding_ptrs, size));
    return;
  }
  for (int i = 0; i < m; ++i)
    ecgpu_cpu::matrix_dotprod(k, w, matrix + i * k, nullptr, k + i, data_ptrs, coding_ptrs, size);
}

int jerasure_matrix_decode(int k, int m, int w, int* matrix, int row_k_ones, int* erasures, char** data_ptrs,
                           char** coding_ptrs, int size) {
  if (w != 8 && w != 16 && w != 32) return -1;
  if (!whole_words(w, size))
    return ecgpu_cpu::matrix_decode(k, m, w, matrix, row_k_ones, erasures, data_ptrs, coding_ptrs, size);
  const int rc = ecgpu_jerasure_matrix_decode(k, m, w, matrix, row_k_ones, erasures, data_ptrs, coding_ptrs, size);
  if (rc == ECGPU_ERR) return -1;
  if (rc != ECGPU_OK) {  // the reference's failure result, with the reason on stderr
    std::fprintf(stderr, "jerasure_matrix_decode: %s (%d): %s%s\n",
                 rc == ECGPU_ERR_ARG ? "arguments rejected" : "MI355X path failed", rc, ecgpu_last_error(),
                 rc == ECGPU_ERR_ARG ? "" : fallback_note());
    return -1;
  }
  return 0;
}

void jerasure_matrix_dotprod(int k, int w, int* matrix_row, int* src_ids, int dest_id, char** data_ptrs,
                             char** coding_ptrs, int size) {
  if (w != 1 && w != 8 && w != 16 && w != 32) {
    std::fprintf(stderr, "ERROR: jerasure_matrix_dotprod() called and w is not 1, 8, 16 or 32\n");
    std::exit(1);
  }
  // w = 1 is byte-exact XOR / copy at any size, like w = 8
  if (w == 1 || whole_words(w, size)) {
    check("jerasure_matrix_dotprod",
          ecgpu_jerasure_matrix_dotprod(k, w, matrix_row, src_ids, dest_id, data_ptrs, coding_ptrs, size));
    return;
  }
  ecgpu_cpu::matrix_dotprod(k, w, matrix_row, src_ids, dest_id, data_ptrs, coding_ptrs, size);
}

void jerasure_do_parity(int k, char** data_ptrs, char* parity_ptr, int size) {
  check("jerasure_do_parity", ecgpu_jerasure_do_parity(k, data_ptrs, parity_ptr, size));
}

int jerasure_make_decoding_matrix(int k, int m, int w, int* matrix, int* erased, int* decoding_matrix, int* dm_ids) {
  return ecgpu_jerasure_make_decoding_matrix(k, m, w, matrix, erased, decoding_matrix, dm_ids);
}
int* jerasure_erasures_to_erased(int k, int m, int* erasures) { return ecgpu_jerasure_erasures_to_erased(k, m, erasures); }
int jerasure_invert_matrix(int* mat, int* inv, int rows, int w) { return ecgpu_jerasure_invert_matrix(mat, inv, rows, w); }
int jerasure_invertible_matrix(int* mat, int rows, int w) { return ecgpu_jerasure_invertible_matrix(mat, rows, w); }
int* jerasure_matrix_multiply(int* m1, int* m2, int r1, int c1, int r2, int c2, int w) {
  return ecgpu_jerasure_matrix_multiply(m1, m2, r1, c1, r2, c2, w);
}

void jerasure_get_stats(double* fill_in) {
  ecgpu_jerasure_get_stats(fill_in);  // GPU-path counters (reset)
  double cpu[3];
  ecgpu_cpu::take_stats(cpu);          // CPU-surface counters (reset)
  for (int i = 0; i < 3; ++i) fill_in[i] += cpu[i];
}
