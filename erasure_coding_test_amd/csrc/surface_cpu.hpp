// surface_cpu.hpp -- CPU side of the drop-in library for the parts of the
// reference surface outside the north-star path (w = 16 / 32 region math,
// field-table accessors, byte counters).  The w = 8 hot path never comes
// here; see jerasure_dropin.cpp.
#pragma once

namespace ecgpu_cpu {

int create_log_tables(int w);
int create_mult_tables(int w);
int* mult_table(int w);
int* div_table(int w);
int* log_table(int w);
int* ilog_table(int w);
int shift_multiply(int a, int b, int w);
int shift_inverse(int a, int w);

// galois.cpp:469-546 / :667-729 semantics, exact on [0, nbytes).
void region_multiply_w16(char* region, int multby, int nbytes, char* r2, int add);
void region_multiply_w32(char* region, int multby, int nbytes, char* r2, int add);
void region_xor(const char* r1, const char* r2, char* r3, long nbytes);

// jerasure.cpp:561-620 for w in {16, 32} (ragged sizes); :153-254 for w in {16, 32}.
void matrix_dotprod(int k, int w, const int* row, const int* src_ids, int dest_id, char** data, char** coding,
                    int size);
int matrix_decode(int k, int m, int w, int* matrix, int row_k_ones, int* erasures, char** data, char** coding,
                  int size);
// reed_sol.cpp:200-225 for w in {16, 32}.
int r6_encode(int k, int w, char** data, char** coding, int size);

void count(double xor_b, double gf_b, double memcpy_b);
void take_stats(double out[3]);

}  // namespace ecgpu_cpu
