// matrix_host.hpp -- host-side coding / decoding matrix construction.
//
// Everything here runs once per (k, m, erasure pattern) in microseconds and
// stays on the host; only the resulting coefficients travel to the GPU.
// Matrices are row-major int arrays allocated with malloc (callers free()),
// exactly the ownership of the reference API (jerasure.h:43-70, reed_sol.h).
#pragma once

namespace ecgpu {

// reed_sol.cpp:227-255 / :257-352 / :63-84 / :43-61
int* extended_vandermonde_matrix(int rows, int cols, int w);
int* big_vandermonde_distribution_matrix(int rows, int cols, int w);
int* vandermonde_coding_matrix(int k, int m, int w);
int* r6_coding_matrix(int k, int w);

// jerasure.cpp:360-445 (destroys mat), :447-502, :1126-1141
int invert_matrix(int* mat, int* inv, int rows, int w);
int invertible_matrix(int* mat, int rows, int w);
int* matrix_multiply(const int* m1, const int* m2, int r1, int c1, int r2, int c2, int w);

// jerasure.cpp:507-532, :84-112
int* erasures_to_erased(int k, int m, const int* erasures);
int make_decoding_matrix(int k, int m, int w, const int* matrix, const int* erased, int* decoding_matrix,
                         int* dm_ids);

// GF(2) bit-matrix helpers: jerasure.cpp:257-283, :1034-1123, :115-151
int* matrix_to_bitmatrix(int k, int m, int w, const int* matrix);
int invert_bitmatrix(int* mat, int* inv, int rows);
int invertible_bitmatrix(int* mat, int rows);
int make_decoding_bitmatrix(int k, int m, int w, const int* matrix, const int* erased, int* decoding_matrix,
                            int* dm_ids);

}  // namespace ecgpu
