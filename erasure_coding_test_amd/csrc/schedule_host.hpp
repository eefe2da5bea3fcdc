// schedule_host.hpp -- GF(2) XOR-schedule construction (host only): the
// reference's dumb / smart bit-matrix-to-schedule conversions
// (jerasure.cpp:1194-1344), the survivor layout and decoding schedule of
// scheduled decoding (jerasure.cpp:705-933) and the two-erasure schedule
// cache (jerasure.cpp:997-1032, :543-559).  A schedule is the reference's
// int**: malloc'd rows {src dev, src packet, dst dev, dst packet, xor?},
// terminated by a row whose first entry is -1.  Execution is on the GPU
// (ecgpu_schedule_run).
#pragma once
#include <vector>

namespace ecgpu {

int** dumb_bitmatrix_to_schedule(int k, int m, int w, const int* bitmatrix);
int** smart_bitmatrix_to_schedule(int k, int m, int w, const int* bitmatrix);
void free_schedule(int** schedule);

// Slot layout of scheduled decoding; false if the erasures are not decodable.
bool schedule_layout(int k, int m, const int* erasures, std::vector<int>& row_ids, std::vector<int>& ind_to_row);
// malloc'd k+m pointer table in slot order (NULL for unused slots).
char** schedule_ptrs(int k, int m, const int* erasures, char** data, char** coding);
// One schedule that rebuilds every erased device (NULL if not decodable).
int** decoding_schedule(int k, int m, int w, const int* bitmatrix, const int* erasures, int smart);
// m must be 2 (NULL otherwise); free with free_schedule_cache (-1 if m != 2).
int*** generate_schedule_cache(int k, int m, int w, const int* bitmatrix, int smart);
int free_schedule_cache(int k, int m, int*** cache);

}  // namespace ecgpu
