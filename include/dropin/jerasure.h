/* jerasure.h (drop-in) -- erasure-coding surface of libjerasure_amd.so, same
 * signatures as the reference's include/jerasure.h:113-282.  Conventions
 * (k data + m coding devices, ids 0..k+m-1, -1 terminated erasure lists,
 * m x k row-major matrices, malloc'd results) are the reference's. */
#ifndef ECGPU_DROPIN_JERASURE_H
#define ECGPU_DROPIN_JERASURE_H
#include "galois.h"

/* bit-matrices and XOR schedules (host) */
int *jerasure_matrix_to_bitmatrix(int k, int m, int w, int *matrix);
int **jerasure_dumb_bitmatrix_to_schedule(int k, int m, int w, int *bitmatrix);
int **jerasure_smart_bitmatrix_to_schedule(int k, int m, int w, int *bitmatrix);
int ***jerasure_generate_schedule_cache(int k, int m, int w, int *bitmatrix, int smart);
void jerasure_free_schedule(int **schedule);
void jerasure_free_schedule_cache(int k, int m, int ***cache);

/* encoding */
void jerasure_do_parity(int k, char **data_ptrs, char *parity_ptr, int size);
void jerasure_matrix_encode(int k, int m, int w, int *matrix, char **data_ptrs, char **coding_ptrs, int size);
void jerasure_bitmatrix_encode(int k, int m, int w, int *bitmatrix, char **data_ptrs, char **coding_ptrs, int size,
                               int packetsize);
void jerasure_schedule_encode(int k, int m, int w, int **schedule, char **data_ptrs, char **coding_ptrs, int size,
                              int packetsize);

/* decoding (0 on success, -1 on failure) */
int jerasure_matrix_decode(int k, int m, int w, int *matrix, int row_k_ones, int *erasures, char **data_ptrs,
                           char **coding_ptrs, int size);
int jerasure_bitmatrix_decode(int k, int m, int w, int *bitmatrix, int row_k_ones, int *erasures, char **data_ptrs,
                              char **coding_ptrs, int size, int packetsize);
int jerasure_schedule_decode_lazy(int k, int m, int w, int *bitmatrix, int *erasures, char **data_ptrs,
                                  char **coding_ptrs, int size, int packetsize, int smart);
int jerasure_schedule_decode_cache(int k, int m, int w, int ***scache, int *erasures, char **data_ptrs,
                                   char **coding_ptrs, int size, int packetsize);
int jerasure_make_decoding_matrix(int k, int m, int w, int *matrix, int *erased, int *decoding_matrix, int *dm_ids);
int jerasure_make_decoding_bitmatrix(int k, int m, int w, int *matrix, int *erased, int *decoding_matrix,
                                     int *dm_ids);
int *jerasure_erasures_to_erased(int k, int m, int *erasures);

/* dot products and schedules */
void jerasure_matrix_dotprod(int k, int w, int *matrix_row, int *src_ids, int dest_id, char **data_ptrs,
                             char **coding_ptrs, int size);
void jerasure_bitmatrix_dotprod(int k, int w, int *bitmatrix_row, int *src_ids, int dest_id, char **data_ptrs,
                                char **coding_ptrs, int size, int packetsize);
void jerasure_do_scheduled_operations(char **ptrs, int **schedule, int packetsize);

/* inversion */
int jerasure_invert_matrix(int *mat, int *inv, int rows, int w);
int jerasure_invert_bitmatrix(int *mat, int *inv, int rows);
int jerasure_invertible_matrix(int *mat, int rows, int w);
int jerasure_invertible_bitmatrix(int *mat, int rows);

/* misc */
void jerasure_print_matrix(int *matrix, int rows, int cols, int w);
void jerasure_print_bitmatrix(int *matrix, int rows, int cols, int w);
int *jerasure_matrix_multiply(int *m1, int *m2, int r1, int c1, int r2, int c2, int w);

/* stats: [0] bytes XORed, [1] bytes GF-multiplied, [2] bytes copied; resets */
void jerasure_get_stats(double *fill_in);

#endif
