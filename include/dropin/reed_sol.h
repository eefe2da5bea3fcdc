/* reed_sol.h (drop-in) -- Reed-Solomon matrix surface of libjerasure_amd.so,
 * same signatures as the reference's include/reed_sol.h:33-42. */
#ifndef ECGPU_DROPIN_REED_SOL_H
#define ECGPU_DROPIN_REED_SOL_H

int *reed_sol_vandermonde_coding_matrix(int k, int m, int w);
int *reed_sol_extended_vandermonde_matrix(int rows, int cols, int w);
int *reed_sol_big_vandermonde_distribution_matrix(int rows, int cols, int w);

int reed_sol_r6_encode(int k, int w, char **data_ptrs, char **coding_ptrs, int size);
int *reed_sol_r6_coding_matrix(int k, int w);

void reed_sol_galois_w08_region_multby_2(char *region, int nbytes);
void reed_sol_galois_w16_region_multby_2(char *region, int nbytes);
void reed_sol_galois_w32_region_multby_2(char *region, int nbytes);

#endif
