/* galois.h (drop-in) -- GF(2^w) surface of libjerasure_amd.so.
 * Declares, with identical signatures, the functions of the reference's
 * include/galois.h:41-95 so reference callers compile and link unchanged.
 * Implementation: erasure_coding_test_amd/csrc/jerasure_dropin.cpp
 * (w=8 region ops run on the MI355X through include/ecgpu.h). */
#ifndef ECGPU_DROPIN_GALOIS_H
#define ECGPU_DROPIN_GALOIS_H
#include <stdio.h>
#include <stdlib.h>

int galois_single_multiply(int a, int b, int w);
int galois_single_divide(int a, int b, int w);
int galois_log(int value, int w);
int galois_ilog(int value, int w);

int galois_create_log_tables(int w);
int galois_logtable_multiply(int x, int y, int w);
int galois_logtable_divide(int x, int y, int w);

int galois_create_mult_tables(int w);
int galois_multtable_multiply(int x, int y, int w);
int galois_multtable_divide(int x, int y, int w);

int galois_shift_multiply(int x, int y, int w);
int galois_shift_divide(int x, int y, int w);

int galois_create_split_w8_tables();
int galois_split_w8_multiply(int x, int y);

int galois_inverse(int x, int w);
int galois_shift_inverse(int y, int w);

int *galois_get_mult_table(int w);
int *galois_get_div_table(int w);
int *galois_get_log_table(int w);
int *galois_get_ilog_table(int w);

/* r3 = r1 ^ r2 over nbytes (r3 may alias r1 or r2). */
void galois_region_xor(char *r1, char *r2, char *r3, int nbytes);

/* r2 (^)= multby * region, or region *= multby in place when r2 == NULL. */
void galois_w08_region_multiply(char *region, int multby, int nbytes, char *r2, int add);
void galois_w16_region_multiply(char *region, int multby, int nbytes, char *r2, int add);
void galois_w32_region_multiply(char *region, int multby, int nbytes, char *r2, int add);

#endif
