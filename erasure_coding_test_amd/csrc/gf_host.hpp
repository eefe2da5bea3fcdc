// gf_host.hpp -- host-side Galois-field arithmetic GF(2^w), w = 1..32.
//
// Same fields as the reference (galois.cpp:48-81: one primitive polynomial
// per w, generator 2), so every product, quotient, log and inverse is the
// same number.  Layout of the exported tables follows the reference API
// (galois.h:53-56): mult/div tables are int[(x << w) | y], ilog is offset so
// that indices [-(2^w-1), 2*(2^w-1)) are valid (galois.cpp:185-189).
//
// Thread-safe: all tables are built once under std::call_once / a mutex,
// unlike the reference's unsynchronised lazy statics (galois.cpp:329-336).
#pragma once
#include <cstdint>

namespace ecgpu {

// Low w bits of the primitive polynomial for GF(2^w) (x^w term implicit).
uint32_t prim_poly(int w);

// Carry-less multiply of a*b reduced modulo prim_poly(w).
uint32_t gf_mul_poly(uint32_t a, uint32_t b, int w);

// GF(2^8) dense tables, built once.
struct Gf8Tables {
  uint8_t mul[256][256];  // mul[a][b] = a*b
  uint8_t inv[256];       // inv[0] = 0 (caller handles the -1 convention)
  int16_t log[256];       // log[0] = 255 (reference convention, galois.cpp:168-171)
  uint8_t exp[255];
};
const Gf8Tables& gf8();

// Scalar ops with the reference's edge conventions (galois.cpp:322-398, :597-603).
int single_multiply(int a, int b, int w);
int single_divide(int a, int b, int w);  // b == 0 -> -1
int inverse(int a, int w);               // a == 0 -> -1
int shift_multiply(int a, int b, int w);
int shift_inverse(int a, int w);

// Table accessors with the reference API's layout and lifetime (never freed).
// Return nullptr where the reference returns NULL / -1 (mult w >= 14, log w > 30).
int* mult_table(int w);
int* div_table(int w);
int* log_table(int w);
int* ilog_table(int w);  // already offset: valid index range [-(2^w-1), 2*(2^w-1))
int create_log_tables(int w);   // 0 / -1
int create_mult_tables(int w);  // 0 / -1
// galois.cpp:756-809: the seven 2^16-entry byte-pair product tables of
// GF(2^32) (built once, thread-safely; 0, or -1 if they cannot be allocated)
// and the w = 32 multiply that reads them (computed directly while they are
// not built, where the reference would dereference NULL).
int create_split_w8_tables();
int split_w8_multiply(int x, int y);

}  // namespace ecgpu
