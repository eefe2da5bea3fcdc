// gf_kernels.hpp -- CDNA4 (gfx950) kernels for the fused GF(2^8) matrix apply
//
//     dst[s][r][x] = XOR_j  coef[r][j] * src[s][j][x]      (GF(2^8), poly 0x11D)
//
// for every stripe s, output row r < R (<= 4 per launch) and byte x.  This
// one primitive carries jerasure_matrix_encode, _decode, _dotprod and the
// galois region ops (see planner.hpp).  It is HBM-bound integer byte work:
// no MFMA; 16-byte coalesced loads/stores; all K source columns of a lane
// are loaded before any arithmetic so a wave has K*16 B per lane in flight.
//
// Multiply engines:
//  * gf_apply<K,R,UNITS> (production, w = 8): c*x is GF(2)-linear in x, so a
//    byte splits into bit slices [0:2], [3:5], [6:7] and
//    c*x = T0[x&7] ^ T1[(x>>3)&7] ^ T2[x>>6] with Tp[e] = c*(e << 3p); one
//    v_perm_b32 looks up four bytes at once from tables held in scalar
//    registers (3 v_perm per coefficient-dword), terms fold three at a time
//    with v_bitop3 (XOR3), and unit coefficients are plain XORs from a
//    compile-time structure the host checks per launch.  K and R are
//    compile-time; gf_apply_perm_generic covers K > 16 and gf_apply_bytes
//    shard tails and misaligned pointers.
//  * gf_apply_lds<K,R> (w = 8, selectable; the bench's independent
//    self-check engine): the north star's nibble tables T_lo[x] = c*x,
//    T_hi[x] = c*(x<<4) staged in LDS, one 4-byte entry serving all R rows
//    of a nibble (2 ds_read_b32 per source byte for every row together).
//  * gf_apply_wide_nib<R> / gf_apply_wide<W,R> (w = 16 / 32) and
//    gf_xor_packets16 / gf_xor_packets (GF(2) bit-matrix / schedule coding):
//    see their sections below.
// gf_apply_perm (2-bit slices, runtime coefficient classes) and the LDS-DMA
// form are kept for the A/B probes of the diagnostic library.
//
// The kernels live in three headers: gf_kernels_w8.hpp (shared vocabulary and
// every w = 8 kernel), gf_kernels_wide.hpp (w = 16 / 32), gf_kernels_packets.hpp
// (GF(2) packet coding).
#pragma once
#include "gf_kernels_w8.hpp"
#include "gf_kernels_wide.hpp"
#include "gf_kernels_packets.hpp"
