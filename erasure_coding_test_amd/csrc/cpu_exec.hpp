// cpu_exec.hpp -- the library's own CPU executor of a planned fused map
// (planner.hpp).  It serves three callers, all for synchronous calls whose
// buffers are host memory:
//   * small calls below ECGPU_MIN_OFFLOAD_KIB bytes moved, where the GPU
//     round trip (launch + sync + staging) costs more than the arithmetic
//     (the measured crossover);
//   * every such call when ECGPU_GPU=0;
//   * SURVEY.md §8b's failure contract (cpu_fallback.hpp).
// Nothing here comes from oracle/ or the reference.
//
// GF(2^w) multiplication by a constant c is GF(2)-linear, so on hosts with
// AVX-512 + GFNI one vgf2p8affineqb applies c's 8x8 bit matrix to 64 bytes
// (any field polynomial: the matrix is built from the reference's own
// products, gf_host).  w = 16 / 32 words are B x B blocks of such matrices
// over byte rotations of the word.  Without GFNI: w = 8 by the north star's
// nibble split on AVX2 (two vpshufb per 32 bytes, rows grouped like the
// GFNI path: each source loaded once per 32-byte column), then scalar.
//
// Semantics: dst[r] = XOR_j coef[r][j] * src[j]; every byte column is
// independent and every source column is read before any output column is
// written, so an output that is also a source reads its original bytes (the
// kernels' order, and the reference's sequential result for identical
// buffers).  Outputs with no terms become zero.  Host-only (g++).
#pragma once
#include <cstdint>
#include <vector>

#include "planner.hpp"

namespace ecgpu {
namespace __attribute__((visibility("hidden"))) rt {

// SIMD level the executor runs at: 2 AVX-512BW + GFNI, 1 AVX2, 0 scalar --
// the host's best, lowered by the ECGPU_CPU_SIMD knob (tests run every level).
int cpu_simd_level();

// size: a whole number of w/8-byte words.
void cpu_apply(const FusedOp& op, int64_t size);
// The same at a given SIMD level (capped at the host's; the tests' hook).
void cpu_apply(const FusedOp& op, int64_t size, int level);

// The GF(2) packet form (PacketTracker keys): slot s's packet row r of
// super-packet sp is ptrs[s] + sp * spstride + r * ps.
void cpu_apply_packets(const FusedOp& op, const std::vector<char*>& ptrs, int64_t nsp, int64_t spstride, int64_t ps);
void cpu_apply_packets(const FusedOp& op, const std::vector<char*>& ptrs, int64_t nsp, int64_t spstride, int64_t ps,
                       int level);

// The 8x8 GF(2) matrix of y -> c * y restricted to input byte b -> output
// byte a of a w-bit word (w = 8: a = b = 0), in vgf2p8affineqb's layout: byte
// 7 - i of the qword selects the input bits whose parity is output bit i.
uint64_t gf_affine_block(uint32_t c, int w, int a, int b);

}  // namespace rt
}  // namespace ecgpu
