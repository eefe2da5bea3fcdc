// cpu_fallback.hpp -- SURVEY.md §8b's failure contract: "the GPU layer must
// add no new failure modes; on any HIP error it falls back to the CPU and
// records it in stats / logs".
//
// A synchronous call (ecgpu_jerasure_*, ecgpu_galois_*, ecgpu_reed_sol_*,
// and so every drop-in name of libjerasure_amd.so) that gets a HIP error
// while every buffer it names is host memory and before any byte of the
// caller's memory has been written is completed here, on the CPU, by the
// library's OWN code: the same fused map (planner.hpp) the kernel would have
// applied, read-all-sources-then-write per byte column like the kernel, so
// aliasing and the byte counters are exactly the GPU path's.  Nothing here
// comes from oracle/ or the reference.  A call whose outputs were already
// partly written keeps the error (the drop-in then exits, the reference's
// channel).  A sticky HIP error (the device or its context is gone) marks the
// device lost, and later calls on it go straight to the CPU.
//
// Gated by the ECGPU_CPU_FALLBACK knob (1 by default, so a deployed
// datanode keeps running; the bench, smoke() and the -m gpu session set 0 and
// assert ecgpu_fallback_count() == 0, so no measured or parity-tested result
// ever comes from here).  ECGPU_TEST_INJECT_HIP (tests only) fails calls
// with ECGPU_ERR_HIP on purpose: 1 before the first launch, 2 the same and
// the device marked lost, 3 after the call has started writing caller
// memory.  Host-only code (the sanitizer harness builds it).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "planner.hpp"

namespace ecgpu {
namespace __attribute__((visibility("hidden"))) rt {

// dst[r] = XOR_j coef[r][j] * src[j] over GF(2^op.w), byte columns
// independent: every source column is read before any output column is
// written (an output that is also a source reads its original bytes).  size
// is a whole number of w/8-byte words.  Outputs with no terms become zero.
void cpu_apply(const FusedOp& op, int64_t size);

// The GF(2) packet form (PacketTracker keys): slot s's packet row r of
// super-packet sp is ptrs[s] + sp * spstride + r * ps.
void cpu_apply_packets(const FusedOp& op, const std::vector<char*>& ptrs, int64_t nsp, int64_t spstride, int64_t ps);

// ---- per-call trace (thread-local: a split call's ranges run on their own threads)
void trace_begin();
void note_caller_write();  // about to write caller memory (D2H, or a kernel writing it in place)
bool caller_written();

// ---- devices whose HIP context hit a sticky error
void mark_device_lost(int device);
bool device_lost(int device);

bool fallback_enabled();
// ECGPU_TEST_INJECT_HIP at a point of the call: `stage` 0 = before the first
// launch, 1 = after caller memory has started to be written.  Returns
// ECGPU_ERR_HIP (with the message set) where the knob asks for a failure.
int injected_failure(int device, int stage);

// Counts the fallback; the first one of the process prints one stderr line.
void record_fallback(const char* call, const std::string& why);
int64_t fallback_count();

}  // namespace rt
}  // namespace ecgpu
