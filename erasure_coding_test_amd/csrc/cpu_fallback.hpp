// cpu_fallback.hpp -- when a synchronous call runs on the CPU executor
// (cpu_exec.hpp) instead of the GPU, and the bookkeeping of it.
//
// 1. SURVEY.md §8b's failure contract: "the GPU layer must add no new failure
//    modes; on any HIP error it falls back to the CPU and records it in stats
//    / logs".  A synchronous call (ecgpu_jerasure_*, ecgpu_galois_*,
//    ecgpu_reed_sol_*, and so every drop-in name of libjerasure_amd.so) that
//    gets a HIP error while every buffer it names is host memory is completed
//    on the CPU by the library's OWN executor: the same fused map (planner.hpp)
//    the kernel would have applied, read-all-sources-then-write per byte column
//    like the kernel, so aliasing and the byte counters are exactly the GPU
//    path's.  Nothing here comes from oracle/ or the reference.  The map reads
//    its sources only, so a call whose outputs are identical to none of its
//    sources stays recoverable even after the GPU wrote part of an output; a
//    call with such an alias keeps the error once it started writing caller
//    memory (the drop-in then exits, the reference's channel).  A sticky HIP
//    error (the device or its context is gone) marks the device lost, and
//    later calls on it go straight to the CPU.
//
//    Gated by the ECGPU_CPU_FALLBACK knob (1 by default, so a deployed
//    datanode keeps running; the bench, smoke() and the -m gpu session set 0
//    and assert ecgpu_fallback_count() == 0, so no measured or parity-tested
//    result ever comes from here).  The test_inject_hip knob (tests only, set
//    through ecgpu_set_knob, never read from the environment) fails calls with
//    ECGPU_ERR_HIP on purpose: 1 before the first launch, 2 the same and the
//    device marked lost, 3 after the call has started writing caller memory.
//
// 2. By choice (cpu_by_choice): a host-memory call that moves fewer than
//    ECGPU_MIN_OFFLOAD_KIB bytes (distinct buffers x size), where the GPU round
//    trip costs more than the arithmetic (the measured
//    crossover), or any host-memory call with ECGPU_GPU=0.  Counted by
//    ecgpu_cpu_call_count(); the Python package (tests, smoke(), bench) sets
//    the threshold to 0 and asserts the count stays 0.
//
// Host-only code (the sanitizer harness builds it).
#pragma once
#include <cstdint>
#include <string>

#include "cpu_exec.hpp"

namespace ecgpu {
namespace __attribute__((visibility("hidden"))) rt {

// ---- per-call trace (thread-local: a split call's ranges run on their own threads)
void trace_begin();
void note_caller_write();  // started writing caller memory in a call with an output that is also a source
bool caller_written();

// ---- devices whose HIP context hit a sticky error (ordinals 0..1023; others are never lost)
void mark_device_lost(int device);
bool device_lost(int device);

bool fallback_enabled();
// test_inject_hip at a point of the call: `stage` 0 = before the first
// launch, 1 = after caller memory has started to be written.  Returns
// ECGPU_ERR_HIP (with the message set) where the knob asks for a failure.
int injected_failure(int device, int stage);

// Counts the fallback; the first one of a process prints one stderr line.
void record_fallback(const char* call, const std::string& why);
int64_t fallback_count();

// Does a host-memory call moving `bytes_moved` bytes run on the CPU executor
// by choice (ECGPU_GPU=0, or below ECGPU_MIN_OFFLOAD_KIB)?
bool cpu_by_choice(int64_t bytes_moved);
// The threshold in force (ecgpu_min_offload_bytes).
int64_t min_offload_bytes();
void record_cpu_call();
int64_t cpu_call_count();

}  // namespace rt
}  // namespace ecgpu
