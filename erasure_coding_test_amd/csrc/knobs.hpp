// knobs.hpp -- the library's tuning and A/B switches (ECGPU_* environment
// variables), read ONCE per process and settable at run time through
// ecgpu_set_knob (include/ecgpu.h).
//
// Every dispatch decision that has a measured alternative (residency cap,
// store policy, engine, wide-word forms, staging thresholds, shard skew) is a
// knob, so an A/B compares both arms in one process -- between processes the
// same launch varies by 3-5 % -- without re-reading the
// environment on the hot path (getenv racing a setenv is undefined, and it
// cost a lookup per launch).  Host-only (no HIP).
#pragma once

namespace ecgpu {

enum class Knob : int {
  kCap,             // ECGPU_CAP: residency cap rule -1 auto (cap_for), 0 never, 1 always
  kBlocksPerCu,     // ECGPU_BLOCKS_PER_CU: capped launches' workgroups per CU, -1 auto (4 / 3 by shard streams), 0 none
  kKernel,          // ECGPU_KERNEL: w = 8 engine of new plans, 0 v_perm (production), 1 LDS nibble tables
  kNt,              // ECGPU_NT: store policy of new plans, 0 plain, 1 non-temporal
  kWidePerm,        // ECGPU_WIDE: 1 forces the w = 16 / 32 v_perm engine
  kNib16,           // ECGPU_NIB16: w = 16 packed-pair LDS kernel (1) or the 32-bit-entry form (0)
  kWideUnits,       // ECGPU_WIDE_UNITS: w = 32 unit-structure kernel when row 0 / column 0 are ones
  kWidePipe,        // ECGPU_WIDE_PIPE: pipelined wide kernel, 0 never, 1 measured rule, 2 every whole-block launch
  kWide16Bpcu,      // ECGPU_WIDE16_BPCU: w = 16 persistent grid's workgroups per CU (0 = occupancy)
  kWide16Units,     // ECGPU_WIDE16_UNITS: w = 16 unit-structure kernel (gf_apply_wide_nib16<R, 1>)
  kDevice,          // ECGPU_DEVICE: device of the synchronous calls (-1 = the caller's current device)
  kBounceKib,       // ECGPU_BOUNCE_KIB: staged bytes up to which a call goes through the pinned bounce
  kZcKib,           // ECGPU_ZC_KIB: staged bytes up to which a call is zero-copy
  kZcOutKib,        // ECGPU_ZC_OUT_KIB: staged output bytes written straight to coherent memory
  kZcOutShardKib,   // ECGPU_ZC_OUT_SHARD_KIB: ... per output
  kZcPinned,        // ECGPU_ZC_PINNED: pinned / registered host buffers used in place
  kZcGrid,          // ECGPU_ZC_GRID: workgroups of a launch reading host memory in place (0 = uncapped)
  kInline,          // ECGPU_INLINE: one-stripe calls carry pointers and tables in the kernel arguments
  kPipe2d,          // ECGPU_PIPE_2D: evenly spaced host shards cross PCIe as one 2-D copy
  kPipeD2hWorker,   // ECGPU_PIPE_D2H_WORKER: pipelines issue pageable D2H from a worker thread
  kPacket,          // ECGPU_PACKET: packet kernel, 0 production (unit form where the map allows), 1 8-B
                    // lanes, 2 unpipelined 16-B, 3 the general pipelined 16-B kernel only
  kShardSkewKib,    // ECGPU_SHARD_SKEW_KIB: one shard skew for every size (-1 = the measured table)
  kSplit,           // ECGPU_SPLIT: synchronous host-memory calls cut into byte ranges run concurrently,
                    // 0 off, -1 one range per visible device, N > 0 N ranges over the devices in turn
  kSplitMinKib,     // ECGPU_SPLIT_MIN_KIB: smallest range of a split call
  kTestD2hDelayUs,  // tests only, set with ecgpu_set_knob (no environment variable): the D2H
                    // worker sleeps this long before issuing a job (widens a race window)
  kCpuFallback,     // ECGPU_CPU_FALLBACK: a synchronous host-memory call that hits a HIP error before
                    // writing caller memory completes on the CPU (cpu_fallback.hpp), 1 on (default), 0 off
  kTestInjectHip,   // test_inject_hip (tests only, ecgpu_set_knob; never read from the environment):
                    // synchronous calls fail with ECGPU_ERR_HIP, 1 before the first launch, 2 the same and
                    // the device marked lost, 3 after writing caller memory
  kGpu,             // ECGPU_GPU: 0 runs every synchronous host-memory call on the CPU executor (cpu_exec.hpp)
  kMinOffloadKib,   // ECGPU_MIN_OFFLOAD_KIB: a synchronous host-memory call moving fewer bytes (distinct
                    // buffers x size) runs on the CPU executor; 0 = every call on the GPU; -1 (default) = the
                    // measured crossover for the executor's SIMD level, 16 MiB GFNI / 4 MiB AVX2 / 256 KiB
                    // scalar (cpu_fallback.cpp min_offload_bytes)
  kCpuSimd,         // ECGPU_CPU_SIMD: the CPU executor's SIMD level, -1 the host's best, 2 AVX-512 + GFNI,
                    // 1 AVX2, 0 scalar (never above what the host has)
  kPipeZc,          // ECGPU_PIPE_ZC: host pipelines over pinned host shards -- 0 DMA in and out, 1 DMA in and
                    // the kernel writes the outputs into the pinned host buffers, 2 the kernel reads the
                    // sources and writes the outputs in host memory (no DMA); read at pipeline creation
  kPipeContig,      // ECGPU_PIPE_CONTIG: host pipelines lay a ring slot's shards back to back (size % 256 == 0),
                    // so contiguous host stripes move as one 1-D copy; 0 = the skewed shard stride (read at creation)
  kPipeFlat,        // ECGPU_PIPE_FLAT: runs contiguous on both sides move as one 1-D copy (copy_shards); 0 = as a
                    // 2-D copy anyway (HIP's 2-D device->pinned copy: +4 % for one process, collapsing when
                    // processes share the GPU)
  kLinkCalls,       // ECGPU_LINK_CALLS: host-memory synchronous calls allowed in flight on one device's link before
                    // a further one runs on the CPU executor (0 = no limit)
  kCount
};

int knob(Knob k);

// name -> knob ("ECGPU_CAP" or "cap"); false for an unknown name
bool knob_by_name(const char* name, Knob* out);

}  // namespace ecgpu
