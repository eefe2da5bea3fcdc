// shard_stride.hpp -- the HBM layout advice behind
// ecgpu_recommended_shard_stride (include/ecgpu.h), header-only so the
// measurement labs (tools/*_lab.hip) lay their slabs out exactly as the
// library does.
//
// Shard-stride skew.  A lane reads the same column of every shard, so the
// k + m concurrent accesses sit one stride apart; when that stride lines up
// with the HBM channel / bank hash they collide.  The effect is a
// deterministic function of the stride: an in-process sweep (RS(10,4), ~5 GiB
// per launch, every skew's slab interleaved, tools/skew_sweep.sh) gave the same
// numbers within ~1 % on three MI355X boxes (profiles/r03_skew_sweep_*.jsonl),
// including sharp dips of 15-30 % (e.g. +12 KiB at 1 and 3 MiB shards, +8 KiB
// at 2 and 6 MiB, +14 KiB at 512 KiB, no skew from 4 MiB up), and again on
// independent random shards (profiles/r03_skew_sweep_random.jsonl; the first
// sweeps filled every shard from one buffer, and HBM throughput depends on the
// data).  For the shard sizes measured, the skew with the best
// rate; tie-breaks from the BASELINE configs' own A/Bs on random data:
// RS(6,3) 1 MiB none (1-3 % over +10 KiB, profiles/r03_skew_ab_random.jsonl);
// RS(10,4) 4 MiB +6 KiB, the best bench step (encode + decode{0}) on three
// boxes, 0.6-1 % over the +14 KiB first chosen on the old fill
// (profiles/r03_skew_step_ab.jsonl); RS(12,4) 16 MiB +8 KiB (4 %).  Other
// sizes keep +10 KiB, within 1-4 % of the best at every size measured and
// never near a dip.
//
// Small shards (round 5, profiles/r05_skew_small.jsonl: 4-341 KiB at
// RS(4,2) / RS(6,3) / RS(10,4)): from 8 to 256 KiB NO skew is the best or
// within 2 % of it at every size and scheme (at 4 KiB 3-5 % ahead of +10
// KiB), and +10 KiB loses 3-22 % (e.g. RS(6,3)
// 32 KiB 0.820 vs 0.670 of peak, C1's RS(4,2) 64 KiB 0.825 vs 0.747): a
// stripe of small shards is one short contiguous run, and the skew's gaps
// only break it up.  From ~341 KiB (the ECX block) +10 KiB is back on top.
// At 512 KiB (profiles/r05_skew_mid.jsonl) none is best for RS(4,2) / RS(6,3)
// / RS(12,4) too (+7 / +1 / +4 % over +8 KiB) -- but not at 341 KiB, where
// +10 KiB leads by 0-3 %, so 512 KiB is a table class, not part of the rule.
// RS(10,4), which the round-3 table was tuned on, keeps its +12 KiB at 256
// and +8 KiB at 512 KiB (1-3 % ahead of none on four sweeps) as per-scheme
// entries (shard_stride(size, k + m)).
#pragma once
#include <cstdint>

namespace ecgpu {

struct SkewClass {
  int64_t size, skew;
};
constexpr SkewClass kSkewTable[] = {
    {256 << 10, 0},        {512 << 10, 0},  {1 << 20, 0},          {2 << 20, 12 << 10},
    {3 << 20, 8 << 10},    {4 << 20, 6 << 10},   {6 << 20, 12 << 10},   {8 << 20, 12 << 10},
    {12 << 20, 8 << 10},   {16 << 20, 8 << 10},   {32 << 20, 8 << 10},   {64 << 20, 8 << 10},
};
constexpr int64_t kDefaultSkew = 10 << 10;
// shards up to this size (+1/16, like the table's classes) take no skew
constexpr int64_t kNoSkewUpTo = 256 << 10;

// Per-scheme entries (shards = k + m), ahead of the rule and the table.
struct SchemeSkew {
  int64_t size;
  int shards;
  int64_t skew;
};
constexpr SchemeSkew kSchemeSkewTable[] = {{256 << 10, 14, 12 << 10}, {512 << 10, 14, 8 << 10}};

inline bool in_class(int64_t rounded, int64_t size) { return rounded >= size - size / 16 && rounded <= size + size / 16; }

// round_up(size, 256) + a skew: the scheme's entry for that size (+-1/16) when
// `shards` (k + m) has one, else none up to kNoSkewUpTo (+1/16), else the
// table's skew for that size, or kDefaultSkew elsewhere.  shards = 0: no
// scheme (the size-only advice).
inline int64_t shard_stride(int64_t size, int shards = 0) {
  if (size < 0) size = 0;
  const int64_t rounded = (size + 255) & ~int64_t(255);
  for (const SchemeSkew& c : kSchemeSkewTable)
    if (c.shards == shards && in_class(rounded, c.size)) return rounded + c.skew;
  if (rounded <= kNoSkewUpTo + kNoSkewUpTo / 16) return rounded;
  int64_t skew = kDefaultSkew;
  for (const SkewClass& c : kSkewTable)
    if (in_class(rounded, c.size)) skew = c.skew;
  return rounded + skew;
}

}  // namespace ecgpu
