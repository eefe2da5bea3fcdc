// contract_host.cpp -- the buffer contract (buffer_contract.hpp) at every
// entry point that takes caller buffers.  Host-only: each check runs before
// the call touches the GPU, so a rejected call has launched and copied
// nothing (and the checks run in the CPU test suite without a GPU).
#include <cstdint>
#include <string>
#include <vector>

#include "buffer_contract.hpp"
#include "ecgpu.h"
#include "planner.hpp"

namespace ecgpu {
namespace __attribute__((visibility("hidden"))) rt {

int fail(int code, const std::string& msg);  // capi_host.cpp

// A synchronous call: the buffers the replayed reference sequence named.
// Identical pointers are one buffer to the tracker (the planner reproduces
// the reference's sequential semantics on them), so only partial overlaps
// involving a written buffer remain to reject.
int check_op_buffers(const char* call, const FusedOp& op, int64_t size) {
  if (size <= 0 || op.touched.size() < 2) return ECGPU_OK;
  std::vector<Span> s(op.touched.size());
  for (size_t i = 0; i < s.size(); ++i)
    s[i] = Span{op.touched[i], size, i < op.touched_written.size() && op.touched_written[i] != 0, int(i)};
  const auto c = find_conflict(s);
  if (c.first < 0) return ECGPU_OK;
  return fail(ECGPU_ERR_ARG, conflict_message(call, s, c, [&](int t) {
                return std::string(s[size_t(t)].written ? "written region" : "read region");
              }));
}

// One stripe of a host pipeline: the shards it reads (src_ids) and writes
// (out_ids), id < k in data_ptrs, else coding_ptrs.  An output may not share
// bytes with any other shard of the stripe, identical pointers included: the
// pipeline's plan is fixed when it is created (the coding matrix, or one
// decode pattern's fused map) and runs every stripe from the ORIGINAL bytes of
// its sources, whereas the reference's sequence over an output that is also a
// source reads the bytes it has just written (jerasure.cpp:285-299: coding[0]
// overwrites an aliased data shard before coding[1] reads it).  Only the
// synchronous calls replay that order per call (planner.hpp), so only they
// accept identical pointers.
int check_stripe_buffers(const char* call, int k, char** data, char** coding, const std::vector<int>& src_ids,
                         const std::vector<int>& out_ids, int64_t size) {
  if (size <= 0 || out_ids.empty()) return ECGPU_OK;
  std::vector<Span> s;
  s.reserve(src_ids.size() + out_ids.size());
  auto ptr = [&](int id) -> const void* { return id < k ? data[id] : coding[id - k]; };
  for (int id : src_ids) s.push_back(Span{ptr(id), size, false, id});
  for (int id : out_ids) s.push_back(Span{ptr(id), size, true, id});
  const auto c = find_conflict(s);
  if (c.first < 0) return ECGPU_OK;
  return fail(ECGPU_ERR_ARG, conflict_message(call, s, c, [&](int id) {
                return id < k ? "data_ptrs[" + std::to_string(id) + "]"
                              : "coding_ptrs[" + std::to_string(id - k) + "]";
              }));
}

// GF(2) packet calls: device slot sl covers [ptrs[sl], ptrs[sl] + extent[sl]).
// The packet tracker models slots, not pointers, so two slots on the same
// memory are rejected too when either is written.
int check_slot_buffers(const char* call, const std::vector<char*>& ptrs, const std::vector<int>& slots,
                       const std::vector<int64_t>& extent, const std::vector<char>& is_out) {
  std::vector<Span> s;
  for (int sl : slots)
    s.push_back(Span{ptrs[size_t(sl)], extent[size_t(sl)], is_out[size_t(sl)] != 0, sl});
  const auto c = find_conflict(s);
  if (c.first < 0) return ECGPU_OK;
  return fail(ECGPU_ERR_ARG,
              conflict_message(call, s, c, [](int sl) { return "device pointer " + std::to_string(sl); }));
}

}  // namespace rt
}  // namespace ecgpu

extern "C" {

// The batched plan API (ecgpu_plan_bind calls this first): srcs / dsts are
// stripe-major tables of `size`-byte buffers.  An output may be identical to
// a source of its own stripe when the plan runs as one launch (rows <= 4: a
// lane reads its column of every source before it writes); any other shared
// byte between an output and another buffer of the bind is rejected, since
// the stripes' workgroups run in no defined order.
ECGPU_API int ecgpu_plan_check_buffers(int rows, int nsrc, int stripes, const uint8_t* const* src_ptrs,
                                       uint8_t* const* dst_ptrs, int64_t size) {
  using namespace ecgpu;
  if (rows <= 0 || nsrc <= 0 || stripes < 0 || size < 0 || (stripes && (!src_ptrs || !dst_ptrs)))
    return rt::fail(ECGPU_ERR_ARG, "ecgpu_plan_check_buffers: bad arguments");
  if (size == 0 || stripes == 0) return ECGPU_OK;
  const int per = nsrc + rows;
  std::vector<Span> s;
  s.reserve(size_t(stripes) * size_t(per));
  for (int st = 0; st < stripes; ++st) {
    for (int j = 0; j < nsrc; ++j) s.push_back(Span{src_ptrs[size_t(st) * nsrc + j], size, false, st * per + j});
    for (int r = 0; r < rows; ++r)
      s.push_back(Span{dst_ptrs[size_t(st) * rows + r], size, true, st * per + nsrc + r});
  }
  constexpr int kOneLaunchRows = 4;  // gf_kernels.hpp kMaxRows
  const auto c = find_conflict(s, [&](const Span& a, const Span& b) {
    return a.written != b.written && a.tag / per == b.tag / per && rows <= kOneLaunchRows;
  });
  if (c.first < 0) return ECGPU_OK;
  return rt::fail(ECGPU_ERR_ARG, conflict_message("ecgpu_plan_bind", s, c, [&](int t) {
                    const int st = t / per, i = t % per;
                    return (i < nsrc ? "source " + std::to_string(i) : "destination " + std::to_string(i - nsrc)) +
                           " of stripe " + std::to_string(st);
                  }));
}

}  // extern "C"
