// packets.hip -- GF(2) bit-matrix / schedule coding on the GPU
// (gf_xor_packets* kernels, gf_kernels.hpp).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "buffer_contract.hpp"
#include "cpu_fallback.hpp"
#include "ecgpu.h"
#include "gf_host.hpp"
#include "matrix_host.hpp"
#include "planner.hpp"
#include "schedule_host.hpp"
#include "runtime.hpp"

using namespace ecgpu;
using namespace ecgpu::rt;

using dev::u32x4;

// ------------------------------------------- GF(2) packet coding ----
// Bit-matrix / schedule coding (jerasure.cpp:301-345, :623-703, :1153-1192,
// :1346-1363).  The reference's memcpy / XOR sequence over packet rows is
// replayed by the LinearTracker on virtual buffers "packet row r of device
// slot s" (one super-packet), and the fused map runs once over every
// super-packet (gf_xor_packets).
namespace {

inline int pslot(const void* k) { return PacketTracker::key_slot(k); }
inline int prow(const void* k) { return PacketTracker::key_row(k); }
constexpr int kMaxPacketRow = (1 << 20) - 1;

constexpr int kPacketRows = 32;  // output packet rows per launch (uint32 masks)

// The map of a w = 8 Vandermonde bit-matrix encode, exactly (the unit form
// gf_xor_packets16u relies on it): 32 output rows, sources device-major in
// whole devices of 8 bits, bit b of every device feeding output row b (the
// identity blocks of coding device 0) and device 0's bit b feeding row b of
// every coding device.
bool unit_packet_map(const uint32_t* m, int nsrc) {
  if (nsrc < 8 || nsrc % 8 != 0) return false;
  for (int j = 0; j < nsrc; ++j) {
    const uint32_t bit = 1u << (j % 8);
    if ((m[j] & 0xFFu) != bit) return false;
    if (j < 8 && m[j] != bit * 0x01010101u) return false;
  }
  return true;
}

int execute_packets_gpu(const FusedOp& op, const std::vector<char*>& ptrs, int64_t nsp, int64_t spstride, int64_t ps,
                        int device, const std::vector<int>& slots, const std::vector<int64_t>& extent,
                        const std::vector<char>& is_out);

// Slot s's packet row r of super-packet sp is ptrs[s] + sp * spstride + r * ps.
int execute_packets(const FusedOp& op, const std::vector<char*>& ptrs, int64_t nsp, int64_t spstride, int64_t ps,
                    const char* call) {
  if (op.dsts.empty() || nsp <= 0 || ps <= 0) {
    add_stats(op);
    return ECGPU_OK;
  }
  // Slots touched and their byte extents.
  std::vector<int> slots;
  std::vector<int64_t> maxrow(ptrs.size(), -1);
  std::vector<char> is_out(ptrs.size(), 0);
  auto touch = [&](const void* key, bool out) -> int {
    const int sl = pslot(key), r = prow(key);
    if (sl < 0 || size_t(sl) >= ptrs.size() || !ptrs[size_t(sl)])
      return fail(ECGPU_ERR_ARG, "packet op references a missing device pointer");
    if (maxrow[size_t(sl)] < 0) slots.push_back(sl);
    maxrow[size_t(sl)] = std::max<int64_t>(maxrow[size_t(sl)], r);
    if (out) is_out[size_t(sl)] = 1;
    return ECGPU_OK;
  };
  for (void* k : op.srcs)
    if (int rc = touch(k, false)) return rc;
  for (void* k : op.dsts)
    if (int rc = touch(k, true)) return rc;
  std::vector<int64_t> extent(ptrs.size(), 0);
  for (int sl : slots) extent[size_t(sl)] = (nsp - 1) * spstride + (maxrow[size_t(sl)] + 1) * ps;
  // identical or disjoint device buffers, checked before anything touches the GPU
  if (int rc = check_slot_buffers(call, ptrs, slots, extent, is_out)) return rc;
  add_stats(op);
  std::vector<void*> slot_ptrs;
  for (int sl : slots) slot_ptrs.push_back(ptrs[size_t(sl)]);
  // small host-memory calls (and all of them with ECGPU_GPU=0) on the CPU
  // executor, as for the w = 8 calls (execute)
  int64_t moved = 0;
  for (int sl : slots) moved += extent[size_t(sl)];
  if (cpu_by_choice(moved) && all_host(slot_ptrs)) {
    record_cpu_call();
    cpu_apply_packets(op, ptrs, nsp, spstride, ps);
    return ECGPU_OK;
  }
  const int device = call_device(slot_ptrs, {});
  // SURVEY §8b's failure contract, as for the w = 8 calls (cpu_fallback.hpp):
  // host-memory calls complete on the CPU after a HIP error that came before
  // a source was overwritten, or at once on a device marked lost
  trace_begin();
  CallDeviceScope scope(device);
  const bool fallback = fallback_enabled();
  if (fallback && device_lost(device) && all_host(slot_ptrs)) {
    record_fallback(call, "device " + std::to_string(device) + " marked lost by an earlier HIP error");
    cpu_apply_packets(op, ptrs, nsp, spstride, ps);
    return ECGPU_OK;
  }
  const int rc = execute_packets_gpu(op, ptrs, nsp, spstride, ps, device, slots, extent, is_out);
  if (rc != ECGPU_ERR_HIP || !fallback || caller_written() || !all_host(slot_ptrs)) return rc;
  record_fallback(call, "HIP error: " + t_err);
  cpu_apply_packets(op, ptrs, nsp, spstride, ps);
  t_err = std::string(call) + ": completed on the CPU after a HIP error: " + t_err;
  return ECGPU_OK;
}

int packets_on_ctx(Ctx* c, const FusedOp& op, const std::vector<char*>& ptrs, int64_t nsp, int64_t spstride,
                   int64_t ps, int device, const std::vector<int>& slots, const std::vector<int64_t>& extent,
                   const std::vector<char>& is_out);

// The GPU part of execute_packets: staging, one launch per 32 output rows,
// the copies back.  A failure returns with nothing of the call in flight.
int execute_packets_gpu(const FusedOp& op, const std::vector<char*>& ptrs, int64_t nsp, int64_t spstride, int64_t ps,
                        int device, const std::vector<int>& slots, const std::vector<int64_t>& extent,
                        const std::vector<char>& is_out) {
  CtxLease lease(device);
  if (!lease.c) return lease.rc;
  DeviceGuard g(device);
  const int rc = packets_on_ctx(lease.c, op, ptrs, nsp, spstride, ps, device, slots, extent, is_out);
  if (rc != ECGPU_OK) {
    (void)hipStreamSynchronize(lease.c->stream);
    (void)hipGetLastError();
  }
  return rc;
}

int packets_on_ctx(Ctx* c, const FusedOp& op, const std::vector<char*>& ptrs, int64_t nsp, int64_t spstride,
                   int64_t ps, int device, const std::vector<int>& slots, const std::vector<int64_t>& extent,
                   const std::vector<char>& is_out) {
  const int rows = int(op.dsts.size()), nsrc = int(op.srcs.size());
  const bool via_temp = op.dst_is_src && rows > kPacketRows;
  const int ngroups = (rows + kPacketRows - 1) / kPacketRows;

  // Staging slab: staged slots, temporaries, then the pointer / mask tables.
  std::vector<uint8_t*> base(ptrs.size(), nullptr);
  std::vector<char> staged(ptrs.size(), 0);
  size_t off = 0;
  for (int sl : slots) {
    bool on_dev = false;
    if (int rc = classify(ptrs[size_t(sl)], device, &on_dev)) return rc;
    if (on_dev) {
      base[size_t(sl)] = reinterpret_cast<uint8_t*>(ptrs[size_t(sl)]);
    } else {
      staged[size_t(sl)] = 1;
      base[size_t(sl)] = reinterpret_cast<uint8_t*>(off);  // offset, rebased below
      off += (size_t(extent[size_t(sl)]) + 255) & ~size_t(255);
    }
  }
  if (int rc = injected_failure(device, 0)) return rc;
  const size_t temp_off = off;
  if (via_temp) off += size_t(rows) * size_t(nsp * ps + 255 & ~int64_t(255));
  const size_t tab_off = off;
  const size_t tab_bytes = sizeof(void*) * size_t(nsrc + rows) + sizeof(uint32_t) * size_t(nsrc) * ngroups;
  off += tab_bytes;
  if (int rc = ensure_stage(c, off)) return rc;
  for (int sl : slots)
    if (staged[size_t(sl)]) {
      base[size_t(sl)] = c->stage + reinterpret_cast<size_t>(base[size_t(sl)]);
      // outputs too: packets the op does not write must come back unchanged
      ECGPU_HIP(hipMemcpyAsync(base[size_t(sl)], ptrs[size_t(sl)], size_t(extent[size_t(sl)]),
                               hipMemcpyHostToDevice, c->stream));
    }

  std::vector<const uint8_t*> sb(static_cast<size_t>(nsrc));
  std::vector<uint8_t*> db(static_cast<size_t>(rows));
  const int64_t temp_stride = (nsp * ps + 255) & ~int64_t(255);
  // sources in (slot, packet row) order -- device-major, bit-minor for a
  // bit-matrix call, whatever order the tracker met them in -- so the map of
  // a Vandermonde encode has the layout the unit kernel checks for (the
  // XOR of the sources does not depend on their order)
  std::vector<int> sorder(static_cast<size_t>(nsrc));
  for (int j = 0; j < nsrc; ++j) sorder[size_t(j)] = j;
  std::stable_sort(sorder.begin(), sorder.end(), [&](int x, int y) {
    const void* kx = op.srcs[size_t(x)];
    const void* ky = op.srcs[size_t(y)];
    return pslot(kx) != pslot(ky) ? pslot(kx) < pslot(ky) : prow(kx) < prow(ky);
  });
  for (int j = 0; j < nsrc; ++j) {
    const void* key = op.srcs[size_t(sorder[size_t(j)])];
    sb[size_t(j)] = base[size_t(pslot(key))] + prow(key) * ps;
  }
  for (int r = 0; r < rows; ++r)
    db[size_t(r)] = via_temp ? c->stage + temp_off + size_t(r) * size_t(temp_stride)
                             : base[size_t(pslot(op.dsts[size_t(r)]))] + prow(op.dsts[size_t(r)]) * ps;
  std::vector<uint32_t> masks(size_t(nsrc) * ngroups, 0u);
  for (int r = 0; r < rows; ++r)
    for (int j = 0; j < nsrc; ++j)
      if (op.coef[size_t(r) * nsrc + sorder[size_t(j)]])
        masks[size_t(r / kPacketRows) * nsrc + j] |= 1u << (r % kPacketRows);
  // one upload of [src bases | dst bases | masks]
  std::vector<uint8_t> host_tab(tab_bytes);
  std::memcpy(host_tab.data(), sb.data(), sizeof(void*) * nsrc);
  std::memcpy(host_tab.data() + sizeof(void*) * nsrc, db.data(), sizeof(void*) * rows);
  std::memcpy(host_tab.data() + sizeof(void*) * size_t(nsrc + rows), masks.data(), masks.size() * sizeof(uint32_t));
  uint8_t* tab = c->stage + tab_off;
  auto* d_src = reinterpret_cast<const uint8_t**>(tab);
  auto* d_dst = reinterpret_cast<uint8_t**>(tab + sizeof(void*) * nsrc);
  auto* d_mask = reinterpret_cast<uint32_t*>(tab + sizeof(void*) * size_t(nsrc + rows));
  ECGPU_HIP(hipMemcpyAsync(tab, host_tab.data(), tab_bytes, hipMemcpyHostToDevice, c->stream));

  const int64_t dstride = via_temp ? ps : spstride;
  bool aligned = ps % 8 == 0 && spstride % 8 == 0 && dstride % 8 == 0;
  for (auto* p : sb) aligned &= (reinterpret_cast<uintptr_t>(p) & 7u) == 0;
  for (auto* p : db) aligned &= (reinterpret_cast<uintptr_t>(p) & 7u) == 0;
  // 16-B lanes when everything is 16-B aligned, in the unit form when the map
  // is a Vandermonde encode's; ECGPU_PACKET=1 forces 8-B lanes, 2 the
  // unpipelined 16-B kernel, 3 the general pipelined 16-B kernel (A/B, RS(10,4) w = 8 64 MiB
  // bit-matrix encode on MI355X: pipelined 16-B lanes 180.5 us, unpipelined
  // with 8 rows in flight 187, 8-B lanes 190; profiles/r02_packet_ab.txt)
  const int packet_kind = knob(Knob::kPacket);
  bool wide16 = aligned && packet_kind != 1 && ps % 16 == 0 && spstride % 16 == 0 && dstride % 16 == 0;
  for (auto* p : sb) wide16 &= (reinterpret_cast<uintptr_t>(p) & 15u) == 0;
  for (auto* p : db) wide16 &= (reinterpret_cast<uintptr_t>(p) & 15u) == 0;
  for (int g0 = 0; g0 < ngroups; ++g0) {
    const int R = std::min(kPacketRows, rows - g0 * kPacketRows);
    dev::PacketArgs a{};
    a.src = d_src;
    a.dst = d_dst + size_t(g0) * kPacketRows;
    a.mask = d_mask + size_t(g0) * nsrc;
    a.sstride = spstride;
    a.dstride = dstride;
    a.nsrc = nsrc;
    a.R = R;
    a.cpp = wide16 ? ps / 16 : aligned ? ps / 8 : ps;
    a.ncols = nsp * a.cpp;
    if (nsrc == 0) {  // every output packet is zero
      for (int r = 0; r < R; ++r)
        ECGPU_HIP(hipMemset2DAsync(db[size_t(g0 * kPacketRows + r)], size_t(nsp > 1 ? dstride : ps), 0, size_t(ps),
                                   size_t(nsp), c->stream));
      continue;
    }
    void* fn = nullptr;
    if (wide16 && packet_kind == 0 && R == kPacketRows &&
        unit_packet_map(masks.data() + size_t(g0) * nsrc, nsrc))
      fn = reinterpret_cast<void*>(&dev::gf_xor_packets16u<32>);
    else if (wide16 && packet_kind == 2)
      fn = R <= 8    ? reinterpret_cast<void*>(&dev::gf_xor_packets16<8, 8>)
           : R <= 16 ? reinterpret_cast<void*>(&dev::gf_xor_packets16<16, 8>)
                     : reinterpret_cast<void*>(&dev::gf_xor_packets16<32, 8>);
    else if (wide16)
      fn = R <= 8    ? reinterpret_cast<void*>(&dev::gf_xor_packets16p<8>)
           : R <= 16 ? reinterpret_cast<void*>(&dev::gf_xor_packets16p<16>)
                     : reinterpret_cast<void*>(&dev::gf_xor_packets16p<32>);
    else
      fn = aligned ? (R <= 8    ? reinterpret_cast<void*>(&dev::gf_xor_packets<8>)
                      : R <= 16 ? reinterpret_cast<void*>(&dev::gf_xor_packets<16>)
                                : reinterpret_cast<void*>(&dev::gf_xor_packets<32>))
                   : reinterpret_cast<void*>(&dev::gf_xor_packets_bytes);
    void* args[] = {&a};
    const dim3 grid(unsigned((a.ncols + dev::kBlock - 1) / dev::kBlock));
    ECGPU_HIP(hipLaunchKernel(fn, grid, dim3(dev::kBlock), args, 0, c->stream));
  }
  if (via_temp)
    for (int r = 0; r < rows; ++r) {
      uint8_t* real = base[size_t(pslot(op.dsts[size_t(r)]))] + prow(op.dsts[size_t(r)]) * ps;
      ECGPU_HIP(hipMemcpy2DAsync(real, size_t(nsp > 1 ? spstride : ps), db[size_t(r)], size_t(ps), size_t(ps),
                                 size_t(nsp), hipMemcpyDeviceToDevice, c->stream));
    }
  // the launches above wrote device slots in place; the copies below write
  // host ones (a slot's packets that are not outputs come back unchanged):
  // only an output that is also a source loses bytes the CPU would need
  if (op.dst_is_src) note_caller_write();
  if (int rc = injected_failure(device, 1)) return rc;
  for (int sl : slots)
    if (staged[size_t(sl)] && is_out[size_t(sl)])
      ECGPU_HIP(hipMemcpyAsync(ptrs[size_t(sl)], base[size_t(sl)], size_t(extent[size_t(sl)]), hipMemcpyDeviceToHost,
                               c->stream));
  ECGPU_HIP(hipStreamSynchronize(c->stream));
  ECGPU_HIP(hipGetLastError());
  return ECGPU_OK;
}

// jerasure_bitmatrix_dotprod (jerasure.cpp:301-345) for ONE super-packet on
// virtual packet rows; byte counters scaled by the super-packet count.
void record_bitmatrix_dotprod(PacketTracker& t, int k, int w, const int* row, const int* src_ids, int dest_id,
                              int64_t ps, int64_t nsp) {
  int index = 0;
  for (int j = 0; j < w; ++j) {
    bool started = false;
    for (int x = 0; x < k; ++x) {
      const int dev = src_ids ? src_ids[x] : x;
      for (int y = 0; y < w; ++y, ++index) {
        if (!row[index]) continue;
        if (!started) {
          t.copy(dest_id, j, dev, y);
          t.count(0, 0, double(ps) * double(nsp));
          started = true;
        } else {
          t.xor_into(dest_id, j, dev, y);
          t.count(double(ps) * double(nsp), 0, 0);
        }
      }
    }
  }
}

std::vector<char*> device_ptrs(int k, int n, char** data, char** coding) {
  std::vector<char*> p(static_cast<size_t>(n), nullptr);
  for (int i = 0; i < n; ++i) p[size_t(i)] = i < k ? data[i] : coding[i - k];
  return p;
}

// Devices and packet rows a schedule names (ops[i] = {src dev, src packet,
// dst dev, dst packet, xor?}, terminated by ops[i][0] < 0).
int schedule_extent(int** ops, int* max_dev, int* max_row) {
  *max_dev = -1;
  *max_row = -1;
  for (int i = 0; ops[i][0] >= 0; ++i) {
    const int* o = ops[i];
    if (o[1] < 0 || o[3] < 0 || o[1] > kMaxPacketRow || o[3] > kMaxPacketRow || o[2] < 0)
      return fail(ECGPU_ERR_ARG, "schedule op out of range");
    *max_dev = std::max(*max_dev, std::max(o[0], o[2]));
    *max_row = std::max(*max_row, std::max(o[1], o[3]));
  }
  return ECGPU_OK;
}

// Replays a schedule for one super-packet.
void record_schedule(PacketTracker& t, int** ops, int64_t ps, int64_t nsp) {
  for (int i = 0; ops[i][0] >= 0; ++i) {
    const int* o = ops[i];
    if (o[4]) {
      t.xor_into(o[2], o[3], o[0], o[1]);
      t.count(double(ps) * double(nsp), 0, 0);
    } else {
      t.copy(o[2], o[3], o[0], o[1]);
      t.count(0, 0, double(ps) * double(nsp));
    }
  }
}

}  // namespace

extern "C" {

ECGPU_API int ecgpu_jerasure_bitmatrix_dotprod(int k, int w, int* bitmatrix_row, int* src_ids, int dest_id,
                                               char** data_ptrs, char** coding_ptrs, int size, int packetsize) {
  if (k <= 0 || w <= 0 || packetsize <= 0 || !bitmatrix_row || size % (w * packetsize) != 0)
    return fail(ECGPU_ERR_ARG, "ecgpu_jerasure_bitmatrix_dotprod: size % (w*packetsize) must be 0");
  const int64_t nsp = size / (int64_t(w) * packetsize);
  int n = std::max(k, dest_id + 1);
  if (src_ids)
    for (int x = 0; x < k; ++x) n = std::max(n, src_ids[x] + 1);
  PacketTracker t(n, w);
  record_bitmatrix_dotprod(t, k, w, bitmatrix_row, src_ids, dest_id, packetsize, nsp);
  // ids >= k index coding_ptrs; only the ids the op touches are dereferenced
  std::vector<char*> p(static_cast<size_t>(n), nullptr);
  auto put = [&](int id) { p[size_t(id)] = id < k ? data_ptrs[id] : coding_ptrs[id - k]; };
  put(dest_id);
  for (int x = 0; x < k; ++x) put(src_ids ? src_ids[x] : x);
  return execute_packets(t.finish(), p, nsp, int64_t(w) * packetsize, packetsize, "jerasure_bitmatrix_dotprod");
}

ECGPU_API int ecgpu_jerasure_bitmatrix_encode(int k, int m, int w, int* bitmatrix, char** data_ptrs,
                                              char** coding_ptrs, int size, int packetsize) {
  if (k <= 0 || m <= 0 || w <= 0 || packetsize <= 0 || !bitmatrix || size % (w * packetsize) != 0)
    return fail(ECGPU_ERR_ARG, "ecgpu_jerasure_bitmatrix_encode: size % (packetsize*w) must be 0");
  const int64_t nsp = size / (int64_t(w) * packetsize);
  PacketTracker t(k + m, w);
  for (int i = 0; i < m; ++i)
    record_bitmatrix_dotprod(t, k, w, bitmatrix + size_t(i) * k * w * w, nullptr, k + i, packetsize, nsp);
  return execute_packets(t.finish(), device_ptrs(k, k + m, data_ptrs, coding_ptrs), nsp, int64_t(w) * packetsize,
                         packetsize, "jerasure_bitmatrix_encode");
}

// jerasure.cpp:623-703 as one fused GF(2) map.
ECGPU_API int ecgpu_jerasure_bitmatrix_decode(int k, int m, int w, int* bitmatrix, int row_k_ones, int* erasures,
                                              char** data_ptrs, char** coding_ptrs, int size, int packetsize) {
  if (k <= 0 || m <= 0 || w <= 0 || packetsize <= 0 || !bitmatrix || !erasures || size % (w * packetsize) != 0)
    return fail(ECGPU_ERR_ARG, "ecgpu_jerasure_bitmatrix_decode: bad arguments");
  int* erased = erasures_to_erased(k, m, erasures);
  if (!erased) return ECGPU_ERR;
  const int64_t nsp = size / (int64_t(w) * packetsize);
  int edd = 0, lastdrive = k;
  for (int i = 0; i < k; ++i)
    if (erased[i]) {
      ++edd;
      lastdrive = i;
    }
  if (row_k_ones != 1 || erased[k]) lastdrive = k;
  const size_t blk = size_t(k) * w * w;
  std::vector<int> dm, ids;
  if (edd > 1 || (edd > 0 && (row_k_ones != 1 || erased[k]))) {
    dm.resize(blk * k);
    ids.resize(size_t(k));
    if (make_decoding_bitmatrix(k, m, w, bitmatrix, erased, dm.data(), ids.data()) < 0) {
      std::free(erased);
      return ECGPU_ERR;
    }
  }
  PacketTracker t(k + m, w);
  for (int i = 0; edd > 0 && i < lastdrive; ++i)
    if (erased[i]) {
      record_bitmatrix_dotprod(t, k, w, dm.data() + i * blk, ids.data(), i, packetsize, nsp);
      --edd;
    }
  if (edd > 0) {
    std::vector<int> tmp(static_cast<size_t>(k));
    for (int i = 0; i < k; ++i) tmp[size_t(i)] = i < lastdrive ? i : i + 1;
    record_bitmatrix_dotprod(t, k, w, bitmatrix, tmp.data(), lastdrive, packetsize, nsp);
  }
  for (int i = 0; i < m; ++i)
    if (erased[k + i]) record_bitmatrix_dotprod(t, k, w, bitmatrix + i * blk, nullptr, k + i, packetsize, nsp);
  std::free(erased);
  return execute_packets(t.finish(), device_ptrs(k, k + m, data_ptrs, coding_ptrs), nsp, int64_t(w) * packetsize,
                         packetsize, "jerasure_bitmatrix_decode");
}

// jerasure.cpp:1153-1176: one super-packet at ptrs.
ECGPU_API int ecgpu_jerasure_do_scheduled_operations(char** ptrs, int** operations, int packetsize) {
  if (!ptrs || !operations || packetsize <= 0)
    return fail(ECGPU_ERR_ARG, "ecgpu_jerasure_do_scheduled_operations: bad arguments");
  int max_dev = -1, max_row = -1;
  if (int rc = schedule_extent(operations, &max_dev, &max_row)) return rc;
  if (max_dev < 0) return ECGPU_OK;
  PacketTracker t(max_dev + 1, max_row + 1);
  record_schedule(t, operations, packetsize, 1);
  std::vector<char*> p(ptrs, ptrs + (max_dev + 1));
  return execute_packets(t.finish(), p, 1, 0, packetsize, "jerasure_do_scheduled_operations");
}

// jerasure.cpp:1178-1192 over nptrs device pointers (NULL where unused), and
// the decode-time schedules of jerasure.cpp:935-995.
ECGPU_API int ecgpu_schedule_run(int nptrs, char** ptrs, int** operations, int w, int size, int packetsize) {
  if (nptrs <= 0 || !ptrs || !operations || w <= 0 || packetsize <= 0 || size % (w * packetsize) != 0)
    return fail(ECGPU_ERR_ARG, "ecgpu_schedule_run: size % (w*packetsize) must be 0");
  const int64_t nsp = size / (int64_t(w) * packetsize);
  int max_dev = -1, max_row = -1;
  if (int rc = schedule_extent(operations, &max_dev, &max_row)) return rc;
  if (max_dev >= nptrs) return fail(ECGPU_ERR_ARG, "ecgpu_schedule_run: schedule names a device >= nptrs");
  if (max_dev < 0) return ECGPU_OK;
  PacketTracker t(max_dev + 1, max_row + 1);
  record_schedule(t, operations, packetsize, nsp);
  std::vector<char*> p(ptrs, ptrs + nptrs);
  return execute_packets(t.finish(), p, nsp, int64_t(w) * packetsize, packetsize, "jerasure_schedule");
}

ECGPU_API int ecgpu_jerasure_schedule_encode(int k, int m, int w, int** schedule, char** data_ptrs, char** coding_ptrs,
                                             int size, int packetsize) {
  if (k <= 0 || m <= 0) return fail(ECGPU_ERR_ARG, "ecgpu_jerasure_schedule_encode: bad arguments");
  std::vector<char*> p = device_ptrs(k, k + m, data_ptrs, coding_ptrs);
  return ecgpu_schedule_run(k + m, p.data(), schedule, w, size, packetsize);
}

}  // extern "C"
