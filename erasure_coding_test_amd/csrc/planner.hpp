// planner.hpp -- symbolic replay of the reference's region-op sequences.
//
// The reference computes encode/decode as a SEQUENCE of whole-region ops
// (memcpy, XOR, multiply-add) over caller buffers (jerasure.cpp:561-620,
// :153-254).  Every op is GF(2^w)-linear (w = 8, 16 or 32; the word size only
// changes the field the coefficients live in), so the final content of each
// written buffer is a fixed linear combination of the ORIGINAL contents of
// the buffers involved.  The tracker replays the sequence on coefficient
// vectors (one per buffer, indexed by buffer identity = pointer) and emits a
// single fused op: outputs x sources coefficient matrix.  One GPU launch then
// reads every source once and writes every output once -- bit-identical to the
// sequential reference, including aliasing (a destination that is also a
// source) and the "all-zero row leaves the destination untouched" rule.
#pragma once
#include <cstddef>
#include <cstdint>
#include <unordered_map>
#include <vector>

namespace ecgpu {

struct FusedOp {
  std::vector<void*> srcs;     // buffers whose ORIGINAL contents are read
  std::vector<void*> dsts;     // buffers written (final contents)
  std::vector<uint32_t> coef;  // dsts.size() x srcs.size(), row-major, GF(2^w) elements
  int w = 8;                   // field / word size of the coefficients
  // Reference byte counters (jerasure.cpp:42-44): xor, gf-multiply, memcpy.
  double xor_bytes = 0, gf_bytes = 0, memcpy_bytes = 0;
  bool dst_is_src = false;     // some output buffer is also read
  // Every buffer the replayed sequence named (first-use order) and whether the
  // sequence wrote it -- what the buffer contract is checked on
  // (buffer_contract.hpp), including buffers whose terms cancel out of the map.
  std::vector<void*> touched;
  std::vector<char> touched_written;
};

class LinearTracker {
 public:
  explicit LinearTracker(int w = 8) : w_(w) {}
  int w() const { return w_; }

  // Registers (or finds) a buffer; identity is the pointer value.
  int id(void* p);

  // Whole-region primitives over GF(2^w).
  void copy(void* dst, void* src);                 // dst = src
  void xor3(void* r1, void* r2, void* r3);         // r3 = r1 ^ r2
  void mul(void* src, int c, void* dst, bool add);  // dst (^)= c * src

  // jerasure_matrix_dotprod semantics (jerasure.cpp:561-620), any w, with
  // its stats accounting.  size only feeds the byte counters.
  void dotprod(int k, const int* row, const int* src_ids, int dest_id, char** data, char** coding, int64_t size);

  // Adds to the byte counters like jerasure_do_parity etc. do.
  void count(double xor_b, double gf_b, double memcpy_b) {
    xor_ += xor_b;
    gf_ += gf_b;
    memcpy_ += memcpy_b;
  }

  FusedOp finish() const;

 private:
  using Vec = std::vector<uint32_t>;
  int w_ = 8;
  Vec& state(int b);
  std::vector<void*> bufs_;
  static constexpr std::size_t kScanIds = 32;  // id(): linear scan up to this many buffers, then the map
  std::unordered_map<void*, int> idx_;     // filled only past kScanIds
  std::vector<Vec> state_;
  std::vector<char> written_;
  double xor_ = 0, gf_ = 0, memcpy_ = 0;
};

// GF(2) specialisation for packet coding (bit-matrices and schedules,
// jerasure.cpp:301-345, :1153-1192): buffers are the dense "packet row r of
// device slot s" (s < nslots, r < nrows), every coefficient is 0/1, so a
// state is a bitset and an op is a few word XORs -- schedules replay
// thousands of ops per call.  finish() returns the same FusedOp shape with
// srcs / dsts holding packet keys (see packet_key) and 0/1 coefficients.
class PacketTracker {
 public:
  PacketTracker(int nslots, int nrows);
  void copy(int dslot, int drow, int sslot, int srow);  // dst = src
  void xor_into(int dslot, int drow, int sslot, int srow);  // dst ^= src
  void count(double xor_b, double gf_b, double memcpy_b) {
    xor_ += xor_b;
    gf_ += gf_b;
    memcpy_ += memcpy_b;
  }
  FusedOp finish() const;
  static void* packet_key(int slot, int row);
  static int key_slot(const void* key);
  static int key_row(const void* key);

 private:
  int idx(int slot, int row) const { return slot * nrows_ + row; }
  int nslots_, nrows_, n_, words_;
  std::vector<uint64_t> bits_;  // n_ states of words_ words each
  std::vector<char> written_;
  double xor_ = 0, gf_ = 0, memcpy_ = 0;
};

// jerasure_matrix_encode (jerasure.cpp:285-299) as a fused op, w = t.w().
void plan_encode(LinearTracker& t, int k, int m, const int* matrix, char** data, char** coding, int64_t size);

// jerasure_matrix_decode (jerasure.cpp:153-254) as a fused op, w = t.w().
// Returns 0, or -1 where the reference returns -1 (too many erasures,
// singular survivor matrix); nothing is recorded in that case.
int plan_decode(LinearTracker& t, int k, int m, const int* matrix, int row_k_ones, const int* erasures, char** data,
                char** coding, int64_t size);

}  // namespace ecgpu
