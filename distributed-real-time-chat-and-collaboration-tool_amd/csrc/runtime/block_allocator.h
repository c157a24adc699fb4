// Paged-KV block allocator (host side of the engine's memory manager).
//
// LIFO free list (recently freed blocks are reused first: their lines may
// still sit in the 256 MiB Infinity Cache) + per-block reference counts so a
// block can be shared by several sequences (prefix sharing / forked
// sampling).  Not thread-safe by design: the engine's scheduler thread is
// its only caller.
#pragma once
#include <cstdint>
#include <stdexcept>
#include <vector>

namespace drtc {

class BlockAllocator {
 public:
  BlockAllocator(int32_t num_blocks, int32_t reserved)
      : num_blocks_(num_blocks), reserved_(reserved), refcnt_(num_blocks, 0) {
    if (num_blocks <= reserved || reserved < 0)
      throw std::invalid_argument("BlockAllocator: num_blocks must exceed reserved");
    free_.reserve(num_blocks);
    for (int32_t b = num_blocks - 1; b >= reserved; --b) free_.push_back(b);
  }

  int32_t num_blocks() const { return num_blocks_; }
  int32_t num_free() const { return (int32_t)free_.size(); }
  int32_t num_used() const { return num_blocks_ - reserved_ - num_free(); }
  bool can_allocate(int32_t n) const { return n <= (int32_t)free_.size(); }

  std::vector<int32_t> allocate(int32_t n) {
    if (n < 0 || n > (int32_t)free_.size())
      throw std::runtime_error("BlockAllocator: out of KV-cache blocks");
    std::vector<int32_t> out(n);
    for (int32_t i = 0; i < n; ++i) {
      out[i] = free_.back();
      free_.pop_back();
      refcnt_[out[i]] = 1;
    }
    return out;
  }

  int32_t allocate_one() {
    if (free_.empty()) throw std::runtime_error("BlockAllocator: out of KV-cache blocks");
    int32_t b = free_.back();
    free_.pop_back();
    refcnt_[b] = 1;
    return b;
  }

  void incref(const std::vector<int32_t>& blocks) {
    for (int32_t b : blocks) {
      check(b);
      if (refcnt_[b] <= 0) throw std::runtime_error("BlockAllocator: incref of a free block");
      ++refcnt_[b];
    }
  }

  // Decrement; blocks reaching zero return to the free list.
  void free(const std::vector<int32_t>& blocks) {
    for (int32_t b : blocks) {
      check(b);
      if (refcnt_[b] <= 0) throw std::runtime_error("BlockAllocator: double free");
      if (--refcnt_[b] == 0) free_.push_back(b);
    }
  }

  int32_t refcount(int32_t b) const {
    check(b);
    return refcnt_[b];
  }

 private:
  void check(int32_t b) const {
    if (b < reserved_ || b >= num_blocks_)
      throw std::out_of_range("BlockAllocator: block id out of range");
  }
  int32_t num_blocks_, reserved_;
  std::vector<int32_t> refcnt_;
  std::vector<int32_t> free_;
};

}  // namespace drtc
