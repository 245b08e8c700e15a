// Paged KV-cache block manager with automatic prefix caching (E6/E7 in
// SURVEY.md §2.3; replaces vLLM's --gpu-memory-utilization / --swap-space
// block pool that the reference configures in docker-compose.vllm.yml:44,49).
//
// * Blocks are fixed-size token pages of the per-layer KV tensors.
// * A *full* block is identified by a chained 64-bit hash of (parent hash,
//   its block_size token ids) and its token ids are stored for verification,
//   so a hash collision can never alias two different prefixes.
// * Freed blocks that carry a hash are not wiped: they park in an LRU list and
//   are handed back (refcount++) when a later request starts with the same
//   prefix -- that is what turns turn N+1 of a conversation into a prefill of
//   only the new message (multi-turn KV reuse, Appendix D Q18).
// * Allocation takes never-hashed blocks first, then evicts the least recently
//   used cached block.
#pragma once

#include <cstdint>
#include <unordered_map>
#include <vector>

namespace ftrt {

class BlockManager {
 public:
  BlockManager(int num_blocks, int block_size, bool enable_prefix_caching);

  int num_blocks() const { return num_blocks_; }
  int block_size() const { return block_size_; }
  int num_free() const { return (int)free_.size() + lru_size_; }
  int num_free_uncached() const { return (int)free_.size(); }
  int num_cached() const { return (int)hash_to_block_.size(); }
  bool can_allocate(int n) const { return n <= num_free(); }

  // Longest cached prefix of `tokens` made of full blocks, at most max_blocks
  // blocks.  The returned blocks are referenced (refcount++).
  std::vector<int> match_prefix(const int32_t* tokens, int64_t n_tokens, int max_blocks);

  // n fresh blocks (refcount 1).  Returns empty vector if not enough blocks.
  std::vector<int> allocate(int n);

  void incref(const std::vector<int>& blocks);
  void free(const std::vector<int>& blocks);

  // Register the hashes of the full blocks [first_block, n_tokens / block_size)
  // of a sequence whose block table is `blocks` and token ids are `tokens`.
  void commit(const int* blocks, int n_blocks, const int32_t* tokens, int64_t n_tokens,
              int first_block);

  void reset_prefix_cache();

  // stats
  int64_t hits() const { return hit_blocks_; }
  int64_t queries() const { return query_blocks_; }
  int refcount(int b) const { return refcnt_[b]; }

 private:
  uint64_t chain_hash(uint64_t parent, const int32_t* toks) const;
  void lru_push_back(int b);
  void lru_remove(int b);
  int lru_pop_front();
  void drop_hash(int b);

  int num_blocks_, block_size_;
  bool prefix_caching_;
  std::vector<int> refcnt_;
  std::vector<uint64_t> block_hash_;   // 0 = none
  std::vector<int32_t> block_tokens_;  // num_blocks * block_size, valid when hashed
  std::vector<int> free_;              // stack of un-hashed free blocks
  std::vector<int> prev_, next_;       // LRU links (-1 = none)
  std::vector<uint8_t> in_lru_;
  int lru_head_ = -1, lru_tail_ = -1, lru_size_ = 0;
  std::unordered_map<uint64_t, int> hash_to_block_;
  int64_t hit_blocks_ = 0, query_blocks_ = 0;
};

}  // namespace ftrt
