#include "block_manager.h"

#include <algorithm>
#include <cstring>
#include <stdexcept>

namespace ftrt {

BlockManager::BlockManager(int num_blocks, int block_size, bool enable_prefix_caching)
    : num_blocks_(num_blocks),
      block_size_(block_size),
      prefix_caching_(enable_prefix_caching),
      refcnt_(num_blocks, 0),
      block_hash_(num_blocks, 0),
      block_tokens_(enable_prefix_caching ? (size_t)num_blocks * block_size : 0, 0),
      prev_(num_blocks, -1),
      next_(num_blocks, -1),
      in_lru_(num_blocks, 0) {
  if (num_blocks <= 0 || block_size <= 0) throw std::invalid_argument("bad block pool size");
  free_.reserve(num_blocks);
  for (int b = num_blocks - 1; b >= 0; --b) free_.push_back(b);
}

uint64_t BlockManager::chain_hash(uint64_t parent, const int32_t* toks) const {
  // 64-bit multiply-xorshift mixing (splitmix-style) over the parent and tokens
  uint64_t h = parent ^ 0x9E3779B97F4A7C15ull;
  for (int i = 0; i < block_size_; ++i) {
    h ^= (uint64_t)(uint32_t)toks[i] + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2);
    h *= 0xBF58476D1CE4E5B9ull;
    h ^= h >> 31;
  }
  return h ? h : 1;  // 0 is reserved for "no hash"
}

void BlockManager::lru_push_back(int b) {
  prev_[b] = lru_tail_;
  next_[b] = -1;
  if (lru_tail_ >= 0) next_[lru_tail_] = b;
  lru_tail_ = b;
  if (lru_head_ < 0) lru_head_ = b;
  in_lru_[b] = 1;
  ++lru_size_;
}

void BlockManager::lru_remove(int b) {
  if (!in_lru_[b]) return;
  if (prev_[b] >= 0) next_[prev_[b]] = next_[b]; else lru_head_ = next_[b];
  if (next_[b] >= 0) prev_[next_[b]] = prev_[b]; else lru_tail_ = prev_[b];
  prev_[b] = next_[b] = -1;
  in_lru_[b] = 0;
  --lru_size_;
}

int BlockManager::lru_pop_front() {
  const int b = lru_head_;
  if (b >= 0) lru_remove(b);
  return b;
}

void BlockManager::drop_hash(int b) {
  const uint64_t h = block_hash_[b];
  if (!h) return;
  auto it = hash_to_block_.find(h);
  if (it != hash_to_block_.end() && it->second == b) hash_to_block_.erase(it);
  block_hash_[b] = 0;
}

std::vector<int> BlockManager::match_prefix(const int32_t* tokens, int64_t n_tokens,
                                            int max_blocks) {
  std::vector<int> out;
  if (!prefix_caching_) return out;
  const int64_t nfull = n_tokens / block_size_;
  uint64_t h = 0;
  for (int64_t i = 0; i < nfull && (int)out.size() < max_blocks; ++i) {
    const int32_t* t = tokens + i * block_size_;
    h = chain_hash(h, t);
    ++query_blocks_;
    auto it = hash_to_block_.find(h);
    if (it == hash_to_block_.end()) break;
    const int b = it->second;
    if (std::memcmp(&block_tokens_[(size_t)b * block_size_], t, sizeof(int32_t) * block_size_) != 0)
      break;
    if (refcnt_[b] == 0) lru_remove(b);
    ++refcnt_[b];
    ++hit_blocks_;
    out.push_back(b);
  }
  return out;
}

std::vector<int> BlockManager::allocate(int n) {
  std::vector<int> out;
  if (n <= 0) return out;
  if (!can_allocate(n)) return out;
  out.reserve(n);
  for (int i = 0; i < n; ++i) {
    int b;
    if (!free_.empty()) {
      b = free_.back();
      free_.pop_back();
    } else {
      b = lru_pop_front();
      drop_hash(b);
    }
    refcnt_[b] = 1;
    out.push_back(b);
  }
  return out;
}

void BlockManager::incref(const std::vector<int>& blocks) {
  for (int b : blocks) {
    if (refcnt_[b] == 0) lru_remove(b);
    ++refcnt_[b];
  }
}

void BlockManager::free(const std::vector<int>& blocks) {
  // release in reverse so the tail of a sequence is evicted before its head
  for (auto it = blocks.rbegin(); it != blocks.rend(); ++it) {
    const int b = *it;
    if (b < 0 || b >= num_blocks_) throw std::out_of_range("block id");
    if (refcnt_[b] <= 0) throw std::logic_error("double free of KV block");
    if (--refcnt_[b] == 0) {
      if (prefix_caching_ && block_hash_[b]) lru_push_back(b);
      else free_.push_back(b);
    }
  }
}

void BlockManager::commit(const int* blocks, int n_blocks, const int32_t* tokens,
                          int64_t n_tokens, int first_block) {
  if (!prefix_caching_) return;
  const int64_t nfull = std::min<int64_t>(n_tokens / block_size_, n_blocks);
  uint64_t h = 0;
  for (int64_t i = 0; i < nfull; ++i) {
    const int32_t* t = tokens + i * block_size_;
    h = chain_hash(h, t);
    if (i < first_block) continue;
    const int b = blocks[i];
    if (block_hash_[b] == h) continue;
    if (block_hash_[b]) drop_hash(b);
    if (hash_to_block_.count(h)) continue;  // identical content already cached elsewhere
    hash_to_block_[h] = b;
    block_hash_[b] = h;
    std::memcpy(&block_tokens_[(size_t)b * block_size_], t, sizeof(int32_t) * block_size_);
  }
}

void BlockManager::reset_prefix_cache() {
  while (lru_head_ >= 0) {
    const int b = lru_pop_front();
    drop_hash(b);
    free_.push_back(b);
  }
  for (int b = 0; b < num_blocks_; ++b) drop_hash(b);
  hash_to_block_.clear();
}

}  // namespace ftrt
