// Paged-KV block manager with automatic prefix caching.
//
// The KV cache is one pool of fixed-size blocks (block_size tokens each) in
// HBM; every sequence owns a block table.  A full block whose tokens are all
// prompt tokens is content-addressed by a chained 64-bit hash of
// (parent hash, its tokens) and stays cached after the sequence is freed,
// so the next round's prompt of the same agent -- whose system prompt and
// chat header are byte-identical -- reuses those blocks and
// skips their prefill.  Cached blocks with refcount 0 are evicted LRU-first
// only when the free list is empty.
//
// Tokens of every cached block are stored and compared on lookup, so a hash
// collision can never alias two prompts.

#include <algorithm>
#include <cstring>
#include <stdexcept>

#include "runtime.h"

namespace bcg {

static inline uint64_t mix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return x;
}

uint64_t BlockManager::hash_block(uint64_t parent, const int32_t* toks, int n) {
  uint64_t h = mix64(parent ^ 0x9e3779b97f4a7c15ULL);
  for (int i = 0; i < n; ++i) h = mix64(h ^ (static_cast<uint64_t>(static_cast<uint32_t>(toks[i])) + 0x632be59bd9b4e019ULL * (i + 1)));
  return h;
}

BlockManager::BlockManager(int num_blocks, int block_size)
    : num_blocks_(num_blocks), block_size_(block_size), meta_(num_blocks) {
  if (num_blocks <= 0 || block_size <= 0) throw std::invalid_argument("bad BlockManager geometry");
  free_.reserve(num_blocks);
  for (int b = num_blocks - 1; b >= 0; --b) free_.push_back(b);
}

int BlockManager::num_free_blocks() const {
  return static_cast<int>(free_.size() + evictable_.size());
}

int BlockManager::take_block() {
  if (!free_.empty()) {
    int b = free_.back();
    free_.pop_back();
    return b;
  }
  if (evictable_.empty()) return -1;
  int b = evictable_.front();  // least recently released
  evictable_.pop_front();
  Meta& m = meta_[b];
  m.in_lru = false;
  auto it = cache_.find(m.hash);
  if (it != cache_.end() && it->second == b) cache_.erase(it);
  m.hashed = false;
  ++evictions_;
  return b;
}

void BlockManager::lru_remove(int b) {
  Meta& m = meta_[b];
  if (!m.in_lru) return;
  evictable_.erase(m.lru_pos);
  m.in_lru = false;
}

Allocation BlockManager::allocate(const std::vector<int32_t>& prompt, int max_new_tokens,
                                  bool use_cache) {
  const int n = static_cast<int>(prompt.size());
  const int total = n + std::max(max_new_tokens, 0);
  const int need = (total + block_size_ - 1) / block_size_;
  Allocation a;
  a.blocks.reserve(need);
  uint64_t parent = 0;
  // reuse cached full prompt blocks, but always leave >= 1 token to compute
  const int max_cached_blocks = use_cache ? (n - 1) / block_size_ : 0;
  int hit = 0;
  for (; hit < max_cached_blocks; ++hit) {
    const int32_t* toks = prompt.data() + hit * block_size_;
    const uint64_t h = hash_block(parent, toks, block_size_);
    auto it = cache_.find(h);
    if (it == cache_.end()) break;
    Meta& m = meta_[it->second];
    if (std::memcmp(m.tokens.data(), toks, sizeof(int32_t) * block_size_) != 0) break;
    parent = h;
    lru_remove(it->second);
    ++m.ref;
    a.blocks.push_back(it->second);
  }
  a.num_cached_tokens = hit * block_size_;
  if (need - hit > num_free_blocks()) {
    // roll back the hits; caller must wait for memory
    for (int b : a.blocks) release_one(b);
    a.blocks.clear();
    a.num_cached_tokens = 0;
    a.ok = false;
    return a;
  }
  for (int i = hit; i < need; ++i) {
    int b = take_block();
    meta_[b].ref = 1;
    meta_[b].hashed = false;
    a.blocks.push_back(b);
  }
  a.ok = true;
  hits_ += hit;
  lookups_ += max_cached_blocks;
  return a;
}

void BlockManager::commit_prompt(const std::vector<int>& blocks, const std::vector<int32_t>& prompt) {
  // register every full prompt block (content now resident in HBM)
  const int full = static_cast<int>(prompt.size()) / block_size_;
  uint64_t parent = 0;
  for (int i = 0; i < full && i < static_cast<int>(blocks.size()); ++i) {
    const int32_t* toks = prompt.data() + i * block_size_;
    const uint64_t h = hash_block(parent, toks, block_size_);
    parent = h;
    Meta& m = meta_[blocks[i]];
    if (m.hashed) continue;
    auto it = cache_.find(h);
    if (it != cache_.end()) continue;  // an identical block is already cached
    m.hashed = true;
    m.hash = h;
    m.tokens.assign(toks, toks + block_size_);
    cache_[h] = blocks[i];
  }
}

void BlockManager::release_one(int b) {
  Meta& m = meta_[b];
  if (m.ref <= 0) throw std::logic_error("double free of KV block");
  if (--m.ref > 0) return;
  if (m.hashed) {
    evictable_.push_back(b);
    m.lru_pos = std::prev(evictable_.end());
    m.in_lru = true;
  } else {
    free_.push_back(b);
  }
}

void BlockManager::free(const std::vector<int>& blocks) {
  // release in reverse so deeper (less shared) blocks are evicted first
  for (auto it = blocks.rbegin(); it != blocks.rend(); ++it) release_one(*it);
}

void BlockManager::reset_cache() {
  for (int b : std::vector<int>(evictable_.begin(), evictable_.end())) {
    meta_[b].in_lru = false;
    meta_[b].hashed = false;
    free_.push_back(b);
  }
  evictable_.clear();
  for (auto& kv : cache_) meta_[kv.second].hashed = false;
  cache_.clear();
}

}  // namespace bcg
