// Native runtime of the BCG MI355X engine (host side, C++17).
#pragma once

#include <cstdint>
#include <list>
#include <string>
#include <unordered_map>
#include <vector>

namespace bcg {

// ---------------------------------------------------------------- token FSM
struct TokenFsmTables {
  int num_states = 0;
  int vocab_rows = 0;
  std::vector<int16_t> next;  // [num_states * vocab_rows], -1 = forbidden
  std::vector<int16_t> dist;  // [num_states], INT16_MAX = cannot finish
};

TokenFsmTables compile_token_fsm(const int32_t* trans, const uint8_t* accept, int num_states,
                                 const std::vector<std::string>& tokens, int vocab_rows);

// ------------------------------------------------------------ block manager
struct Allocation {
  bool ok = false;
  std::vector<int> blocks;
  int num_cached_tokens = 0;
};

class BlockManager {
 public:
  BlockManager(int num_blocks, int block_size);
  Allocation allocate(const std::vector<int32_t>& prompt, int max_new_tokens, bool use_cache);
  void commit_prompt(const std::vector<int>& blocks, const std::vector<int32_t>& prompt);
  void free(const std::vector<int>& blocks);
  void reset_cache();
  int num_free_blocks() const;
  int num_blocks() const { return num_blocks_; }
  int block_size() const { return block_size_; }
  int64_t hits() const { return hits_; }
  int64_t lookups() const { return lookups_; }
  int64_t evictions() const { return evictions_; }
  int cached_blocks() const { return static_cast<int>(cache_.size()); }

  static uint64_t hash_block(uint64_t parent, const int32_t* toks, int n);

 private:
  struct Meta {
    int ref = 0;
    bool hashed = false;
    bool in_lru = false;
    uint64_t hash = 0;
    std::vector<int32_t> tokens;
    std::list<int>::iterator lru_pos;
  };
  int take_block();
  void lru_remove(int b);
  void release_one(int b);

  int num_blocks_;
  int block_size_;
  std::vector<Meta> meta_;
  std::vector<int> free_;
  std::list<int> evictable_;
  std::unordered_map<uint64_t, int> cache_;
  int64_t hits_ = 0, lookups_ = 0, evictions_ = 0;
};

}  // namespace bcg
