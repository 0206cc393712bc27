// Paged-KV block allocator with hash-chained prefix caching (native runtime component).
//
// The KV cache is a pool of fixed-size blocks (block_size tokens of K and V for every layer).
// A sequence owns a list of block ids (its block table).  Full blocks of PROMPT tokens can be
// shared between sequences: each full block is identified by a hash chained over the token ids
// of every block before it, so two prompts that share the same first N*block_size tokens (the
// scheduler's long system prompt) share the same N blocks and skip their prefill.
//
// Lifecycle: allocate() reserves blocks for prompt + max_new_tokens (decode never allocates, so a
// decode step needs no host work and can be replayed from a hipGraph); commit_prefix() publishes
// the hashes of blocks whose KV has actually been written (a block is never shared before its KV
// exists); release() drops references -- hashed blocks with no users stay cached (LRU) until
// their space is needed.
//
// Sub-block prefix: a shared prefix rarely ends on a block boundary (the scheduler's system prompt
// and chat header end 11 tokens into a block, and the pod-specific text follows in the same block).
// Every published block is also indexed under its parent chain hash, so after the full-block hits
// allocate() looks for a cached block with the same parent whose leading tokens match the next
// tokens of the new prompt; the longest such run is reported (copy_src / copy_tokens) and counted
// as cached: the caller copies those positions' K/V into the new sequence's own block before its
// prefill (no sharing, so the block stays private and writable).
#pragma once
#include <cstdint>
#include <list>
#include <stdexcept>
#include <unordered_map>
#include <vector>

namespace k8sllm {

class BlockAllocator {
 public:
  BlockAllocator(int num_blocks, int block_size, bool prefix_caching);

  struct Allocation {
    std::vector<int32_t> blocks;
    int cached_tokens = 0;  // leading prompt tokens whose KV is already cached (shared blocks + copy_tokens)
    int copy_src = -1;      // sub-block prefix: copy positions [0, copy_tokens) of this block's K/V ...
    int copy_tokens = 0;    // ... into blocks[cached_tokens / block_size] before the prefill
  };

  // Reserve ceil(total_tokens / block_size) blocks for a sequence whose prompt is `tokens`.
  // Throws std::runtime_error when the pool cannot satisfy the request.
  Allocation allocate(const std::vector<int32_t>& tokens, int total_tokens);
  // Would allocate() succeed right now (counting prefix hits)?
  bool can_allocate(const std::vector<int32_t>& tokens, int total_tokens) const;
  // Publish hashes for the full prompt blocks among the first `num_tokens` tokens.
  void commit_prefix(const std::vector<int32_t>& blocks, const std::vector<int32_t>& tokens, int num_tokens);
  void release(const std::vector<int32_t>& blocks);

  int num_blocks() const { return num_blocks_; }
  int block_size() const { return block_size_; }
  int num_free() const { return (int)free_.size() + (int)evictable_.size(); }
  int num_cached() const { return (int)hash_to_block_.size(); }
  int refcount(int block) const { return ref_[block]; }
  uint64_t hits() const { return hits_; }
  uint64_t queries() const { return queries_; }
  void reset_prefix_cache();

 private:
  uint64_t chain_hash(uint64_t parent, const int32_t* toks, int n) const;
  int take_block();
  int prefix_hits(const std::vector<int32_t>& tokens, std::vector<int>* blocks, uint64_t* last = nullptr) const;
  int sub_block_hit(const std::vector<int32_t>& tokens, int start, uint64_t parent, int* src) const;
  void unindex(int block);

  int num_blocks_, block_size_;
  bool prefix_caching_;
  std::vector<int> ref_;
  std::vector<uint64_t> block_hash_;  // 0 == not hashed
  std::vector<int> free_;             // never hashed / invalidated blocks (stack)
  std::list<int> evictable_;          // hashed, refcount 0, LRU order (front = oldest)
  std::vector<std::list<int>::iterator> evict_pos_;
  std::vector<bool> in_evictable_;
  std::unordered_map<uint64_t, int> hash_to_block_;
  // sub-block prefix index: parent chain hash -> the most recent published blocks under it (their tokens kept)
  static constexpr int kChildren = 8;
  std::unordered_map<uint64_t, std::vector<int>> children_;
  std::vector<uint64_t> block_parent_;
  std::vector<std::vector<int32_t>> block_tokens_;
  uint64_t hits_ = 0, queries_ = 0;
};

}  // namespace k8sllm
