#include "block_allocator.h"

#include <algorithm>
#include <string>

namespace k8sllm {

BlockAllocator::BlockAllocator(int num_blocks, int block_size, bool prefix_caching)
    : num_blocks_(num_blocks), block_size_(block_size), prefix_caching_(prefix_caching) {
  if (num_blocks <= 0 || block_size <= 0) throw std::invalid_argument("num_blocks and block_size must be > 0");
  ref_.assign(num_blocks, 0);
  block_hash_.assign(num_blocks, 0);
  block_parent_.assign(num_blocks, 0);
  block_tokens_.resize(num_blocks);
  evict_pos_.resize(num_blocks);
  in_evictable_.assign(num_blocks, false);
  free_.reserve(num_blocks);
  for (int b = num_blocks - 1; b >= 0; --b) free_.push_back(b);  // pop_back() yields 0, 1, 2, ...
}

uint64_t BlockAllocator::chain_hash(uint64_t parent, const int32_t* toks, int n) const {
  // FNV-1a over (parent, tokens) followed by a splitmix finaliser; never returns 0.
  uint64_t h = 1469598103934665603ull ^ parent;
  for (int i = 0; i < n; ++i) {
    h ^= (uint64_t)(uint32_t)toks[i];
    h *= 1099511628211ull;
  }
  h ^= h >> 30; h *= 0xbf58476d1ce4e5b9ull;
  h ^= h >> 27; h *= 0x94d049bb133111ebull;
  h ^= h >> 31;
  return h ? h : 1;
}

int BlockAllocator::prefix_hits(const std::vector<int32_t>& tokens, std::vector<int>* blocks, uint64_t* last) const {
  if (last) *last = 0;
  if (!prefix_caching_) return 0;
  // The last prompt token is always recomputed (its logits start decoding), so at most
  // (len - 1) tokens can come from the cache.
  const int usable = ((int)tokens.size() - 1) / block_size_;
  uint64_t h = 0;
  int n = 0;
  for (int i = 0; i < usable; ++i) {
    h = chain_hash(h, tokens.data() + (size_t)i * block_size_, block_size_);
    auto it = hash_to_block_.find(h);
    if (it == hash_to_block_.end()) break;
    if (blocks) blocks->push_back(it->second);
    if (last) *last = h;
    ++n;
  }
  return n;
}

int BlockAllocator::sub_block_hit(const std::vector<int32_t>& tokens, int start, uint64_t parent, int* src) const {
  *src = -1;
  auto it = children_.find(parent);
  if (it == children_.end()) return 0;
  // at most (len - 1) prompt tokens may come from the cache (the last one is recomputed for its logits)
  const int maxn = std::min(block_size_, (int)tokens.size() - 1 - start);
  int best = 0;
  for (int b : it->second) {
    const std::vector<int32_t>& t = block_tokens_[b];
    int l = 0;
    while (l < maxn && l < (int)t.size() && t[l] == tokens[start + l]) ++l;
    if (l > best) {
      best = l;
      *src = b;
    }
  }
  return best;
}

void BlockAllocator::unindex(int b) {
  auto it = children_.find(block_parent_[b]);
  if (it != children_.end()) {
    auto& v = it->second;
    v.erase(std::remove(v.begin(), v.end(), b), v.end());
    if (v.empty()) children_.erase(it);
  }
  block_tokens_[b].clear();
}

bool BlockAllocator::can_allocate(const std::vector<int32_t>& tokens, int total_tokens) const {
  std::vector<int> hit;
  const int nhit = prefix_hits(tokens, &hit);
  const int need = (total_tokens + block_size_ - 1) / block_size_;
  int hits_from_evictable = 0;
  for (int b : hit)
    if (ref_[b] == 0) ++hits_from_evictable;
  return need - nhit <= num_free() - hits_from_evictable;
}

int BlockAllocator::take_block() {
  int b;
  if (!free_.empty()) {
    b = free_.back();
    free_.pop_back();
  } else if (!evictable_.empty()) {
    b = evictable_.front();
    evictable_.pop_front();
    in_evictable_[b] = false;
    hash_to_block_.erase(block_hash_[b]);
    block_hash_[b] = 0;
    unindex(b);
  } else {
    throw std::runtime_error("KV cache exhausted");
  }
  ref_[b] = 1;
  return b;
}

BlockAllocator::Allocation BlockAllocator::allocate(const std::vector<int32_t>& tokens, int total_tokens) {
  if (total_tokens < (int)tokens.size()) throw std::invalid_argument("total_tokens < prompt length");
  if (!can_allocate(tokens, total_tokens)) throw std::runtime_error("KV cache exhausted");
  Allocation a;
  std::vector<int> hit;
  uint64_t parent = 0;
  const int nhit = prefix_hits(tokens, &hit, &parent);
  ++queries_;
  if (nhit) ++hits_;
  for (int b : hit) {
    if (ref_[b] == 0 && in_evictable_[b]) {
      evictable_.erase(evict_pos_[b]);
      in_evictable_[b] = false;
    }
    ++ref_[b];
    a.blocks.push_back(b);
  }
  a.cached_tokens = nhit * block_size_;
  // the source of a sub-block hit is read (copied) by the caller before anything can overwrite it: pick it now,
  // before taking this sequence's own blocks (which may evict cached ones)
  const int need = (total_tokens + block_size_ - 1) / block_size_;
  int src = -1;
  int sub = prefix_caching_ ? sub_block_hit(tokens, nhit * block_size_, parent, &src) : 0;
  if (sub > 0 && ref_[src] == 0 && in_evictable_[src]) {
    // keep the source out of this call's evictions -- only when the pool has room without it (can_allocate counted
    // it as evictable space)
    if (need - nhit <= num_free() - 1) {
      evictable_.erase(evict_pos_[src]);
      in_evictable_[src] = false;
    } else {
      sub = 0;
    }
  }
  for (int i = nhit; i < need; ++i) a.blocks.push_back(take_block());
  if (sub > 0) {
    a.copy_src = src;
    a.copy_tokens = sub;
    a.cached_tokens += sub;
    if (ref_[src] == 0 && !in_evictable_[src]) {   // back into the LRU (as the most recently used)
      evictable_.push_back(src);
      evict_pos_[src] = std::prev(evictable_.end());
      in_evictable_[src] = true;
    }
  }
  return a;
}

void BlockAllocator::commit_prefix(const std::vector<int32_t>& blocks, const std::vector<int32_t>& tokens,
                                   int num_tokens) {
  if (!prefix_caching_) return;
  const int nfull = std::min((int)blocks.size(), std::min(num_tokens, (int)tokens.size()) / block_size_);
  uint64_t h = 0;
  for (int i = 0; i < nfull; ++i) {
    const uint64_t parent = h;
    h = chain_hash(h, tokens.data() + (size_t)i * block_size_, block_size_);
    const int b = blocks[i];
    if (block_hash_[b] == h) continue;  // already published (shared prefix block)
    if (block_hash_[b] != 0) continue;  // block carries another chain; leave it
    auto it = hash_to_block_.find(h);
    if (it != hash_to_block_.end()) continue;  // an identical block is already published
    block_hash_[b] = h;
    hash_to_block_[h] = b;
    // sub-block index: under its parent (the chain hash before it), with its tokens
    block_parent_[b] = parent;
    block_tokens_[b].assign(tokens.begin() + (size_t)i * block_size_, tokens.begin() + (size_t)(i + 1) * block_size_);
    auto& v = children_[parent];
    if ((int)v.size() >= kChildren) v.erase(v.begin());   // (the oldest stays published, just not indexed)
    v.push_back(b);
  }
}

void BlockAllocator::release(const std::vector<int32_t>& blocks) {
  for (int b : blocks) {
    if (b < 0 || b >= num_blocks_) throw std::out_of_range("block id " + std::to_string(b));
    if (ref_[b] <= 0) throw std::logic_error("double free of block " + std::to_string(b));
    if (--ref_[b] == 0) {
      if (block_hash_[b] != 0) {
        evictable_.push_back(b);
        evict_pos_[b] = std::prev(evictable_.end());
        in_evictable_[b] = true;
      } else {
        free_.push_back(b);
      }
    }
  }
}

void BlockAllocator::reset_prefix_cache() {
  for (int b : evictable_) {
    in_evictable_[b] = false;
    free_.push_back(b);
  }
  evictable_.clear();
  for (int b = 0; b < num_blocks_; ++b) {
    block_hash_[b] = 0;
    block_parent_[b] = 0;
    block_tokens_[b].clear();
  }
  hash_to_block_.clear();
  children_.clear();
}

}  // namespace k8sllm
