#include "block_manager.h"

#include <algorithm>
#include <functional>
#include <stdexcept>

namespace lmxrt {

const std::vector<int32_t> BlockManager::empty_;

uint64_t page_hash(uint64_t prev, const int32_t* toks, int n) {
  // FNV-1a over the previous hash and the page tokens, finished by a 64-bit mix
  uint64_t h = 1469598103934665603ULL ^ (prev * 0x9E3779B97F4A7C15ULL);
  for (int i = 0; i < n; ++i) {
    h ^= (uint64_t)(uint32_t)toks[i];
    h *= 1099511628211ULL;
  }
  h ^= h >> 33;
  h *= 0xff51afd7ed558ccdULL;
  h ^= h >> 33;
  return h ? h : 1;  // 0 is reserved for "not cached"
}

BlockManager::BlockManager(int num_blocks, int block_size, bool enable_prefix_cache)
    : num_blocks_(num_blocks), block_size_(block_size), prefix_(enable_prefix_cache) {
  if (num_blocks <= 0 || block_size <= 0) throw std::invalid_argument("bad block manager size");
  free_.reserve(num_blocks);
  for (int i = 0; i < num_blocks; ++i) free_.push_back(i);  // ascending = a min-heap
  ref_.assign(num_blocks, 0);
  page_hash_.assign(num_blocks, 0);
  lru_pos_.resize(num_blocks);
  in_lru_.assign(num_blocks, false);
}

int BlockManager::alloc_page() {
  int p;
  if (!free_.empty()) {
    std::pop_heap(free_.begin(), free_.end(), std::greater<int32_t>());
    p = free_.back();
    free_.pop_back();
  } else if (!lru_.empty()) {
    p = lru_.front();  // evict the least recently used cached page
    lru_.pop_front();
    in_lru_[p] = false;
    if (page_hash_[p]) {
      auto it = cache_.find(page_hash_[p]);
      if (it != cache_.end() && it->second == p) cache_.erase(it);
      page_hash_[p] = 0;
    }
  } else {
    return -1;
  }
  ref_[p] = 1;
  return p;
}

void BlockManager::release_page(int p) {
  if (--ref_[p] > 0) return;
  if (prefix_ && page_hash_[p]) {
    lru_.push_back(p);
    lru_pos_[p] = std::prev(lru_.end());
    in_lru_[p] = true;
  } else {
    page_hash_[p] = 0;
    free_.push_back(p);
    std::push_heap(free_.begin(), free_.end(), std::greater<int32_t>());
  }
}

int BlockManager::match_prefix(int64_t seq, const int32_t* tokens, int n) {
  SeqPages& sp = tables_[seq];
  if (!prefix_ || !sp.pages.empty()) return (int)sp.pages.size() * block_size_;
  uint64_t h = 0;
  int matched = 0;
  // never match the page holding the last prompt token: its logits are needed
  const int full = (n - 1) / block_size_;
  for (int i = 0; i < full; ++i) {
    const uint64_t nh = page_hash(h, tokens + (long)i * block_size_, block_size_);
    auto it = cache_.find(nh);
    if (it == cache_.end()) break;
    const int p = it->second;
    if (in_lru_[p]) {
      lru_.erase(lru_pos_[p]);
      in_lru_[p] = false;
    }
    ++ref_[p];
    sp.pages.push_back(p);
    h = nh;
    ++matched;
  }
  sp.hashed = matched;
  sp.last_hash = h;
  prefix_hits_ += matched;
  return matched * block_size_;
}

int BlockManager::pages_needed(int64_t seq, int n_tokens) const {
  const int want = (n_tokens + block_size_ - 1) / block_size_;
  auto it = tables_.find(seq);
  const int have = it == tables_.end() ? 0 : (int)it->second.pages.size();
  return want > have ? want - have : 0;
}

bool BlockManager::ensure(int64_t seq, int n_tokens) {
  const int need = pages_needed(seq, n_tokens);
  if (need > num_free()) return false;
  SeqPages& sp = tables_[seq];
  for (int i = 0; i < need; ++i) {
    const int p = alloc_page();
    if (p < 0) throw std::runtime_error("block manager accounting error");
    sp.pages.push_back(p);
  }
  return true;
}

void BlockManager::commit(int64_t seq, const int32_t* tokens, int n_computed) {
  if (!prefix_) return;
  auto it = tables_.find(seq);
  if (it == tables_.end()) return;
  SeqPages& sp = it->second;
  const int full = n_computed / block_size_;
  while (sp.hashed < full && sp.hashed < (int)sp.pages.size()) {
    const int i = sp.hashed;
    const uint64_t nh = page_hash(sp.last_hash, tokens + (long)i * block_size_, block_size_);
    const int p = sp.pages[i];
    if (!cache_.count(nh) && page_hash_[p] == 0) {
      cache_[nh] = p;
      page_hash_[p] = nh;
    }
    sp.last_hash = nh;
    ++sp.hashed;
  }
}

void BlockManager::free_seq(int64_t seq) {
  auto it = tables_.find(seq);
  if (it == tables_.end()) return;
  // release in reverse so the tail of a prefix is evicted before its head
  for (auto p = it->second.pages.rbegin(); p != it->second.pages.rend(); ++p) release_page(*p);
  tables_.erase(it);
}

const std::vector<int32_t>& BlockManager::table(int64_t seq) const {
  auto it = tables_.find(seq);
  return it == tables_.end() ? empty_ : it->second.pages;
}

}  // namespace lmxrt
