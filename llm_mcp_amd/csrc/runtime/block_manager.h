// Paged KV-cache block manager (native runtime).
//
// Owns the mapping sequence -> list of physical KV pages of the device cache
// (see csrc/kernels/rope_cache.hip for the page layout) with
//   * O(log n) allocate / free from a min-heap of free pages: a page is always
//     the lowest free one, so a prompt's pages form ascending runs and every
//     wave reuses the same compact region instead of the previous wave's pages
//     in reverse release order (a LIFO stack); level with the stack on the
//     headline (same box, profiles/r5_serving.md), but the layout no longer
//     depends on the release history,
//   * reference counts, so full pages can be shared between sequences,
//   * automatic prefix caching: every *full* page is identified by a chained
//     64-bit hash of its tokens (h_i = H(h_{i-1}, tokens of page i)); a new
//     prompt reuses cached pages for its longest cached prefix, and pages whose
//     refcount drops to zero stay cached (LRU) until the free stack runs dry.
//
// Admission is by pages, i.e. by HBM: the engine sizes num_blocks from the
// 288 GB device after weights (the reference admits by a fixed
// DEVICE_MAX_CONCURRENCY, core/internal/api/handlers.go:192-246).
#pragma once
#include <cstdint>
#include <list>
#include <unordered_map>
#include <vector>

namespace lmxrt {

class BlockManager {
 public:
  BlockManager(int num_blocks, int block_size, bool enable_prefix_cache);

  int num_blocks() const { return num_blocks_; }
  int block_size() const { return block_size_; }
  // pages that can be handed out right now (free + evictable cached)
  int num_free() const { return (int)free_.size() + (int)lru_.size(); }
  double usage() const { return 1.0 - (double)num_free() / (double)num_blocks_; }

  // Reuse cached pages for the longest cached prefix of `tokens` (full pages
  // only). Returns the number of tokens covered; the pages are attached to seq.
  int match_prefix(int64_t seq, const int32_t* tokens, int n);
  // Ensure seq owns pages for its first n_tokens tokens. False (and no change)
  // if not enough free pages.
  bool ensure(int64_t seq, int n_tokens);
  int pages_needed(int64_t seq, int n_tokens) const;
  // Register the full pages of seq among its first n_computed tokens in the
  // prefix cache.
  void commit(int64_t seq, const int32_t* tokens, int n_computed);
  void free_seq(int64_t seq);
  const std::vector<int32_t>& table(int64_t seq) const;
  bool has(int64_t seq) const { return tables_.count(seq) != 0; }
  int64_t prefix_hits() const { return prefix_hits_; }

 private:
  int alloc_page();
  void release_page(int p);

  int num_blocks_, block_size_;
  bool prefix_;
  std::vector<int32_t> free_;         // min-heap (std::greater)
  std::vector<int32_t> ref_;
  std::vector<uint64_t> page_hash_;   // 0 = not cached
  std::unordered_map<uint64_t, int32_t> cache_;  // hash -> page
  std::list<int32_t> lru_;            // cached pages with ref 0 (front = oldest)
  std::vector<std::list<int32_t>::iterator> lru_pos_;
  std::vector<bool> in_lru_;
  struct SeqPages {
    std::vector<int32_t> pages;
    int hashed = 0;        // leading pages already registered / matched
    uint64_t last_hash = 0;
  };
  std::unordered_map<int64_t, SeqPages> tables_;
  int64_t prefix_hits_ = 0;
  static const std::vector<int32_t> empty_;
};

uint64_t page_hash(uint64_t prev, const int32_t* toks, int n);

}  // namespace lmxrt
