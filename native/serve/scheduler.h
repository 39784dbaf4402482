// Continuous-batching scheduler + paged-KV block allocator for kgs.serve (the
// native runtime behind the Llama serving stand-in of BASELINE config 5).
//
// The model runner (kgs/serve/engine.py) asks for one step at a time:
//   * PREFILL: admitted waiting sequences, each padded to a multiple of
//     `pad_multiple` tokens (the flash-attention prefill kernel's q-block), with
//     per-token positions and KV-cache slots (-1 for padding rows);
//   * DECODE: every running sequence's last token, its position, the slot the
//     new k/v goes to, its block table and context length.
//   * MIXED (SchedulerConfig::chunk_tokens > 0, chunked prefill): every
//     decode-ready sequence's token PLUS prompt chunks of sequences still
//     prefilling, within a per-step token budget -- a long prompt is split over
//     steps (chunks are multiples of pad_multiple except the last), so decode
//     steps never wait behind a whole prefill. Prefill rows come first.
// Pages are PAGE_SIZE tokens; page 0 is reserved as the null page that padded
// decode rows point at (never handed out). When a decode step cannot get a new
// page, the most recently admitted running sequence is preempted: its pages are
// freed and it goes back to the front of the waiting queue with its generated
// tokens appended to the prompt (recompute on re-admission).
#pragma once

#include <cstdint>
#include <deque>
#include <list>
#include <string>
#include <unordered_map>
#include <vector>

namespace kgs {
namespace serve {

// Pages carry a reference count: with prefix caching, sequences whose prompts
// share leading pages share those pages. A page whose count drops to zero goes
// back to the free stack -- or, if it holds a registered (hashed) full prompt
// page, to an LRU list of evictable cached pages that a later prompt with the
// same prefix can re-acquire. alloc() takes free pages first, then evicts the
// least recently released cached page.
class BlockAllocator {
 public:
  explicit BlockAllocator(int num_pages);
  int alloc();                   // -1 when exhausted
  void free(int page);           // drop one reference
  void acquire(int page);        // one more reference (revives an evictable cached page)
  int num_free() const { return (int)free_.size() + (int)lru_.size(); }  // allocatable
  int num_pages() const { return num_pages_; }
  int refs(int page) const { return page > 0 && page < num_pages_ ? ref_[page] : 0; }
  bool is_free(int page) const { return page > 0 && page < num_pages_ && ref_[page] == 0; }
  // prefix cache: a full page's content key (chained hash + its tokens)
  void register_page(int page, uint64_t hash, uint64_t parent, const int32_t* tokens, int n);
  int lookup(uint64_t hash, uint64_t parent, const int32_t* tokens, int n) const;  // -1 if absent
  int num_cached() const { return (int)by_hash_.size(); }

 private:
  void forget(int page);
  int num_pages_;
  std::vector<int> free_;      // LIFO stack (recently freed pages are reused first: warm in L2/MALL)
  std::vector<int> ref_;
  std::list<int> lru_;         // evictable cached pages, most recently released first
  std::vector<std::list<int>::iterator> lru_pos_;
  std::vector<uint8_t> in_lru_;
  std::unordered_map<uint64_t, int> by_hash_;
  std::vector<uint64_t> hash_, parent_;
  std::vector<uint8_t> hashed_;
  std::vector<std::vector<int32_t>> toks_;
};

enum class SeqState : int { kWaiting = 0, kRunning = 1, kFinished = 2 };

struct Sequence {
  int64_t id = 0;
  std::vector<int32_t> tokens;  // prompt + generated
  int prompt_len = 0;
  int max_new = 0;
  int generated = 0;
  int64_t arrival = 0;          // admission order (preemption picks the newest)
  std::vector<int32_t> pages;
  int cached = 0;               // tokens whose k/v are in the cache
  SeqState state = SeqState::kWaiting;
  int preemptions = 0;
  int hashed = 0;               // leading pages registered in the prefix cache
  uint64_t tail_hash = 0;       // chained hash of those pages
};

struct StepPlan {
  int kind = 0;  // 0 idle, 1 prefill, 2 decode, 3 mixed (chunked prefill + decode)
  std::vector<int64_t> seq_ids;
  // prefill (flattened over sequences, each padded to pad_multiple)
  std::vector<int32_t> tokens, positions, slots;
  std::vector<int32_t> seq_starts, seq_lens, padded_lens;
  // decode
  std::vector<int32_t> block_tables;  // [B, max_pages]
  std::vector<int32_t> ctx_lens;
  int max_pages = 0;
  std::vector<int64_t> preempted;
  // mixed: seq_ids[0 .. n_prefill) are prefill chunks (rows first, with
  // seq_starts / seq_lens / padded_lens), the rest decode rows (block_tables /
  // ctx_lens); ctx_starts = tokens cached before the chunk, last_chunk = the
  // chunk completes the prompt (its last row is sampled), pf_block_tables
  // [n_prefill, pf_max_pages] the chunk sequences' pages
  int n_prefill = 0;
  std::vector<int32_t> ctx_starts;
  std::vector<uint8_t> last_chunk;
  std::vector<int32_t> pf_block_tables;
  int pf_max_pages = 0;
};

struct SchedulerConfig {
  int num_pages = 1024;
  int page_size = 32;
  int max_batch = 256;            // decode sequences per step
  int max_prefill_tokens = 16384; // padded tokens per prefill step
  int max_model_len = 8192;
  int pad_multiple = 128;
  int chunk_tokens = 0;           // > 0: mixed steps of at most this many rows (chunked prefill)
  bool prefix_caching = false;    // share full prompt pages across sequences (implies chunked prefill)
};

class Scheduler {
 public:
  explicit Scheduler(const SchedulerConfig& cfg);
  // returns false if the request can never fit (prompt + max_new > max_model_len
  // or more pages than the cache has)
  bool add(int64_t id, const std::vector<int32_t>& prompt, int max_new_tokens);
  bool abort(int64_t id);
  StepPlan schedule();
  // one sampled token per sequence of the last plan (same order); eos[i] != 0
  // finishes sequence i early. Returns the ids that finished.
  std::vector<int64_t> update(const std::vector<int64_t>& ids, const std::vector<int32_t>& toks,
                              const std::vector<uint8_t>& eos);
  // Two-phase update for an engine that plans step t+1 while step t still runs
  // on the GPU (kgs/serve/engine.py, EngineConfig.overlap): update_pending()
  // advances every sequence of step t by one PENDING token (kPendingToken:
  // lengths, page needs and length stops as update() with no eos), so the next
  // step can be scheduled before the sampled values are known; fill_pending()
  // writes the values in once they are (a sequence's pending token is always
  // its last one: nothing else appends between the two calls). With prefix
  // caching, a full page holding a pending token is registered by fill_pending
  // (its hash needs the value). A stop on EOS,
  // seen one step late, goes through abort(). Returns the ids that finished /
  // the number of tokens filled.
  static constexpr int32_t kPendingToken = -1;
  std::vector<int64_t> update_pending(const std::vector<int64_t>& ids);
  int fill_pending(const std::vector<int64_t>& ids, const std::vector<int32_t>& toks);
  const Sequence* get(int64_t id) const;
  void release(int64_t id);  // drop a finished sequence's record
  int num_waiting() const { return (int)waiting_.size(); }
  int num_running() const { return (int)running_.size(); }
  int num_free_pages() const { return alloc_.num_free(); }
  int64_t prefix_hit_tokens() const { return prefix_hits_; }
  int num_cached_pages() const { return alloc_.num_cached(); }
  const SchedulerConfig& config() const { return cfg_; }
  std::string check_invariants() const;  // "" when consistent (tests)

 private:
  int pages_for(int tokens) const { return (tokens + cfg_.page_size - 1) / cfg_.page_size; }
  bool try_prefill(StepPlan& plan);
  void build_decode(StepPlan& plan);
  StepPlan schedule_mixed();
  bool decode_ready(const Sequence& s) const { return s.cached == (int)s.tokens.size() - 1; }
  void preempt(Sequence& s, StepPlan& plan);
  void free_pages(Sequence& s);

  SchedulerConfig cfg_;
  BlockAllocator alloc_;
  std::unordered_map<int64_t, Sequence> seqs_;
  std::deque<int64_t> waiting_;
  std::vector<int64_t> running_;  // admission order
  int64_t next_arrival_ = 0;
  int64_t prefix_hits_ = 0;
  int match_prefix(Sequence& s);     // acquire cached leading pages; returns tokens matched
  void register_full_pages(Sequence& s);
};

}  // namespace serve
}  // namespace kgs
