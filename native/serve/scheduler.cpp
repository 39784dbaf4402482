// kgs.serve native scheduler: see scheduler.h for the model.
#include "scheduler.h"

#include <algorithm>
#include <sstream>

namespace kgs {
namespace serve {

BlockAllocator::BlockAllocator(int num_pages)
    : num_pages_(num_pages), ref_(num_pages > 0 ? num_pages : 0, 0), lru_pos_(num_pages > 0 ? num_pages : 0),
      in_lru_(num_pages > 0 ? num_pages : 0, 0), hash_(num_pages > 0 ? num_pages : 0, 0),
      parent_(num_pages > 0 ? num_pages : 0, 0), hashed_(num_pages > 0 ? num_pages : 0, 0),
      toks_(num_pages > 0 ? num_pages : 0) {
  // page 0 is the null page: never handed out
  if (num_pages_ > 0) ref_[0] = 1;
  free_.reserve(num_pages_);
  for (int p = num_pages_ - 1; p >= 1; --p) free_.push_back(p);
}

void BlockAllocator::forget(int page) {
  if (!hashed_[page]) return;
  auto it = by_hash_.find(hash_[page]);
  if (it != by_hash_.end() && it->second == page) by_hash_.erase(it);
  hashed_[page] = 0;
  toks_[page].clear();
}

int BlockAllocator::alloc() {
  int p;
  if (!free_.empty()) {
    p = free_.back();
    free_.pop_back();
  } else if (!lru_.empty()) {  // evict the least recently released cached page
    p = lru_.back();
    lru_.pop_back();
    in_lru_[p] = 0;
    forget(p);
  } else {
    return -1;
  }
  ref_[p] = 1;
  return p;
}

void BlockAllocator::free(int page) {
  if (page <= 0 || page >= num_pages_ || ref_[page] == 0) return;  // double free / null page: ignore
  if (--ref_[page] > 0) return;
  if (hashed_[page]) {
    lru_.push_front(page);
    lru_pos_[page] = lru_.begin();
    in_lru_[page] = 1;
  } else {
    free_.push_back(page);
  }
}

void BlockAllocator::acquire(int page) {
  if (page <= 0 || page >= num_pages_) return;
  if (in_lru_[page]) {
    lru_.erase(lru_pos_[page]);
    in_lru_[page] = 0;
  }
  ++ref_[page];
}

void BlockAllocator::register_page(int page, uint64_t hash, uint64_t parent, const int32_t* tokens, int n) {
  if (page <= 0 || page >= num_pages_ || hashed_[page] || by_hash_.count(hash)) return;
  by_hash_[hash] = page;
  hash_[page] = hash;
  parent_[page] = parent;
  hashed_[page] = 1;
  toks_[page].assign(tokens, tokens + n);
}

int BlockAllocator::lookup(uint64_t hash, uint64_t parent, const int32_t* tokens, int n) const {
  auto it = by_hash_.find(hash);
  if (it == by_hash_.end()) return -1;
  const int p = it->second;
  // exact check: the same parent chain and the same tokens (no trust in the hash alone)
  if (parent_[p] != parent || (int)toks_[p].size() != n || !std::equal(tokens, tokens + n, toks_[p].begin()))
    return -1;
  return p;
}

namespace {
// FNV-1a over (parent hash, the page's token ids)
uint64_t page_hash(uint64_t parent, const int32_t* t, int n) {
  uint64_t h = 1469598103934665603ull ^ parent;
  h *= 1099511628211ull;
  for (int i = 0; i < n; ++i) {
    uint32_t v = (uint32_t)t[i];
    for (int b = 0; b < 4; ++b) {
      h ^= (v >> (8 * b)) & 0xff;
      h *= 1099511628211ull;
    }
  }
  return h;
}
}  // namespace

int Scheduler::match_prefix(Sequence& s) {
  // leading full pages already cached; keep the last token to compute (its
  // logits), and an even page count: a chunk's context must be a multiple of
  // the attention kernel's 64-key tile
  const int ps = cfg_.page_size, len = (int)s.tokens.size();
  uint64_t h = 0;
  std::vector<int> hit;
  std::vector<uint64_t> hs;
  for (int j = 0; (j + 1) * ps <= len - 1; ++j) {
    const int32_t* t = s.tokens.data() + j * ps;
    const uint64_t hj = page_hash(h, t, ps);
    const int p = alloc_.lookup(hj, h, t, ps);
    if (p < 0) break;
    hit.push_back(p);
    hs.push_back(hj);
    h = hj;
  }
  const int keep = (int)hit.size() / 2 * 2;
  if (keep == 0) return 0;
  for (int j = 0; j < keep; ++j) {
    alloc_.acquire(hit[j]);
    s.pages.push_back(hit[j]);
  }
  s.hashed = keep;
  s.tail_hash = hs[keep - 1];
  s.cached = keep * ps;
  return s.cached;
}

void Scheduler::register_full_pages(Sequence& s) {
  const int ps = cfg_.page_size;
  while ((s.hashed + 1) * ps <= s.cached && s.hashed < (int)s.pages.size() &&
         (s.hashed + 1) * ps <= (int)s.tokens.size()) {
    const int32_t* t = s.tokens.data() + s.hashed * ps;
    // a page whose last generated token is still pending (overlapped engine
    // steps) is registered by fill_pending, once the value is known
    if (std::find(t, t + ps, kPendingToken) != t + ps) break;
    const uint64_t h = page_hash(s.tail_hash, t, ps);
    alloc_.register_page(s.pages[s.hashed], h, s.tail_hash, t, ps);
    s.tail_hash = h;
    s.hashed++;
  }
}

Scheduler::Scheduler(const SchedulerConfig& cfg) : cfg_(cfg), alloc_(cfg.num_pages) {
  // a (re-)prefill of any sequence up to max_model_len must fit one step
  const int pad = std::max(1, cfg_.pad_multiple);
  cfg_.pad_multiple = pad;
  cfg_.max_prefill_tokens = std::max(cfg_.max_prefill_tokens, (cfg_.max_model_len + pad - 1) / pad * pad);
  // prefix caching skips cached leading pages with a chunk over the cached
  // context: it runs on mixed steps
  if (cfg_.prefix_caching && cfg_.chunk_tokens <= 0) cfg_.chunk_tokens = cfg_.max_prefill_tokens;
  // a mixed step always has room for one padded chunk
  if (cfg_.chunk_tokens > 0) cfg_.chunk_tokens = std::max(cfg_.chunk_tokens, pad);
}

bool Scheduler::add(int64_t id, const std::vector<int32_t>& prompt, int max_new_tokens) {
  if (prompt.empty() || max_new_tokens < 1) return false;
  if (seqs_.count(id)) return false;
  const int total = (int)prompt.size() + max_new_tokens;
  if ((int)prompt.size() >= cfg_.max_model_len || pages_for(std::min(total, cfg_.max_model_len)) > cfg_.num_pages - 1)
    return false;
  Sequence s;
  s.id = id;
  s.tokens = prompt;
  s.prompt_len = (int)prompt.size();
  s.max_new = max_new_tokens;
  seqs_.emplace(id, std::move(s));
  waiting_.push_back(id);
  return true;
}

void Scheduler::free_pages(Sequence& s) {
  for (int p : s.pages) alloc_.free(p);
  s.pages.clear();
  s.cached = 0;
  s.hashed = 0;
  s.tail_hash = 0;
}

bool Scheduler::abort(int64_t id) {
  auto it = seqs_.find(id);
  if (it == seqs_.end() || it->second.state == SeqState::kFinished) return false;
  Sequence& s = it->second;
  if (s.state == SeqState::kWaiting) {
    waiting_.erase(std::remove(waiting_.begin(), waiting_.end(), id), waiting_.end());
  } else {
    running_.erase(std::remove(running_.begin(), running_.end(), id), running_.end());
    free_pages(s);
  }
  s.state = SeqState::kFinished;
  return true;
}

void Scheduler::preempt(Sequence& s, StepPlan& plan) {
  free_pages(s);
  s.state = SeqState::kWaiting;
  s.preemptions++;
  running_.erase(std::remove(running_.begin(), running_.end(), s.id), running_.end());
  waiting_.push_front(s.id);
  plan.preempted.push_back(s.id);
}

bool Scheduler::try_prefill(StepPlan& plan) {
  const int ps = cfg_.page_size, pad = cfg_.pad_multiple;
  // keep ~1% of the cache free after admission so running sequences can grow
  const int watermark = std::max(1, (cfg_.num_pages - 1) / 100);
  int budget = cfg_.max_prefill_tokens;
  while (!waiting_.empty() && (int)running_.size() < cfg_.max_batch) {
    Sequence& s = seqs_.at(waiting_.front());
    const int len = (int)s.tokens.size();
    const int padded = (len + pad - 1) / pad * pad;
    const int need = pages_for(len + 1);
    if (padded > budget) break;
    if (alloc_.num_free() - need < (running_.empty() && plan.seq_ids.empty() ? 0 : watermark)) break;
    waiting_.pop_front();
    budget -= padded;
    for (int i = 0; i < need; ++i) s.pages.push_back(alloc_.alloc());
    const int start = (int)plan.tokens.size();
    plan.seq_ids.push_back(s.id);
    plan.seq_starts.push_back(start);
    plan.seq_lens.push_back(len);
    plan.padded_lens.push_back(padded);
    for (int t = 0; t < padded; ++t) {
      const bool real = t < len;
      plan.tokens.push_back(real ? s.tokens[t] : 0);
      plan.positions.push_back(t);
      plan.slots.push_back(real ? s.pages[t / ps] * ps + t % ps : -1);
    }
    s.cached = len;
    s.state = SeqState::kRunning;
    s.arrival = next_arrival_++;
    running_.push_back(s.id);
  }
  if (plan.seq_ids.empty()) return false;
  plan.kind = 1;
  return true;
}

void Scheduler::build_decode(StepPlan& plan) {
  const int ps = cfg_.page_size;
  // make sure every running sequence has a slot for one more token, preempting
  // the newest sequences when the cache is full (oldest keep making progress)
  for (size_t i = 0; i < running_.size();) {
    Sequence& s = seqs_.at(running_[i]);
    if (pages_for(s.cached + 1) <= (int)s.pages.size()) {
      ++i;
      continue;
    }
    int p = alloc_.alloc();
    while (p < 0) {
      Sequence& victim = seqs_.at(running_.back());
      const bool self = victim.id == s.id;
      preempt(victim, plan);
      if (self) break;
      p = alloc_.alloc();
    }
    if (p < 0) continue;  // s itself was preempted (running_ shrank)
    s.pages.push_back(p);
    ++i;
  }
  if (running_.empty()) return;
  plan.kind = 2;
  int maxp = 0;
  for (int64_t id : running_) maxp = std::max(maxp, (int)seqs_.at(id).pages.size());
  plan.max_pages = maxp;
  plan.block_tables.assign(running_.size() * (size_t)maxp, 0);
  for (size_t i = 0; i < running_.size(); ++i) {
    Sequence& s = seqs_.at(running_[i]);
    const int pos = s.cached;
    plan.seq_ids.push_back(s.id);
    plan.tokens.push_back(s.tokens.back());
    plan.positions.push_back(pos);
    plan.slots.push_back(s.pages[pos / ps] * ps + pos % ps);
    plan.ctx_lens.push_back(pos + 1);
    std::copy(s.pages.begin(), s.pages.end(), plan.block_tables.begin() + i * maxp);
    s.cached = pos + 1;
  }
}

StepPlan Scheduler::schedule_mixed() {
  StepPlan plan;
  const int ps = cfg_.page_size, pad = cfg_.pad_multiple;
  // 1) every decode-ready sequence gets a slot for one more token (preempting
  //    the newest sequences when the cache is full, as build_decode does)
  for (size_t i = 0; i < running_.size();) {
    Sequence& s = seqs_.at(running_[i]);
    if (!decode_ready(s) || pages_for(s.cached + 1) <= (int)s.pages.size()) {
      ++i;
      continue;
    }
    int p = alloc_.alloc();
    while (p < 0) {
      Sequence& victim = seqs_.at(running_.back());
      const bool self = victim.id == s.id;
      preempt(victim, plan);
      if (self) break;
      p = alloc_.alloc();
    }
    if (p < 0) continue;
    s.pages.push_back(p);
    ++i;
  }
  std::vector<int64_t> dec;
  for (int64_t id : running_)
    if (decode_ready(seqs_.at(id))) dec.push_back(id);
  // 2) prompt chunks within the remaining row budget: sequences already
  //    prefilling (admission order), then newly admitted ones
  int budget = std::max(pad, cfg_.chunk_tokens - (int)dec.size());
  const int watermark = std::max(1, (cfg_.num_pages - 1) / 100);
  std::vector<int64_t> pf;
  auto add_chunk = [&](Sequence& s) -> bool {
    int matched = 0;
    if (cfg_.prefix_caching && s.cached == 0 && s.pages.empty()) matched = match_prefix(s);
    auto undo = [&]() {
      if (matched) free_pages(s);
      return false;
    };
    const int len = (int)s.tokens.size(), rem = len - s.cached;
    const bool last = rem <= budget;
    const int n = last ? rem : budget / pad * pad;  // non-final chunks: whole q-blocks
    if (n <= 0) return undo();
    const int padded = (n + pad - 1) / pad * pad;
    const int need = pages_for(s.cached + n + (last ? 1 : 0)) - (int)s.pages.size();
    if (need > 0 && alloc_.num_free() - need < (dec.empty() && pf.empty() ? 0 : watermark)) return undo();
    prefix_hits_ += matched;
    for (int i = 0; i < need; ++i) s.pages.push_back(alloc_.alloc());
    const int start = (int)plan.tokens.size();
    plan.seq_ids.push_back(s.id);
    plan.seq_starts.push_back(start);
    plan.seq_lens.push_back(n);
    plan.padded_lens.push_back(padded);
    plan.ctx_starts.push_back(s.cached);
    plan.last_chunk.push_back(last ? 1 : 0);
    for (int t = 0; t < padded; ++t) {
      const int pos = s.cached + t;
      const bool real = t < n;
      plan.tokens.push_back(real ? s.tokens[pos] : 0);
      plan.positions.push_back(pos);
      plan.slots.push_back(real ? s.pages[pos / ps] * ps + pos % ps : -1);
    }
    s.cached += n;
    if (cfg_.prefix_caching) register_full_pages(s);  // written by this step, before any later step reads them
    budget -= padded;
    pf.push_back(s.id);
    return true;
  };
  auto fill = [&]() {
    for (int64_t id : running_) {
      Sequence& s = seqs_.at(id);
      if (budget < pad) break;
      if (!decode_ready(s) && s.cached < (int)s.tokens.size()) add_chunk(s);
    }
    while (!waiting_.empty() && budget >= pad && (int)running_.size() < cfg_.max_batch) {
      Sequence& s = seqs_.at(waiting_.front());
      if (!add_chunk(s)) break;
      waiting_.pop_front();
      s.state = SeqState::kRunning;
      s.arrival = next_arrival_++;
      running_.push_back(s.id);
    }
  };
  fill();
  // every running sequence is mid-prompt and none can get pages for its next
  // chunk: free the newest (recompute later) so the others progress
  while (dec.empty() && pf.empty() && !running_.empty()) {
    preempt(seqs_.at(running_.back()), plan);
    fill();
  }
  plan.n_prefill = (int)pf.size();
  // 3) decode rows after the chunks
  if (!pf.empty()) {
    int maxp = 0;
    for (int64_t id : pf) maxp = std::max(maxp, (int)seqs_.at(id).pages.size());
    plan.pf_max_pages = maxp;
    plan.pf_block_tables.assign(pf.size() * (size_t)maxp, 0);
    for (size_t i = 0; i < pf.size(); ++i) {
      const Sequence& s = seqs_.at(pf[i]);
      std::copy(s.pages.begin(), s.pages.end(), plan.pf_block_tables.begin() + i * maxp);
    }
  }
  int maxp = 0;
  for (int64_t id : dec) maxp = std::max(maxp, (int)seqs_.at(id).pages.size());
  plan.max_pages = maxp;
  plan.block_tables.assign(dec.size() * (size_t)maxp, 0);
  for (size_t i = 0; i < dec.size(); ++i) {
    Sequence& s = seqs_.at(dec[i]);
    const int pos = s.cached;
    plan.seq_ids.push_back(s.id);
    plan.tokens.push_back(s.tokens.back());
    plan.positions.push_back(pos);
    plan.slots.push_back(s.pages[pos / ps] * ps + pos % ps);
    plan.ctx_lens.push_back(pos + 1);
    std::copy(s.pages.begin(), s.pages.end(), plan.block_tables.begin() + i * maxp);
    s.cached = pos + 1;
    // a page filled by generated tokens is cacheable too (multi-turn chat:
    // the next turn's prompt starts with this one's prompt + answer)
    if (cfg_.prefix_caching && s.cached % ps == 0) register_full_pages(s);
  }
  // no chunk this step: a plain decode plan (the engine replays its hipGraph)
  plan.kind = plan.seq_ids.empty() ? 0 : pf.empty() ? 2 : 3;
  return plan;
}

StepPlan Scheduler::schedule() {
  if (cfg_.chunk_tokens > 0) return schedule_mixed();
  StepPlan plan;
  if (!waiting_.empty() && try_prefill(plan)) return plan;
  build_decode(plan);
  return plan;
}

std::vector<int64_t> Scheduler::update(const std::vector<int64_t>& ids, const std::vector<int32_t>& toks,
                                       const std::vector<uint8_t>& eos) {
  std::vector<int64_t> done;
  for (size_t i = 0; i < ids.size() && i < toks.size(); ++i) {
    auto it = seqs_.find(ids[i]);
    if (it == seqs_.end() || it->second.state != SeqState::kRunning) continue;  // aborted / preempted meanwhile
    Sequence& s = it->second;
    s.tokens.push_back(toks[i]);
    s.generated++;
    const bool stop = (i < eos.size() && eos[i]) || s.generated >= s.max_new ||
                      (int)s.tokens.size() >= cfg_.max_model_len;
    if (stop) {
      running_.erase(std::remove(running_.begin(), running_.end(), s.id), running_.end());
      free_pages(s);
      s.state = SeqState::kFinished;
      done.push_back(s.id);
    }
  }
  return done;
}

std::vector<int64_t> Scheduler::update_pending(const std::vector<int64_t>& ids) {
  return update(ids, std::vector<int32_t>(ids.size(), kPendingToken), {});
}

int Scheduler::fill_pending(const std::vector<int64_t>& ids, const std::vector<int32_t>& toks) {
  int n = 0;
  for (size_t i = 0; i < ids.size() && i < toks.size(); ++i) {
    auto it = seqs_.find(ids[i]);
    if (it == seqs_.end()) continue;  // released meanwhile
    std::vector<int32_t>& t = it->second.tokens;
    if (!t.empty() && t.back() == kPendingToken) {
      t.back() = toks[i];
      ++n;
      if (cfg_.prefix_caching && it->second.state == SeqState::kRunning) register_full_pages(it->second);
    }
  }
  return n;
}

const Sequence* Scheduler::get(int64_t id) const {
  auto it = seqs_.find(id);
  return it == seqs_.end() ? nullptr : &it->second;
}

void Scheduler::release(int64_t id) {
  auto it = seqs_.find(id);
  if (it != seqs_.end() && it->second.state == SeqState::kFinished) seqs_.erase(it);
}

std::string Scheduler::check_invariants() const {
  std::ostringstream err;
  std::vector<int> owners(cfg_.num_pages, 0);
  for (const auto& kv : seqs_) {
    const Sequence& s = kv.second;
    if (s.state != SeqState::kRunning && !s.pages.empty()) err << "seq " << s.id << " not running but holds pages; ";
    if (s.state == SeqState::kRunning && pages_for(s.cached) > (int)s.pages.size())
      err << "seq " << s.id << " cached " << s.cached << " beyond its pages; ";
    std::vector<int> mine(s.pages);
    std::sort(mine.begin(), mine.end());
    if (std::adjacent_find(mine.begin(), mine.end()) != mine.end()) err << "seq " << s.id << " holds a page twice; ";
    for (int p : s.pages) {
      if (p <= 0 || p >= cfg_.num_pages) {
        err << "seq " << s.id << " holds bad page " << p << "; ";
        continue;
      }
      owners[p]++;
      if (alloc_.is_free(p)) err << "page " << p << " both free and owned; ";
    }
  }
  int owned = 0;
  for (int p = 1; p < cfg_.num_pages; ++p) {
    if (owners[p] != alloc_.refs(p)) err << "page " << p << " refs " << alloc_.refs(p) << " owners " << owners[p] << "; ";
    if (!cfg_.prefix_caching && owners[p] > 1) err << "page " << p << " shared without prefix caching; ";
    owned += owners[p] > 0;
  }
  if (owned + alloc_.num_free() != cfg_.num_pages - 1) err << "page leak: owned " << owned << " free " << alloc_.num_free() << "; ";
  if ((int)running_.size() > cfg_.max_batch) err << "running over max_batch; ";
  for (int64_t id : running_)
    if (seqs_.at(id).state != SeqState::kRunning) err << "running list has non-running " << id << "; ";
  for (int64_t id : waiting_)
    if (seqs_.at(id).state != SeqState::kWaiting) err << "waiting list has non-waiting " << id << "; ";
  return err.str();
}

}  // namespace serve
}  // namespace kgs
