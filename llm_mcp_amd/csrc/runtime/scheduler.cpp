#include "scheduler.h"

#include <climits>

#include <algorithm>
#include <stdexcept>

namespace lmxrt {

Scheduler::Scheduler(int num_blocks, int block_size, int max_num_seqs, int max_batched_tokens,
                     int max_model_len, bool prefix_cache)
    : bm_(num_blocks, block_size, prefix_cache),
      max_num_seqs_(max_num_seqs),
      max_batched_tokens_(max_batched_tokens),
      max_model_len_(max_model_len) {
  if (max_num_seqs <= 0 || max_batched_tokens <= 0 || max_model_len <= 0)
    throw std::invalid_argument("bad scheduler limits");
  max_blocks_ = (max_model_len + block_size - 1) / block_size;
}

void Scheduler::add(int64_t id, const std::vector<int32_t>& prompt, int max_new,
                    const std::vector<int32_t>& stop_ids, bool ignore_eos, int priority,
                    float temperature, int top_k, float top_p, int64_t seed) {
  if (seqs_.count(id)) throw std::invalid_argument("duplicate sequence id");
  if (prompt.empty()) throw std::invalid_argument("empty prompt");
  if ((int)prompt.size() >= max_model_len_)
    throw std::invalid_argument("prompt longer than max_model_len");
  const int pages = ((int)prompt.size() + bm_.block_size()) / bm_.block_size();
  if (pages > bm_.num_blocks()) throw std::invalid_argument("prompt larger than the KV cache");
  auto s = std::make_unique<Seq>();
  s->id = id;
  s->tokens = prompt;
  s->prompt_len = (int)prompt.size();
  s->max_new = std::max(1, std::min(max_new, max_model_len_ - (int)prompt.size()));
  s->stop_ids = stop_ids;
  s->ignore_eos = ignore_eos;
  s->priority = priority;
  s->temperature = temperature;
  s->top_k = top_k;
  s->top_p = top_p;
  s->seed = seed;
  s->arrival = arrival_++;
  s->arrival_step = steps_;
  Seq* raw = s.get();
  seqs_[id] = std::move(s);
  // priority first (higher earlier), FIFO inside a priority
  auto it = waiting_.end();
  while (it != waiting_.begin() && (*(it - 1))->priority < priority) --it;
  waiting_.insert(it, raw);
}

bool Scheduler::set_penalties(int64_t id, float repetition, float presence, float frequency,
                              int last_n) {
  auto it = seqs_.find(id);
  if (it == seqs_.end()) return false;
  if (!(repetition > 0.f)) throw std::invalid_argument("repetition penalty must be > 0");
  Seq* s = it->second.get();
  s->rep_pen = repetition;
  s->pres_pen = presence;
  s->freq_pen = frequency;
  s->pen_last_n = std::max(0, std::min(last_n, kPenWindow));
  return true;
}

const Seq* Scheduler::get(int64_t id) const {
  auto it = seqs_.find(id);
  return it == seqs_.end() ? nullptr : it->second.get();
}

bool Scheduler::abort(int64_t id) {
  auto it = seqs_.find(id);
  if (it == seqs_.end()) return false;
  Seq* s = it->second.get();
  if (s->zombie) return false;    // already finished, awaiting its plan's consumption
  auto w = std::find(waiting_.begin(), waiting_.end(), s);
  if (w != waiting_.end()) waiting_.erase(w);
  auto r = std::find(running_.begin(), running_.end(), s);
  if (r != running_.end()) running_.erase(r);
  bm_.free_seq(id);
  // lookahead: a sample of it awaiting patch() is dropped; a row of it in the
  // plan in flight keeps the object alive until update_lookahead() consumes it
  for (Seq*& q : inflight_)
    if (q == s) q = nullptr;
  if (in_plan(s)) {
    s->status = FINISHED;
    s->finish = FR_ABORT;
    s->zombie = true;
    return true;
  }
  seqs_.erase(it);
  return true;
}

bool Scheduler::in_plan(const Seq* s) const {
  return std::find(plan_seqs_.begin(), plan_seqs_.end(), s) != plan_seqs_.end();
}

bool Scheduler::length_done(const Seq* s) const {
  return s->num_generated >= s->max_new || (int)s->tokens.size() >= max_model_len_ ||
         // a sequence longer than the whole KV cache could never be re-admitted
         (int)s->tokens.size() >= bm_.num_blocks() * bm_.block_size();
}

void Scheduler::preempt(Seq* s) {
  bm_.free_seq(s->id);
  s->num_computed = 0;
  s->scheduled = 0;
  s->status = WAITING;
  auto r = std::find(running_.begin(), running_.end(), s);
  if (r != running_.end()) running_.erase(r);
  waiting_.push_front(s);
  plan_.preempted.push_back(s->id);
  ++preemptions_;
}

void Scheduler::finish(Seq* s, int reason) {
  s->status = FINISHED;
  s->finish = reason;
  bm_.free_seq(s->id);
  auto r = std::find(running_.begin(), running_.end(), s);
  if (r != running_.end()) running_.erase(r);
  // lookahead: a sequence preempted by the plan after the one that sampled
  // its stop token sits in waiting_ when patch() finishes it; it must leave
  // that queue before its Seq is erased
  auto w = std::find(waiting_.begin(), waiting_.end(), s);
  if (w != waiting_.end()) waiting_.erase(w);
}

const StepPlan& Scheduler::schedule(int q_per_tile) {
  if (q_per_tile <= 0) q_per_tile = 16;
  StepPlan& p = plan_;
  p.input_ids.clear(); p.positions.clear(); p.slots.clear(); p.input_src.clear();
  p.num_pending_inputs = 0;
  p.seq_ids.clear(); p.qlens.clear(); p.context_lens.clear(); p.cu_q.clear();
  p.block_tables.clear(); p.sample_rows.clear(); p.sample_seq.clear();
  p.sample_temp.clear(); p.sample_topp.clear(); p.sample_topk.clear(); p.sample_off.clear();
  p.sample_seed.clear();
  p.prefill_tiles.clear(); p.preempted.clear();
  p.any_penalty = false;
  p.pen_window.clear(); p.pen_ngen.clear(); p.pen_params.clear();
  p.num_decode = 0; p.num_tokens = 0; p.num_prefill_tokens = 0; p.max_context = 0;
  p.max_blocks = max_blocks_;
  plan_seqs_.clear();

  int budget = max_batched_tokens_;
  // mixed steps: with at least mixed_min_decodes_ decode rows running, the
  // step's prefill tokens are capped (a long prefill chunk stalls every
  // decoding stream for the whole step); a step without decodes -- an idle
  // engine taking a burst -- keeps the full max_batched_tokens
  int prefill_left = INT_MAX;
  ++steps_;
  if (mixed_prefill_cap_ > 0) {
    // the newest request with prompt tokens left (running chunks, waiting)
    int64_t newest = -1;
    if (mixed_later_ > 0) {
      for (Seq* s : running_)
        if ((int)s->tokens.size() - s->num_computed > 1) newest = std::max(newest, s->arrival_step);
      for (Seq* s : waiting_) newest = std::max(newest, s->arrival_step);
    }
    int nd = 0;
    for (Seq* s : running_)
      nd += ((int)s->tokens.size() - s->num_computed) == 1 &&
            (mixed_later_ == 0 || newest - s->arrival_step >= mixed_later_);
    if (nd >= mixed_min_decodes_) prefill_left = mixed_prefill_cap_;
  }
  std::vector<Seq*> decodes, prefills;
  // 1. running sequences, oldest first
  for (size_t i = 0; i < running_.size() && budget > 0;) {
    Seq* s = running_[i];
    const int remaining = (int)s->tokens.size() - s->num_computed;
    if (remaining <= 0) { ++i; continue; }
    int n = std::min(remaining, budget);
    if (remaining > 1) n = std::min(n, prefill_left);
    if (n <= 0) { ++i; continue; }       // prefill capped this step: wait for the next
    bool preempted_self = false;
    while (!bm_.ensure(s->id, s->num_computed + n)) {
      Seq* victim = running_.back();
      preempt(victim);
      if (victim == s) { preempted_self = true; break; }
    }
    if (preempted_self) break;
    s->scheduled = n;
    budget -= n;
    if (remaining > 1) prefill_left -= n;
    (n == 1 ? decodes : prefills).push_back(s);
    ++i;
  }
  // 2. admit waiting sequences
  while (!waiting_.empty() && budget > 0 && (int)running_.size() < max_num_seqs_) {
    Seq* s = waiting_.front();
    if (s->num_computed == 0 && !bm_.has(s->id))
      s->num_computed = bm_.match_prefix(s->id, s->tokens.data(), (int)s->tokens.size());
    const int remaining = (int)s->tokens.size() - s->num_computed;
    int n = std::min(remaining, budget);
    if (remaining > 1) n = std::min(n, prefill_left);
    if (n <= 0) break;
    if (!bm_.ensure(s->id, s->num_computed + n)) {
      // a waiting sequence must not keep the prefix pages it just matched:
      // with every runner preempted, waiting sequences each pinning their
      // cached prefix could fill the cache and admit nobody (deadlock)
      bm_.free_seq(s->id);
      s->num_computed = 0;
      break;
    }
    waiting_.pop_front();
    s->status = RUNNING;
    running_.push_back(s);
    s->scheduled = n;
    budget -= n;
    if (remaining > 1) prefill_left -= n;
    (n == 1 ? decodes : prefills).push_back(s);
  }

  // 3. flatten (decode rows first).  Block-table rows are only as wide as
  // the longest table in this plan (the kernels take the row stride), so the
  // per-step upload scales with the live context, not with max_model_len.
  const int bs = bm_.block_size();
  int width = 1;
  for (Seq* s : decodes) width = std::max(width, (int)bm_.table(s->id).size());
  for (Seq* s : prefills) width = std::max(width, (int)bm_.table(s->id).size());
  p.max_blocks = width;
  p.cu_q.push_back(0);
  auto emit = [&](Seq* s, bool is_prefill, int prefill_idx) {
    const int n = s->scheduled;
    const std::vector<int32_t>& tab = bm_.table(s->id);
    const int row0 = p.num_tokens;
    const int pend_t = s->pend >= 0 ? (int)s->tokens.size() - 1 : -1;
    for (int t = s->num_computed; t < s->num_computed + n; ++t) {
      if (t == pend_t) {          // the in-flight plan's sample: filled on the device
        p.input_ids.push_back(0);
        p.input_src.push_back(s->pend);
        ++p.num_pending_inputs;
      } else {
        p.input_ids.push_back(s->tokens[t]);
        p.input_src.push_back(-1);
      }
      p.positions.push_back(t);
      p.slots.push_back(tab[t / bs] * bs + t % bs);
    }
    p.num_tokens += n;
    const int ctx = s->num_computed + n;
    p.seq_ids.push_back(s->id);
    p.qlens.push_back(n);
    p.context_lens.push_back(ctx);
    p.cu_q.push_back(p.num_tokens);
    p.max_context = std::max(p.max_context, ctx);
    const size_t off = p.block_tables.size();
    p.block_tables.resize(off + width, 0);
    std::copy(tab.begin(), tab.end(), p.block_tables.begin() + off);
    if (ctx == (int)s->tokens.size()) {
      p.sample_rows.push_back(row0 + n - 1);
      p.sample_seq.push_back((int)plan_seqs_.size());
      p.sample_temp.push_back(s->temperature);
      p.sample_topk.push_back(s->top_k);
      p.sample_topp.push_back(s->top_p);
      p.sample_seed.push_back(s->seed);
      p.sample_off.push_back(s->num_generated);
      p.any_penalty |= s->penalized();
    }
    if (is_prefill) {
      p.num_prefill_tokens += n;
      for (int q0 = 0; q0 < n; q0 += q_per_tile) {
        p.prefill_tiles.push_back(prefill_idx);
        p.prefill_tiles.push_back(q0);
      }
    }
    plan_seqs_.push_back(s);
  };
  for (Seq* s : decodes) emit(s, false, 0);
  p.num_decode = (int)decodes.size();
  int j = 0;
  for (Seq* s : prefills) emit(s, true, j++);
  if (p.any_penalty) {
    const size_t n = p.sample_rows.size();
    p.pen_window.assign(n * kPenWindow, -1);
    p.pen_ngen.assign(n, 0);
    p.pen_params.assign(n * 3, 0.f);
    for (size_t i = 0; i < n; ++i) {
      const Seq* s = plan_seqs_[p.sample_seq[i]];
      p.pen_params[3 * i] = 1.f;
      if (!s->penalized()) continue;
      const int len = (int)s->tokens.size(), w = std::min(s->pen_last_n, len);
      std::copy(s->tokens.end() - w, s->tokens.end(),
                p.pen_window.begin() + (i + 1) * kPenWindow - w);
      p.pen_ngen[i] = std::min(w, s->num_generated);
      p.pen_params[3 * i] = s->rep_pen;
      p.pen_params[3 * i + 1] = s->pres_pen;
      p.pen_params[3 * i + 2] = s->freq_pen;
    }
  }
  return p;
}

std::vector<std::pair<int64_t, int>> Scheduler::update(const int32_t* sampled, int n) {
  std::vector<std::pair<int64_t, int>> done;
  if (n != (int)plan_.sample_rows.size()) throw std::invalid_argument("sample count mismatch");
  for (Seq* s : plan_seqs_) {
    s->num_computed += s->scheduled;
    s->scheduled = 0;
    bm_.commit(s->id, s->tokens.data(), s->num_computed);
  }
  for (int i = 0; i < n; ++i) {
    Seq* s = plan_seqs_[plan_.sample_seq[i]];
    const int32_t tok = sampled[i];
    s->tokens.push_back(tok);
    s->num_generated++;
    int reason = FR_NONE;
    if (!s->ignore_eos &&
        std::find(s->stop_ids.begin(), s->stop_ids.end(), tok) != s->stop_ids.end())
      reason = FR_STOP;
    else if (length_done(s))
      reason = FR_LENGTH;
    if (reason != FR_NONE) {
      finish(s, reason);
      done.emplace_back(s->id, reason);
    }
  }
  for (auto& d : done) seqs_.erase(d.first);
  plan_seqs_.clear();
  return done;
}

void Scheduler::update_lookahead() {
  if (!inflight_.empty()) throw std::logic_error("update_lookahead before patch of the last plan");
  for (Seq* s : plan_seqs_) {
    if (s->zombie) continue;
    s->num_computed += s->scheduled;
    s->scheduled = 0;
    bm_.commit(s->id, s->tokens.data(), s->num_computed);
  }
  const int n = (int)plan_.sample_rows.size();
  inflight_.assign(n, nullptr);
  for (int i = 0; i < n; ++i) {
    Seq* s = plan_seqs_[plan_.sample_seq[i]];
    if (s->zombie) continue;     // finished after this plan was launched: sample dropped
    s->tokens.push_back(0);      // placeholder until patch()
    s->num_generated++;
    s->pend = i;
    inflight_[i] = s;
    // its last token: pages freed now (no further row), reason (stop or
    // length, stop first as in update()) reported by patch()
    if (length_done(s)) finish(s, FR_LENGTH);
  }
  for (Seq* s : plan_seqs_)
    if (s->zombie) seqs_.erase(s->id);
  plan_seqs_.clear();
}

std::vector<std::pair<int64_t, int>> Scheduler::patch(const int32_t* sampled, int n) {
  if (n != (int)inflight_.size()) throw std::invalid_argument("sample count mismatch");
  std::vector<std::pair<int64_t, int>> done;
  for (int i = 0; i < n; ++i) {
    Seq* s = inflight_[i];
    if (s == nullptr) continue;
    const int32_t tok = sampled[i];
    s->tokens.back() = tok;
    s->pend = -1;
    const bool stop = !s->ignore_eos &&
        std::find(s->stop_ids.begin(), s->stop_ids.end(), tok) != s->stop_ids.end();
    if (s->status == FINISHED) {  // its last token (update_lookahead freed it)
      done.emplace_back(s->id, stop ? FR_STOP : FR_LENGTH);
      seqs_.erase(s->id);
      continue;
    }
    if (stop) {
      finish(s, FR_STOP);
      done.emplace_back(s->id, FR_STOP);
      if (in_plan(s)) s->zombie = true;
      else seqs_.erase(s->id);
    }
  }
  inflight_.clear();
  return done;
}

void Scheduler::discard_lookahead() {
  for (Seq* s : inflight_) {
    if (s == nullptr) continue;
    s->pend = -1;
    if (s->status == FINISHED) seqs_.erase(s->id);
  }
  inflight_.clear();
  for (Seq* s : plan_seqs_) {
    s->scheduled = 0;
    if (s->zombie) seqs_.erase(s->id);
  }
  plan_seqs_.clear();
}

}  // namespace lmxrt
