// Continuous-batching step scheduler (native runtime).
//
// One instance per engine (per GPU, or per TP group on its leader rank).  Every
// engine step asks `schedule()` for a StepPlan: a token-budgeted batch in which
//   * every running sequence gets its next token (decode) or its next prefill
//     chunk (chunked prefill, bounded by max_batched_tokens),
//   * waiting sequences are admitted FIFO (priority first) while KV pages,
//     batch slots and the token budget allow, reusing cached prefix pages,
//   * when pages run out a running sequence is preempted by recompute (its
//     pages are freed, it re-enters the front of the waiting queue with its
//     generated tokens appended to the prompt).
// The plan is written into flat int32 arrays in the exact layout the GPU
// kernels consume (decode rows first, then prefill rows), so the Python side
// does one host->device copy per step and no per-token Python work.
//
// This replaces the reference's one-job-per-worker execution
// (worker/llm_worker/main.py:558-599): a GPU worker serves many claimed jobs
// at once and admission is by KV pages rather than DEVICE_MAX_CONCURRENCY.
#pragma once
#include <cstdint>
#include <deque>
#include <memory>
#include <unordered_map>
#include <vector>

#include "block_manager.h"

namespace lmxrt {

enum SeqStatus { WAITING = 0, RUNNING = 1, FINISHED = 2 };
enum FinishReason { FR_NONE = 0, FR_STOP = 1, FR_LENGTH = 2, FR_ABORT = 3 };

struct Seq {
  int64_t id = 0;
  std::vector<int32_t> tokens;  // prompt + generated
  int prompt_len = 0;
  int num_computed = 0;         // tokens whose KV is resident
  int max_new = 0;
  int num_generated = 0;
  int priority = 0;
  int64_t arrival = 0;
  int64_t arrival_step = 0;     // the scheduler step count when it was added
  bool ignore_eos = false;
  std::vector<int32_t> stop_ids;
  // sampling parameters travel with the sequence so the plan carries them
  // as flat per-sample-row arrays (no per-request host work per step)
  float temperature = 1.f, top_p = 1.f;
  int top_k = 0;
  int64_t seed = 0;
  // repetition (HF / Ollama repeat_penalty), presence and frequency (OpenAI)
  // penalties over the last pen_last_n context tokens (<= kPenWindow)
  float rep_pen = 1.f, pres_pen = 0.f, freq_pen = 0.f;
  int pen_last_n = 0;
  bool penalized() const { return pen_last_n > 0 && (rep_pen != 1.f || pres_pen != 0.f || freq_pen != 0.f); }
  int status = WAITING;
  int finish = FR_NONE;
  int scheduled = 0;            // tokens scheduled in the current plan
  // lookahead stepping: tokens.back() is the sample `pend` of the plan in
  // flight, not yet read back (-1: every token is known)
  int pend = -1;
  // finished (stop token / abort) while the plan in flight still holds a row
  // of it: the object lives until that plan is consumed
  bool zombie = false;
};

constexpr int kPenWindow = 64;   // token window of the penalty kernel (one wave per row)

struct StepPlan {
  // per token rows (T)
  std::vector<int32_t> input_ids, positions, slots;
  // lookahead stepping: -1, or the previous plan's sample index whose token
  // (still on the device) is this row's input; input_ids holds 0 there
  std::vector<int32_t> input_src;
  int num_pending_inputs = 0;
  // per scheduled sequence (S), decode sequences first
  std::vector<int64_t> seq_ids;
  std::vector<int32_t> qlens, context_lens, cu_q;  // cu_q has S+1 entries
  std::vector<int32_t> block_tables;               // S x max_blocks (0-padded)
  std::vector<int32_t> sample_rows;                // token rows whose logits are sampled
  std::vector<int32_t> sample_seq;                 // index into seq_ids for each sample row
  std::vector<float> sample_temp, sample_topp;     // per sample row
  std::vector<int32_t> sample_topk, sample_off;    // sample_off = tokens generated so far
  std::vector<int64_t> sample_seed;
  std::vector<int32_t> prefill_tiles;              // (prefill-seq index, q_start) pairs
  // penalties (filled only when some sampled row is penalised): per sample
  // row the last kPenWindow context tokens right-aligned (-1 padded), how
  // many of them are generated tokens, and (repetition, presence, frequency)
  bool any_penalty = false;
  std::vector<int32_t> pen_window, pen_ngen;
  std::vector<float> pen_params;
  int num_decode = 0;                              // first num_decode sequences have qlen 1
  int max_blocks = 0;                              // row width of block_tables (this plan)
  int num_tokens = 0;
  int num_prefill_tokens = 0;
  int max_context = 0;
  std::vector<int64_t> preempted;
};

class Scheduler {
 public:
  Scheduler(int num_blocks, int block_size, int max_num_seqs, int max_batched_tokens,
            int max_model_len, bool prefix_cache);

  void add(int64_t id, const std::vector<int32_t>& prompt, int max_new,
           const std::vector<int32_t>& stop_ids, bool ignore_eos, int priority,
           float temperature = 1.f, int top_k = 0, float top_p = 1.f, int64_t seed = 0);
  bool abort(int64_t id);
  bool set_penalties(int64_t id, float repetition, float presence, float frequency, int last_n);
  // q_per_tile: queries per prefill workgroup (64 / G for the paged prefill kernel)
  const StepPlan& schedule(int q_per_tile);
  // sampled[i] is the token for plan.sample_rows[i]; returns finished (id, reason)
  std::vector<std::pair<int64_t, int>> update(const int32_t* sampled, int n);
  // Lookahead stepping (the engine launches plan n+1 before it has read plan
  // n's tokens):
  //   update_lookahead()  consume the plan just launched with its sampled
  //                       tokens still unknown: a placeholder is appended per
  //                       sample and the next schedule() points the rows that
  //                       read it at the sample (plan.input_src); a sequence
  //                       at its length limit is finished here (no next row);
  //   patch(sampled, n)   the tokens of the plan consumed by the last
  //                       update_lookahead(): placeholders filled, that plan's
  //                       finishes returned (stop before length, as update()).  A sequence that stops while the
  //                       next plan (already launched) holds a row of it is
  //                       finished at once (pages freed: the in-flight write
  //                       lands before any later step in stream order) and its
  //                       extra sample is dropped by the next update_lookahead.
  void update_lookahead();
  std::vector<std::pair<int64_t, int>> patch(const int32_t* sampled, int n);
  int num_inflight_samples() const { return (int)inflight_.size(); }
  // drop the lookahead state (engine failure): pending samples and the plan
  // in flight are forgotten, finished objects released
  void discard_lookahead();

  // prefill tokens of a step that also carries >= min_decodes decode rows
  // (0: no cap beyond max_batched_tokens).  later_steps > 0: only decode rows
  // whose request was added at least later_steps scheduler steps before the
  // newest request with prefill work count -- streams interrupted by LATER
  // arrivals (steady serving); the rows of one burst, prefilled together,
  // never cap each other (a wave keeps the full token budget)
  void set_mixed_prefill_cap(int tokens, int min_decodes, int later_steps = 0) {
    mixed_prefill_cap_ = tokens > 0 ? tokens : 0;
    mixed_min_decodes_ = min_decodes > 0 ? min_decodes : 1;
    mixed_later_ = later_steps > 0 ? later_steps : 0;
  }
  int64_t steps() const { return steps_; }
  int num_waiting() const { return (int)waiting_.size(); }
  int num_running() const { return (int)running_.size(); }
  bool has_work() const { return !waiting_.empty() || !running_.empty(); }
  BlockManager& blocks() { return bm_; }
  const Seq* get(int64_t id) const;
  int64_t preemptions() const { return preemptions_; }

 private:
  void preempt(Seq* s);
  void finish(Seq* s, int reason);
  bool in_plan(const Seq* s) const;
  bool length_done(const Seq* s) const;

  BlockManager bm_;
  int max_num_seqs_, max_batched_tokens_, max_model_len_, max_blocks_;
  int mixed_prefill_cap_ = 0, mixed_min_decodes_ = 1, mixed_later_ = 0;
  int64_t steps_ = 0;
  std::unordered_map<int64_t, std::unique_ptr<Seq>> seqs_;
  std::deque<Seq*> waiting_;
  std::vector<Seq*> running_;
  std::vector<Seq*> plan_seqs_;
  std::vector<Seq*> inflight_;   // samples awaiting patch() (nullptr: dropped)
  StepPlan plan_;
  int64_t arrival_ = 0;
  int64_t preemptions_ = 0;
};

}  // namespace lmxrt
