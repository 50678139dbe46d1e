// Durable lease job queue (native runtime) -- the in-process equivalent of the
// reference's Postgres `jobs` / `job_attempts` queue with
// `FOR UPDATE SKIP LOCKED` claims (core/internal/api/handlers.go:173-445,
// core/internal/grpcserver/server.go:126-274).
//
// Semantics kept from the reference:
//   claim order   priority DESC, queued_at ASC; queued jobs and running jobs
//                 whose lease expired are both claimable; kinds filter;
//                 per-device concurrency (DEVICE_MAX_CONCURRENCY CTE) and
//                 "device must be online" for device-pinned jobs;
//   claim effect  status=running, attempts+1, lease_until=now+lease, a new
//                 job_attempts row;
//   fail          requeue while attempts < max_attempts, else status=error.
// Defects of the reference fixed here:
//   * every claim path enforces device concurrency/online (the gRPC claim did
//     not);
//   * lease ownership: claim returns an attempt token; heartbeat / complete /
//     fail must present it (a worker whose lease expired cannot overwrite the
//     new owner's result);
//   * attempts are bounded at claim time and deadline_at is enforced
//     (expired jobs become error "deadline_exceeded").
// Durability: optional append-only journal (one full-row record per
// mutation, last write wins on replay, compactable), fsync policy by caller.
// Thread safety: one mutex; `wait_change` blocks (GIL released by the binding)
// until the version counter moves -- the NOTIFY job_update equivalent.
#pragma once
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace lmxrt {

struct JobRow {
  std::string id, kind, payload, source, status, result, error;
  std::string device_id, model_id;  // placement (running/last device) / payload->>'model_id'
  std::string pin_device;           // payload->>'device_id': the submitter's pin ("" = any)
  std::string worker_id, lease_token;
  int32_t priority = 0, attempts = 0, max_attempts = 3;
  int64_t lease_until = 0, deadline_at = 0, queued_at = 0, updated_at = 0;  // ms, 0 = NULL
  int64_t seq = 0;  // insertion order tie-break
};

struct AttemptRow {
  std::string id, job_id, worker_id, status, error, metrics;
  int64_t started_at = 0, finished_at = 0;
};

struct ClaimFilter {
  std::vector<std::string> kinds;             // empty = any
  std::string worker_device;                  // device of the claiming worker ("" = none)
  std::set<std::string> online_devices;       // devices that may receive pinned jobs
  bool check_online = false;
  int device_max_concurrency = 0;             // 0 = unlimited
  std::map<std::string, int> device_limits;   // per-device override
};

class JobQueue {
 public:
  explicit JobQueue(const std::string& journal_path = "");
  ~JobQueue();

  std::string submit(const std::string& kind, const std::string& payload, int priority,
                     const std::string& source, int max_attempts, int64_t deadline_at,
                     const std::string& device_id, const std::string& model_id, int64_t now,
                     const std::string& status = "queued", const std::string& forced_id = "");
  bool get(const std::string& id, JobRow* out) const;
  // returns false when nothing is claimable
  bool claim(const std::string& worker_id, const ClaimFilter& f, int64_t lease_ms, int64_t now,
             JobRow* out, std::string* attempt_id);
  bool heartbeat(const std::string& id, const std::string& worker_id, const std::string& token,
                 int64_t extend_ms, int64_t now);
  bool complete(const std::string& id, const std::string& worker_id, const std::string& token,
                const std::string& result, const std::string& metrics, int64_t now);
  // returns "queued" (requeued), "error" (exhausted) or "" (not owner / unknown)
  std::string fail(const std::string& id, const std::string& worker_id, const std::string& token,
                   const std::string& error, const std::string& metrics, int64_t now);
  // offline device: clear leases of its running jobs so they are reclaimable now
  int release_device(const std::string& device_id, int64_t now);
  int expire_deadlines(int64_t now);
  int purge_finished(int64_t older_than);  // retention cleanup (planner)

  std::map<std::string, int> counts() const;
  // jobs per status whose kind starts with ``prefix`` (dashboard benchmark
  // counts without converting every row)
  std::map<std::string, int> kind_counts(const std::string& prefix) const;
  // queued + running rows whose device is ``device`` (O(1), indexed)
  int active_on(const std::string& device) const;
  // v_device_stats from the rows: finished jobs of ``device`` updated at or
  // after ``since`` -> {total, done, ms_sum, ms_n} (ms from the done
  // attempts' metrics)
  std::map<std::string, int64_t> device_stats(const std::string& device, int64_t since) const;
  int stuck(int64_t now) const;  // running with expired lease
  std::vector<JobRow> list(const std::string& status, int limit) const;
  std::vector<AttemptRow> attempts(const std::string& job_id) const;
  int running_on(const std::string& device_id, int64_t now) const;  // live leases
  int64_t version() const;
  int64_t wait_change(int64_t since, int64_t timeout_ms);  // returns current version
  void notify_change();  // wake wait_change() for state kept outside the queue (job progress)
  void compact();
  size_t size() const;

 private:
  typedef std::tuple<int32_t, int64_t, int64_t, std::string> ReadyKey;  // (-prio, queued, seq, id)
  void index_insert(const JobRow& j);
  void index_erase(const JobRow& j);
  void journal(const JobRow& j);
  void journal_attempt(const AttemptRow& a);
  void journal_delete(const std::string& id);
  void replay();
  void bump();
  std::string new_id();

  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::unordered_map<std::string, JobRow> jobs_;
  std::set<ReadyKey> claimable_;  // queued + running (lease may expire)
  std::unordered_map<std::string, std::vector<AttemptRow>> attempts_;
  std::unordered_map<std::string, std::unordered_set<std::string>> running_per_device_;
  // queued + running rows placed on each device (the router's load signal)
  std::unordered_map<std::string, int> active_per_device_;
  int live_running(const std::string& dev, int64_t now, const std::string& except) const;
  std::string path_;
  FILE* jf_ = nullptr;
  int64_t seq_ = 0;
  int64_t version_ = 0;
  uint64_t rng_;
};

}  // namespace lmxrt
