// Native runtime stress test, built with host sanitizers (TSan for races,
// ASan+UBSan for memory errors) by `python -m llm_mcp_amd.build
// --sanitize-runtime`.  The MI355X-side equivalent of the reference's
// `go test -race ./...` (.github/workflows/ci.yml:60-63): the lease queue is
// hammered by concurrent workers (claim / heartbeat / complete / fail /
// release_device / wait_change) and the KV block manager + scheduler run a
// randomized admission/preemption workload, with invariants checked.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "../job_queue.h"
#include "../scheduler.h"

using namespace lmxrt;

#define CHECK(c)                                                      \
  do {                                                                \
    if (!(c)) {                                                       \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::exit(1);                                                   \
    }                                                                 \
  } while (0)

static int queue_stress(int n_jobs, int n_workers) {
  JobQueue q("");
  std::atomic<int64_t> clock{1000};
  for (int i = 0; i < n_jobs; ++i) {
    const std::string dev = (i % 3 == 0) ? "n:gpu" + std::to_string(i % 4) : "";
    q.submit(i % 5 == 0 ? "engine.embed" : "engine.generate", "{}", i % 7, "stress", 3, 0, dev,
             "m", clock.load());
  }
  std::atomic<int> done{0}, lost{0};
  std::atomic<bool> stop{false};
  std::vector<std::thread> ts;
  for (int w = 0; w < n_workers; ++w) {
    ts.emplace_back([&, w] {
      std::mt19937 rng(w * 7919 + 1);
      ClaimFilter f;
      f.worker_device = "n:gpu" + std::to_string(w % 4);
      f.device_max_concurrency = 8;
      while (!stop.load()) {
        JobRow j;
        std::string tok;
        const int64_t now = clock.fetch_add(1);
        if (!q.claim("w" + std::to_string(w), f, 60000, now, &j, &tok)) {
          auto c = q.counts();
          if (c["queued"] + c["running"] == 0) break;
          q.wait_change(q.version(), 1);
          continue;
        }
        CHECK(j.status == "running");
        CHECK(q.running_on(f.worker_device, now) <= 8);
        q.heartbeat(j.id, "w" + std::to_string(w), tok, 60000, clock.load());
        // a stale token must never complete someone else's lease
        CHECK(!q.complete(j.id, "w" + std::to_string(w), "bogus", "{}", "{}", clock.load()));
        // release_device (chaos thread) may have handed the lease to another
        // worker: then this worker's complete/fail must be refused
        if (rng() % 4 == 0) {
          std::string st = q.fail(j.id, "w" + std::to_string(w), tok, "boom", "{}",
                                  clock.load());
          CHECK(st == "queued" || st == "error" || st.empty());
          if (st.empty()) lost.fetch_add(1);
        } else if (q.complete(j.id, "w" + std::to_string(w), tok, "{\"ok\":true}",
                              "{\"ms\":1}", clock.load())) {
          done.fetch_add(1);
        } else {
          lost.fetch_add(1);
        }
      }
    });
  }
  std::thread chaos([&] {
    for (int i = 0; i < 200 && !stop.load(); ++i) {
      q.release_device("n:gpu" + std::to_string(i % 4), clock.load());
      (void)q.counts();
      (void)q.stuck(clock.load());
      std::this_thread::yield();
    }
  });
  for (auto& t : ts) t.join();
  stop.store(true);
  chaos.join();
  auto c = q.counts();
  CHECK(c["done"] + c["error"] == n_jobs);  // every job finished exactly once
  CHECK(c["done"] == done.load());            // no completion double-counted
  CHECK(c["queued"] == 0 && c["running"] == 0);
  std::printf("queue: %d done, %d error, %d lost leases refused\n", c["done"], c["error"],
              lost.load());
  return 0;
}

static int scheduler_stress(int steps) {
  Scheduler s(96, 32, 16, 256, 1024, true);
  std::mt19937 rng(5);
  int64_t next = 1;
  int finished = 0;
  std::set<int64_t> live;
  for (int it = 0; it < steps; ++it) {
    if (live.size() < 24 && rng() % 2 == 0) {
      std::vector<int32_t> prompt(1 + rng() % 300);
      const int shared = rng() % 3;  // shared prefixes exercise the prefix cache
      for (size_t i = 0; i < prompt.size(); ++i)
        prompt[i] = (int32_t)(i < 64 && shared ? shared : rng() % 1000);
      s.add(next, prompt, 1 + rng() % 40, {7}, rng() % 2 == 0, rng() % 3);
      live.insert(next++);
    }
    if (!live.empty() && rng() % 17 == 0) {
      auto it2 = live.begin();
      std::advance(it2, rng() % live.size());
      s.abort(*it2);
      live.erase(it2);
    }
    if (!s.has_work()) continue;
    const StepPlan& p = s.schedule(16);
    CHECK(p.num_tokens <= 256);
    CHECK((int)p.cu_q.size() == (int)p.seq_ids.size() + 1);
    CHECK((int)p.block_tables.size() == (int)p.seq_ids.size() * p.max_blocks);
    std::set<int32_t> slots;
    for (int32_t sl : p.slots) {
      CHECK(sl >= 0 && sl < 96 * 32);
      CHECK(slots.insert(sl).second);  // no two tokens write the same KV slot
    }
    std::vector<int32_t> toks(p.sample_rows.size());
    for (auto& t : toks) t = (int32_t)(rng() % 1000);
    for (auto& d : s.update(toks.data(), (int)toks.size())) {
      live.erase(d.first);
      ++finished;
    }
    CHECK(s.blocks().num_free() <= 96);
  }
  std::printf("scheduler: %d finished, %lld preemptions, %lld prefix hits\n", finished,
              (long long)s.preemptions(), (long long)s.blocks().prefix_hits());
  return 0;
}


// Lookahead protocol (update_lookahead / schedule / patch) under KV pressure:
// stop tokens are frequent, so in-flight samples of sequences the next plan
// preempted or already carries turn out to be STOP (a preempted
// sequence finished by patch() used to stay in the waiting queue after its
// Seq was freed).  Run under ASan this reports any such use-after-free.
static int lookahead_stress(int steps) {
  Scheduler s(12, 16, 16, 128, 512, true);
  std::mt19937 rng(11);
  int64_t next = 1;
  int finished = 0;
  std::set<int64_t> live;
  std::vector<int32_t> prev;     // samples of the plan in flight, read back one step late
  bool inflight = false;
  for (int it = 0; it < steps; ++it) {
    if (live.size() < 20 && rng() % 2 == 0) {
      std::vector<int32_t> prompt(1 + rng() % 60);
      for (auto& t : prompt) t = (int32_t)(10 + rng() % 1000);
      s.add(next, prompt, 1 + rng() % 80, {7}, false, 0);
      live.insert(next++);
    }
    if (!live.empty() && rng() % 23 == 0) {
      auto it2 = live.begin();
      std::advance(it2, rng() % live.size());
      if (s.abort(*it2)) live.erase(it2);
    }
    if (inflight) s.update_lookahead();
    const StepPlan& p = s.schedule(16);
    std::vector<int32_t> toks(p.sample_rows.size());
    for (auto& t : toks) t = rng() % 9 == 0 ? 7 : (int32_t)(10 + rng() % 1000);
    if (inflight) {
      for (auto& d : s.patch(prev.data(), (int)prev.size())) {
        live.erase(d.first);
        ++finished;
      }
    }
    inflight = p.num_tokens > 0;
    prev = toks;
    if (!inflight) continue;
    std::set<int32_t> slots;
    for (int32_t sl : p.slots) {
      CHECK(sl >= 0 && sl < 12 * 16);
      CHECK(slots.insert(sl).second);
    }
  }
  if (inflight) s.discard_lookahead();
  std::printf("lookahead: %d finished, %lld preemptions\n", finished, (long long)s.preemptions());
  return 0;
}

int main(int argc, char** argv) {
  const int jobs = argc > 1 ? std::atoi(argv[1]) : 3000;
  queue_stress(jobs, 8);
  scheduler_stress(argc > 2 ? std::atoi(argv[2]) : 4000);
  lookahead_stress(argc > 2 ? std::atoi(argv[2]) : 4000);
  std::printf("ok\n");
  return 0;
}
