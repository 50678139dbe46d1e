#include "job_queue.h"

#include <cctype>
#include <cstdlib>

#include <algorithm>
#include <chrono>
#include <random>
#include <stdexcept>

namespace lmxrt {

namespace {

std::string esc(const std::string& s) {
  std::string o;
  o.reserve(s.size() + 8);
  for (char c : s) {
    if (c == '\\') o += "\\\\";
    else if (c == '\n') o += "\\n";
    else if (c == '\x1f') o += "\\u";
    else o += c;
  }
  return o;
}

std::string unesc(const std::string& s) {
  std::string o;
  o.reserve(s.size());
  for (size_t i = 0; i < s.size(); ++i) {
    if (s[i] == '\\' && i + 1 < s.size()) {
      const char n = s[++i];
      o += n == 'n' ? '\n' : (n == 'u' ? '\x1f' : n);
    } else {
      o += s[i];
    }
  }
  return o;
}

std::vector<std::string> split(const std::string& line) {
  std::vector<std::string> f;
  size_t b = 0;
  for (size_t i = 0; i <= line.size(); ++i) {
    if (i == line.size() || line[i] == '\x1f') {
      f.push_back(unesc(line.substr(b, i - b)));
      b = i + 1;
    }
  }
  return f;
}

}  // namespace

JobQueue::JobQueue(const std::string& journal_path) : path_(journal_path) {
  std::random_device rd;
  rng_ = ((uint64_t)rd() << 32) ^ rd() ^
         (uint64_t)std::chrono::steady_clock::now().time_since_epoch().count();
  if (!path_.empty()) {
    replay();
    jf_ = fopen(path_.c_str(), "a");
    if (!jf_) throw std::runtime_error("cannot open job journal " + path_);
  }
}

JobQueue::~JobQueue() {
  if (jf_) fclose(jf_);
}

std::string JobQueue::new_id() {
  auto next = [this]() {
    rng_ ^= rng_ << 13;
    rng_ ^= rng_ >> 7;
    rng_ ^= rng_ << 17;
    return rng_;
  };
  const uint64_t a = next(), b = next();
  unsigned char u[16];
  for (int i = 0; i < 8; ++i) { u[i] = (a >> (8 * i)) & 0xff; u[8 + i] = (b >> (8 * i)) & 0xff; }
  u[6] = (u[6] & 0x0f) | 0x40;  // version 4
  u[8] = (u[8] & 0x3f) | 0x80;  // variant
  static const char* hx = "0123456789abcdef";
  std::string s;
  for (int i = 0; i < 16; ++i) {
    if (i == 4 || i == 6 || i == 8 || i == 10) s += '-';
    s += hx[u[i] >> 4];
    s += hx[u[i] & 15];
  }
  return s;
}

void JobQueue::bump() {
  ++version_;
  cv_.notify_all();
}

void JobQueue::index_insert(const JobRow& j) {
  if (j.status == "queued" || j.status == "running")
    claimable_.insert(ReadyKey(-j.priority, j.queued_at, j.seq, j.id));
  if (j.status == "running" && !j.device_id.empty()) running_per_device_[j.device_id].insert(j.id);
  if ((j.status == "queued" || j.status == "running") && !j.device_id.empty())
    ++active_per_device_[j.device_id];
}

void JobQueue::index_erase(const JobRow& j) {
  claimable_.erase(ReadyKey(-j.priority, j.queued_at, j.seq, j.id));
  if (j.status == "running" && !j.device_id.empty()) {
    auto it = running_per_device_.find(j.device_id);
    if (it != running_per_device_.end()) {
      it->second.erase(j.id);
      if (it->second.empty()) running_per_device_.erase(it);
    }
  }
  if ((j.status == "queued" || j.status == "running") && !j.device_id.empty()) {
    auto it = active_per_device_.find(j.device_id);
    if (it != active_per_device_.end() && --it->second <= 0) active_per_device_.erase(it);
  }
}

// running jobs on a device whose lease is still live (the reference's
// running_per_device CTE counts lease_until > now())
int JobQueue::live_running(const std::string& dev, int64_t now, const std::string& except) const {
  auto it = running_per_device_.find(dev);
  if (it == running_per_device_.end()) return 0;
  int n = 0;
  for (const std::string& id : it->second) {
    if (id == except) continue;
    auto j = jobs_.find(id);
    if (j != jobs_.end() && j->second.lease_until >= now) ++n;
  }
  return n;
}

void JobQueue::journal(const JobRow& j) {
  if (!jf_) return;
  const char S = '\x1f';
  std::string line = "J";
  for (const std::string* f : {&j.id, &j.kind, &j.payload, &j.source, &j.status, &j.result,
                               &j.error, &j.device_id, &j.model_id, &j.worker_id, &j.lease_token}) {
    line += S;
    line += esc(*f);
  }
  for (int64_t v : {(int64_t)j.priority, (int64_t)j.attempts, (int64_t)j.max_attempts,
                    j.lease_until, j.deadline_at, j.queued_at, j.updated_at, j.seq}) {
    line += S;
    line += std::to_string(v);
  }
  line += S;
  line += esc(j.pin_device);
  line += '\n';
  fwrite(line.data(), 1, line.size(), jf_);
  fflush(jf_);
}

void JobQueue::journal_attempt(const AttemptRow& a) {
  if (!jf_) return;
  const char S = '\x1f';
  std::string line = "A";
  for (const std::string* f : {&a.id, &a.job_id, &a.worker_id, &a.status, &a.error, &a.metrics}) {
    line += S;
    line += esc(*f);
  }
  line += S + std::to_string(a.started_at) + S + std::to_string(a.finished_at) + "\n";
  fwrite(line.data(), 1, line.size(), jf_);
  fflush(jf_);
}

void JobQueue::journal_delete(const std::string& id) {
  if (!jf_) return;
  std::string line = "D\x1f" + esc(id) + "\n";
  fwrite(line.data(), 1, line.size(), jf_);
  fflush(jf_);
}

void JobQueue::replay() {
  FILE* f = fopen(path_.c_str(), "r");
  if (!f) return;
  std::string line;
  int c;
  auto apply = [&](const std::string& l) {
    if (l.empty()) return;
    std::vector<std::string> v = split(l);
    if (v[0] == "J" && (v.size() == 20 || v.size() == 21)) {
      JobRow j;
      j.id = v[1]; j.kind = v[2]; j.payload = v[3]; j.source = v[4]; j.status = v[5];
      j.result = v[6]; j.error = v[7]; j.device_id = v[8]; j.model_id = v[9];
      j.worker_id = v[10]; j.lease_token = v[11];
      j.priority = std::stoi(v[12]); j.attempts = std::stoi(v[13]);
      j.max_attempts = std::stoi(v[14]); j.lease_until = std::stoll(v[15]);
      j.deadline_at = std::stoll(v[16]); j.queued_at = std::stoll(v[17]);
      j.updated_at = std::stoll(v[18]); j.seq = std::stoll(v[19]);
      // journals written before the pin field: a placed device counts as a pin
      j.pin_device = v.size() == 21 ? v[20] : j.device_id;
      auto it = jobs_.find(j.id);
      if (it != jobs_.end()) index_erase(it->second);
      jobs_[j.id] = j;
      index_insert(jobs_[j.id]);
      seq_ = std::max(seq_, j.seq + 1);
    } else if (v[0] == "A" && v.size() == 9) {
      AttemptRow a;
      a.id = v[1]; a.job_id = v[2]; a.worker_id = v[3]; a.status = v[4]; a.error = v[5];
      a.metrics = v[6]; a.started_at = std::stoll(v[7]); a.finished_at = std::stoll(v[8]);
      auto& lst = attempts_[a.job_id];
      auto it = std::find_if(lst.begin(), lst.end(), [&](const AttemptRow& x) { return x.id == a.id; });
      if (it != lst.end()) *it = a; else lst.push_back(a);
    } else if (v[0] == "D" && v.size() == 2) {
      auto it = jobs_.find(v[1]);
      if (it != jobs_.end()) { index_erase(it->second); jobs_.erase(it); }
      attempts_.erase(v[1]);
    }
  };
  while ((c = fgetc(f)) != EOF) {
    if (c == '\n') { apply(line); line.clear(); }
    else line += (char)c;
  }
  apply(line);
  fclose(f);
}

void JobQueue::compact() {
  std::lock_guard<std::mutex> g(mu_);
  if (path_.empty()) return;
  const std::string tmp = path_ + ".tmp";
  FILE* old = jf_;
  jf_ = fopen(tmp.c_str(), "w");
  if (!jf_) { jf_ = old; return; }
  for (auto& kv : jobs_) journal(kv.second);
  for (auto& kv : attempts_) for (auto& a : kv.second) journal_attempt(a);
  fclose(jf_);
  if (old) fclose(old);
  std::rename(tmp.c_str(), path_.c_str());
  jf_ = fopen(path_.c_str(), "a");
}

std::string JobQueue::submit(const std::string& kind, const std::string& payload, int priority,
                             const std::string& source, int max_attempts, int64_t deadline_at,
                             const std::string& device_id, const std::string& model_id,
                             int64_t now, const std::string& status, const std::string& forced_id) {
  std::lock_guard<std::mutex> g(mu_);
  JobRow j;
  j.id = forced_id.empty() ? new_id() : forced_id;
  if (jobs_.count(j.id)) throw std::invalid_argument("duplicate job id");
  j.kind = kind;
  j.payload = payload;
  j.priority = priority;
  j.source = source;
  j.status = status;
  j.max_attempts = max_attempts > 0 ? max_attempts : 3;
  j.deadline_at = deadline_at;
  j.device_id = device_id;
  j.pin_device = device_id;
  j.model_id = model_id;
  j.queued_at = now;
  j.updated_at = now;
  j.seq = seq_++;
  jobs_[j.id] = j;
  index_insert(jobs_[j.id]);
  journal(j);
  bump();
  return j.id;
}

bool JobQueue::get(const std::string& id, JobRow* out) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = jobs_.find(id);
  if (it == jobs_.end()) return false;
  *out = it->second;
  return true;
}

bool JobQueue::claim(const std::string& worker_id, const ClaimFilter& f, int64_t lease_ms,
                     int64_t now, JobRow* out, std::string* attempt_id) {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<std::string> to_error_deadline, to_error_attempts;
  JobRow* pick = nullptr;
  for (const ReadyKey& k : claimable_) {
    JobRow& j = jobs_[std::get<3>(k)];
    if (j.status == "running" && j.lease_until >= now) continue;  // leased: SKIP LOCKED
    if (!f.kinds.empty() && std::find(f.kinds.begin(), f.kinds.end(), j.kind) == f.kinds.end())
      continue;
    if (j.deadline_at > 0 && now > j.deadline_at) { to_error_deadline.push_back(j.id); continue; }
    if (j.attempts >= j.max_attempts) { to_error_attempts.push_back(j.id); continue; }
    // only the submitter's pin restricts placement: a requeued or lease-lapsed
    // job goes to any device, not back to the one it failed on
    const std::string& dev = !j.pin_device.empty() ? j.pin_device : f.worker_device;
    if (!j.pin_device.empty() && !f.worker_device.empty() && j.pin_device != f.worker_device)
      continue;  // pinned to another device
    if (!dev.empty()) {
      if (f.check_online && !j.pin_device.empty() && !f.online_devices.count(dev)) continue;
      int limit = f.device_max_concurrency;
      auto li = f.device_limits.find(dev);
      if (li != f.device_limits.end()) limit = li->second;
      if (limit > 0 && live_running(dev, now, j.id) >= limit) continue;
    }
    pick = &j;
    break;
  }
  auto set_error = [&](const std::string& id, const char* msg) {
    JobRow& j = jobs_[id];
    index_erase(j);
    j.status = "error";
    j.error = msg;
    j.lease_until = 0;
    j.lease_token.clear();
    j.updated_at = now;
    index_insert(j);
    journal(j);
  };
  for (auto& id : to_error_deadline) set_error(id, "deadline_exceeded");
  for (auto& id : to_error_attempts) set_error(id, "attempts_exhausted");
  if (!pick) {
    if (!to_error_deadline.empty() || !to_error_attempts.empty()) bump();
    return false;
  }
  JobRow& j = *pick;
  index_erase(j);
  if (j.status == "running" && !j.lease_token.empty()) {
    // previous owner lost its lease: close that attempt
    auto& lst = attempts_[j.id];
    for (auto& a : lst)
      if (a.id == j.lease_token && a.status == "running") {
        a.status = "lease_expired";
        a.finished_at = now;
        journal_attempt(a);
      }
  }
  j.status = "running";
  j.attempts += 1;
  j.lease_until = now + lease_ms;
  j.worker_id = worker_id;
  j.device_id = j.pin_device.empty() ? f.worker_device : j.pin_device;  // placement
  j.lease_token = new_id();
  j.updated_at = now;
  index_insert(j);
  AttemptRow a;
  a.id = j.lease_token;
  a.job_id = j.id;
  a.worker_id = worker_id;
  a.status = "running";
  a.started_at = now;
  attempts_[j.id].push_back(a);
  journal(j);
  journal_attempt(a);
  *out = j;
  *attempt_id = a.id;
  bump();
  return true;
}

static bool owns(const JobRow& j, const std::string& worker_id, const std::string& token) {
  if (j.status != "running") return false;
  if (!token.empty()) return j.lease_token == token;
  return j.worker_id == worker_id;
}

bool JobQueue::heartbeat(const std::string& id, const std::string& worker_id,
                         const std::string& token, int64_t extend_ms, int64_t now) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = jobs_.find(id);
  if (it == jobs_.end() || !owns(it->second, worker_id, token)) return false;
  it->second.lease_until = now + extend_ms;
  it->second.updated_at = now;
  journal(it->second);
  return true;
}

bool JobQueue::complete(const std::string& id, const std::string& worker_id,
                        const std::string& token, const std::string& result,
                        const std::string& metrics, int64_t now) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = jobs_.find(id);
  if (it == jobs_.end() || !owns(it->second, worker_id, token)) return false;
  JobRow& j = it->second;
  const std::string tok = j.lease_token;
  index_erase(j);
  j.status = "done";
  j.result = result;
  j.lease_until = 0;
  j.updated_at = now;
  index_insert(j);
  journal(j);
  for (auto& a : attempts_[id])
    if (a.id == tok) {
      a.status = "done";
      a.finished_at = now;
      a.metrics = metrics;
      journal_attempt(a);
    }
  bump();
  return true;
}

std::string JobQueue::fail(const std::string& id, const std::string& worker_id,
                           const std::string& token, const std::string& error,
                           const std::string& metrics, int64_t now) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = jobs_.find(id);
  if (it == jobs_.end() || !owns(it->second, worker_id, token)) return "";
  JobRow& j = it->second;
  const std::string tok = j.lease_token;
  index_erase(j);
  j.error = error;
  j.lease_until = 0;
  j.lease_token.clear();
  j.updated_at = now;
  j.status = j.attempts < j.max_attempts ? "queued" : "error";
  if (j.status == "queued") j.device_id = j.pin_device;   // placement dropped on requeue
  index_insert(j);
  journal(j);
  for (auto& a : attempts_[id])
    if (a.id == tok) {
      a.status = "error";
      a.error = error;
      a.finished_at = now;
      a.metrics = metrics;
      journal_attempt(a);
    }
  bump();
  return j.status;
}

int JobQueue::release_device(const std::string& device_id, int64_t now) {
  std::lock_guard<std::mutex> g(mu_);
  int n = 0;
  for (auto& kv : jobs_) {
    JobRow& j = kv.second;
    if (j.status == "running" && j.device_id == device_id) {
      j.lease_until = 0;  // reclaimable immediately (offline_handler.go:20-26)
      j.updated_at = now;
      journal(j);
      ++n;
    }
  }
  if (n) bump();
  return n;
}

int JobQueue::expire_deadlines(int64_t now) {
  std::lock_guard<std::mutex> g(mu_);
  int n = 0;
  for (auto& kv : jobs_) {
    JobRow& j = kv.second;
    if ((j.status == "queued" || j.status == "running") && j.deadline_at > 0 &&
        now > j.deadline_at) {
      index_erase(j);
      j.status = "error";
      j.error = "deadline_exceeded";
      j.lease_until = 0;
      j.lease_token.clear();
      j.updated_at = now;
      index_insert(j);
      journal(j);
      ++n;
    }
  }
  if (n) bump();
  return n;
}

int JobQueue::purge_finished(int64_t older_than) {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<std::string> del;
  for (auto& kv : jobs_)
    if ((kv.second.status == "done" || kv.second.status == "error") &&
        kv.second.updated_at < older_than)
      del.push_back(kv.first);
  for (auto& id : del) {
    index_erase(jobs_[id]);
    jobs_.erase(id);
    attempts_.erase(id);
    journal_delete(id);
  }
  if (!del.empty()) bump();
  return (int)del.size();
}

std::map<std::string, int> JobQueue::counts() const {
  std::lock_guard<std::mutex> g(mu_);
  std::map<std::string, int> c{{"queued", 0}, {"running", 0}, {"done", 0}, {"error", 0}};
  for (auto& kv : jobs_) c[kv.second.status]++;
  return c;
}

std::map<std::string, int> JobQueue::kind_counts(const std::string& prefix) const {
  std::lock_guard<std::mutex> g(mu_);
  std::map<std::string, int> c;
  for (auto& kv : jobs_)
    if (kv.second.kind.compare(0, prefix.size(), prefix) == 0) c[kv.second.status]++;
  return c;
}

int JobQueue::active_on(const std::string& device) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = active_per_device_.find(device);
  return it == active_per_device_.end() ? 0 : it->second;
}

// the number after "ms": in a metrics JSON object (-1: absent / not a number)
static double metrics_ms(const std::string& m) {
  const size_t k = m.find("\"ms\"");
  if (k == std::string::npos) return -1;
  size_t i = k + 4;
  while (i < m.size() && (m[i] == ' ' || m[i] == ':')) ++i;
  if (i >= m.size() || !(std::isdigit((unsigned char)m[i]) || m[i] == '-' || m[i] == '.'))
    return -1;
  return std::strtod(m.c_str() + i, nullptr);
}

std::map<std::string, int64_t> JobQueue::device_stats(const std::string& device,
                                                      int64_t since) const {
  std::lock_guard<std::mutex> g(mu_);
  int64_t total = 0, done = 0, ms_n = 0;
  double ms_sum = 0;
  for (auto& kv : jobs_) {
    const JobRow& j = kv.second;
    if (j.device_id != device || j.updated_at < since) continue;
    if (j.status != "done" && j.status != "error") continue;
    ++total;
    if (j.status != "done") continue;
    ++done;
    auto it = attempts_.find(j.id);
    if (it == attempts_.end()) continue;
    for (auto& a : it->second)
      if (a.status == "done") {
        const double ms = metrics_ms(a.metrics);
        if (ms >= 0) { ms_sum += ms; ++ms_n; }
      }
  }
  return {{"total", total}, {"done", done}, {"ms_sum", (int64_t)ms_sum}, {"ms_n", ms_n}};
}

int JobQueue::stuck(int64_t now) const {
  std::lock_guard<std::mutex> g(mu_);
  int n = 0;
  for (auto& kv : jobs_)
    if (kv.second.status == "running" && kv.second.lease_until < now) ++n;
  return n;
}

std::vector<JobRow> JobQueue::list(const std::string& status, int limit) const {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<JobRow> v;
  for (auto& kv : jobs_)
    if (status.empty() || kv.second.status == status) v.push_back(kv.second);
  std::sort(v.begin(), v.end(), [](const JobRow& a, const JobRow& b) {
    return a.updated_at != b.updated_at ? a.updated_at > b.updated_at : a.seq > b.seq;
  });
  if (limit > 0 && (int)v.size() > limit) v.resize(limit);
  return v;
}

std::vector<AttemptRow> JobQueue::attempts(const std::string& job_id) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = attempts_.find(job_id);
  return it == attempts_.end() ? std::vector<AttemptRow>{} : it->second;
}

int JobQueue::running_on(const std::string& device_id, int64_t now) const {
  std::lock_guard<std::mutex> g(mu_);
  return live_running(device_id, now, "");
}

int64_t JobQueue::version() const {
  std::lock_guard<std::mutex> g(mu_);
  return version_;
}

int64_t JobQueue::wait_change(int64_t since, int64_t timeout_ms) {
  std::unique_lock<std::mutex> g(mu_);
  cv_.wait_for(g, std::chrono::milliseconds(timeout_ms), [&] { return version_ != since; });
  return version_;
}

void JobQueue::notify_change() {
  std::lock_guard<std::mutex> g(mu_);
  bump();
}

size_t JobQueue::size() const {
  std::lock_guard<std::mutex> g(mu_);
  return jobs_.size();
}

}  // namespace lmxrt
