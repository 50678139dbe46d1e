// pybind11 bindings of the native runtime (_lmx_runtime).
#include <charconv>
#include <cmath>
#include <string>

#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "block_manager.h"
#include "job_queue.h"
#include "scheduler.h"

namespace py = pybind11;
using namespace lmxrt;

template <typename T>
static py::array_t<T> to_np(const std::vector<T>& v) {
  py::array_t<T> a(v.size());
  if (!v.empty()) std::memcpy(a.mutable_data(), v.data(), v.size() * sizeof(T));
  return a;
}

static py::dict job_dict(const JobRow& j) {
  py::dict d;
  d["id"] = j.id; d["kind"] = j.kind; d["payload"] = j.payload; d["source"] = j.source;
  d["status"] = j.status; d["result"] = j.result; d["error"] = j.error;
  d["device_id"] = j.device_id; d["model_id"] = j.model_id; d["worker_id"] = j.worker_id;
  d["lease_token"] = j.lease_token; d["priority"] = j.priority; d["attempts"] = j.attempts;
  d["max_attempts"] = j.max_attempts; d["lease_until"] = j.lease_until;
  d["deadline_at"] = j.deadline_at; d["queued_at"] = j.queued_at; d["updated_at"] = j.updated_at;
  return d;
}

static py::dict attempt_dict(const AttemptRow& a) {
  py::dict d;
  d["id"] = a.id; d["job_id"] = a.job_id; d["worker_id"] = a.worker_id; d["status"] = a.status;
  d["error"] = a.error; d["metrics"] = a.metrics; d["started_at"] = a.started_at;
  d["finished_at"] = a.finished_at;
  return d;
}

PYBIND11_MODULE(_lmx_runtime, m) {
  m.doc() = "llm_mcp_amd native runtime: lease job queue, KV block manager, batch scheduler";

  py::class_<BlockManager>(m, "BlockManager")
      .def(py::init<int, int, bool>(), py::arg("num_blocks"), py::arg("block_size"),
           py::arg("prefix_cache") = true)
      .def_property_readonly("num_blocks", &BlockManager::num_blocks)
      .def_property_readonly("block_size", &BlockManager::block_size)
      .def_property_readonly("num_free", &BlockManager::num_free)
      .def_property_readonly("usage", &BlockManager::usage)
      .def_property_readonly("prefix_hits", &BlockManager::prefix_hits)
      .def("match_prefix", [](BlockManager& b, int64_t seq, const std::vector<int32_t>& t) {
        return b.match_prefix(seq, t.data(), (int)t.size());
      })
      .def("ensure", &BlockManager::ensure)
      .def("commit", [](BlockManager& b, int64_t seq, const std::vector<int32_t>& t, int n) {
        b.commit(seq, t.data(), n);
      })
      .def("free_seq", &BlockManager::free_seq)
      .def("table", [](const BlockManager& b, int64_t s) { return b.table(s); });

  // /v1/embeddings response bodies: each row of a float32 matrix as a JSON
  // array in shortest round-trip form (std::to_chars), ~10x faster than
  // json.dumps over Python floats, which held the API process at one core
  // (7.4 ms per 16 x 768 response); non-finite values become null
  m.def("f32_json_rows", [](py::array_t<float, py::array::c_style | py::array::forcecast> a) {
    if (a.ndim() != 2) throw std::invalid_argument("f32_json_rows: 2-D array expected");
    auto r = a.unchecked<2>();
    py::list out;
    std::string s;
    char buf[32];
    for (py::ssize_t i = 0; i < r.shape(0); ++i) {
      s.clear();
      s.push_back('[');
      for (py::ssize_t j = 0; j < r.shape(1); ++j) {
        if (j) s.push_back(',');
        const float v = r(i, j);
        if (!std::isfinite(v)) {
          s += "null";
          continue;
        }
        const auto res = std::to_chars(buf, buf + sizeof buf, v);
        s.append(buf, res.ptr);
      }
      s.push_back(']');
      out.append(py::str(s));
    }
    return out;
  });

  py::class_<Scheduler>(m, "Scheduler")
      .def(py::init<int, int, int, int, int, bool>(), py::arg("num_blocks"),
           py::arg("block_size"), py::arg("max_num_seqs"), py::arg("max_batched_tokens"),
           py::arg("max_model_len"), py::arg("prefix_cache") = true)
      .def("add", &Scheduler::add, py::arg("id"), py::arg("prompt"), py::arg("max_new"),
           py::arg("stop_ids"), py::arg("ignore_eos") = false, py::arg("priority") = 0,
           py::arg("temperature") = 1.f, py::arg("top_k") = 0, py::arg("top_p") = 1.f,
           py::arg("seed") = 0)
      .def("abort", &Scheduler::abort)
      .def("set_mixed_prefill_cap", &Scheduler::set_mixed_prefill_cap, py::arg("tokens"),
           py::arg("min_decodes"), py::arg("later_steps") = 0)
      .def_property_readonly("steps", &Scheduler::steps)
      .def("set_penalties", &Scheduler::set_penalties, py::arg("id"), py::arg("repetition"),
           py::arg("presence"), py::arg("frequency"), py::arg("last_n"))
      .def("schedule", [](Scheduler& s, int q_per_tile) {
        const StepPlan& p = s.schedule(q_per_tile);
        py::dict d;
        d["input_ids"] = to_np(p.input_ids);
        d["positions"] = to_np(p.positions);
        d["slots"] = to_np(p.slots);
        d["input_src"] = to_np(p.input_src);
        d["num_pending_inputs"] = p.num_pending_inputs;
        d["seq_ids"] = to_np(p.seq_ids);
        d["qlens"] = to_np(p.qlens);
        d["context_lens"] = to_np(p.context_lens);
        d["cu_q"] = to_np(p.cu_q);
        d["block_tables"] = to_np(p.block_tables);
        d["sample_rows"] = to_np(p.sample_rows);
        d["sample_seq"] = to_np(p.sample_seq);
        d["temp"] = to_np(p.sample_temp);
        d["topk"] = to_np(p.sample_topk);
        d["topp"] = to_np(p.sample_topp);
        d["seeds"] = to_np(p.sample_seed);
        d["offs"] = to_np(p.sample_off);
        d["prefill_tiles"] = to_np(p.prefill_tiles);
        d["any_penalty"] = p.any_penalty;
        if (p.any_penalty) {
          d["pen_window"] = to_np(p.pen_window);
          d["pen_ngen"] = to_np(p.pen_ngen);
          d["pen_params"] = to_np(p.pen_params);
        }
        d["pen_window_len"] = kPenWindow;
        d["num_decode"] = p.num_decode;
        d["max_blocks"] = p.max_blocks;
        d["num_tokens"] = p.num_tokens;
        d["num_prefill_tokens"] = p.num_prefill_tokens;
        d["max_context"] = p.max_context;
        d["preempted"] = p.preempted;
        return d;
      })
      .def("update", [](Scheduler& s, py::array_t<int32_t, py::array::c_style | py::array::forcecast> a) {
        return s.update(a.data(), (int)a.size());
      })
      .def("update_lookahead", &Scheduler::update_lookahead)
      .def("patch", [](Scheduler& s, py::array_t<int32_t, py::array::c_style | py::array::forcecast> a) {
        return s.patch(a.data(), (int)a.size());
      })
      .def_property_readonly("num_inflight_samples", &Scheduler::num_inflight_samples)
      .def("discard_lookahead", &Scheduler::discard_lookahead)
      .def_property_readonly("num_waiting", &Scheduler::num_waiting)
      .def_property_readonly("num_running", &Scheduler::num_running)
      .def_property_readonly("has_work", &Scheduler::has_work)
      .def_property_readonly("preemptions", &Scheduler::preemptions)
      .def_property_readonly("kv_usage", [](Scheduler& s) { return s.blocks().usage(); })
      .def_property_readonly("kv_free_blocks", [](Scheduler& s) { return s.blocks().num_free(); })
      .def_property_readonly("prefix_hits", [](Scheduler& s) { return s.blocks().prefix_hits(); })
      .def("seq_tokens", [](const Scheduler& s, int64_t id) {
        const Seq* q = s.get(id);
        return q ? q->tokens : std::vector<int32_t>{};
      });

  py::class_<JobQueue>(m, "JobQueue")
      .def(py::init<const std::string&>(), py::arg("journal_path") = "")
      .def("submit", &JobQueue::submit, py::arg("kind"), py::arg("payload"), py::arg("priority"),
           py::arg("source"), py::arg("max_attempts"), py::arg("deadline_at"),
           py::arg("device_id"), py::arg("model_id"), py::arg("now"),
           py::arg("status") = "queued", py::arg("forced_id") = "")
      .def("get", [](const JobQueue& q, const std::string& id) -> py::object {
        JobRow j;
        if (!q.get(id, &j)) return py::none();
        return job_dict(j);
      })
      .def("claim", [](JobQueue& q, const std::string& worker, const std::vector<std::string>& kinds,
                       const std::string& worker_device, const std::vector<std::string>& online,
                       bool check_online, int max_conc, const std::map<std::string, int>& limits,
                       int64_t lease_ms, int64_t now) -> py::object {
        ClaimFilter f;
        f.kinds = kinds;
        f.worker_device = worker_device;
        f.online_devices.insert(online.begin(), online.end());
        f.check_online = check_online;
        f.device_max_concurrency = max_conc;
        f.device_limits = limits;
        JobRow j;
        std::string aid;
        bool ok;
        {
          py::gil_scoped_release rel;
          ok = q.claim(worker, f, lease_ms, now, &j, &aid);
        }
        if (!ok) return py::none();
        py::dict d = job_dict(j);
        d["attempt_id"] = aid;
        return d;
      })
      .def("heartbeat", &JobQueue::heartbeat)
      .def("complete", &JobQueue::complete)
      .def("fail", &JobQueue::fail)
      .def("release_device", &JobQueue::release_device)
      .def("expire_deadlines", &JobQueue::expire_deadlines)
      .def("purge_finished", &JobQueue::purge_finished)
      .def("counts", &JobQueue::counts)
      .def("kind_counts", &JobQueue::kind_counts)
      .def("active_on", &JobQueue::active_on, py::call_guard<py::gil_scoped_release>())
      .def("device_stats", &JobQueue::device_stats)
      .def("stuck", &JobQueue::stuck)
      .def("list", [](const JobQueue& q, const std::string& status, int limit) {
        py::list l;
        for (auto& j : q.list(status, limit)) l.append(job_dict(j));
        return l;
      })
      .def("attempts", [](const JobQueue& q, const std::string& id) {
        py::list l;
        for (auto& a : q.attempts(id)) l.append(attempt_dict(a));
        return l;
      })
      .def("running_on", &JobQueue::running_on)
      .def_property_readonly("version", &JobQueue::version)
      .def("wait_change", &JobQueue::wait_change, py::call_guard<py::gil_scoped_release>())
      .def("notify_change", &JobQueue::notify_change)
      .def("compact", &JobQueue::compact)
      .def("__len__", &JobQueue::size);
}
