#include <random>
#include "controller.h"

#include <cstdlib>
#include <thread>

#include "log.h"

namespace tfop {

Json crd_manifest() {
  const char* text = R"JSON({
  "apiVersion": "apiextensions.k8s.io/v1",
  "kind": "CustomResourceDefinition",
  "metadata": {"name": "tfjobs.tensorflow.org"},
  "spec": {
    "group": "tensorflow.org",
    "scope": "Namespaced",
    "names": {"plural": "tfjobs", "singular": "tfjob", "kind": "TfJob", "shortNames": ["tfj"]},
    "versions": [{
      "name": "v1alpha1", "served": true, "storage": true,
      "schema": {"openAPIV3Schema": {"type": "object", "x-kubernetes-preserve-unknown-fields": true}},
      "additionalPrinterColumns": [
        {"name": "Phase", "type": "string", "jsonPath": ".status.phase"},
        {"name": "State", "type": "string", "jsonPath": ".status.state"},
        {"name": "RuntimeId", "type": "string", "jsonPath": ".spec.RuntimeId"},
        {"name": "Age", "type": "date", "jsonPath": ".metadata.creationTimestamp"}
      ]
    }]
  }
})JSON";
  return Json::parse(text);
}

Controller::Controller(KubeApi& api, ControllerConfig cfg, ControllerOptions opts)
    : api_(api), cfg_(std::move(cfg)), opts_(std::move(opts)) {
  if (opts_.informers) {
    // every replica Job / Pod the operator creates carries the `tensorflow.org` label (replicas.cc Labels)
    InformerOptions io;
    io.watch_timeout = opts_.watch_timeout;
    io.watch_idle_grace = opts_.watch_idle_grace;
    io.resync_period = opts_.resync_period;  // same relist period as the TfJob loop (--resync-period)
    jobs_inf_ = std::make_unique<Informer>(api_, group_path("batch/v1", opts_.ns, "jobs"), "tensorflow.org", io);
    pods_inf_ = std::make_unique<Informer>(api_, core_path(opts_.ns, "pods"), "tensorflow.org", io);
    jobs_inf_->set_on_change([this](const std::string&, const Json& o) { poke_owner(o); });
    pods_inf_->set_on_change([this](const std::string&, const Json& o) { poke_owner(o); });
    opts_.reconcile.jobs_cache = jobs_inf_.get();
    opts_.reconcile.pods_cache = pods_inf_.get();
  }
}

Controller::~Controller() {
  {
    std::lock_guard<std::mutex> g(mu_);
    for (auto& kv : jobs_) kv.second->stop();
  }
  // the informers' callbacks take mu_: stop them before the workers go away
  if (jobs_inf_) jobs_inf_->stop();
  if (pods_inf_) pods_inf_->stop();
  std::lock_guard<std::mutex> g(mu_);
  jobs_.clear();
  retiring_.clear();  // each finishes its requested delete, then joins
}

void Controller::poke_owner(const Json& obj) {
  const Json* m = obj.find("metadata");
  const Json* l = m ? m->find("labels") : nullptr;
  const Json* n = l ? l->find("tf_job_name") : nullptr;
  if (!n || !n->is_string()) return;
  const std::string key = get_str(*m, "namespace") + "/" + n->as_string();
  std::lock_guard<std::mutex> g(mu_);
  auto it = jobs_.find(key);
  if (it != jobs_.end() && !it->second->finished()) it->second->poke();
}

static bool crd_established(const Json& crd) {
  const Json* st = crd.find("status");
  if (!st) return false;
  const Json* conds = st->find("conditions");
  if (!conds || !conds->is_array()) return false;
  for (auto& c : conds->as_array())
    if (get_str(c, "type") == "Established" && get_str(c, "status") == "True") return true;
  return false;
}

std::string Controller::init_resource() {
  if (opts_.create_crd) {
    Json crd = crd_manifest();
    ApiResult r = api_.post(crd_path(), crd);
    if (!r.ok() && !r.already_exists()) return "create CRD: " + r.message();
    const auto deadline = std::chrono::steady_clock::now() + opts_.crd_timeout;
    while (true) {
      ApiResult g = api_.get(crd_path(crd_name()));
      if (g.ok() && crd_established(g.body)) break;
      if (std::chrono::steady_clock::now() > deadline) {
        if (r.ok()) api_.del(crd_path(crd_name()));  // we created it; do not leave a half-initialised CRD
        return "CRD " + crd_name() + " did not become Established";
      }
      std::this_thread::sleep_for(opts_.crd_poll);
    }
  }
  return "";
}

std::string Controller::find_all_jobs(std::string& rv) {
  ApiResult r = api_.get(list_path());
  if (!r.ok()) return "list tfjobs: " + r.message();
  if (const Json* m = r.body.find("metadata")) rv = get_str(*m, "resourceVersion");
  if (const Json* items = r.body.find("items"); items && items->is_array()) {
    for (auto& it : items->as_array()) handle_event("ADDED", it);
  }
  return "";
}

void Controller::handle_event(const std::string& type, const Json& obj) {
  TfJob job;
  try {
    job = tfjob_from_json(obj);
  } catch (const std::exception& e) {
    log_error("bad TfJob object in %s event: %s", type.c_str(), e.what());
    return;
  }
  const std::string key = job.ns() + "/" + job.name();
  std::lock_guard<std::mutex> g(mu_);
  job_rvs_[key] = job.resource_version();
  if (type == "DELETED") {
    auto it = jobs_.find(key);
    if (it != jobs_.end()) it->second->request_delete();
    job_rvs_.erase(key);
    return;
  }
  // Failed jobs are ignored until deleted (controller.go:126-133)
  if (job.status.state == "Failed" && !jobs_.count(key)) return;
  auto it = jobs_.find(key);
  if (it != jobs_.end() && !it->second->finished()) {
    if (job_uids_[key] == job.uid() || job.uid().empty()) {
      if (type == "MODIFIED") it->second->update(job);
      return;
    }
    // same name, new object (deleted and re-created while no watch event reached us): retire the old worker
    log_info("TfJob %s was re-created (uid %s -> %s)", key.c_str(), job_uids_[key].c_str(), job.uid().c_str());
    it->second->request_delete();
    retiring_.push_back(std::move(it->second));  // keeps running its delete; reaped by reap_finished
    jobs_.erase(it);
  }
  if (type == "ADDED" || type == "MODIFIED") {
    log_info("Starting TfJob %s (phase=%s)", key.c_str(), job.status.phase.c_str());
    auto tj = std::make_unique<TrainingJob>(api_, job, cfg_, opts_.reconcile);
    jobs_[key] = std::make_unique<JobWorker>(std::move(tj), opts_.reconcile.interval);
    job_uids_[key] = job.uid();
  }
}

void Controller::reap_finished() {
  std::vector<std::unique_ptr<JobWorker>> done;  // joined after mu_ is released
  {
    std::lock_guard<std::mutex> g(mu_);
    for (auto it = jobs_.begin(); it != jobs_.end();) {
      if (it->second->finished() && !job_rvs_.count(it->first)) {
        job_uids_.erase(it->first);
        done.push_back(std::move(it->second));
        it = jobs_.erase(it);
      } else {
        ++it;
      }
    }
    for (auto it = retiring_.begin(); it != retiring_.end();) {
      if ((*it)->finished()) {
        done.push_back(std::move(*it));
        it = retiring_.erase(it);
      } else {
        ++it;
      }
    }
  }
}

size_t Controller::num_jobs() {
  std::lock_guard<std::mutex> g(mu_);
  return jobs_.size();
}

std::map<std::string, TfJobStatus> Controller::statuses() {
  std::lock_guard<std::mutex> g(mu_);
  std::map<std::string, TfJobStatus> out;
  for (auto& kv : jobs_) out[kv.first] = kv.second->job().status();
  return out;
}

void Controller::watchdog_loop() {
  const long long limit = std::chrono::duration_cast<std::chrono::nanoseconds>(opts_.event_watchdog).count();
  while (!stop_) {
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
    const long long t0 = handler_started_ns_.load();
    if (t0 && std::chrono::steady_clock::now().time_since_epoch().count() - t0 > limit) {
      log_error("panicTimer: handling a TfJob event has taken longer than %lld ms; aborting",
                (long long)opts_.event_watchdog.count());
      std::abort();
    }
  }
}

bool Controller::relist(std::string& rv) {
  std::map<std::string, std::string> before;
  {
    std::lock_guard<std::mutex> g(mu_);
    before = job_rvs_;
  }
  ApiResult l = api_.get(list_path());
  if (!l.ok()) {
    log_warn("relist failed: HTTP %d", l.code);
    return false;
  }
  std::map<std::string, bool> seen;
  if (const Json* items = l.body.find("items"); items && items->is_array())
    for (auto& it : items->as_array()) {
      TfJob j = tfjob_from_json(it);
      seen[j.ns() + "/" + j.name()] = true;
      handle_event("ADDED", it);  // idempotent for a job that already has a worker
    }
  for (auto& kv : before)
    if (!seen.count(kv.first)) {
      std::lock_guard<std::mutex> g(mu_);
      auto jt = jobs_.find(kv.first);
      if (jt != jobs_.end()) jt->second->request_delete();
      job_rvs_.erase(kv.first);
    }
  if (const Json* m = l.body.find("metadata")) rv = get_str(*m, "resourceVersion");
  return true;
}

std::string Controller::run() {
  std::thread watchdog(&Controller::watchdog_loop, this);
  struct Joiner {
    Controller* c;
    std::thread& t;
    ~Joiner() {
      c->stop_ = true;
      t.join();
    }
  } joiner{this, watchdog};
  // initResource with retry (controller.go:86-96)
  while (!stop_) {
    std::string err = init_resource();
    if (err.empty()) break;
    log_error("initResource failed: %s; retrying in %lld ms", err.c_str(), (long long)opts_.init_retry.count());
    for (int i = 0; i < opts_.init_retry.count() / 100 && !stop_; ++i)
      std::this_thread::sleep_for(std::chrono::milliseconds(100));
  }
  if (jobs_inf_) {
    jobs_inf_->start();
    pods_inf_->start();
    // re-adopted jobs read their replicas from the caches from the first tick (a cache that is slow to sync is
    // not waited for: get_status reads the API server until it is)
    jobs_inf_->wait_synced(std::chrono::milliseconds(5000));
    pods_inf_->wait_synced(std::chrono::milliseconds(5000));
  }
  std::string rv;
  while (!stop_) {
    std::string err = find_all_jobs(rv);
    if (err.empty()) break;
    log_error("%s; retrying", err.c_str());
    std::this_thread::sleep_for(std::chrono::seconds(1));
  }
  std::mt19937 rng(std::random_device{}());
  using clock = std::chrono::steady_clock;
  auto last_relist = clock::now();
  while (!stop_) {
    std::string err;
    const long tmin = std::max<long>(1, (long)(opts_.watch_timeout.count() / 1000));
    const long timeout_s = std::uniform_int_distribution<long>(tmin, 2 * tmin - 1 > tmin ? 2 * tmin - 1 : tmin)(rng);
    auto w = api_.watch(list_path() + "?watch=true&resourceVersion=" + rv + "&timeoutSeconds=" +
                            std::to_string(timeout_s), err);
    if (!w) {
      log_warn("watch failed: %s; retrying", err.c_str());
      std::this_thread::sleep_for(std::chrono::seconds(1));
      continue;
    }
    // the server ends this watch after timeout_s; still open past the grace = nobody is on the other end
    const auto dead_after = clock::now() + std::chrono::seconds(timeout_s) + opts_.watch_idle_grace;
    while (!stop_) {
      if (clock::now() > dead_after) {
        log_warn("watch open %lds past its timeoutSeconds=%ld: half-open connection, re-watching from rv=%s",
                 (long)(opts_.watch_idle_grace.count() / 1000), timeout_s, rv.c_str());
        break;
      }
      if (opts_.resync_period.count() > 0 && clock::now() - last_relist > opts_.resync_period) {
        last_relist = clock::now();
        log_v(1, "periodic resync: relisting TfJobs");
        if (relist(rv)) break;  // re-watch from the list's resourceVersion
      }
      Json ev;
      if (!w->next(ev, 1000, err)) {
        log_v(1, "watch stream ended: %s; re-watching from %s", err.c_str(), rv.c_str());
        break;
      }
      reap_finished();
      if (ev.is_null()) continue;  // timeout tick
      const std::string type = get_str(ev, "type");
      const Json* obj = ev.find("object");
      if (type == "ERROR") {
        const int code = obj ? (int)(obj->find("code") ? obj->at("code").as_int() : 0) : 0;
        if (code == 410) {
          // resourceVersion too old: relist and diff (removed jobs are deleted, new ones started)
          log_warn("watch 410 Gone at rv=%s: relisting", rv.c_str());
          relist(rv);
          last_relist = clock::now();
          break;
        }
        log_error("watch ERROR event: %s", obj ? obj->dump().c_str() : "");
        break;
      }
      if (!obj) continue;
      if (const Json* m = obj->find("metadata")) rv = get_str(*m, "resourceVersion");
      // panicTimer: armed while the handler runs; the watchdog thread aborts a wedged handler
      handler_started_ns_ = std::chrono::steady_clock::now().time_since_epoch().count();
      if (opts_.inject_handler_stall.count() > 0) std::this_thread::sleep_for(opts_.inject_handler_stall);
      handle_event(type, *obj);
      handler_started_ns_ = 0;
    }
    w->close();
  }
  return "";
}

}  // namespace tfop
