#include "reconciler.h"

#include <random>

#include "election.h"
#include "log.h"

namespace tfop {

std::string rand_string(int n) {
  static const char* letters = "0123456789abcdefghijklmnopqrstuvwxyz";
  static thread_local std::mt19937_64 rng{std::random_device{}() ^
                                          (uint64_t)std::chrono::steady_clock::now().time_since_epoch().count()};
  std::string s;
  for (int i = 0; i < n; ++i) s += letters[rng() % 36];
  return s;
}

TrainingJob::TrainingJob(KubeApi& api, TfJob job, ControllerConfig cfg, ReconcileOptions opts)
    : api_(api), job_(std::move(job)), cfg_(std::move(cfg)), opts_(std::move(opts)) {
  status_ = job_.status;
}

ApiResult TrainingJob::call(const std::string& method, const std::string& path, const Json* body) {
  ++api_calls_;
  return api_.request(method, path, body);
}

std::string TrainingJob::chief_type() const {
  if (job_.spec.termination_policy && job_.spec.termination_policy->chief)
    return job_.spec.termination_policy->chief->replica_name;
  return "MASTER";
}

std::string TrainingJob::build_replica_sets() {
  replicas_.clear();
  for (auto& r : job_.spec.replica_specs) {
    // NewTFReplicaSet validation (replicas.go:55-88)
    if (r.type == "MASTER" && r.replicas.value_or(1) != 1) return "The MASTER must have Replicas = 1";
    if (!r.tf_port) return "tfReplicaSpec.TfPort can't be nil.";
    if (!r.tmpl && r.type != "PS") return "tfReplicaSpec.Template can't be nil for replica type " + r.type + ".";
    if (replica_type_from(r.type) == ReplicaType::INVALID)
      return "tfReplicaSpec.TfReplicaType is " + r.type + " but must be one of [MASTER PS WORKER]";
    replicas_.push_back(r);
  }
  tensorboard_ = false;
  if (job_.spec.tensorboard) {
    if (job_.spec.tensorboard->log_dir.empty()) return "tbReplicaSpec.LogDir must be specified";
    tensorboard_ = true;
  }
  return "";
}

void TrainingJob::setup() {
  std::string err;
  if (status_.phase.empty()) {
    err = set_defaults(job_.spec);
    if (!err.empty()) err = "there was a problem setting defaults for job spec: " + err;
    if (err.empty()) {
      err = validate(job_.spec);
      if (!err.empty()) err = "invalid job spec: " + err;
    }
    if (err.empty()) err = build_replica_sets();
    if (err.empty()) {
      err = configure_accelerators(job_.spec, cfg_.accelerators);
      if (!err.empty()) err = "ConfigureAccelerators(...) error; " + err;
      else err = build_replica_sets();  // pick up the injected volumes/env
    }
    if (err.empty() && job_.spec.runtime_id.empty()) job_.spec.runtime_id = rand_string(4);
    if (!err.empty()) {
      status_.reason = err;
      status_.phase = "Failed";
      status_.state = "Failed";
      setup_ok_ = false;
      record_event("Warning", "Failed", "TfJob " + job_.name() + " cannot run: " + err);
    } else {
      status_.phase = "Creating";
      status_.state = "Running";
      status_.append_condition("Creating", "replica resources are being created");
      setup_ok_ = true;
      record_event("Normal", "Created", "Creating the replica resources of TfJob " + job_.name() + " (RuntimeId " +
                                            job_.spec.runtime_id + ")");
    }
    return;
  }
  // Q1: re-adopted job (phase already set): rebuild from the persisted, already-defaulted spec
  if (status_.phase != "Failed") {
    err = build_replica_sets();
    setup_ok_ = err.empty();
    if (!err.empty()) log_warn("job %s: cannot rebuild replica sets: %s", key().c_str(), err.c_str());
  }
}

bool TrainingJob::create_if_absent(const std::string& collection, const std::string& name, const Json& obj,
                                   bool* created) {
  const std::string k = collection + "/" + name;
  if (created) *created = false;
  if (existing_.count(k)) return true;
  ApiResult r = call("POST", collection, &obj);
  if (r.ok()) {
    existing_.insert(k);
    if (created) *created = true;
    log_info("Created %s", k.c_str());
    return true;
  }
  if (r.already_exists()) {
    existing_.insert(k);
    return true;
  }
  log_error("Creating %s returned error: %s", k.c_str(), r.message().c_str());
  return false;
}

void TrainingJob::create_resources() {
  const std::string ns = job_.ns();
  const ClusterSpec cs = cluster_spec(job_);
  bool all = true;
  for (auto& r : replicas_) {
    if (r.is_default_ps) {
      all &= create_if_absent(core_path(ns, "configmaps"), default_ps_configmap_name(job_),
                              make_ps_configmap(job_, opts_.ps_server_source), nullptr);
    }
    const int n = r.replicas.value_or(1);
    for (int i = 0; i < n; ++i) {
      const std::string name = replica_job_name(job_, r.type, i);
      all &= create_if_absent(core_path(ns, "services"), name, make_replica_service(job_, r, i), nullptr);
      all &= create_if_absent(group_path("batch/v1", ns, "jobs"), name,
                              make_replica_job(job_, r, i, cs, opts_.ps_script_path), nullptr);
    }
  }
  if (tensorboard_) {
    all &= create_if_absent(core_path(ns, "services"), tb_name(job_), make_tb_service(job_), nullptr);
    all &= create_if_absent(group_path("apps/v1", ns, "deployments"), tb_name(job_), make_tb_deployment(job_),
                            nullptr);
  }
  if (all && status_.phase == "Creating") {
    status_.phase = "Running";
    status_.append_condition("Running", "all replica resources created");
    record_event("Normal", "Running", "All replica resources of TfJob " + job_.name() + " exist");
  }
}

void TrainingJob::get_status(std::string& state, std::vector<TfReplicaStatus>& out) {
  const std::string ns = job_.ns();
  // the caches count only once synced (a reconcile racing the operator's start reads the API server)
  // a cache that is not fresh (its watch keeps failing and no list succeeded lately) is bypassed: direct GET / LIST
  const Informer* jobs_cache = opts_.jobs_cache && opts_.jobs_cache->fresh() ? opts_.jobs_cache : nullptr;
  const Informer* pods_cache = opts_.pods_cache && opts_.pods_cache->fresh() ? opts_.pods_cache : nullptr;
  out.clear();
  for (auto& r : replicas_) {
    TfReplicaStatus st;
    st.type = r.type;
    st.state = "Unknown";
    const int n = r.replicas.value_or(1);
    for (int i = 0; i < n; ++i) {
      const std::string name = replica_job_name(job_, r.type, i);
      Json jobj;
      if (jobs_cache && jobs_cache->get(ns, name, jobj)) {
        ++cache_reads_;
      } else {  // no cache, or not in it yet: ask the API server
        ApiResult jr = call("GET", group_path("batch/v1", ns, "jobs", name));
        if (!jr.ok()) {
          if (jr.not_found()) existing_.erase(group_path("batch/v1", ns, "jobs") + "/" + name);  // recreate
          st.replicas_states["Unknown"]++;
          continue;
        }
        jobj = jr.body;
      }
      const Json* js = jobj.find("status");
      if (js && js->find("succeeded") && js->at("succeeded").is_number() && js->at("succeeded").as_int() >= 1) {
        st.replicas_states["Succeeded"]++;
        continue;
      }
      const Labels tl = task_labels(job_, r.type, i);
      if (pods_cache) {
        ++cache_reads_;
        st.replicas_states[replica_state_from_pods(pods_cache->list(ns, tl), kTensorflowContainer)]++;
        continue;
      }
      ApiResult pl = call("GET", core_path(ns, "pods") + "?labelSelector=" + url_escape(selector_string(tl)));
      if (!pl.ok()) {
        st.replicas_states["Unknown"]++;  // Q6: transient API error is not a failure
        continue;
      }
      const Json* items = pl.body.find("items");
      st.replicas_states[replica_state_from_pods(items ? *items : Json::array(), kTensorflowContainer)]++;
    }
    st.state = aggregate_replica_states(st.replicas_states, n);
    out.push_back(st);
  }
  state = job_state_from_replicas(out, chief_type());
}

bool TrainingJob::update_status() {
  TfJob want = job_;
  want.metadata = job_.metadata.clone();
  want.status = status_;
  if (tfjob_to_json(want) == tfjob_to_json(job_)) return true;
  for (int attempt = 0; attempt < 5; ++attempt) {
    Json body = tfjob_to_json(want);
    ApiResult r = call("PUT", tfjobs_path(job_.ns(), job_.name()), &body);
    if (r.ok()) {
      job_ = tfjob_from_json(r.body);
      return true;
    }
    if (r.conflict()) {  // Q3: re-GET, keep our spec edits and status, retry
      ApiResult g = call("GET", tfjobs_path(job_.ns(), job_.name()));
      if (!g.ok()) return false;
      TfJob cur = tfjob_from_json(g.body);
      if (!job_.uid().empty() && cur.uid() != job_.uid()) {
        // the name now belongs to a re-created object: never write this (old) job's spec / status onto it
        log_warn("Job %s: uid changed (%s -> %s); dropping the status write of the old object", key().c_str(),
                 job_.uid().c_str(), cur.uid().c_str());
        return false;
      }
      want.metadata = cur.metadata.clone();
      continue;
    }
    log_warn("Job %s: failed to update TfJob status: %s", key().c_str(), r.message().c_str());
    return false;
  }
  return false;
}

void TrainingJob::record_event(const std::string& type, const std::string& reason, const std::string& message) {
  const std::string ev_key = reason + "\n" + message;
  const std::string now = now_rfc3339();
  const std::string ns = job_.ns();
  auto it = events_.find(ev_key);
  if (it != events_.end()) {  // seen before: count + 1 on the stored object (carries its resourceVersion)
    Json ev = it->second.clone();
    ev["count"] = (long long)(ev.find("count") && ev.at("count").is_number() ? ev.at("count").as_int() : 1) + 1;
    ev["lastTimestamp"] = now;
    const std::string name = ev.find("metadata") ? get_str(ev.at("metadata"), "name") : "";
    ApiResult r = call("PUT", core_path(ns, "events", name), &ev);
    if (r.ok()) it->second = r.body;
    else log_v(1, "job %s: could not update event %s: HTTP %d", key().c_str(), name.c_str(), r.code);
    return;
  }
  Json ev = Json::object();
  ev["apiVersion"] = "v1";
  ev["kind"] = "Event";
  Json md = Json::object();
  md["name"] = job_.name() + "." + rand_string(8);  // kubectl-style <object>.<unique suffix>
  md["namespace"] = ns;
  ev["metadata"] = md;
  Json io = Json::object();
  io["apiVersion"] = "tensorflow.org/v1alpha1";
  io["kind"] = "TfJob";
  io["name"] = job_.name();
  io["namespace"] = ns;
  if (!job_.uid().empty()) io["uid"] = job_.uid();
  ev["involvedObject"] = io;
  ev["type"] = type;
  ev["reason"] = reason;
  ev["message"] = message;
  ev["firstTimestamp"] = now;
  ev["lastTimestamp"] = now;
  ev["count"] = 1;
  Json src = Json::object();
  src["component"] = "tf-operator";
  ev["source"] = src;
  ApiResult r = call("POST", core_path(ns, "events"), &ev);
  if (r.ok()) events_[ev_key] = r.body.is_object() ? r.body : ev;
  else log_v(1, "job %s: could not record event %s: HTTP %d", this->key().c_str(), reason.c_str(), r.code);
}

// Phase / state transitions are recorded as Events where they happen (README.md:466-476 phases and states):
// Created (setup done, resources being created), Running (every replica resource exists), Succeeded / Failed (the
// chief's outcome, or a spec that cannot run)
void TrainingJob::reconcile() { reconcile_once(); }

void TrainingJob::reconcile_once() {
  if (status_.phase.empty() || !setup_ok_) {
    const bool first = status_.phase.empty();
    setup();
    if (first) update_status();
  }
  if (setup_ok_ && (status_.phase == "Creating" || status_.phase == "Running")) {
    create_resources();
    std::string state;
    std::vector<TfReplicaStatus> rs;
    get_status(state, rs);
    status_.replica_statuses = rs;
    status_.replica_statuses_null = false;
    if (state == "Failed") {
      log_error("Master failed Job: %s.", job_.name().c_str());
      status_.phase = "Done";
      status_.state = "Failed";
      status_.append_condition("Done", "chief replica failed");
      record_event("Warning", "Failed", "TfJob " + job_.name() + " failed: the " + chief_type() + " replica failed");
    } else if (state == "Succeeded") {
      log_info("Master succeeded Job: %s.", job_.name().c_str());
      status_.phase = "Done";
      status_.state = "Succeeded";
      status_.append_condition("Done", "chief replica succeeded");
      record_event("Normal", "Succeeded", "TfJob " + job_.name() + " succeeded: the " + chief_type() +
                                              " replica exited 0");
    }
  }
  update_status();
}

void TrainingJob::update_object(const TfJob& j) {
  // keep our own status as the source of truth; adopt the newer metadata (resourceVersion)
  job_.metadata = j.metadata.clone();
}

void TrainingJob::delete_resources() {
  const std::string ns = job_.ns();
  if (replicas_.empty() && !job_.spec.replica_specs.empty()) build_replica_sets();
  bool failures = false;
  Json opts = Json::object();
  opts["kind"] = "DeleteOptions";
  opts["apiVersion"] = "v1";
  opts["propagationPolicy"] = "Background";
  for (auto& r : replicas_) {
    const std::string sel = url_escape(selector_string(replica_labels(job_, r.type)));
    ApiResult a = call("DELETE", group_path("batch/v1", ns, "jobs") + "?labelSelector=" + sel, &opts);
    if (!a.ok() && !a.not_found()) failures = true;
    ApiResult b = call("DELETE", core_path(ns, "pods") + "?labelSelector=" + sel);
    if (!b.ok() && !b.not_found()) failures = true;
    const int n = r.replicas.value_or(1);
    for (int i = 0; i < n; ++i) {
      ApiResult c = call("DELETE", core_path(ns, "services", replica_job_name(job_, r.type, i)));
      if (!c.ok() && !c.not_found()) failures = true;
    }
    if (r.is_default_ps) call("DELETE", core_path(ns, "configmaps", default_ps_configmap_name(job_)));
  }
  if (tensorboard_) {
    Json fg = Json::object();
    fg["propagationPolicy"] = "Foreground";
    call("DELETE", group_path("apps/v1", ns, "deployments", tb_name(job_)), &fg);
    call("DELETE", core_path(ns, "services", tb_name(job_)));
  }
  existing_.clear();
  if (failures) log_error("Job %s: some of the replicas resources could not be deleted", key().c_str());
}

// ------------------------------------------------------------------ worker thread
JobWorker::JobWorker(std::unique_ptr<TrainingJob> job, std::chrono::milliseconds interval)
    : job_(std::move(job)), interval_(interval) {
  th_ = std::thread([this] { run(); });
}

JobWorker::~JobWorker() {
  stop();
  if (th_.joinable()) th_.join();
}

void JobWorker::poke() {
  std::lock_guard<std::mutex> g(mu_);
  poked_ = true;
  cv_.notify_all();
}

void JobWorker::request_delete() {
  std::lock_guard<std::mutex> g(mu_);
  deleted_ = true;
  cv_.notify_all();
}

void JobWorker::update(const TfJob& j) {
  std::lock_guard<std::mutex> g(mu_);
  // metadata refresh only (resourceVersion); MODIFIED events caused by our own status writes must not
  // trigger a reconcile storm -- spec edits are ignored like the reference (controller.go:154-159)
  pending_update_ = std::make_unique<TfJob>(j);
}

void JobWorker::stop() {
  std::lock_guard<std::mutex> g(mu_);
  stop_ = true;
  cv_.notify_all();
}

void JobWorker::run() {
  try {
    job_->reconcile();
    while (true) {
      std::unique_ptr<TfJob> upd;
      bool del = false;
      {
        std::unique_lock<std::mutex> lk(mu_);
        // system_clock deadline: libstdc++ maps steady_clock waits to pthread_cond_clockwait, which GCC 11's
        // ThreadSanitizer does not intercept (it then misreports the mutex as double-locked); a wall-clock
        // jump only moves one resync tick
        cv_.wait_until(lk, std::chrono::system_clock::now() + interval_, [&] { return poked_ || deleted_ || stop_; });
        del = deleted_;  // a requested delete is carried out even when a stop arrives with it (retired workers)
        if (stop_ && !del) break;
        poked_ = false;
        upd.swap(pending_update_);
      }
      if (del) {
        log_info("TfJob %s deleted by the user", job_->key().c_str());
        job_->delete_resources();
        break;
      }
      if (upd) job_->update_object(*upd);
      job_->reconcile();
    }
  } catch (const std::exception& e) {
    log_error("job %s worker crashed: %s", job_->key().c_str(), e.what());
  }
  finished_ = true;
}

}  // namespace tfop
