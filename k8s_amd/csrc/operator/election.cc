#include "election.h"

#include <ctime>
#include <random>
#include <thread>

#include "log.h"

namespace tfop {

std::string now_rfc3339() {
  std::time_t t = std::time(nullptr);
  std::tm tm;
  gmtime_r(&t, &tm);
  char buf[64];
  strftime(buf, sizeof buf, "%Y-%m-%dT%H:%M:%SZ", &tm);
  return buf;
}

Json LeaderElectionRecord::to_json() const {
  Json j = Json::object();
  j["holderIdentity"] = holder_identity;
  j["leaseDurationSeconds"] = lease_duration_seconds;
  j["acquireTime"] = acquire_time;
  j["renewTime"] = renew_time;
  j["leaderTransitions"] = leader_transitions;
  return j;
}

LeaderElectionRecord LeaderElectionRecord::from_json(const Json& j) {
  LeaderElectionRecord r;
  r.holder_identity = get_str(j, "holderIdentity");
  if (const Json* v = j.find("leaseDurationSeconds"); v && v->is_number()) r.lease_duration_seconds = (int)v->as_int();
  r.acquire_time = get_str(j, "acquireTime");
  r.renew_time = get_str(j, "renewTime");
  if (const Json* v = j.find("leaderTransitions"); v && v->is_number()) r.leader_transitions = (int)v->as_int();
  return r;
}

LeaderElector::LeaderElector(KubeApi& api, ElectionConfig cfg) : api_(api), cfg_(std::move(cfg)) {}

std::string LeaderElector::check() const {
  if (cfg_.lease <= cfg_.renew_deadline) return "leaseDuration must be greater than renewDeadline";
  if (cfg_.renew_deadline.count() <= (long)(1.2 * cfg_.retry.count()))
    return "renewDeadline must be greater than retryPeriod*JitterFactor";
  if (cfg_.identity.empty()) return "Lock identity is empty";
  return "";
}

bool LeaderElector::try_acquire_or_renew() {
  const std::string path = core_path(cfg_.ns, "endpoints", cfg_.name);
  const std::string now = now_rfc3339();
  LeaderElectionRecord rec;
  rec.holder_identity = cfg_.identity;
  rec.lease_duration_seconds = (int)(cfg_.lease.count() / 1000);
  rec.acquire_time = now;
  rec.renew_time = now;
  ApiResult g = api_.get(path);
  if (g.not_found()) {
    Json ep = Json::object();
    ep["apiVersion"] = "v1";
    ep["kind"] = "Endpoints";
    Json md = Json::object();
    md["name"] = cfg_.name;
    md["namespace"] = cfg_.ns;
    Json ann = Json::object();
    ann[kLeaderAnnotation] = rec.to_json().dump();
    md["annotations"] = ann;
    ep["metadata"] = md;
    ApiResult c = api_.post(core_path(cfg_.ns, "endpoints"), ep);
    if (!c.ok()) return false;
    observed_ = rec;
    observed_time_ = std::chrono::steady_clock::now();
    return leader_ = true;
  }
  if (!g.ok()) return leader_ = false;
  Json ep = g.body;
  Json& md = ep["metadata"];
  LeaderElectionRecord old;
  if (const Json* ann = md.find("annotations"); ann && ann->find(kLeaderAnnotation)) {
    try {
      old = LeaderElectionRecord::from_json(Json::parse(ann->at(kLeaderAnnotation).as_string()));
    } catch (...) {
    }
  }
  if (old.to_json() != observed_.to_json()) {
    observed_ = old;
    observed_time_ = std::chrono::steady_clock::now();
  }
  const bool held_by_other = !old.holder_identity.empty() && old.holder_identity != cfg_.identity;
  if (held_by_other &&
      observed_time_ + std::chrono::seconds(old.lease_duration_seconds) > std::chrono::steady_clock::now())
    return leader_ = false;
  if (old.holder_identity == cfg_.identity) {
    rec.acquire_time = old.acquire_time;
    rec.leader_transitions = old.leader_transitions;
  } else {
    rec.leader_transitions = old.leader_transitions + 1;
  }
  md["annotations"][kLeaderAnnotation] = rec.to_json().dump();
  ApiResult u = api_.put(path, ep);  // carries metadata.resourceVersion: optimistic CAS
  if (!u.ok()) return leader_ = false;
  observed_ = rec;
  observed_time_ = std::chrono::steady_clock::now();
  return leader_ = true;
}

// resourcelock/endpointslock.go RecordEvent: a Normal "LeaderElection" Event "<identity> <what>" on the
// Endpoints lock (best effort: a failed POST does not affect the election).
void LeaderElector::record_event(const std::string& what) {
  static std::atomic<unsigned> seq{0};
  const std::string now = now_rfc3339();
  Json ev = Json::object();
  ev["apiVersion"] = "v1";
  ev["kind"] = "Event";
  Json md = Json::object();
  md["name"] = cfg_.name + "." + cfg_.identity + "." + std::to_string(std::time(nullptr)) + "." +
               std::to_string(seq++);
  md["namespace"] = cfg_.ns;
  ev["metadata"] = md;
  Json io = Json::object();
  io["kind"] = "Endpoints";
  io["namespace"] = cfg_.ns;
  io["name"] = cfg_.name;
  io["apiVersion"] = "v1";
  ev["involvedObject"] = io;
  ev["reason"] = "LeaderElection";
  ev["message"] = cfg_.identity + " " + what;
  ev["type"] = "Normal";
  ev["firstTimestamp"] = now;
  ev["lastTimestamp"] = now;
  ev["count"] = 1;
  Json src = Json::object();
  src["component"] = "tf-operator";
  ev["source"] = src;
  ApiResult r = api_.post(core_path(cfg_.ns, "events"), ev);
  if (!r.ok()) log_info("could not record leader-election event: %d", r.code);
}

void LeaderElector::run(const std::function<void()>& on_started, const std::function<void()>& on_stopped,
                        const std::atomic<bool>& stop) {
  std::mt19937 rng{std::random_device{}()};
  std::uniform_real_distribution<double> jitter(1.0, 1.2);
  while (!stop && !try_acquire_or_renew())
    std::this_thread::sleep_for(std::chrono::milliseconds((long)(cfg_.retry.count() * jitter(rng))));
  if (stop) return;
  log_info("became leader: %s", cfg_.identity.c_str());
  record_event("became leader");
  std::thread worker(on_started);
  worker.detach();
  auto last_ok = std::chrono::steady_clock::now();
  while (!stop) {
    std::this_thread::sleep_for(cfg_.retry);
    if (try_acquire_or_renew()) {
      last_ok = std::chrono::steady_clock::now();
    } else if (std::chrono::steady_clock::now() - last_ok > cfg_.renew_deadline) {
      log_error("leader election lost");
      break;
    }
  }
  leader_ = false;
  record_event("stopped leading");
  on_stopped();
}

}  // namespace tfop
