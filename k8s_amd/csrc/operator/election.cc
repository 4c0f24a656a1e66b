#include <vector>
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

// MicroTime as the Lease API wants it (RFC3339 with microseconds)
static std::string now_micro() {
  using namespace std::chrono;
  const auto t = system_clock::now();
  const std::time_t s = system_clock::to_time_t(t);
  const long us = (long)(duration_cast<microseconds>(t.time_since_epoch()).count() % 1000000);
  std::tm tm;
  gmtime_r(&s, &tm);
  char buf[64];
  strftime(buf, sizeof buf, "%Y-%m-%dT%H:%M:%S", &tm);
  char out[96];
  snprintf(out, sizeof out, "%s.%06ldZ", buf, us);
  return out;
}

// Lock object <-> record. Endpoints: JSON in the leader annotation. Lease: the spec fields.
static LeaderElectionRecord record_of(const Json& obj, bool lease) {
  LeaderElectionRecord r;
  if (lease) {
    const Json* sp = obj.find("spec");
    if (!sp) return r;
    r.holder_identity = get_str(*sp, "holderIdentity");
    if (const Json* v = sp->find("leaseDurationSeconds"); v && v->is_number()) r.lease_duration_seconds = (int)v->as_int();
    r.acquire_time = get_str(*sp, "acquireTime");
    r.renew_time = get_str(*sp, "renewTime");
    if (const Json* v = sp->find("leaseTransitions"); v && v->is_number()) r.leader_transitions = (int)v->as_int();
    return r;
  }
  const Json* md = obj.find("metadata");
  if (md)
    if (const Json* ann = md->find("annotations"); ann && ann->find(kLeaderAnnotation)) {
      try {
        r = LeaderElectionRecord::from_json(Json::parse(ann->at(kLeaderAnnotation).as_string()));
      } catch (...) {
      }
    }
  return r;
}

static void store_record(Json& obj, const LeaderElectionRecord& rec, bool lease) {
  if (lease) {
    Json sp = Json::object();
    sp["holderIdentity"] = rec.holder_identity;
    sp["leaseDurationSeconds"] = rec.lease_duration_seconds;
    sp["acquireTime"] = rec.acquire_time;
    sp["renewTime"] = rec.renew_time;
    sp["leaseTransitions"] = rec.leader_transitions;
    obj["spec"] = sp;
  } else {
    obj["metadata"]["annotations"][kLeaderAnnotation] = rec.to_json().dump();
  }
}

bool LeaderElector::try_acquire_or_renew(int timeout_ms) {
  // lock objects this elector holds: the Lease, the Endpoints annotation, or both (client-go's
  // "endpointsleases" MultiLock: an operator that takes BOTH is mutually exclusive with an older operator that
  // only knows either one, so a rolling upgrade from an Endpoints-lock or a Lease-lock release cannot produce two
  // leaders)
  std::vector<bool> kinds;
  if (cfg_.lock_type == "endpoints") kinds = {false};
  else if (cfg_.lock_type == "leases") kinds = {true};
  else kinds = {false, true};
  RequestTimeout bound(timeout_ms);  // every API call below gives up by the caller's deadline
  struct Held {
    bool lease;
    std::string coll, path;
    ApiResult got;
    LeaderElectionRecord old;
  };
  std::vector<Held> locks;
  const auto now_steady = std::chrono::steady_clock::now();
  for (bool lease : kinds) {
    Held h;
    h.lease = lease;
    h.coll = lease ? group_path("coordination.k8s.io/v1", cfg_.ns, "leases") : core_path(cfg_.ns, "endpoints");
    h.path = h.coll + "/" + cfg_.name;
    h.got = api_.get(h.path);
    if (!h.got.ok() && !h.got.not_found()) return leader_ = false;
    if (h.got.ok()) h.old = record_of(h.got.body, lease);
    LeaderElectionRecord& seen = lease ? observed_lease_ : observed_;
    auto& seen_time = lease ? observed_lease_time_ : observed_time_;
    if (h.old.to_json() != seen.to_json()) {
      seen = h.old;
      seen_time = now_steady;
    }
    // the lease is judged by OUR clock since we last saw the record change (election.go:232-236), never by
    // the holder's timestamps: no clock-skew assumptions between replicas
    const bool held_by_other = !h.old.holder_identity.empty() && h.old.holder_identity != cfg_.identity;
    if (held_by_other && seen_time + std::chrono::seconds(h.old.lease_duration_seconds) > now_steady)
      return leader_ = false;
    locks.push_back(std::move(h));
  }
  for (auto& h : locks) {
    const std::string now = h.lease ? now_micro() : now_rfc3339();
    LeaderElectionRecord rec;
    rec.holder_identity = cfg_.identity;
    rec.lease_duration_seconds = std::max(1, (int)(cfg_.lease.count() / 1000));
    rec.acquire_time = now;
    rec.renew_time = now;
    if (h.got.not_found()) {
      Json obj = Json::object();
      obj["apiVersion"] = h.lease ? "coordination.k8s.io/v1" : "v1";
      obj["kind"] = h.lease ? "Lease" : "Endpoints";
      Json md = Json::object();
      md["name"] = cfg_.name;
      md["namespace"] = cfg_.ns;
      if (!h.lease) md["annotations"] = Json::object();
      obj["metadata"] = md;
      store_record(obj, rec, h.lease);
      if (!api_.post(h.coll, obj).ok()) return leader_ = false;
    } else {
      if (h.old.holder_identity == cfg_.identity) {
        rec.acquire_time = h.old.acquire_time;
        rec.leader_transitions = h.old.leader_transitions;
      } else {
        rec.leader_transitions = h.old.leader_transitions + 1;
      }
      Json obj = h.got.body;
      if (!h.lease && !obj["metadata"].find("annotations")) obj["metadata"]["annotations"] = Json::object();
      store_record(obj, rec, h.lease);
      if (!api_.put(h.path, obj).ok()) return leader_ = false;  // carries resourceVersion: optimistic CAS
    }
    (h.lease ? observed_lease_ : observed_) = rec;
    (h.lease ? observed_lease_time_ : observed_time_) = std::chrono::steady_clock::now();
  }
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
  io["kind"] = cfg_.lock_type == "leases" ? "Lease" : "Endpoints";
  io["namespace"] = cfg_.ns;
  io["name"] = cfg_.name;
  io["apiVersion"] = cfg_.lock_type == "leases" ? "coordination.k8s.io/v1" : "v1";
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
  // acquire: every attempt bounded by the retry period, then JitterUntil's sleep (election.go:175-189)
  while (!stop && !try_acquire_or_renew((int)cfg_.retry.count()))
    std::this_thread::sleep_for(std::chrono::milliseconds((long)(cfg_.retry.count() * jitter(rng))));
  if (stop) return;
  log_info("became leader: %s", cfg_.identity.c_str());
  record_event("became leader");
  std::thread worker(on_started);
  worker.detach();
  // renew: Poll(retry) until RenewDeadline passes without a successful renewal (election.go:192-208). Each
  // attempt's API calls are bounded by the time left before that deadline, so a stalled API server makes the
  // leader give up at renew_deadline -- strictly before a standby may take the lease (lease > renew_deadline).
  auto last_ok = std::chrono::steady_clock::now();
  while (!stop) {
    std::this_thread::sleep_for(cfg_.retry);
    const auto left = std::chrono::duration_cast<std::chrono::milliseconds>(
        last_ok + cfg_.renew_deadline - std::chrono::steady_clock::now());
    if (left.count() > 0 && try_acquire_or_renew((int)left.count())) {
      last_ok = std::chrono::steady_clock::now();
    } else if (std::chrono::steady_clock::now() - last_ok >= cfg_.renew_deadline) {
      log_error("leader election lost: no renewal within the %lld ms renew deadline",
                (long long)cfg_.renew_deadline.count());
      break;
    }
  }
  leader_ = false;
  {
    RequestTimeout bound(1000);  // best effort: the API server may be the reason we lost the lease
    record_event("stopped leading");
  }
  on_stopped();
}

}  // namespace tfop
