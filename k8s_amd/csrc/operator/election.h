// Leader election for operator HA.
//
// Parity: /root/reference/pkg/util/k8sutil/election/election.go (acquire /
// renew / tryAcquireOrRenew :141-265, lease > renew > 1.2 x retry check
// :73-86, renew Poll until RenewDeadline :192-208) and resourcelock/
// endpointslock.go + interface.go (record stored as JSON in the Endpoints
// annotation control-plane.alpha.kubernetes.io/leader; that record format is
// unchanged). Added: a coordination.k8s.io/v1 Lease lock, the default
// "endpointsleases" multi-lock that takes and renews BOTH objects (client-go's
// migration lock: mutually exclusive with an operator that only knows the
// Endpoints lock -- the reference, round 1 -- or only the Lease, so a rolling
// upgrade cannot run two leaders), and renews whose API calls are bounded by
// the time left before the renew deadline, so a hung API server cannot keep a
// leader that can no longer renew (no split brain: the standby only acquires
// after a full lease duration without renewals).
#pragma once

#include <atomic>
#include <chrono>
#include <functional>
#include <string>

#include "kube_api.h"

namespace tfop {

constexpr const char* kLeaderAnnotation = "control-plane.alpha.kubernetes.io/leader";

struct LeaderElectionRecord {
  std::string holder_identity;
  int lease_duration_seconds = 0;
  std::string acquire_time, renew_time;  // RFC3339
  int leader_transitions = 0;
  Json to_json() const;
  static LeaderElectionRecord from_json(const Json& j);
};

struct ElectionConfig {
  std::string ns, name, identity;
  std::chrono::milliseconds lease{15000}, renew_deadline{5000}, retry{3000};
  // "endpointsleases" (both locks, the default), "leases" (coordination.k8s.io/v1 Lease only) or "endpoints"
  // (the reference's Endpoints annotation lock, pkg/util/k8sutil/election/resourcelock/endpointslock.go)
  std::string lock_type = "endpointsleases";
};

class LeaderElector {
 public:
  LeaderElector(KubeApi& api, ElectionConfig cfg);
  // error text if the durations are inconsistent (lease > renew > 1.2*retry)
  std::string check() const;
  // one acquire/renew attempt, every API call bounded by timeout_ms (-1: the client default); true if we hold
  // the lock afterwards
  bool try_acquire_or_renew(int timeout_ms = -1);
  // Blocks: acquire, run on_started (in this thread's caller's stead: a separate thread), renew until lost.
  // Returns when leadership is lost or stop is set.
  void run(const std::function<void()>& on_started, const std::function<void()>& on_stopped,
           const std::atomic<bool>& stop);
  bool is_leader() const { return leader_; }
  void record_event(const std::string& what);

 private:
  KubeApi& api_;
  ElectionConfig cfg_;
  LeaderElectionRecord observed_;  // the Endpoints record (or the only lock's)
  std::chrono::steady_clock::time_point observed_time_;
  LeaderElectionRecord observed_lease_;  // the Lease record
  std::chrono::steady_clock::time_point observed_lease_time_;
  bool leader_ = false;
};

std::string now_rfc3339();

}  // namespace tfop
