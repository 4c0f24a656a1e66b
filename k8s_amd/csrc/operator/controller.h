// TfJob controller: CRD registration, list + re-adopt, watch, dispatch.
//
// Parity: /root/reference/pkg/controller/controller.go (Run :80-121,
// handleTfJobEvent :123-170, findAllTfJobs :172-201, initResource/createCRD
// :213-286, watch + 410 relist :292-376) and pkg/controller/util.go
// (pollEvent, panicTimer watchdog).
//
// Differences by design: CRD is apiextensions.k8s.io/v1 (v1beta1 is gone
// since K8s 1.22); jobs are keyed by namespace/name everywhere (Q4/Q5 fix);
// a 410 Gone relists and diffs instead of tearing the controller down.
#pragma once

#include <atomic>
#include <chrono>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "kube_api.h"
#include "reconciler.h"
#include "spec.h"

namespace tfop {

struct ControllerOptions {
  std::string ns;               // namespace to manage ("" = all namespaces)
  ReconcileOptions reconcile;   // per-job options (interval, PS server)
  std::chrono::milliseconds init_retry{30000};
  std::chrono::milliseconds crd_poll{500};
  std::chrono::milliseconds crd_timeout{60000};
  std::chrono::milliseconds event_watchdog{60000};  // panicTimer: abort if one event takes longer
  std::chrono::milliseconds inject_handler_stall{0};  // fault injection: every event handler sleeps this long
  bool create_crd = true;
  // Watch liveness (controller.go:292-361 re-watches on EOF; client-go's reflector asks the server to end every
  // watch after a random 5-10 min timeoutSeconds). Each watch asks for timeoutSeconds in [watch_timeout,
  // 2 * watch_timeout); a stream still open watch_idle_grace after that is a half-open connection (dropped by a
  // NAT / load balancer without a FIN) and is closed and re-established from the last resourceVersion.
  std::chrono::milliseconds watch_timeout{300000};
  std::chrono::milliseconds watch_idle_grace{30000};
  // full relist + diff (the 410 path) this often, so an event lost anywhere is still picked up (0 = off)
  std::chrono::milliseconds resync_period{300000};
  // shared watch caches of the replica Jobs / Pods (informer.h): reconcile ticks read them instead of per-replica
  // GET / LIST requests, and a change to a job's Job or Pod pokes its worker at once. false: the reference's
  // polling reads (kept for A/B and for API servers that refuse cluster-wide watches).
  bool informers = true;
};

Json crd_manifest();  // the CustomResourceDefinition the operator installs

class Controller {
 public:
  Controller(KubeApi& api, ControllerConfig cfg, ControllerOptions opts);
  ~Controller();

  // Blocks until stop() is called (or a fatal error). Returns an error message ("" on clean stop).
  std::string run();
  void stop() { stop_ = true; }

  // introspection for tests
  size_t num_jobs();
  const Informer* jobs_cache() const { return jobs_inf_.get(); }
  const Informer* pods_cache() const { return pods_inf_.get(); }
  std::map<std::string, TfJobStatus> statuses();

  // one-shot pieces, public for tests
  std::string init_resource();
  std::string find_all_jobs(std::string& resource_version);
  void handle_event(const std::string& type, const Json& obj);

 private:
  std::string list_path() const { return tfjobs_path(opts_.ns); }
  void reap_finished();
  // relist every TfJob, start the new ones, delete the vanished ones; updates rv. false on an API error.
  bool relist(std::string& rv);

  KubeApi& api_;
  ControllerConfig cfg_;
  ControllerOptions opts_;
  void watchdog_loop();
  void poke_owner(const Json& obj);  // informer change callback: reconcile the TfJob that owns obj now

  std::atomic<bool> stop_{false};
  // panicTimer (pkg/controller/util.go:50-76): steady-clock ns at which the current event handler started,
  // 0 when idle; a watchdog thread aborts the process while a handler is still running past event_watchdog
  std::atomic<long long> handler_started_ns_{0};
  // declared before the workers: destroyed after them (every worker reads these caches)
  std::unique_ptr<Informer> jobs_inf_, pods_inf_;
  std::mutex mu_;
  std::map<std::string, std::unique_ptr<JobWorker>> jobs_;  // ns/name -> worker
  std::map<std::string, std::string> job_rvs_;               // ns/name -> resourceVersion
  std::map<std::string, std::string> job_uids_;              // ns/name -> uid of the object its worker runs
  // workers of deleted-and-re-created TfJobs: still deleting the old object's children on their own thread;
  // reaped (joined) once finished, never destroyed under mu_ while running
  std::vector<std::unique_ptr<JobWorker>> retiring_;
};

}  // namespace tfop
