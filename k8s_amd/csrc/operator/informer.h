// Shared watch cache ("informer") for the child objects every TfJob reconciler reads.
//
// The reference's TrainingJob reads its replicas' state with one batch Job GET plus one Pod LIST per replica
// index on every 8 s tick (/root/reference/pkg/trainer/replicas.go:415-492, GetStatus), per job. At the design
// target of O(100) concurrent TfJobs (/root/reference/tf_job_design_doc.md:24) that is hundreds of API requests
// per tick, growing with jobs x replicas. client-go's answer (SharedInformer) is what this is: ONE list + watch per
// collection for the whole operator, an in-memory store every reconciler reads, and a change callback that pokes
// the owning job's worker so status changes are seen at watch latency instead of at the next resync tick
// (SURVEY.md §2.7 Q16 / §3.3).
//
// Per collection (batch/v1 jobs, v1 pods; label selector `tensorflow.org`, the label every replica object carries):
// LIST -> store keyed by namespace/name + an index by (namespace, tf_job_name label); WATCH from the list's
// resourceVersion with a server-side timeoutSeconds; a stream that outlives timeoutSeconds by the grace is a
// half-open connection and is re-established; 410 Gone relists, on the stream or on the watch open (as does a 403,
// or a watch open that keeps failing), and a resync period relists a healthy cache too. fresh() tells readers
// whether to trust the cache or to read the API directly (a cache frozen behind a failing watch is not trusted). Readers get immutable shared objects (an update
// replaces the entry, it never mutates one in place).
#pragma once

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "kube_api.h"
#include "replicas.h"

namespace tfop {

struct InformerOptions {
  std::chrono::milliseconds watch_timeout{300000};  // timeoutSeconds in [t, 2t) per watch (client-go reflector)
  std::chrono::milliseconds watch_idle_grace{30000};
  std::chrono::milliseconds retry{1000};            // after a failed list / watch
  // periodic relist even while the watch is healthy (client-go resyncPeriod): bounds how long a missed event can
  // hide a replica's state change. 0 = never.
  std::chrono::milliseconds resync_period{300000};
  // consecutive failed watch OPENS after which the next attempt relists instead of re-watching from the same rv
  // (a 410 / 403 on open relists at once)
  int relist_after_watch_failures{3};
  // fresh(): the cache is trusted while a watch is established, or within this bound of the last successful list /
  // watch open / event; readers fall back to direct API reads past it
  std::chrono::milliseconds stale_after{60000};
};

class Informer {
 public:
  // obj: the object that changed (ADDED / MODIFIED) or was removed (DELETED)
  using OnChange = std::function<void(const std::string& type, const Json& obj)>;

  Informer(KubeApi& api, std::string collection_path, std::string label_selector, InformerOptions opts = {});
  ~Informer();
  Informer(const Informer&) = delete;
  Informer& operator=(const Informer&) = delete;

  void set_on_change(OnChange cb) { on_change_ = std::move(cb); }  // before start()
  void start();
  void stop();

  bool synced() const { return synced_.load(); }
  // synced AND (a watch is open, or the last successful list / watch open / event is within stale_after): what a
  // reader checks before trusting the cache over a direct GET / LIST
  bool fresh() const;
  bool wait_synced(std::chrono::milliseconds timeout);

  // namespace/name lookup; false when the object is not in the cache
  bool get(const std::string& ns, const std::string& name, Json& out) const;
  // objects of namespace ns whose labels match every key of sel (uses the tf_job_name index when sel has it)
  Json list(const std::string& ns, const Labels& sel) const;
  size_t size() const;

  // counters (tests / metrics)
  long long lists() const { return lists_.load(); }
  long long watches() const { return watches_.load(); }
  long long events() const { return events_.load(); }

 private:
  void run();
  bool relist(std::string& rv);
  void apply(const std::string& type, const Json& obj);
  static std::string index_key(const std::string& ns, const Json& obj);

  KubeApi& api_;
  std::string path_, selector_;
  InformerOptions opts_;
  OnChange on_change_;
  mutable std::mutex mu_;
  std::map<std::string, Json> objs_;                  // ns/name -> object
  std::map<std::string, std::set<std::string>> idx_;  // ns/tf_job_name -> {ns/name}
  void touch();  // a successful list / watch open / event: the cache is current as of now

  std::atomic<bool> synced_{false}, stop_{false}, watching_{false};
  std::atomic<long long> last_ok_ns_{0};  // steady_clock of the last touch()
  std::atomic<long long> lists_{0}, watches_{0}, events_{0};
  std::mutex sync_mu_;
  std::condition_variable sync_cv_;
  std::thread th_;
};

}  // namespace tfop
