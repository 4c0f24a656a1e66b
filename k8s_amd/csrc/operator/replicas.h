// Per-replica resource construction and status logic (pure functions).
//
// Parity: /root/reference/pkg/trainer/replicas.go (labels :91-99, default-PS
// cluster spec :102-122, Service/Job/TF_CONFIG construction :124-271,
// ConfigMap :275-296, replicaStatusFromPodList :359-412, GetStatus
// aggregation :415-492, jobName :494-500), pkg/trainer/training.go
// (ClusterSpec :114-128, GetStatus :163-199, isRetryableTerminationState
// :203-238), pkg/trainer/tensorboard.go (:40-194), pkg/trainer/labels.go.
//
// These build Kubernetes objects as JSON; the reconciler (reconciler.h)
// sends them through a KubeApi.
#pragma once

#include <map>
#include <string>
#include <vector>

#include "json.h"
#include "spec.h"

namespace tfop {

using Labels = std::map<std::string, std::string>;  // sorted: deterministic selectors (Q10 fix)
using ClusterSpec = std::map<std::string, std::vector<std::string>>;

std::string selector_string(const Labels& l);  // "k=v,k2=v2" (sorted keys)
bool labels_match(const Labels& selector, const Json& labels_obj);
Labels parse_selector(const std::string& sel);

std::string truncate_name(const std::string& name);  // fmt "%.40s" (first 40 runes)
std::string replica_job_name(const TfJob& job, const std::string& type, int index);
std::string tb_name(const TfJob& job);
std::string default_ps_configmap_name(const TfJob& job);

Labels replica_labels(const TfJob& job, const std::string& type);
Labels task_labels(const TfJob& job, const std::string& type, int index);
Labels tb_labels(const TfJob& job);

ClusterSpec cluster_spec(const TfJob& job);
std::string tf_config_json(const ClusterSpec& cs, const std::string& type_lower, int index);
std::string default_ps_cluster_spec(const ClusterSpec& cs);  // "job|h:p;h:p,job2|..." sorted

// Kubernetes objects
Json make_replica_service(const TfJob& job, const TfReplicaSpec& r, int index);
Json make_replica_job(const TfJob& job, const TfReplicaSpec& r, int index, const ClusterSpec& cs,
                      const std::string& ps_script_path);
Json make_ps_configmap(const TfJob& job, const std::string& server_source);
Json make_tb_service(const TfJob& job);
Json make_tb_deployment(const TfJob& job);

// Status
struct ContainerTermination {
  int exit_code = 0;
  std::string reason;
};
bool is_retryable_termination(const ContainerTermination& t);
// newest pod (by status.startTime) -> replica state for the given container name
std::string replica_state_from_pods(const Json& pod_list_items, const std::string& container);
// aggregate a replica set: any Failed -> Failed; any Running -> Running; all Succeeded -> Succeeded; else Unknown
std::string aggregate_replica_states(const std::map<std::string, int>& counts, int replicas);
// job-level: the chief replica type's state decides (TerminationPolicy.chief, default MASTER).
// Returns Running/Succeeded/Failed.
std::string job_state_from_replicas(const std::vector<TfReplicaStatus>& statuses, const std::string& chief_type);

}  // namespace tfop
