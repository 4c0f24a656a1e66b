// TfJob API types (group tensorflow.org, version v1alpha1, kind TfJob) with
// defaulting, validation and accelerator injection.
//
// Parity: /root/reference/pkg/spec/tf_job.go (types :33-123, Validate
// :126-176, ConfigureAccelerators :179-233, SetDefaults :236-273, default PS
// template :282-301, status types :303-383) and pkg/spec/controller.go.
// Pod templates, volumes and other Kubernetes objects are carried as raw
// JSON: the operator only edits the few fields it owns.
#pragma once

#include <map>
#include <optional>
#include <string>
#include <vector>

#include "json.h"

namespace tfop {

constexpr const char* kCRDKind = "TfJob";
constexpr const char* kCRDKindPlural = "tfjobs";
constexpr const char* kCRDGroup = "tensorflow.org";
constexpr const char* kCRDVersion = "v1alpha1";
constexpr int kDefaultTfPort = 2222;
constexpr int kDefaultReplicas = 1;
constexpr const char* kTensorflowContainer = "tensorflow";
// The reference defaults to tensorflow/tensorflow:1.3.0 (tf_job.go:87); our
// default image is the ROCm PyTorch trainer image that ships k8s_amd.
constexpr const char* kDefaultTfImage = "k8s-amd/trainer:rocm7-gfx950";
constexpr const char* kPSConfigVolume = "ps-config-volume";
constexpr const char* kPSServerMount = "/ps-server";
constexpr const char* kPSServerFile = "grpc_tensorflow_server.py";

std::string crd_name();  // "tfjobs.tensorflow.org"

enum class ReplicaType { MASTER, PS, WORKER, INVALID };
std::string to_string(ReplicaType t);
ReplicaType replica_type_from(const std::string& s);  // exact (case-sensitive) like Go

struct ChiefSpec {
  std::string replica_name;
  int replica_index = 0;
};

struct TerminationPolicy {
  std::optional<ChiefSpec> chief;
};

struct TensorBoardSpec {
  std::string log_dir;
  Json volumes;        // []v1.Volume or null
  Json volume_mounts;  // []v1.VolumeMount or null
  std::string service_type;
};

struct TfReplicaSpec {
  std::optional<int> replicas;
  std::optional<Json> tmpl;  // v1.PodTemplateSpec
  std::optional<int> tf_port;
  std::string type;  // raw string: "" | MASTER | PS | WORKER | anything (validated later)
  bool is_default_ps = false;
};

struct TfJobSpec {
  std::string runtime_id;
  std::optional<TensorBoardSpec> tensorboard;
  std::vector<TfReplicaSpec> replica_specs;
  std::string tf_image;
  std::optional<TerminationPolicy> termination_policy;
};

struct TfJobCondition {
  std::string type, reason, transition_time;
};

struct TfReplicaStatus {
  std::string type;
  std::string state;                    // Unknown|Starting|Running|Failed|Succeeded
  std::map<std::string, int> replicas_states;  // sorted like Go map encoding
};

struct TfJobStatus {
  std::string phase;  // "" | Creating | Running | CleanUp | Failed | Done
  std::string reason;
  bool control_paused = false;
  std::vector<TfJobCondition> conditions;
  bool conditions_null = true;  // Go nil slice -> null
  std::string state;            // Unknown | Running | Succeeded | Failed
  std::vector<TfReplicaStatus> replica_statuses;
  bool replica_statuses_null = true;

  void append_condition(const std::string& type, const std::string& reason);  // keeps the 10 most recent
  bool operator==(const TfJobStatus& o) const;
};

struct TfJob {
  std::string api_version = std::string(kCRDGroup) + "/" + kCRDVersion;
  std::string kind = kCRDKind;
  Json metadata = Json::object();  // metav1.ObjectMeta as JSON
  TfJobSpec spec;
  TfJobStatus status;

  std::string name() const { return get_str(metadata, "name"); }
  std::string ns() const { return get_str(metadata, "namespace", "default"); }
  std::string uid() const { return get_str(metadata, "uid"); }
  std::string resource_version() const { return get_str(metadata, "resourceVersion"); }
  Json as_owner() const;  // OwnerReference, controller=true, blockOwnerDeletion=true
};

// --- wire codec (Go encoding/json semantics: case-insensitive decode, field order/omitempty on encode)
TfJob tfjob_from_json(const Json& j);
Json tfjob_to_json(const TfJob& job);
Json spec_to_json(const TfJobSpec& s);
TfJobSpec spec_from_json(const Json& j);
Json status_to_json(const TfJobStatus& s);
TfJobStatus status_from_json(const Json& j);
Json replica_status_to_json(const TfReplicaStatus& s);

// --- controller config (pkg/spec/controller.go)
struct AcceleratorVolume {
  std::string name, host_path, mount_path;
};
struct EnvVarConfig {
  std::string name, value;
};
struct AcceleratorConfig {
  std::vector<AcceleratorVolume> volumes;
  std::vector<EnvVarConfig> env_vars;
};
struct ControllerConfig {
  std::map<std::string, AcceleratorConfig> accelerators;
  std::string grpc_server_file_path;
};
ControllerConfig controller_config_from_json(const Json& j);  // keys matched case-insensitively
Json controller_config_to_json(const ControllerConfig& c);

// --- behaviour (errors are returned as messages; empty == ok)
std::string set_defaults(TfJobSpec& s);
std::string validate(const TfJobSpec& s);
std::string configure_accelerators(TfJobSpec& s, const std::map<std::string, AcceleratorConfig>& acc);
void set_default_ps_template(TfReplicaSpec& r, const std::string& image);

// Go's util.Pformat: indented JSON
std::string pformat(const Json& j);

}  // namespace tfop
