#include <cstdlib>
#include "replicas.h"

#include <algorithm>
#include <cctype>

namespace tfop {

static std::string lower(std::string s) {
  for (auto& c : s) c = (char)tolower((unsigned char)c);
  return s;
}

std::string selector_string(const Labels& l) {
  std::string out;
  for (auto& kv : l) {
    if (!out.empty()) out += ",";
    out += kv.first + "=" + kv.second;
  }
  return out;
}

Labels parse_selector(const std::string& sel) {
  Labels l;
  size_t i = 0;
  while (i < sel.size()) {
    size_t j = sel.find(',', i);
    if (j == std::string::npos) j = sel.size();
    std::string kv = sel.substr(i, j - i);
    size_t e = kv.find('=');
    if (e != std::string::npos) {
      std::string k = kv.substr(0, e), v = kv.substr(e + 1);
      if (!v.empty() && v[0] == '=') v = v.substr(1);  // "=="
      l[k] = v;
    } else if (!kv.empty()) {
      l[kv] = "\x01exists";
    }
    i = j + 1;
  }
  return l;
}

bool labels_match(const Labels& selector, const Json& labels_obj) {
  for (auto& kv : selector) {
    const Json* v = labels_obj.is_object() ? labels_obj.find(kv.first) : nullptr;
    if (!v || !v->is_string()) return false;
    if (kv.second != "\x01exists" && v->as_string() != kv.second) return false;
  }
  return true;
}

std::string truncate_name(const std::string& name) {
  // first 40 runes of a UTF-8 string
  size_t runes = 0, i = 0;
  while (i < name.size() && runes < 40) {
    unsigned char c = (unsigned char)name[i];
    size_t len = c < 0x80 ? 1 : (c >> 5) == 6 ? 2 : (c >> 4) == 14 ? 3 : (c >> 3) == 30 ? 4 : 1;
    i += len;
    ++runes;
  }
  return name.substr(0, std::min(i, name.size()));
}

std::string replica_job_name(const TfJob& job, const std::string& type, int index) {
  return truncate_name(job.name()) + "-" + lower(type) + "-" + job.spec.runtime_id + "-" + std::to_string(index);
}

std::string tb_name(const TfJob& job) { return truncate_name(job.name()) + "-tensorboard-" + job.spec.runtime_id; }

std::string default_ps_configmap_name(const TfJob& job) { return "cm-ps-" + job.spec.runtime_id; }

Labels replica_labels(const TfJob& job, const std::string& type) {
  return Labels{{"tensorflow.org", ""}, {"job_type", type}, {"runtime_id", job.spec.runtime_id},
                {"tf_job_name", job.name()}};
}

Labels task_labels(const TfJob& job, const std::string& type, int index) {
  Labels l = replica_labels(job, type);
  l["task_index"] = std::to_string(index);
  return l;
}

Labels tb_labels(const TfJob& job) {
  return Labels{{"tensorflow.org", ""}, {"runtime_id", job.spec.runtime_id}, {"app", "tensorboard"},
                {"tf_job_name", job.name()}};
}

static Json labels_json(const Labels& l) {
  Json o = Json::object();
  for (auto& kv : l) o[kv.first] = kv.second;
  return o;
}

ClusterSpec cluster_spec(const TfJob& job) {
  ClusterSpec cs;
  for (auto& r : job.spec.replica_specs) {
    std::vector<std::string> names;
    const int n = r.replicas.value_or(kDefaultReplicas);
    for (int i = 0; i < n; ++i)
      names.push_back(replica_job_name(job, r.type, i) + ":" + std::to_string(r.tf_port.value_or(kDefaultTfPort)));
    cs[lower(r.type)] = names;
  }
  return cs;
}

std::string tf_config_json(const ClusterSpec& cs, const std::string& type_lower, int index) {
  // Go marshals map keys sorted; struct fields in order cluster, task{type,index}, environment.
  Json cluster = Json::object();
  for (auto& kv : cs) {
    Json a = Json::array();
    for (auto& h : kv.second) a.push_back(h);
    cluster[kv.first] = a;
  }
  Json task = Json::object();
  task["type"] = type_lower;
  task["index"] = index;
  Json j = Json::object();
  j["cluster"] = cluster;
  j["task"] = task;
  j["environment"] = "cloud";
  return j.dump();
}

std::string default_ps_cluster_spec(const ClusterSpec& cs) {
  std::string out;
  for (auto& kv : cs) {  // std::map iterates sorted
    if (!out.empty()) out += ",";
    out += kv.first + "|";
    for (size_t i = 0; i < kv.second.size(); ++i) {
      if (i) out += ";";
      out += kv.second[i];
    }
  }
  return out;
}

static Json object_meta(const std::string& name, const Labels& l, const TfJob& job, bool owner = true) {
  Json m = Json::object();
  m["name"] = name;
  m["namespace"] = job.ns();
  m["labels"] = labels_json(l);
  if (owner) m["ownerReferences"] = JsonArray{job.as_owner()};
  return m;
}

Json make_replica_service(const TfJob& job, const TfReplicaSpec& r, int index) {
  Labels l = task_labels(job, r.type, index);
  Json svc = Json::object();
  svc["apiVersion"] = "v1";
  svc["kind"] = "Service";
  svc["metadata"] = object_meta(replica_job_name(job, r.type, index), l, job);
  Json port = Json::object();
  port["name"] = "tf-port";
  port["port"] = r.tf_port.value_or(kDefaultTfPort);
  Json spec = Json::object();
  spec["selector"] = labels_json(l);
  spec["ports"] = JsonArray{port};
  svc["spec"] = spec;
  return svc;
}

// GPUs the `tensorflow` container of a replica template asks for: limits (else requests) of every resource whose
// name contains "gpu" (amd.com/gpu, nvidia.com/gpu, alpha.kubernetes.io/nvidia-gpu).
static int64_t template_gpus(const TfReplicaSpec& r) {
  if (!r.tmpl) return 0;
  const Json* spec = r.tmpl->find("spec");
  const Json* cons = spec ? spec->find("containers") : nullptr;
  if (!cons || !cons->is_array()) return 0;
  for (const auto& c : cons->as_array()) {
    if (get_str(c, "name") != kTensorflowContainer) continue;
    const Json* res = c.find("resources");
    if (!res || !res->is_object()) return 0;
    for (const char* which : {"limits", "requests"}) {
      const Json* m = res->find(which);
      if (!m || !m->is_object()) continue;
      int64_t n = 0;
      for (const auto& kv : m->as_object()) {
        if (kv.first.find("gpu") == std::string::npos) continue;
        if (kv.second.is_number()) n += kv.second.as_int();
        else if (kv.second.is_string()) n += std::atoll(kv.second.as_string().c_str());
      }
      if (n > 0) return n;
    }
    return 0;
  }
  return 0;
}

// TFJOB_TASK_GPUS: {"master": n, "worker": n, "ps": n} -- the GPUs per task of every replica type, so a trainer
// replica that drives several local GPUs (one process per GPU) can place its processes in the global rank order
// without a registration round (TF_CONFIG itself stays byte-identical to the reference's).
std::string task_gpus_json(const TfJob& job) {
  Json j = Json::object();
  for (const auto& r : job.spec.replica_specs) j[lower(r.type)] = template_gpus(r);
  return j.dump();
}

Json make_replica_job(const TfJob& job, const TfReplicaSpec& r, int index, const ClusterSpec& cs,
                      const std::string& ps_script_path) {
  Labels l = task_labels(job, r.type, index);
  // deep copy of the template: the spec's template is never mutated by resource creation
  Json tmpl = r.tmpl ? r.tmpl->clone() : Json::object();
  // insert every top-level key BEFORE taking references into the object (vector storage may move)
  if (!tmpl.find("metadata") || !tmpl["metadata"].is_object()) tmpl["metadata"] = Json::object();
  if (!tmpl.find("spec")) tmpl["spec"] = Json::object();
  Json& pspec = tmpl["spec"];
  if (r.is_default_ps) {
    Json cm = Json::object();
    cm["name"] = default_ps_configmap_name(job);
    Json vol = Json::object();
    vol["name"] = kPSConfigVolume;
    vol["configMap"] = cm;
    pspec["volumes"].push_back(vol);
    Json& cs0 = pspec["containers"][0];
    Json cmd = Json::array();
    for (auto& s : {std::string("python"), ps_script_path, std::string("--cluster_spec"),
                    default_ps_cluster_spec(cs), std::string("--job_name"), std::string("ps"),
                    std::string("--task_id"), std::to_string(index)})
      cmd.push_back(s);
    cs0["command"] = cmd;
  }
  Json& tl = tmpl["metadata"]["labels"];
  if (!tl.is_object()) tl = Json::object();
  for (auto& kv : l) tl[kv.first] = kv.second;
  const std::string tfc = tf_config_json(cs, lower(r.type), index);
  const std::string gpus = task_gpus_json(job);
  if (Json* cons = pspec.find("containers"); cons && cons->is_array()) {
    for (auto& c : cons->as_array()) {
      if (get_str(c, "name") != kTensorflowContainer) continue;
      Json ev = Json::object();
      ev["name"] = "TF_CONFIG";
      ev["value"] = tfc;
      c["env"].push_back(ev);
      Json eg = Json::object();
      eg["name"] = "TFJOB_TASK_GPUS";
      eg["value"] = gpus;
      c["env"].push_back(eg);
    }
  }
  Json jspec = Json::object();
  jspec["completions"] = 1;
  jspec["parallelism"] = 1;
  jspec["template"] = tmpl;
  Json j = Json::object();
  j["apiVersion"] = "batch/v1";
  j["kind"] = "Job";
  j["metadata"] = object_meta(replica_job_name(job, r.type, index), l, job);
  j["spec"] = jspec;
  return j;
}

Json make_ps_configmap(const TfJob& job, const std::string& server_source) {
  Json cm = Json::object();
  cm["apiVersion"] = "v1";
  cm["kind"] = "ConfigMap";
  Json m = Json::object();
  m["name"] = default_ps_configmap_name(job);
  m["namespace"] = job.ns();
  m["ownerReferences"] = JsonArray{job.as_owner()};  // Q9 fix: garbage-collected with the TfJob
  cm["metadata"] = m;
  Json d = Json::object();
  d[kPSServerFile] = server_source;
  cm["data"] = d;
  return cm;
}

Json make_tb_service(const TfJob& job) {
  const TensorBoardSpec& tb = *job.spec.tensorboard;
  Labels l = tb_labels(job);
  Json port = Json::object();
  port["name"] = "tb-port";
  port["port"] = 80;
  port["targetPort"] = 6006;
  Json spec = Json::object();
  spec["type"] = tb.service_type.empty() ? "ClusterIP" : tb.service_type;
  spec["selector"] = labels_json(l);
  spec["ports"] = JsonArray{port};
  Json s = Json::object();
  s["apiVersion"] = "v1";
  s["kind"] = "Service";
  s["metadata"] = object_meta(tb_name(job), l, job);
  s["spec"] = spec;
  return s;
}

Json make_tb_deployment(const TfJob& job) {
  const TensorBoardSpec& tb = *job.spec.tensorboard;
  Labels l = tb_labels(job);
  Json c = Json::object();
  c["name"] = tb_name(job);
  c["image"] = job.spec.tf_image;
  c["command"] = JsonArray{Json("tensorboard"), Json("--logdir"), Json(tb.log_dir), Json("--host"), Json("0.0.0.0")};
  Json cp = Json::object();
  cp["containerPort"] = 6006;
  c["ports"] = JsonArray{cp};
  c["volumeMounts"] = tb.volume_mounts.is_array() ? tb.volume_mounts.clone() : Json::array();
  Json ps = Json::object();
  ps["containers"] = JsonArray{c};
  ps["volumes"] = tb.volumes.is_array() ? tb.volumes.clone() : Json::array();
  Json tm = Json::object();
  tm["name"] = tb_name(job);
  tm["labels"] = labels_json(l);
  Json tmpl = Json::object();
  tmpl["metadata"] = tm;
  tmpl["spec"] = ps;
  Json sel = Json::object();
  sel["matchLabels"] = labels_json(l);
  Json spec = Json::object();
  spec["selector"] = sel;
  spec["replicas"] = 1;
  spec["template"] = tmpl;
  Json d = Json::object();
  d["apiVersion"] = "apps/v1";  // extensions/v1beta1 was removed in K8s 1.16
  d["kind"] = "Deployment";
  d["metadata"] = object_meta(tb_name(job), l, job);
  d["spec"] = spec;
  return d;
}

bool is_retryable_termination(const ContainerTermination& t) {
  if (t.reason == "OOMKilled") return false;
  if (t.exit_code >= 0 && t.exit_code <= 127) return false;
  return true;
}

// Kubernetes RFC3339 timestamps of equal format compare lexicographically.
std::string replica_state_from_pods(const Json& items, const std::string& container) {
  const Json* latest = nullptr;
  std::string latest_t;
  if (items.is_array()) {
    for (auto& p : items.as_array()) {
      std::string t;
      if (const Json* st = p.find("status")) t = get_str(*st, "startTime");
      if (!latest || latest_t < t) {
        latest = &p;
        latest_t = t;
      }
    }
  }
  if (!latest) return "Running";
  Json state;  // chosen ContainerState
  if (const Json* st = latest->find("status")) {
    if (const Json* css = st->find("containerStatuses"); css && css->is_array()) {
      for (auto& cst : css->as_array()) {
        if (get_str(cst, "name") != container) continue;
        if (const Json* s = cst.find("state")) state = *s;
        if (const Json* lt = cst.find("lastState"); lt && lt->is_object() && lt->find("terminated") &&
                                                       !lt->at("terminated").is_null())
          state = *lt;
      }
    }
  }
  if (state.is_object()) {
    auto present = [&](const char* k) {
      const Json* v = state.find(k);
      return v && !v->is_null();
    };
    if (present("running") || present("waiting")) return "Running";
    if (present("terminated")) {
      const Json& t = state.at("terminated");
      ContainerTermination ct;
      if (const Json* e = t.find("exitCode")) ct.exit_code = (int)e->as_int();
      ct.reason = get_str(t, "reason");
      if (ct.exit_code == 0) return "Succeeded";
      if (is_retryable_termination(ct)) return "Running";
      return "Failed";
    }
  }
  return "Unknown";
}

std::string aggregate_replica_states(const std::map<std::string, int>& counts, int replicas) {
  if (counts.count("Failed")) return "Failed";
  if (counts.count("Running")) return "Running";
  auto it = counts.find("Succeeded");
  if (it != counts.end() && it->second == replicas) return "Succeeded";
  return "Unknown";
}

std::string job_state_from_replicas(const std::vector<TfReplicaStatus>& statuses, const std::string& chief_type) {
  for (auto& s : statuses) {
    if (s.type != chief_type) continue;
    if (s.state == "Succeeded") return "Succeeded";
    if (s.state == "Failed") return "Failed";
  }
  return "Running";
}

}  // namespace tfop
