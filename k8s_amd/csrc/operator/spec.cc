#include "spec.h"

#include <chrono>
#include <ctime>

namespace tfop {

std::string crd_name() { return std::string(kCRDKindPlural) + "." + kCRDGroup; }

std::string to_string(ReplicaType t) {
  switch (t) {
    case ReplicaType::MASTER: return "MASTER";
    case ReplicaType::PS: return "PS";
    case ReplicaType::WORKER: return "WORKER";
    default: return "";
  }
}

ReplicaType replica_type_from(const std::string& s) {
  if (s == "MASTER") return ReplicaType::MASTER;
  if (s == "PS") return ReplicaType::PS;
  if (s == "WORKER") return ReplicaType::WORKER;
  return ReplicaType::INVALID;
}

std::string pformat(const Json& j) { return j.dump_pretty(2); }

static std::string rfc3339_now() {
  std::time_t t = std::time(nullptr);
  char buf[64];
  std::tm tm;
  gmtime_r(&t, &tm);
  strftime(buf, sizeof buf, "%Y-%m-%dT%H:%M:%SZ", &tm);
  return buf;
}

void TfJobStatus::append_condition(const std::string& type, const std::string& reason) {
  conditions.push_back({type, reason, rfc3339_now()});
  conditions_null = false;
  if (conditions.size() > 10) conditions.erase(conditions.begin());
}

bool TfJobStatus::operator==(const TfJobStatus& o) const {
  return status_to_json(*this) == status_to_json(o);
}

Json TfJob::as_owner() const {
  Json o = Json::object();
  o["apiVersion"] = api_version;
  o["kind"] = kind;
  o["name"] = name();
  o["uid"] = uid();
  o["controller"] = true;
  o["blockOwnerDeletion"] = true;
  return o;
}

// ------------------------------------------------------------------ codec
static std::optional<int> opt_int(const Json& o, const char* k) {
  const Json* v = o.find_ci(k);
  if (!v || v->is_null()) return std::nullopt;
  return (int)v->as_int();
}

Json spec_to_json(const TfJobSpec& s) {
  Json j = Json::object();
  j["RuntimeId"] = s.runtime_id;
  if (s.tensorboard) {
    Json tb = Json::object();
    tb["logDir"] = s.tensorboard->log_dir;
    tb["volumes"] = s.tensorboard->volumes.clone();
    tb["volumeMounts"] = s.tensorboard->volume_mounts.clone();
    tb["serviceType"] = s.tensorboard->service_type;
    j["tensorboard"] = tb;
  } else {
    j["tensorboard"] = Json();
  }
  Json rs = Json::array();
  for (auto& r : s.replica_specs) {
    Json rj = Json::object();
    if (r.replicas) rj["replicas"] = *r.replicas;
    if (r.tmpl) rj["template"] = r.tmpl->clone();
    if (r.tf_port) rj["tfPort"] = *r.tf_port;
    rj["tfReplicaType"] = r.type;
    rj["IsDefaultPS"] = r.is_default_ps;
    rs.push_back(rj);
  }
  j["replicaSpecs"] = s.replica_specs.empty() ? Json() : rs;
  if (!s.tf_image.empty()) j["tfImage"] = s.tf_image;
  if (s.termination_policy) {
    Json tp = Json::object();
    if (s.termination_policy->chief) {
      Json c = Json::object();
      c["replicaName"] = s.termination_policy->chief->replica_name;
      c["replicaIndex"] = s.termination_policy->chief->replica_index;
      tp["chief"] = c;
    }
    j["terminationPolicy"] = tp;
  }
  return j;
}

TfJobSpec spec_from_json(const Json& j) {
  TfJobSpec s;
  if (!j.is_object()) return s;
  s.runtime_id = get_str(j, "RuntimeId");
  if (const Json* tb = j.find_ci("tensorboard"); tb && tb->is_object()) {
    TensorBoardSpec t;
    t.log_dir = get_str(*tb, "logDir");
    if (const Json* v = tb->find_ci("volumes")) t.volumes = v->clone();
    if (const Json* v = tb->find_ci("volumeMounts")) t.volume_mounts = v->clone();
    t.service_type = get_str(*tb, "serviceType");
    s.tensorboard = t;
  }
  if (const Json* rs = j.find_ci("replicaSpecs"); rs && rs->is_array()) {
    for (auto& rj : rs->as_array()) {
      if (rj.is_null()) continue;
      TfReplicaSpec r;
      r.replicas = opt_int(rj, "replicas");
      if (const Json* t = rj.find_ci("template"); t && !t->is_null()) r.tmpl = t->clone();
      r.tf_port = opt_int(rj, "tfPort");
      r.type = get_str(rj, "tfReplicaType");
      if (const Json* d = rj.find_ci("IsDefaultPS"); d && d->is_bool()) r.is_default_ps = d->as_bool();
      s.replica_specs.push_back(std::move(r));
    }
  }
  s.tf_image = get_str(j, "tfImage");
  if (const Json* tp = j.find_ci("terminationPolicy"); tp && tp->is_object()) {
    TerminationPolicy p;
    if (const Json* c = tp->find_ci("chief"); c && c->is_object()) {
      ChiefSpec cs;
      cs.replica_name = get_str(*c, "replicaName");
      if (auto v = opt_int(*c, "replicaIndex")) cs.replica_index = *v;
      p.chief = cs;
    }
    s.termination_policy = p;
  }
  return s;
}

Json replica_status_to_json(const TfReplicaStatus& r) {
  Json j = Json::object();
  j["tf_replica_type"] = r.type;
  j["state"] = r.state;
  Json m = Json::object();
  for (auto& kv : r.replicas_states) m[kv.first] = kv.second;
  j["ReplicasStates"] = m;
  return j;
}

Json status_to_json(const TfJobStatus& s) {
  Json j = Json::object();
  j["phase"] = s.phase;
  j["reason"] = s.reason;
  j["controlPaused"] = s.control_paused;
  if (s.conditions_null && s.conditions.empty()) {
    j["conditions"] = Json();
  } else {
    Json c = Json::array();
    for (auto& x : s.conditions) {
      Json cj = Json::object();
      cj["type"] = x.type;
      cj["reason"] = x.reason;
      cj["transitionTime"] = x.transition_time;
      c.push_back(cj);
    }
    j["conditions"] = c;
  }
  j["state"] = s.state;
  if (s.replica_statuses_null && s.replica_statuses.empty()) {
    j["replicaStatuses"] = Json();
  } else {
    Json a = Json::array();
    for (auto& r : s.replica_statuses) a.push_back(replica_status_to_json(r));
    j["replicaStatuses"] = a;
  }
  return j;
}

TfJobStatus status_from_json(const Json& j) {
  TfJobStatus s;
  if (!j.is_object()) return s;
  s.phase = get_str(j, "phase");
  s.reason = get_str(j, "reason");
  if (const Json* v = j.find_ci("controlPaused"); v && v->is_bool()) s.control_paused = v->as_bool();
  if (const Json* c = j.find_ci("conditions"); c && c->is_array()) {
    s.conditions_null = false;
    for (auto& x : c->as_array())
      s.conditions.push_back({get_str(x, "type"), get_str(x, "reason"), get_str(x, "transitionTime")});
  }
  s.state = get_str(j, "state");
  if (const Json* r = j.find_ci("replicaStatuses"); r && r->is_array()) {
    s.replica_statuses_null = false;
    for (auto& x : r->as_array()) {
      TfReplicaStatus rs;
      rs.type = get_str(x, "tf_replica_type");
      rs.state = get_str(x, "state");
      if (const Json* m = x.find_ci("ReplicasStates"); m && m->is_object())
        for (auto& kv : m->as_object()) rs.replicas_states[kv.first] = (int)kv.second.as_int();
      s.replica_statuses.push_back(rs);
    }
  }
  return s;
}

TfJob tfjob_from_json(const Json& j) {
  TfJob t;
  if (!j.is_object()) throw JsonError("TfJob must be a JSON object");
  t.api_version = get_str(j, "apiVersion", t.api_version);
  t.kind = get_str(j, "kind", t.kind);
  if (const Json* m = j.find_ci("metadata"); m && m->is_object()) t.metadata = m->clone();
  if (const Json* s = j.find_ci("spec")) t.spec = spec_from_json(*s);
  if (const Json* s = j.find_ci("status")) t.status = status_from_json(*s);
  return t;
}

Json tfjob_to_json(const TfJob& t) {
  Json j = Json::object();
  if (!t.api_version.empty()) j["apiVersion"] = t.api_version;
  if (!t.kind.empty()) j["kind"] = t.kind;
  j["metadata"] = t.metadata.clone();
  j["spec"] = spec_to_json(t.spec);
  j["status"] = status_to_json(t.status);
  return j;
}

ControllerConfig controller_config_from_json(const Json& j) {
  ControllerConfig c;
  if (!j.is_object()) return c;
  c.grpc_server_file_path = get_str(j, "grpcServerFilePath");
  if (const Json* a = j.find_ci("accelerators"); a && a->is_object()) {
    for (auto& kv : a->as_object()) {
      AcceleratorConfig ac;
      if (const Json* vs = kv.second.find_ci("volumes"); vs && vs->is_array())
        for (auto& v : vs->as_array())
          ac.volumes.push_back({get_str(v, "name"), get_str(v, "hostPath"), get_str(v, "mountPath")});
      if (const Json* es = kv.second.find_ci("envVars"); es && es->is_array())
        for (auto& e : es->as_array()) ac.env_vars.push_back({get_str(e, "name"), get_str(e, "value")});
      c.accelerators[kv.first] = ac;
    }
  }
  return c;
}

Json controller_config_to_json(const ControllerConfig& c) {
  Json j = Json::object();
  Json acc = Json::object();
  for (auto& kv : c.accelerators) {
    Json a = Json::object();
    Json vs = Json::array();
    for (auto& v : kv.second.volumes) {
      Json vj = Json::object();
      vj["Name"] = v.name;
      vj["HostPath"] = v.host_path;
      vj["MountPath"] = v.mount_path;
      vs.push_back(vj);
    }
    Json es = Json::array();
    for (auto& e : kv.second.env_vars) {
      Json ej = Json::object();
      ej["Name"] = e.name;
      ej["Value"] = e.value;
      es.push_back(ej);
    }
    a["Volumes"] = vs;
    a["EnvVars"] = es;
    acc[kv.first] = a;
  }
  j["Accelerators"] = acc;
  j["GrpcServerFilePath"] = c.grpc_server_file_path;
  return j;
}

// ------------------------------------------------------------------ behaviour
static Json replica_debug(const TfReplicaSpec& r) {
  TfJobSpec s;
  s.replica_specs.push_back(r);
  return spec_to_json(s)["replicaSpecs"][0];
}

static const Json* containers_of(const Json& tmpl) {
  const Json* spec = tmpl.find_ci("spec");
  if (!spec) return nullptr;
  const Json* cs = spec->find_ci("containers");
  return (cs && cs->is_array()) ? cs : nullptr;
}

std::string validate(const TfJobSpec& s) {
  for (auto& r : s.replica_specs) {
    if (!r.tmpl && r.type != "PS") return "Replica is missing Template; " + pformat(replica_debug(r));
    if (r.type == "MASTER" && r.replicas && *r.replicas != 1) return "The MASTER must have Replicas = 1";
    if (!r.tf_port) return "tfReplicaSpec.TfPort can't be nil.";
    if (replica_type_from(r.type) == ReplicaType::INVALID)
      return "tfReplicaSpec.TfReplicaType is " + r.type + " but must be one of [MASTER PS WORKER]";
    bool found = false;
    if (r.tmpl) {
      if (const Json* cs = containers_of(*r.tmpl))
        for (auto& c : cs->as_array())
          if (get_str(c, "name") == kTensorflowContainer) {
            found = true;
            break;
          }
    }
    if (!found) return "Replica type " + r.type + " is missing a container named " + kTensorflowContainer;
  }
  if (s.termination_policy) {
    if (!s.termination_policy->chief) return "invalid termination policy, Chief cannot be nil";
    if (s.termination_policy->chief->replica_name != "MASTER" || s.termination_policy->chief->replica_index != 0)
      return "invalid termination policy, Chief should have replicaName=MASTER and index=0";
  }
  return "";
}

std::string configure_accelerators(TfJobSpec& s, const std::map<std::string, AcceleratorConfig>& acc) {
  for (auto& r : s.replica_specs) {
    if (!r.tmpl) return "Replica is missing Template; " + pformat(replica_debug(r));
    Json* spec = r.tmpl->find("spec");
    if (!spec) continue;
    Json* cs = spec->find("containers");
    if (!cs || !cs->is_array()) continue;
    for (auto& c : cs->as_array()) {
      if (get_str(c, "name") != kTensorflowContainer) continue;
      // accelerator names attached to this container via limits OR requests (sorted, deterministic)
      std::map<std::string, const AcceleratorConfig*> found;
      if (const Json* res = c.find_ci("resources")) {
        for (const char* key : {"limits", "requests"}) {
          const Json* l = res->find_ci(key);
          if (!l || !l->is_object()) continue;
          for (auto& kv : l->as_object()) {
            auto it = acc.find(kv.first);
            if (it != acc.end()) found[kv.first] = &it->second;
          }
        }
      }
      for (auto& kv : found) {
        for (auto& v : kv.second->volumes) {
          Json vol = Json::object();
          vol["name"] = v.name;
          Json hp = Json::object();
          hp["path"] = v.host_path;
          vol["hostPath"] = hp;
          (*spec)["volumes"].push_back(vol);
          Json vm = Json::object();
          vm["name"] = v.name;
          vm["mountPath"] = v.mount_path;
          c["volumeMounts"].push_back(vm);
        }
        for (auto& e : kv.second->env_vars) {
          Json ev = Json::object();
          ev["name"] = e.name;
          ev["value"] = e.value;
          c["env"].push_back(ev);
        }
      }
      break;
    }
  }
  return "";
}

void set_default_ps_template(TfReplicaSpec& r, const std::string& image) {
  r.is_default_ps = true;
  Json vm = Json::object();
  vm["name"] = kPSConfigVolume;
  vm["mountPath"] = kPSServerMount;
  Json c = Json::object();
  c["name"] = kTensorflowContainer;
  c["image"] = image;
  c["resources"] = Json::object();
  c["volumeMounts"] = JsonArray{vm};
  Json spec = Json::object();
  spec["containers"] = JsonArray{c};
  spec["restartPolicy"] = "OnFailure";
  Json t = Json::object();
  t["metadata"] = Json::object();
  t["spec"] = spec;
  r.tmpl = t;
}

std::string set_defaults(TfJobSpec& s) {
  if (s.tf_image.empty()) s.tf_image = kDefaultTfImage;
  for (auto& r : s.replica_specs) {
    if (!r.tmpl && r.type != "PS")
      return "ReplicaType: " + r.type + ", Replica is missing Template; " + pformat(replica_debug(r));
    if (!r.tf_port) r.tf_port = kDefaultTfPort;
    if (r.type.empty()) r.type = "MASTER";
    if (!r.replicas) r.replicas = kDefaultReplicas;
    if (!r.tmpl && r.type == "PS") set_default_ps_template(r, s.tf_image);
  }
  if (!s.termination_policy) {
    TerminationPolicy p;
    p.chief = ChiefSpec{"MASTER", 0};
    s.termination_policy = p;
  }
  return "";
}

}  // namespace tfop
