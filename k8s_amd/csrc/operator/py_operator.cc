// pybind11 module k8s_amd._operator: the C++ control-plane core exposed to
// Python (tests, the tfjob CLI, the fake API server's defaulting path).
// JSON crosses the boundary as strings.
#include <chrono>
#include <thread>
#include <algorithm>

#include <pybind11/functional.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "controller.h"
#include "election.h"
#include "flags.h"
#include "informer.h"
#include "kube_api.h"
#include "reconciler.h"
#include "replicas.h"
#include "spec.h"
#include "yaml_lite.h"

namespace py = pybind11;
using namespace tfop;

namespace {

TfJob job_of(const std::string& s) { return tfjob_from_json(Json::parse(s)); }

// KubeApi backed by a Python callable: fn(method, path, body_json_or_None) -> (code, body_json_str)
class PyKubeApi : public KubeApi {
 public:
  explicit PyKubeApi(py::function fn) : fn_(std::move(fn)) {}
  ApiResult request(const std::string& method, const std::string& path, const Json* body,
                    const std::string&) override {
    py::gil_scoped_acquire g;
    py::object b = body ? py::object(py::str(body->dump())) : py::none();
    py::tuple t = fn_(method, path, b);
    ApiResult r;
    r.code = t[0].cast<int>();
    std::string s = t[1].cast<std::string>();
    if (!s.empty()) r.body = Json::parse(s);
    return r;
  }
  std::unique_ptr<WatchStream> watch(const std::string&, std::string& err) override {
    err = "watch not supported on PyKubeApi";
    return nullptr;
  }

 private:
  py::function fn_;
};

struct PyReconciler {
  std::unique_ptr<PyKubeApi> api;
  std::unique_ptr<TrainingJob> job;
  PyReconciler(py::function fn, const std::string& job_json, const std::string& cfg_json, const std::string& ps_src) {
    api = std::make_unique<PyKubeApi>(std::move(fn));
    ReconcileOptions o;
    o.ps_server_source = ps_src;
    ControllerConfig cfg = cfg_json.empty() ? ControllerConfig{} : controller_config_from_json(Json::parse(cfg_json));
    job = std::make_unique<TrainingJob>(*api, job_of(job_json), cfg, o);
  }
};

// A shared watch cache over the real HTTP transport (tests of the informer's relist / resync / freshness rules
// against the fake API server's fault injection)
struct PyInformer {
  std::unique_ptr<KubeApi> api;
  std::unique_ptr<Informer> inf;
  PyInformer(const std::string& url, const std::string& path, const std::string& selector, int watch_timeout_ms,
             int retry_ms, int resync_ms, int relist_after, int stale_ms) {
    api = make_http_api(parse_master_url(url));
    InformerOptions o;
    o.watch_timeout = std::chrono::milliseconds(watch_timeout_ms);
    o.watch_idle_grace = std::chrono::milliseconds(2000);
    o.retry = std::chrono::milliseconds(retry_ms);
    o.resync_period = std::chrono::milliseconds(resync_ms);
    o.relist_after_watch_failures = relist_after;
    o.stale_after = std::chrono::milliseconds(stale_ms);
    inf = std::make_unique<Informer>(*api, path, selector, o);
  }
};

}  // namespace

PYBIND11_MODULE(_operator, m) {
  m.doc() = "k8s_amd C++17 TfJob control plane (pybind11)";
  m.attr("version") = kVersion;
  m.attr("CRD_GROUP") = kCRDGroup;
  m.attr("CRD_VERSION") = kCRDVersion;
  m.attr("CRD_KIND") = kCRDKind;
  m.attr("CRD_PLURAL") = kCRDKindPlural;
  m.attr("DEFAULT_TF_IMAGE") = kDefaultTfImage;
  m.def("crd_name", &crd_name);
  m.def("crd_manifest", [] { return crd_manifest().dump(); });

  m.def("normalize_tfjob", [](const std::string& s) { return tfjob_to_json(job_of(s)).dump(); },
        "decode (Go semantics) and re-encode a TfJob");
  m.def("set_defaults", [](const std::string& spec_json) {
    TfJobSpec s = spec_from_json(Json::parse(spec_json));
    std::string err = set_defaults(s);
    return py::make_tuple(spec_to_json(s).dump(), err);
  });
  m.def("validate", [](const std::string& spec_json) { return validate(spec_from_json(Json::parse(spec_json))); });
  m.def("configure_accelerators", [](const std::string& spec_json, const std::string& cfg_json) {
    TfJobSpec s = spec_from_json(Json::parse(spec_json));
    ControllerConfig c = controller_config_from_json(Json::parse(cfg_json));
    std::string err = configure_accelerators(s, c.accelerators);
    return py::make_tuple(spec_to_json(s).dump(), err);
  });
  m.def("controller_config", [](const std::string& cfg_json) {
    return controller_config_to_json(controller_config_from_json(Json::parse(cfg_json))).dump();
  });

  m.def("replica_job_name", [](const std::string& j, const std::string& t, int i) {
    return replica_job_name(job_of(j), t, i);
  });
  m.def("tb_name", [](const std::string& j) { return tb_name(job_of(j)); });
  m.def("default_ps_configmap_name", [](const std::string& j) { return default_ps_configmap_name(job_of(j)); });
  m.def("replica_labels", [](const std::string& j, const std::string& t) { return replica_labels(job_of(j), t); });
  m.def("task_labels", [](const std::string& j, const std::string& t, int i) { return task_labels(job_of(j), t, i); });
  m.def("tb_labels", [](const std::string& j) { return tb_labels(job_of(j)); });
  m.def("selector_string", &selector_string);
  m.def("cluster_spec", [](const std::string& j) { return cluster_spec(job_of(j)); });
  m.def("tf_config", &tf_config_json);
  m.def("default_ps_cluster_spec", &default_ps_cluster_spec);
  m.def("truncate_name", &truncate_name);
  m.def("make_replica_service", [](const std::string& j, int r, int i) {
    TfJob job = job_of(j);
    return make_replica_service(job, job.spec.replica_specs.at(r), i).dump();
  });
  m.def("make_replica_job", [](const std::string& j, int r, int i, const std::string& ps_script) {
    TfJob job = job_of(j);
    return make_replica_job(job, job.spec.replica_specs.at(r), i, cluster_spec(job), ps_script).dump();
  });
  m.def("make_ps_configmap", [](const std::string& j, const std::string& src) {
    return make_ps_configmap(job_of(j), src).dump();
  });
  m.def("make_tb_service", [](const std::string& j) { return make_tb_service(job_of(j)).dump(); });
  m.def("make_tb_deployment", [](const std::string& j) { return make_tb_deployment(job_of(j)).dump(); });

  m.def("is_retryable_termination", [](int code, const std::string& reason) {
    return is_retryable_termination(ContainerTermination{code, reason});
  });
  m.def("replica_state_from_pods", [](const std::string& items, const std::string& container) {
    return replica_state_from_pods(Json::parse(items), container);
  });
  m.def("aggregate_replica_states", &aggregate_replica_states);
  m.def("rand_string", &rand_string);
  m.def("yaml_to_json", [](const std::string& text) { return yaml_parse(text).dump(); });
  m.def("yaml_all_to_json", [](const std::string& text) {
    Json a = Json::array();
    for (auto& d : yaml_parse_all(text)) a.push_back(d);
    return a.dump();
  });

  // HTTP client probes (tests of the real transport: TLS verification, timeouts, keep-alive)
  m.def("kubeconfig", [](const std::string& text, const std::string& context) {
    ClusterConfig c = cluster_config_from_kubeconfig(text, context);
    py::dict d;
    d["host"] = c.host;
    d["port"] = c.port;
    d["tls"] = c.tls;
    d["insecure"] = c.insecure;
    d["token"] = c.token;
    d["ca_file"] = c.ca_file;
    d["ca_data"] = c.ca_data;
    d["cert_file"] = c.cert_file;
    d["cert_data"] = c.cert_data;
    d["key_file"] = c.key_file;
    d["key_data"] = c.key_data;
    d["tls_server_name"] = c.tls_server_name;
    return d;
  }, py::arg("text"), py::arg("context") = "");
  // n requests through a client configured from a kubeconfig (credentials: token / tokenFile / exec plugin with
  // refresh), the server address overridden by `url`; returns the HTTP codes
  m.def("kubeconfig_requests", [](const std::string& text, const std::string& url, const std::string& path, int n,
                                  int interval_ms) {
    ClusterConfig c = cluster_config_from_kubeconfig(text, "");
    ClusterConfig u = parse_master_url(url);
    c.host = u.host;
    c.port = u.port;
    c.tls = u.tls;
    auto api = make_http_api(c);
    std::vector<int> codes;
    {
      py::gil_scoped_release nogil;
      for (int i = 0; i < n; ++i) {
        if (i && interval_ms > 0) std::this_thread::sleep_for(std::chrono::milliseconds(interval_ms));
        codes.push_back(api->request("GET", path, nullptr, "application/json").code);
      }
    }
    return codes;
  }, py::arg("text"), py::arg("url"), py::arg("path") = "/version", py::arg("n") = 1, py::arg("interval_ms") = 0);
  m.def("http_request", [](const std::string& url, const std::string& method, const std::string& path,
                           const std::string& ca_data, const std::string& server_name, int timeout_ms, int repeat,
                           const std::string& cert_data, const std::string& key_data) {
    ClusterConfig c = parse_master_url(url);
    c.ca_data = ca_data;
    c.tls_server_name = server_name;
    c.cert_data = cert_data;
    c.key_data = key_data;
    if (timeout_ms > 0) {
      c.timeout_ms = timeout_ms;
      c.connect_timeout_ms = timeout_ms;
    }
    auto api = make_http_api(c);
    ApiResult r;
    {
      py::gil_scoped_release nogil;
      for (int i = 0; i < std::max(1, repeat); ++i) r = api->request(method, path, nullptr, "application/json");
    }
    return py::make_tuple(r.code, r.error, r.body.is_null() ? std::string() : r.body.dump());
  }, py::arg("url"), py::arg("method") = "GET", py::arg("path") = "/", py::arg("ca_data") = "",
     py::arg("server_name") = "", py::arg("timeout_ms") = 0, py::arg("repeat") = 1, py::arg("cert_data") = "",
     py::arg("key_data") = "");

  py::class_<PyInformer>(m, "Informer")
      .def(py::init<std::string, std::string, std::string, int, int, int, int, int>(), py::arg("url"),
           py::arg("path"), py::arg("selector") = "", py::arg("watch_timeout_ms") = 300000,
           py::arg("retry_ms") = 1000, py::arg("resync_ms") = 300000, py::arg("relist_after") = 3,
           py::arg("stale_ms") = 60000)
      .def("start", [](PyInformer& i) { i.inf->start(); })
      .def("stop", [](PyInformer& i) {
        py::gil_scoped_release nogil;
        i.inf->stop();
      })
      .def("wait_synced", [](PyInformer& i, int ms) {
        py::gil_scoped_release nogil;
        return i.inf->wait_synced(std::chrono::milliseconds(ms));
      })
      .def("synced", [](PyInformer& i) { return i.inf->synced(); })
      .def("fresh", [](PyInformer& i) { return i.inf->fresh(); })
      .def("size", [](PyInformer& i) { return i.inf->size(); })
      .def("lists", [](PyInformer& i) { return i.inf->lists(); })
      .def("watches", [](PyInformer& i) { return i.inf->watches(); })
      .def("names", [](PyInformer& i, const std::string& ns) {
        std::vector<std::string> out;
        Json items = i.inf->list(ns, Labels{});
        for (auto& o : items.as_array()) out.push_back(get_str(o.at("metadata"), "name"));
        return out;
      });

  py::class_<PyReconciler>(m, "Reconciler")
      .def(py::init<py::function, std::string, std::string, std::string>(), py::arg("api"), py::arg("job"),
           py::arg("config") = "", py::arg("ps_source") = "")
      .def("setup", [](PyReconciler& r) { r.job->setup(); })
      .def("reconcile", [](PyReconciler& r) { r.job->reconcile(); })
      .def("delete_resources", [](PyReconciler& r) { r.job->delete_resources(); })
      .def("status", [](PyReconciler& r) { return status_to_json(r.job->status()).dump(); })
      .def("job", [](PyReconciler& r) { return tfjob_to_json(r.job->job()).dump(); })
      .def("api_calls", [](PyReconciler& r) { return r.job->api_calls(); });
}
