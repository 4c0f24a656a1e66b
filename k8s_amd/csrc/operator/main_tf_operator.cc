// tf_operator: the TfJob operator binary.
//
// Parity: /root/reference/cmd/tf_operator/main.go (flags :48-54, config
// file :68-85, MY_POD_NAMESPACE / MY_POD_NAME :89-96, signal exit :98-103,
// version :105-116, Endpoints leader election 15s/5s/3s :42-44,125-148,
// controller run loop :153-169). Leader election defaults to a coordination.k8s.io/v1 Lease
// (-leader-elect-resource-lock=endpoints keeps the reference's lock). The chaos monkey the reference left
// commented out (:171-207) is implemented: -chaos-level N deletes a random
// TfJob pod every 30/N seconds (fault injection for the exit-code/restart
// state machine).
#include <signal.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <thread>

#include "controller.h"
#include "election.h"
#include "flags.h"
#include "log.h"
#include "yaml_lite.h"

using namespace tfop;

static std::atomic<bool> g_stop{false};

static long parse_duration_ms(const std::string& s, long def) {
  if (s.empty()) return def;
  size_t i = 0;
  double v = std::stod(s, &i);
  std::string unit = s.substr(i);
  if (unit == "ms") return (long)v;
  if (unit == "s" || unit.empty()) return (long)(v * 1000);
  if (unit == "m") return (long)(v * 60000);
  if (unit == "h") return (long)(v * 3600000);
  return def;
}

static void chaos_loop(KubeApi* api, std::string ns, int level) {
  std::mt19937 rng{std::random_device{}()};
  while (!g_stop) {
    for (int i = 0; i < 300 / level && !g_stop; ++i) std::this_thread::sleep_for(std::chrono::milliseconds(100));
    ApiResult l = api->get(core_path(ns, "pods") + "?labelSelector=tensorflow.org%3D");
    if (!l.ok()) continue;
    const Json* items = l.body.find("items");
    if (!items || !items->is_array() || items->size() == 0) continue;
    const Json& p = (*items)[rng() % items->size()];
    const std::string name = get_str(p.at("metadata"), "name");
    log_warn("chaos: deleting pod %s/%s", ns.c_str(), name.c_str());
    api->del(core_path(ns, "pods", name));
  }
}

int main(int argc, char** argv) {
  Flags fl;
  fl.def("controller_config_file", "", "Path to file containing the controller config.");
  fl.def("version", "false", "Show version and quit", true);
  fl.def("chaos-level", "-1", "DO NOT USE IN PRODUCTION - level of chaos injected into the TfJob created by the operator.");
  fl.def("gc-interval", "10m", "GC interval");
  fl.def("master", "", "API server URL (default: $K8S_AMD_APISERVER, $KUBECONFIG, then in-cluster)");
  fl.def("namespace", "", "Namespace to manage (default $MY_POD_NAMESPACE)");
  fl.def("all-namespaces", "false", "Manage TfJobs in every namespace", true);
  fl.def("reconcile-interval", "8s", "Resync period of every TfJob (reference: 8s)");
  fl.def("leader-elect", "true", "Run leader election on Endpoints tf-operator", true);
  // cmd/tf_operator/main.go:42-44 hard-codes 15s / 5s / 3s; kept as the defaults, settable for HA drills/tests
  fl.def("lease-duration", "15s", "Leader-election lease duration");
  fl.def("renew-deadline", "5s", "Leader-election renew deadline");
  fl.def("retry-period", "3s", "Leader-election retry period");
  fl.def("create-crd", "true", "Register the tfjobs.tensorflow.org CRD at startup", true);
  fl.def("leader-elect-resource-lock", "endpointsleases", "Leader-election lock: endpointsleases (both: safe across upgrades from either), leases (coordination.k8s.io/v1) or endpoints");
  fl.def("request-timeout", "30s", "Deadline of every API request (connect, TLS handshake, response)");
  fl.def("event-watchdog", "60s", "Abort when one TfJob event handler runs longer (reference panicTimer: 1m)");
  fl.def("inject-handler-stall", "0s", "DO NOT USE IN PRODUCTION - fault injection: stall every TfJob event handler this long");
  fl.def("watch-timeout", "5m", "Each TfJob watch asks the server to end it after a random timeoutSeconds in [t, 2t)");
  fl.def("watch-idle-grace", "30s", "A watch still open this long past its timeoutSeconds is half-open: re-watch");
  fl.def("resync-period", "5m", "Full relist of the TfJobs this often (0: never), so a lost watch event is recovered");
  fl.def("informers", "true", "Shared watch caches of the replica Jobs / Pods (false: per-replica GET / LIST every tick)", true);
  std::string err = fl.parse(argc, argv);
  if (!err.empty()) {
    fprintf(stderr, "%s\nUsage of tf_operator:\n%s", err.c_str(), fl.usage().c_str());
    return 2;
  }
  g_verbosity = fl.num("v");
  if (fl.on("version")) {
    printf("tf_operator Version: %s\nGit SHA: %s\nGo Version: n/a (C++17)\nGo OS/Arch: linux/amd64\n", kVersion,
           kGitSHA);
    return 0;
  }
  ControllerConfig cfg;
  if (!fl.str("controller_config_file").empty()) {
    try {
      cfg = controller_config_from_json(yaml_parse(read_file(fl.str("controller_config_file"))));
    } catch (const std::exception& e) {
      log_error("could not read controller config file %s: %s", fl.str("controller_config_file").c_str(), e.what());
      return 1;
    }
  } else {
    log_info("No controller_config_file provided; using empty config.");
  }
  std::string ns = fl.str("namespace");
  if (ns.empty() && getenv("MY_POD_NAMESPACE")) ns = getenv("MY_POD_NAMESPACE");
  if (ns.empty()) {
    log_error("must set env MY_POD_NAMESPACE");
    return 1;
  }
  std::string pod = getenv("MY_POD_NAME") ? getenv("MY_POD_NAME") : "";
  if (pod.empty()) {
    log_error("must set env MY_POD_NAME");
    return 1;
  }
  for (int s : {SIGINT, SIGTERM}) signal(s, [](int sig) {
      log_info("received signal: %d, exiting", sig);
      _exit(1);
    });
  log_info("tf_operator Version: %s", kVersion);

  ClusterConfig cc;
  try {
    cc = cluster_config_from_env(fl.str("master"));
  } catch (const std::exception& e) {
    log_error("cluster config: %s", e.what());
    return 1;
  }
  cc.timeout_ms = (int)parse_duration_ms(fl.str("request-timeout"), 30000);
  cc.connect_timeout_ms = std::min(cc.connect_timeout_ms, cc.timeout_ms);
  cc.user_agent = std::string("tf_operator-amd/") + kVersion + " (" + pod + ")";
  auto api = make_http_api(cc);

  ControllerOptions opts;
  opts.ns = fl.on("all-namespaces") ? "" : ns;
  opts.create_crd = fl.on("create-crd");
  opts.reconcile.interval = std::chrono::milliseconds(parse_duration_ms(fl.str("reconcile-interval"), 8000));
  opts.event_watchdog = std::chrono::milliseconds(parse_duration_ms(fl.str("event-watchdog"), 60000));
  opts.inject_handler_stall = std::chrono::milliseconds(parse_duration_ms(fl.str("inject-handler-stall"), 0));
  opts.watch_timeout = std::chrono::milliseconds(parse_duration_ms(fl.str("watch-timeout"), 300000));
  opts.watch_idle_grace = std::chrono::milliseconds(parse_duration_ms(fl.str("watch-idle-grace"), 30000));
  opts.resync_period = std::chrono::milliseconds(parse_duration_ms(fl.str("resync-period"), 300000));
  opts.informers = fl.on("informers");
  if (!cfg.grpc_server_file_path.empty()) {
    try {
      opts.reconcile.ps_server_source = read_file(cfg.grpc_server_file_path);
    } catch (const std::exception& e) {
      log_error("cannot read grpcServerFilePath %s: %s", cfg.grpc_server_file_path.c_str(), e.what());
    }
  }
  const int chaos = fl.num("chaos-level");
  if (chaos > 0) std::thread(chaos_loop, api.get(), ns, chaos).detach();

  auto run_controller = [&] {
    Controller c(*api, cfg, opts);
    std::string e = c.run();
    if (!e.empty()) {
      log_error("controller Run() ended with failure: %s", e.c_str());
      _exit(1);
    }
  };
  if (!fl.on("leader-elect")) {
    run_controller();
    return 0;
  }
  ElectionConfig ec;
  ec.ns = ns;
  ec.name = "tf-operator";
  ec.identity = pod;
  ec.lease = std::chrono::milliseconds(parse_duration_ms(fl.str("lease-duration"), 15000));
  ec.renew_deadline = std::chrono::milliseconds(parse_duration_ms(fl.str("renew-deadline"), 5000));
  ec.retry = std::chrono::milliseconds(parse_duration_ms(fl.str("retry-period"), 3000));
  ec.lock_type = fl.str("leader-elect-resource-lock");
  if (ec.lock_type != "leases" && ec.lock_type != "endpoints" && ec.lock_type != "endpointsleases") {
    log_error("-leader-elect-resource-lock must be endpointsleases, leases or endpoints");
    return 1;
  }
  LeaderElector el(*api, ec);
  if (std::string e = el.check(); !e.empty()) {
    log_error("leader election config: %s", e.c_str());
    return 1;
  }
  el.run(run_controller, [] {
    log_error("leader election lost");
    _exit(1);
  }, g_stop);
  return 0;
}
