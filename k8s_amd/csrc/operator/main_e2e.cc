// e2e: the helm-test end-to-end binary.
//
// Parity: /root/reference/test/e2e/main.go -- create a TfJob with a MASTER
// (--image), a default PS and a WORKER (--image) plus TensorBoard
// (/tmp/tensorflow); poll every 5 s until Succeeded/Failed or --timeout;
// assert RuntimeId, one batch Job per replica/index, TensorBoard Deployment +
// Service; delete the TfJob and wait for garbage collection; --num_jobs jobs
// in parallel; TAP output ("1..1" / "ok 1 - ...").
// Extra flags for MI355X clusters: --gpus N puts amd.com/gpu: N limits on the
// MASTER/WORKER containers, --command overrides the container command.
#include <chrono>
#include <cstdio>
#include <future>
#include <thread>

#include "flags.h"
#include "kube_api.h"
#include "log.h"
#include "reconciler.h"
#include "replicas.h"
#include "spec.h"

using namespace tfop;
using Clock = std::chrono::steady_clock;

static std::string g_ns = "default";

static Json container(const std::string& image, int gpus, const std::string& command) {
  Json c = Json::object();
  c["name"] = "tensorflow";
  c["image"] = image;
  if (!command.empty()) {
    Json cmd = Json::array();
    for (const char* a : {"sh", "-c"}) cmd.push_back(a);
    cmd.push_back(command);
    c["command"] = cmd;
  }
  if (gpus > 0) {
    Json lim = Json::object();
    lim["amd.com/gpu"] = gpus;
    Json res = Json::object();
    res["limits"] = lim;
    c["resources"] = res;
  }
  return c;
}

static Json replica(const std::string& type, const std::string& image, int gpus, const std::string& command) {
  Json r = Json::object();
  r["replicas"] = 1;
  r["tfPort"] = 2222;
  r["tfReplicaType"] = type;
  if (type != "PS") {
    Json spec = Json::object();
    spec["containers"] = JsonArray{container(image, gpus, command)};
    spec["restartPolicy"] = "OnFailure";
    Json t = Json::object();
    t["spec"] = spec;
    r["template"] = t;
  }
  return r;
}

static std::string run_one(KubeApi& api, const std::string& image, int gpus, const std::string& command,
                           std::chrono::milliseconds timeout, std::string& name) {
  name = "e2e-test-job-" + rand_string(4);
  Json job = Json::object();
  job["apiVersion"] = "tensorflow.org/v1alpha1";
  job["kind"] = "TfJob";
  Json md = Json::object();
  md["name"] = name;
  md["namespace"] = g_ns;
  Json lbl = Json::object();
  lbl["test.mlkube.io"] = "";
  md["labels"] = lbl;
  job["metadata"] = md;
  Json spec = Json::object();
  spec["replicaSpecs"] = JsonArray{replica("MASTER", image, gpus, command), replica("PS", image, 0, ""),
                                   replica("WORKER", image, gpus, command)};
  Json tb = Json::object();
  tb["logDir"] = "/tmp/tensorflow";
  spec["tensorboard"] = tb;
  job["spec"] = spec;
  ApiResult c = api.post(tfjobs_path(g_ns), job);
  if (!c.ok()) return "Creating the job failed; " + c.message();

  TfJob cur;
  const auto deadline = Clock::now() + timeout;
  while (true) {
    ApiResult g = api.get(tfjobs_path(g_ns, name));
    if (g.ok()) {
      cur = tfjob_from_json(g.body);
      log_info("Job %s state=%s phase=%s", name.c_str(), cur.status.state.c_str(), cur.status.phase.c_str());
      if (cur.status.state == "Succeeded" || cur.status.state == "Failed") break;
    }
    if (Clock::now() > deadline) return "timed out waiting for TfJob " + name;
    std::this_thread::sleep_for(std::chrono::seconds(5));
  }
  if (cur.status.state != "Succeeded") return "TfJob " + name + " did not succeed: state=" + cur.status.state;
  if (cur.spec.runtime_id.empty()) return "TfJob " + name + " doesn't have a RuntimeId";
  for (auto& r : cur.spec.replica_specs)
    for (int i = 0; i < r.replicas.value_or(1); ++i) {
      const std::string jn = replica_job_name(cur, r.type, i);
      if (!api.get(group_path("batch/v1", g_ns, "jobs", jn)).ok()) return "Did not find Job " + jn;
    }
  const std::string tbn = tb_name(cur);
  if (!api.get(group_path("apps/v1", g_ns, "deployments", tbn)).ok()) return "TensorBoard deployment not found";
  if (!api.get(core_path(g_ns, "services", tbn)).ok()) return "TensorBoard service not found";

  Json opts = Json::object();
  opts["propagationPolicy"] = "Foreground";
  ApiResult d = api.del(tfjobs_path(g_ns, name), &opts);
  if (!d.ok()) return "Deleting TfJob " + name + " failed; " + d.message();
  // wait for garbage collection of the replica Jobs and the TensorBoard deployment
  while (true) {
    bool gone = true;
    for (auto& r : cur.spec.replica_specs)
      for (int i = 0; i < r.replicas.value_or(1); ++i)
        if (!api.get(group_path("batch/v1", g_ns, "jobs", replica_job_name(cur, r.type, i))).not_found()) gone = false;
    if (!api.get(group_path("apps/v1", g_ns, "deployments", tbn)).not_found()) gone = false;
    if (gone) break;
    if (Clock::now() > deadline) return "timed out waiting for resources of " + name + " to be deleted";
    std::this_thread::sleep_for(std::chrono::seconds(1));
  }
  return "";
}

int main(int argc, char** argv) {
  Flags fl;
  fl.def("image", "", "The Docker image containing the TF program to run.");
  fl.def("num_jobs", "1", "The number of jobs to run.");
  fl.def("timeout", "300", "The timeout for the test in seconds (or 5m / 300s).");
  fl.def("master", "", "API server URL");
  fl.def("namespace", "default", "Namespace");
  fl.def("gpus", "0", "amd.com/gpu limit for MASTER/WORKER containers");
  fl.def("command", "", "Shell command for the MASTER/WORKER containers (overrides the image entrypoint)");
  std::string err = fl.parse(argc, argv);
  if (!err.empty()) {
    fprintf(stderr, "%s\n%s", err.c_str(), fl.usage().c_str());
    return 2;
  }
  g_verbosity = fl.num("v");
  if (fl.str("image").empty()) {
    log_error("--image must be provided.");
    return 1;
  }
  g_ns = fl.str("namespace");
  std::string ts = fl.str("timeout");
  long tmo = 300000;
  if (!ts.empty()) {
    double v = atof(ts.c_str());
    tmo = ts.back() == 'm' ? (long)(v * 60000) : (long)(v * 1000);
  }
  auto api = make_http_api(cluster_config_from_env(fl.str("master")));
  const int n = fl.num("num_jobs");
  std::vector<std::future<std::pair<std::string, std::string>>> futs;
  for (int i = 0; i < n; ++i)
    futs.push_back(std::async(std::launch::async, [&] {
      std::string name;
      std::string e = run_one(*api, fl.str("image"), fl.num("gpus"), fl.str("command"),
                              std::chrono::milliseconds(tmo), name);
      if (!e.empty()) log_error("TfJob %s didn't run successfully; %s", name.c_str(), e.c_str());
      else log_info("TfJob %s ran successfully", name.c_str());
      return std::make_pair(name, e);
    }));
  int ok = 0;
  for (auto& f : futs)
    if (f.get().second.empty()) ++ok;
  printf("1..1\n");
  if (ok == n) {
    printf("ok 1 - Successfully ran TfJob\n");
    return 0;
  }
  printf("not ok 1 - Running TfJobs failed \n");
  return 1;
}
