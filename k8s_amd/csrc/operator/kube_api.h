// Kubernetes API access for the operator.
//
// Parity: /root/reference/pkg/util/k8sutil/k8sutil.go (cluster config,
// in-cluster token, AlreadyExists/NotFound helpers) and
// pkg/util/k8sutil/tf_job_client.go (TfJob REST client: Get/Create/Update/
// Delete/List/Watch on /apis/tensorflow.org/v1alpha1/...).
//
// `KubeApi` is a tiny REST surface (method + path + JSON body) so the same
// reconciler runs against a real API server (HttpKubeApi: HTTP/1.1, TLS via
// OpenSSL, bearer token) or the in-memory fake API server used by the tests
// and the local kubelet (k8s_amd/fakeapi).
#pragma once

#include <functional>
#include <memory>
#include <string>

#include "json.h"

namespace tfop {

struct ApiResult {
  int code = 0;  // HTTP status; 0 = transport error
  Json body;
  std::string error;
  bool ok() const { return code >= 200 && code < 300; }
  bool not_found() const { return code == 404; }
  bool already_exists() const { return code == 409 && reason() == "AlreadyExists"; }
  bool conflict() const { return code == 409 && reason() != "AlreadyExists"; }
  bool gone() const { return code == 410; }
  std::string reason() const { return body.is_object() ? get_str(body, "reason") : ""; }
  std::string message() const;
};

// A line-delimited JSON watch stream ({"type":..., "object":...} per line).
class WatchStream {
 public:
  virtual ~WatchStream() = default;
  // false on end-of-stream / error (err set). Blocks up to timeout_ms (-1 forever); returns true with
  // ev null on timeout.
  virtual bool next(Json& ev, int timeout_ms, std::string& err) = 0;
  virtual void close() = 0;
};

class KubeApi {
 public:
  virtual ~KubeApi() = default;
  virtual ApiResult request(const std::string& method, const std::string& path, const Json* body = nullptr,
                            const std::string& content_type = "application/json") = 0;
  virtual std::unique_ptr<WatchStream> watch(const std::string& path, std::string& err) = 0;

  ApiResult get(const std::string& p) { return request("GET", p); }
  ApiResult post(const std::string& p, const Json& b) { return request("POST", p, &b); }
  ApiResult put(const std::string& p, const Json& b) { return request("PUT", p, &b); }
  ApiResult del(const std::string& p, const Json* opts = nullptr) { return request("DELETE", p, opts); }
};

struct ClusterConfig {
  std::string host;  // hostname or IP
  int port = 443;
  bool tls = true;
  bool insecure = false;
  std::string token;
  std::string ca_file, ca_data;      // PEM file / PEM text (kubeconfig certificate-authority[-data])
  std::string cert_file, cert_data;  // client certificate (kubeconfig client-certificate[-data])
  std::string key_file, key_data;    // client key (kubeconfig client-key[-data])
  std::string tls_server_name;       // overrides the name checked against the server certificate
  // credential refresh (client-go re-runs an exec plugin when its token expires or a request gets 401, and
  // re-reads a rotated service-account / tokenFile token): the exec block as JSON, the token's expiry (unix
  // seconds from status.expirationTimestamp, 0 = none), the token file
  std::string exec_config;
  long long token_expiry = 0;
  std::string token_file;
  int exec_timeout_ms = 30000;       // an exec plugin that has not answered by then is killed
  int connect_timeout_ms = 10000;    // TCP connect + TLS handshake
  int timeout_ms = 30000;            // whole request (client-go's default REST timeout is similar)
  std::string user_agent = "tf_operator-amd/0.3.0";
};

// $KUBECONFIG (current-context server + credentials: token / tokenFile, client certificates, inline *-data,
// exec credential plugins), --master URL, or the in-cluster service account. Parity:
// /root/reference/pkg/util/k8sutil/k8sutil.go:45-65 (clientcmd.BuildConfigFromFlags / InClusterConfig).
ClusterConfig cluster_config_from_env(const std::string& master_url = "");
ClusterConfig parse_master_url(const std::string& url);
ClusterConfig cluster_config_from_kubeconfig(const std::string& text, const std::string& context = "");
// (Re)run the exec credential plugin of cfg.exec_config into cfg.token / cert / key / token_expiry.
void refresh_exec_credential(ClusterConfig& cfg);

// Per-thread request deadline override (milliseconds) for the HTTP client, e.g. a leader-election renew that
// must give up by the renew deadline: RequestTimeout t(remaining_ms); api.put(...);
class RequestTimeout {
 public:
  explicit RequestTimeout(int ms);
  ~RequestTimeout();
  static int current();  // -1: none

 private:
  int prev_;
};

std::string base64_decode(const std::string& in);

std::unique_ptr<KubeApi> make_http_api(const ClusterConfig& cfg);

// ---- REST paths
std::string core_path(const std::string& ns, const std::string& resource, const std::string& name = "");
std::string group_path(const std::string& group_version, const std::string& ns, const std::string& resource,
                       const std::string& name = "");
std::string tfjobs_path(const std::string& ns, const std::string& name = "");  // ns "" => all namespaces
std::string crd_path(const std::string& name = "");
std::string url_escape(const std::string& s);

}  // namespace tfop
