#include <ctime>
#include <signal.h>
#include "kube_api.h"

#include <condition_variable>
#include <thread>
#include "log.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <openssl/err.h>
#include <openssl/pem.h>
#include <openssl/ssl.h>
#include <openssl/x509v3.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/wait.h>
#include <unistd.h>

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <sstream>
#include <stdexcept>
#include <vector>

#include "spec.h"
#include "yaml_lite.h"

namespace tfop {

std::string ApiResult::message() const {
  if (!error.empty()) return error;
  if (body.is_object()) {
    std::string m = get_str(body, "message");
    if (!m.empty()) return m;
  }
  return "HTTP " + std::to_string(code);
}

std::string url_escape(const std::string& s) {
  static const char* hex = "0123456789ABCDEF";
  std::string o;
  for (unsigned char c : s) {
    if (isalnum(c) || c == '-' || c == '_' || c == '.' || c == '~' || c == '/') {
      o += (char)c;
    } else {
      o += '%';
      o += hex[c >> 4];
      o += hex[c & 15];
    }
  }
  return o;
}

std::string core_path(const std::string& ns, const std::string& resource, const std::string& name) {
  std::string p = "/api/v1";
  if (!ns.empty()) p += "/namespaces/" + ns;
  p += "/" + resource;
  if (!name.empty()) p += "/" + name;
  return p;
}

std::string group_path(const std::string& gv, const std::string& ns, const std::string& resource,
                       const std::string& name) {
  std::string p = "/apis/" + gv;
  if (!ns.empty()) p += "/namespaces/" + ns;
  p += "/" + resource;
  if (!name.empty()) p += "/" + name;
  return p;
}

std::string tfjobs_path(const std::string& ns, const std::string& name) {
  return group_path(std::string(kCRDGroup) + "/" + kCRDVersion, ns, kCRDKindPlural, name);
}

std::string crd_path(const std::string& name) {
  return "/apis/apiextensions.k8s.io/v1/customresourcedefinitions" + (name.empty() ? "" : "/" + name);
}

// ------------------------------------------------------------------ config
ClusterConfig parse_master_url(const std::string& url) {
  ClusterConfig c;
  std::string u = url;
  if (u.rfind("http://", 0) == 0) {
    c.tls = false;
    c.port = 80;
    u = u.substr(7);
  } else if (u.rfind("https://", 0) == 0) {
    c.tls = true;
    c.port = 443;
    u = u.substr(8);
  }
  size_t slash = u.find('/');
  if (slash != std::string::npos) u = u.substr(0, slash);
  size_t colon = u.rfind(':');
  if (colon != std::string::npos && u.find(']') == std::string::npos) {
    c.port = atoi(u.substr(colon + 1).c_str());
    u = u.substr(0, colon);
  }
  c.host = u;
  return c;
}

static std::string env(const char* k) {
  const char* v = getenv(k);
  return v ? v : "";
}

std::string base64_decode(const std::string& in) {
  static int8_t T[256];
  static std::once_flag once;
  std::call_once(once, [] {
    for (int i = 0; i < 256; ++i) T[i] = -1;
    const char* a = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
    for (int i = 0; i < 64; ++i) T[(unsigned char)a[i]] = (int8_t)i;
    T[(unsigned char)'-'] = 62;  // url-safe alphabet too
    T[(unsigned char)'_'] = 63;
  });
  std::string out;
  unsigned val = 0;
  int bits = -8;
  for (unsigned char c : in) {
    if (c == '=') break;
    if (T[c] < 0) continue;  // whitespace / newlines
    val = (val << 6) | (unsigned)T[c];
    bits += 6;
    if (bits >= 0) {
      out.push_back((char)((val >> bits) & 0xFF));
      bits -= 8;
    }
  }
  return out;
}

// ---- exec credential plugin (client.authentication.k8s.io ExecCredential): run the command, read
// status.{token, clientCertificateData, clientKeyData, expirationTimestamp} from its stdout. A plugin that has not
// finished within out.exec_timeout_ms is killed (a hung plugin must not block the operator forever).
static long long parse_rfc3339(const std::string& t) {
  struct tm tmv = {};
  if (t.size() < 19 || !strptime(t.c_str(), "%Y-%m-%dT%H:%M:%S", &tmv)) return 0;
  return (long long)timegm(&tmv);
}

static void run_exec_plugin(const Json& ex, ClusterConfig& out) {
  std::vector<std::string> argv{get_str(ex, "command")};
  if (argv[0].empty()) throw std::runtime_error("kubeconfig exec: no command");
  if (const Json* a = ex.find("args"); a && a->is_array())
    for (auto& v : a->as_array()) argv.push_back(v.as_string());
  std::vector<std::pair<std::string, std::string>> envs;
  if (const Json* e = ex.find("env"); e && e->is_array())
    for (auto& v : e->as_array()) envs.emplace_back(get_str(v, "name"), get_str(v, "value"));
  int pfd[2];
  if (pipe(pfd) != 0) throw std::runtime_error("kubeconfig exec: pipe failed");
  pid_t pid = fork();
  if (pid < 0) throw std::runtime_error("kubeconfig exec: fork failed");
  if (pid == 0) {
    dup2(pfd[1], 1);
    ::close(pfd[0]);
    ::close(pfd[1]);
    for (auto& kv : envs) setenv(kv.first.c_str(), kv.second.c_str(), 1);
    setenv("KUBERNETES_EXEC_INFO",
           "{\"apiVersion\":\"client.authentication.k8s.io/v1\",\"kind\":\"ExecCredential\",\"spec\":"
           "{\"interactive\":false}}", 1);
    std::vector<char*> av;
    for (auto& a : argv) av.push_back(const_cast<char*>(a.c_str()));
    av.push_back(nullptr);
    execvp(av[0], av.data());
    _exit(127);
  }
  ::close(pfd[1]);
  std::string text;
  char buf[4096];
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(out.exec_timeout_ms);
  bool timed_out = false;
  for (;;) {
    const long left = (long)std::chrono::duration_cast<std::chrono::milliseconds>(
                          deadline - std::chrono::steady_clock::now()).count();
    if (left <= 0) {
      timed_out = true;
      break;
    }
    struct pollfd p{pfd[0], POLLIN, 0};
    const int pr = poll(&p, 1, (int)std::min<long>(left, 1000));
    if (pr < 0 && errno != EINTR) break;
    if (pr <= 0) continue;
    const long n = ::read(pfd[0], buf, sizeof buf);
    if (n <= 0) break;
    text.append(buf, (size_t)n);
  }
  ::close(pfd[0]);
  if (timed_out) kill(pid, SIGKILL);
  int status = 0;
  waitpid(pid, &status, 0);
  if (timed_out) throw std::runtime_error("kubeconfig exec plugin " + argv[0] + " timed out");
  if (!WIFEXITED(status) || WEXITSTATUS(status) != 0)
    throw std::runtime_error("kubeconfig exec plugin " + argv[0] + " failed");
  Json cred = Json::parse(text);
  const Json* st = cred.find("status");
  if (!st) throw std::runtime_error("kubeconfig exec plugin: no status in ExecCredential");
  if (std::string t = get_str(*st, "token"); !t.empty()) out.token = t;
  if (std::string c = get_str(*st, "clientCertificateData"); !c.empty()) out.cert_data = c;
  if (std::string k = get_str(*st, "clientKeyData"); !k.empty()) out.key_data = k;
  out.token_expiry = parse_rfc3339(get_str(*st, "expirationTimestamp"));
}

void refresh_exec_credential(ClusterConfig& cfg) {
  if (cfg.exec_config.empty()) return;
  run_exec_plugin(Json::parse(cfg.exec_config), cfg);
}

ClusterConfig cluster_config_from_kubeconfig(const std::string& text, const std::string& context) {
  Json cfg = yaml_parse(text);
  std::string cur = context.empty() ? get_str(cfg, "current-context") : context;
  std::string cluster_name, user_name;
  if (const Json* ctxs = cfg.find("contexts"); ctxs && ctxs->is_array())
    for (auto& c : ctxs->as_array())
      if (get_str(c, "name") == cur || cur.empty()) {
        if (const Json* cc = c.find("context")) {
          cluster_name = get_str(*cc, "cluster");
          user_name = get_str(*cc, "user");
        }
        break;
      }
  ClusterConfig out;
  if (const Json* cl = cfg.find("clusters"); cl && cl->is_array())
    for (auto& c : cl->as_array())
      if (get_str(c, "name") == cluster_name || cluster_name.empty()) {
        if (const Json* cc = c.find("cluster")) {
          out = parse_master_url(get_str(*cc, "server"));
          out.ca_file = get_str(*cc, "certificate-authority");
          if (std::string d = get_str(*cc, "certificate-authority-data"); !d.empty()) out.ca_data = base64_decode(d);
          out.tls_server_name = get_str(*cc, "tls-server-name");
          if (const Json* v = cc->find("insecure-skip-tls-verify"); v && v->is_bool()) out.insecure = v->as_bool();
        }
        break;
      }
  if (const Json* us = cfg.find("users"); us && us->is_array())
    for (auto& u : us->as_array())
      if (get_str(u, "name") == user_name || user_name.empty()) {
        if (const Json* uu = u.find("user")) {
          out.token = get_str(*uu, "token");
          if (std::string tf = get_str(*uu, "tokenFile"); out.token.empty() && !tf.empty()) {
            out.token = read_file(tf);
            while (!out.token.empty() && isspace((unsigned char)out.token.back())) out.token.pop_back();
          }
          out.cert_file = get_str(*uu, "client-certificate");
          if (std::string d = get_str(*uu, "client-certificate-data"); !d.empty()) out.cert_data = base64_decode(d);
          out.key_file = get_str(*uu, "client-key");
          if (std::string d = get_str(*uu, "client-key-data"); !d.empty()) out.key_data = base64_decode(d);
          if (std::string tf = get_str(*uu, "tokenFile"); !tf.empty()) out.token_file = tf;
          if (const Json* ex = uu->find("exec"); ex && ex->is_object()) {
            out.exec_config = ex->dump();
            if (const char* t = getenv("K8S_AMD_EXEC_TIMEOUT_MS"); t && atoi(t) > 0) out.exec_timeout_ms = atoi(t);
            run_exec_plugin(*ex, out);
          }
        }
        break;
      }
  return out;
}

ClusterConfig cluster_config_from_env(const std::string& master_url) {
  if (!master_url.empty()) return parse_master_url(master_url);
  if (!env("K8S_AMD_APISERVER").empty()) return parse_master_url(env("K8S_AMD_APISERVER"));
  const std::string kc = env("KUBECONFIG");
  if (!kc.empty()) return cluster_config_from_kubeconfig(read_file(kc.substr(0, kc.find(':'))));
  // in-cluster (pkg/util/k8sutil/k8sutil.go:54-63: default port 443)
  ClusterConfig c;
  c.host = env("KUBERNETES_SERVICE_HOST");
  if (c.host.empty()) c.host = "kubernetes.default.svc";
  const std::string port = env("KUBERNETES_SERVICE_PORT");
  c.port = port.empty() ? 443 : atoi(port.c_str());
  c.tls = true;
  const std::string sa = "/var/run/secrets/kubernetes.io/serviceaccount/";
  try {
    c.token = read_file(sa + "token");
    while (!c.token.empty() && isspace((unsigned char)c.token.back())) c.token.pop_back();
    c.token_file = sa + "token";  // bound service-account tokens are rotated by the kubelet: re-read
  } catch (...) {
  }
  c.ca_file = sa + "ca.crt";
  // the API server certificate names kubernetes.default.svc, not the service IP we dial
  c.tls_server_name = "kubernetes.default.svc";
  return c;
}

// ------------------------------------------------------------------ request deadlines
static thread_local int t_timeout_override = -1;
RequestTimeout::RequestTimeout(int ms) : prev_(t_timeout_override) { t_timeout_override = ms; }
RequestTimeout::~RequestTimeout() { t_timeout_override = prev_; }
int RequestTimeout::current() { return t_timeout_override; }

// ------------------------------------------------------------------ transport
namespace {

std::once_flag ssl_once;
using Clock = std::chrono::steady_clock;

struct Deadline {
  Clock::time_point t;
  bool forever = false;
  static Deadline in_ms(int ms) {
    Deadline d;
    if (ms < 0) d.forever = true;
    else d.t = Clock::now() + std::chrono::milliseconds(ms);
    return d;
  }
  int left_ms() const {  // -1 forever, 0 expired
    if (forever) return -1;
    const long ms = std::chrono::duration_cast<std::chrono::milliseconds>(t - Clock::now()).count();
    return ms <= 0 ? 0 : (int)ms;
  }
};

static bool is_ip_literal(const std::string& h) {
  unsigned char b[16];
  return inet_pton(AF_INET, h.c_str(), b) == 1 || inet_pton(AF_INET6, h.c_str(), b) == 1;
}

static bool load_pem_ca(SSL_CTX* ctx, const std::string& pem) {
  BIO* bio = BIO_new_mem_buf(pem.data(), (int)pem.size());
  X509_STORE* store = SSL_CTX_get_cert_store(ctx);
  int n = 0;
  while (X509* x = PEM_read_bio_X509(bio, nullptr, nullptr, nullptr)) {
    X509_STORE_add_cert(store, x);
    X509_free(x);
    ++n;
  }
  ERR_clear_error();
  BIO_free(bio);
  return n > 0;
}

static std::string ssl_err() {
  char buf[256];
  unsigned long e = ERR_get_error();
  if (!e) return "unknown TLS error";
  ERR_error_string_n(e, buf, sizeof buf);
  ERR_clear_error();
  return buf;
}

class Conn {
 public:
  explicit Conn(const ClusterConfig& cfg) : cfg_(cfg) {}
  ~Conn() { close(); }

  // TCP connect (non-blocking + poll) and TLS handshake, both bounded by the deadline
  bool open(const Deadline& dl, std::string& err) {
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_UNSPEC;
    hints.ai_socktype = SOCK_STREAM;
    int rc = getaddrinfo(cfg_.host.c_str(), std::to_string(cfg_.port).c_str(), &hints, &res);
    if (rc != 0) {
      err = std::string("resolve ") + cfg_.host + ": " + gai_strerror(rc);
      return false;
    }
    err = "connect " + cfg_.host + ":" + std::to_string(cfg_.port) + ": no address";
    for (addrinfo* a = res; a && fd_ < 0; a = a->ai_next) {
      int fd = socket(a->ai_family, a->ai_socktype | SOCK_NONBLOCK | SOCK_CLOEXEC, a->ai_protocol);
      if (fd < 0) continue;
      int r = connect(fd, a->ai_addr, a->ai_addrlen);
      if (r != 0 && errno == EINPROGRESS) {
        pollfd p{fd, POLLOUT, 0};
        int pr = poll(&p, 1, std::min(dl.left_ms() < 0 ? cfg_.connect_timeout_ms : dl.left_ms(),
                                      cfg_.connect_timeout_ms));
        int soerr = 0;
        socklen_t sl = sizeof soerr;
        if (pr == 1 && getsockopt(fd, SOL_SOCKET, SO_ERROR, &soerr, &sl) == 0 && soerr == 0) r = 0;
        else errno = pr == 0 ? ETIMEDOUT : (soerr ? soerr : errno);
      }
      if (r == 0) {
        fd_ = fd;
        break;
      }
      err = "connect " + cfg_.host + ":" + std::to_string(cfg_.port) + ": " + strerror(errno);
      ::close(fd);
    }
    freeaddrinfo(res);
    if (fd_ < 0) return false;
    int one = 1;
    setsockopt(fd_, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    setsockopt(fd_, SOL_SOCKET, SO_KEEPALIVE, &one, sizeof one);
    if (!cfg_.tls) return true;
    std::call_once(ssl_once, [] {
      SSL_library_init();
      SSL_load_error_strings();
    });
    ctx_ = SSL_CTX_new(TLS_client_method());
    if (!cfg_.insecure) {
      bool have_ca = false;
      if (!cfg_.ca_data.empty()) have_ca = load_pem_ca(ctx_, cfg_.ca_data);
      if (!cfg_.ca_file.empty()) have_ca = SSL_CTX_load_verify_locations(ctx_, cfg_.ca_file.c_str(), nullptr) == 1;
      if (!have_ca) SSL_CTX_set_default_verify_paths(ctx_);
      SSL_CTX_set_verify(ctx_, SSL_VERIFY_PEER, nullptr);
    }
    if (!cfg_.cert_data.empty() || !cfg_.cert_file.empty()) {
      bool ok = false;
      if (!cfg_.cert_data.empty()) {
        BIO* b = BIO_new_mem_buf(cfg_.cert_data.data(), (int)cfg_.cert_data.size());
        X509* x = PEM_read_bio_X509(b, nullptr, nullptr, nullptr);
        ok = x && SSL_CTX_use_certificate(ctx_, x) == 1;
        if (x) X509_free(x);
        BIO_free(b);
      } else {
        ok = SSL_CTX_use_certificate_chain_file(ctx_, cfg_.cert_file.c_str()) == 1;
      }
      if (ok && !cfg_.key_data.empty()) {
        BIO* b = BIO_new_mem_buf(cfg_.key_data.data(), (int)cfg_.key_data.size());
        EVP_PKEY* k = PEM_read_bio_PrivateKey(b, nullptr, nullptr, nullptr);
        ok = k && SSL_CTX_use_PrivateKey(ctx_, k) == 1;
        if (k) EVP_PKEY_free(k);
        BIO_free(b);
      } else if (ok) {
        ok = SSL_CTX_use_PrivateKey_file(ctx_, cfg_.key_file.c_str(), SSL_FILETYPE_PEM) == 1;
      }
      if (!ok) {
        err = "client certificate/key: " + ssl_err();
        return false;
      }
    }
    ssl_ = SSL_new(ctx_);
    SSL_set_fd(ssl_, fd_);
    const std::string name = cfg_.tls_server_name.empty() ? cfg_.host : cfg_.tls_server_name;
    if (!is_ip_literal(name)) SSL_set_tlsext_host_name(ssl_, name.c_str());
    if (!cfg_.insecure) {
      // hostname (or IP SAN) verification: a CA-valid certificate for another name is rejected
      X509_VERIFY_PARAM* vp = SSL_get0_param(ssl_);
      if (is_ip_literal(name)) X509_VERIFY_PARAM_set1_ip_asc(vp, name.c_str());
      else SSL_set1_host(ssl_, name.c_str());
    }
    // non-blocking handshake driven by poll, bounded by the connect timeout / deadline
    const Deadline hs = Deadline::in_ms(std::min(dl.left_ms() < 0 ? cfg_.connect_timeout_ms : dl.left_ms(),
                                                 cfg_.connect_timeout_ms));
    while (true) {
      int r = SSL_connect(ssl_);
      if (r == 1) break;
      int e = SSL_get_error(ssl_, r);
      if (e != SSL_ERROR_WANT_READ && e != SSL_ERROR_WANT_WRITE) {
        long vr = SSL_get_verify_result(ssl_);
        err = std::string("TLS handshake: ") + (vr != X509_V_OK ? X509_verify_cert_error_string(vr) : ssl_err());
        return false;
      }
      pollfd p{fd_, (short)(e == SSL_ERROR_WANT_READ ? POLLIN : POLLOUT), 0};
      if (poll(&p, 1, hs.left_ms()) <= 0) {
        err = "TLS handshake: timed out";
        return false;
      }
    }
    return true;
  }

  void close() {
    if (ssl_) {
      SSL_free(ssl_);  // no close_notify: the peer may be gone, and a blocking shutdown could hang
      ssl_ = nullptr;
    }
    if (ctx_) {
      SSL_CTX_free(ctx_);
      ctx_ = nullptr;
    }
    if (fd_ >= 0) {
      ::close(fd_);
      fd_ = -1;
    }
  }

  bool write_all(const std::string& s, const Deadline& dl) {
    size_t off = 0;
    while (off < s.size()) {
      long n;
      if (ssl_) {
        n = SSL_write(ssl_, s.data() + off, (int)(s.size() - off));
        if (n <= 0) {
          int e = SSL_get_error(ssl_, (int)n);
          if (e != SSL_ERROR_WANT_READ && e != SSL_ERROR_WANT_WRITE) return false;
          pollfd p{fd_, (short)(e == SSL_ERROR_WANT_READ ? POLLIN : POLLOUT), 0};
          if (poll(&p, 1, dl.left_ms()) <= 0) return false;
          continue;
        }
      } else {
        n = ::send(fd_, s.data() + off, s.size() - off, MSG_NOSIGNAL);
        if (n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
          pollfd p{fd_, POLLOUT, 0};
          if (poll(&p, 1, dl.left_ms()) <= 0) return false;
          continue;
        }
        if (n <= 0) return false;
      }
      off += (size_t)n;
    }
    return true;
  }

  // -1 error/EOF, 0 timeout, >0 bytes; timeout_ms -1 waits forever
  long read_some(char* buf, size_t n, int timeout_ms) {
    while (true) {
      if (!(ssl_ && SSL_pending(ssl_) > 0)) {
        pollfd p{fd_, POLLIN, 0};
        int r = poll(&p, 1, timeout_ms);
        if (r == 0) return 0;
        if (r < 0) return -1;
      }
      if (ssl_) {
        long k = SSL_read(ssl_, buf, (int)n);
        if (k > 0) return k;
        int e = SSL_get_error(ssl_, (int)k);
        if (e == SSL_ERROR_WANT_READ || e == SSL_ERROR_WANT_WRITE) continue;  // a TLS record was partial
        return -1;
      }
      long k = ::recv(fd_, buf, n, 0);
      if (k < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) continue;
      return k <= 0 ? -1 : k;
    }
  }

  // an idle pooled connection the server closed shows as readable (EOF) without any request in flight
  bool stale() {
    if (fd_ < 0) return true;
    if (ssl_ && SSL_pending(ssl_) > 0) return true;
    pollfd p{fd_, POLLIN, 0};
    return poll(&p, 1, 0) != 0;
  }

 private:
  ClusterConfig cfg_;
  int fd_ = -1;
  SSL_CTX* ctx_ = nullptr;
  SSL* ssl_ = nullptr;
};

// Buffered HTTP/1.1 response reader (Content-Length, chunked, or read-to-close bodies); every read is
// bounded by the request deadline.
class Reader {
 public:
  Reader(Conn& c, Deadline dl) : c_(c), dl_(dl) {}

  // returns -1 err, 0 timeout, 1 ok
  int fill(int timeout_ms) {
    char buf[16384];
    long n = c_.read_some(buf, sizeof buf, timeout_ms);
    if (n == 0) return 0;
    if (n < 0) return -1;
    got_any_ = true;
    buf_.append(buf, (size_t)n);
    return 1;
  }
  int fill() { return fill(dl_.left_ms()); }

  bool line(std::string& out) { return line(out, -2); }
  // timeout_ms -2: the request deadline
  bool line(std::string& out, int timeout_ms) {
    while (true) {
      size_t p = buf_.find("\r\n");
      if (p != std::string::npos) {
        out = buf_.substr(0, p);
        buf_.erase(0, p + 2);
        return true;
      }
      if (fill(timeout_ms == -2 ? dl_.left_ms() : timeout_ms) <= 0) return false;
    }
  }

  bool exact(size_t n, std::string& out) {
    while (buf_.size() < n)
      if (fill() <= 0) return false;
    out = buf_.substr(0, n);
    buf_.erase(0, n);
    return true;
  }

  std::string rest_until_close() {
    while (fill() > 0) {
    }
    std::string o;
    o.swap(buf_);
    return o;
  }

  std::string& buffer() { return buf_; }
  bool got_any() const { return got_any_; }
  bool expired() const { return dl_.left_ms() == 0; }

 private:
  Conn& c_;
  Deadline dl_;
  std::string buf_;
  bool got_any_ = false;
};

struct Head {
  int code = 0;
  bool chunked = false;
  bool close = false;
  long content_length = -1;
};

bool read_head(Reader& r, Head& h, std::string& err) {
  std::string l;
  if (!r.line(l)) {
    err = r.expired() ? "request timed out" : "connection closed before response";
    return false;
  }
  // HTTP/1.1 200 OK
  size_t sp = l.find(' ');
  h.code = sp == std::string::npos ? 0 : atoi(l.c_str() + sp + 1);
  if (l.rfind("HTTP/1.0", 0) == 0) h.close = true;
  while (r.line(l)) {
    if (l.empty()) return true;
    size_t c = l.find(':');
    if (c == std::string::npos) continue;
    std::string k = l.substr(0, c), v = l.substr(c + 1);
    while (!v.empty() && v[0] == ' ') v.erase(0, 1);
    for (auto& ch : k) ch = (char)tolower((unsigned char)ch);
    std::string lv = v;
    for (auto& ch : lv) ch = (char)tolower((unsigned char)ch);
    if (k == "transfer-encoding" && lv.find("chunked") != std::string::npos) h.chunked = true;
    if (k == "content-length") h.content_length = atol(v.c_str());
    if (k == "connection" && lv.find("close") != std::string::npos) h.close = true;
  }
  err = r.expired() ? "request timed out" : "truncated headers";
  return false;
}

std::string build_request(const ClusterConfig& cfg, const std::string& method, const std::string& path,
                          const std::string& body, const std::string& ctype, bool keep) {
  std::ostringstream o;
  o << method << " " << path << " HTTP/1.1\r\n";
  o << "Host: " << cfg.host << ":" << cfg.port << "\r\n";
  o << "User-Agent: " << cfg.user_agent << "\r\n";
  o << "Accept: application/json\r\n";
  if (!cfg.token.empty()) o << "Authorization: Bearer " << cfg.token << "\r\n";
  if (!body.empty() || method == "POST" || method == "PUT" || method == "PATCH") {
    o << "Content-Type: " << ctype << "\r\n";
    o << "Content-Length: " << body.size() << "\r\n";
  }
  o << "Connection: " << (keep ? "keep-alive" : "close") << "\r\n\r\n";
  o << body;
  return o.str();
}

class HttpWatch : public WatchStream {
 public:
  HttpWatch(std::unique_ptr<Conn> c, bool chunked, std::string prefix)
      : conn_(std::move(c)), rd_(*conn_, Deadline::in_ms(-1)), chunked_(chunked) {
    rd_.buffer() = std::move(prefix);  // body bytes already read together with the headers
  }
  bool next(Json& ev, int timeout_ms, std::string& err) override {
    ev = Json();
    while (true) {
      size_t p = lines_.find('\n');
      if (p != std::string::npos) {
        std::string l = lines_.substr(0, p);
        lines_.erase(0, p + 1);
        if (l.find_first_not_of(" \r\t") == std::string::npos) continue;
        try {
          ev = Json::parse(l);
        } catch (const std::exception& e) {
          err = e.what();
          return false;
        }
        return true;
      }
      if (!pull(timeout_ms, err)) return false;
      if (timed_out_) {
        timed_out_ = false;
        return true;
      }
    }
  }
  void close() override { conn_->close(); }

 private:
  // A chunk that started arriving must finish within this long, or the stream is considered dead.
  static constexpr int kChunkTimeoutMs = 60000;
  // move decoded body bytes into lines_; a timeout with nothing buffered sets timed_out_
  bool pull(int timeout_ms, std::string& err) {
    if (rd_.buffer().empty()) {
      const int r = rd_.fill(timeout_ms);
      if (r == 0) {
        timed_out_ = true;
        return true;
      }
      if (r < 0) {
        err = "watch stream closed";
        return false;
      }
    }
    if (!chunked_) {
      lines_ += rd_.buffer();
      rd_.buffer().clear();
      return true;
    }
    // chunked framing: data is arriving, wait (bounded) until the current piece is complete
    while (true) {
      std::string& b = rd_.buffer();
      if (chunk_left_ > 0) {
        if (b.empty() && rd_.fill(kChunkTimeoutMs) <= 0) {
          err = "watch stream closed";
          return false;
        }
        size_t n = std::min<size_t>(chunk_left_, rd_.buffer().size());
        lines_.append(rd_.buffer(), 0, n);
        rd_.buffer().erase(0, n);
        chunk_left_ -= n;
        if (chunk_left_ == 0) need_crlf_ = true;
        return true;
      }
      std::string l;
      if (need_crlf_) {
        if (!rd_.line(l, kChunkTimeoutMs)) {
          err = "watch stream closed";
          return false;
        }
        need_crlf_ = false;
        if (rd_.buffer().empty()) return true;  // next chunk not here yet: go back to the timed wait
      }
      if (!rd_.line(l, kChunkTimeoutMs)) {
        err = "watch stream closed";
        return false;
      }
      long n = strtol(l.c_str(), nullptr, 16);
      if (n == 0) {
        err = "watch stream ended";
        return false;
      }
      chunk_left_ = (size_t)n;
    }
  }

  std::unique_ptr<Conn> conn_;
  Reader rd_;
  bool chunked_;
  std::string lines_;
  size_t chunk_left_ = 0;
  bool need_crlf_ = false;
  bool timed_out_ = false;
};

// HTTP/1.1 client with keep-alive connection reuse (client-go's transport keeps idle connections too: one
// TLS handshake per connection instead of per request) and a deadline on every request.
class HttpKubeApi : public KubeApi {
 public:
  explicit HttpKubeApi(ClusterConfig cfg) : cfg_(std::move(cfg)) {}

  ApiResult request(const std::string& method, const std::string& path, const Json* body,
                    const std::string& ctype) override {
    ApiResult res = request_once(method, path, body, ctype, false);
    // 401 with a refreshable credential: refresh it once and replay (the server rejected the request, it did
    // not run it)
    if (res.code == 401 && (!cfg_.exec_config.empty() || !cfg_.token_file.empty()))
      res = request_once(method, path, body, ctype, true);
    return res;
  }

  // the bearer token to send: an exec-plugin token is re-fetched shortly before its expiry (or when forced by a
  // 401), a token file re-read every minute (client-go's cached token source does the same).
  // The plugin never runs under cred_mu_ (every request and the leader-election renew take that lock): one refresh
  // at a time runs on a background thread and swaps the new credentials in under the lock. A request waits for it
  // only when its token is unusable (expired, or rejected with a 401), and then at most `wait_ms` (the request's
  // own deadline); otherwise it goes out with the cached token. A failed refresh backs off (1 s doubling to 60 s)
  // and the cached token stays in use.
  std::string token(bool force, int wait_ms) {
    std::unique_lock<std::mutex> lk(cred_mu_);
    const long long now = (long long)time(nullptr);
    if (!cfg_.exec_config.empty()) {
      const bool near = cfg_.token_expiry > 0 && now >= cfg_.token_expiry - 60;
      const bool unusable = force || cfg_.token.empty() || (cfg_.token_expiry > 0 && now >= cfg_.token_expiry);
      if ((force || near) && !refreshing_ && (force || mono_ms() >= retry_after_ms_)) start_refresh();
      const int w = wait_ms < 0 ? cfg_.exec_timeout_ms + 1000 : wait_ms;  // -1: a request without a deadline
      if (unusable && refreshing_ && w > 0)
        refresh_cv_.wait_for(lk, std::chrono::milliseconds(w), [&] { return !refreshing_; });
    }
    if (!cfg_.token_file.empty() && (force || now - token_read_ >= 60)) {
      try {
        std::string t = read_file(cfg_.token_file);
        while (!t.empty() && isspace((unsigned char)t.back())) t.pop_back();
        if (!t.empty()) cfg_.token = t;
      } catch (...) {
      }
      token_read_ = now;
    }
    return cfg_.token;
  }

  ~HttpKubeApi() override {
    std::thread t;
    {
      std::lock_guard<std::mutex> g(cred_mu_);
      t.swap(refresher_);
    }
    if (t.joinable()) t.join();
  }

  ApiResult request_once(const std::string& method, const std::string& path, const Json* body,
                         const std::string& ctype, bool force_refresh) {
    const int ovr = RequestTimeout::current();
    const Deadline dl = Deadline::in_ms(ovr >= 0 ? ovr : cfg_.timeout_ms);
    const std::string b = body ? body->dump() : "";
    ClusterConfig rc = cfg_view();
    rc.token = token(force_refresh, (int)dl.left_ms());
    const std::string req = build_request(rc, method, path, b, ctype, true);
    ApiResult res;
    for (int attempt = 0; attempt < 2; ++attempt) {
      bool pooled = false;
      std::unique_ptr<Conn> c = take(pooled);
      if (!c) {
        c = std::make_unique<Conn>(cfg_view());
        if (!c->open(dl, res.error)) return res;
      }
      if (!c->write_all(req, dl)) {
        res.error = dl.left_ms() == 0 ? "request timed out" : "write failed";
        if (pooled && dl.left_ms() != 0) continue;  // a stale keep-alive connection: retry once on a fresh one
        return res;
      }
      Reader r(*c, dl);
      Head h;
      if (!read_head(r, h, res.error)) {
        // a pooled connection the server closed while idle: the request was written but no byte came back, so
        // the server may or may not have processed it. Replay only what is safe to run twice (Go's transport:
        // idempotent methods); a POST (create, event) is reported and retried by its caller's own logic, which
        // tolerates AlreadyExists.
        const bool replayable = method == "GET" || method == "HEAD" || method == "PUT" || method == "DELETE";
        if (pooled && replayable && !r.got_any() && !r.expired()) continue;
        return res;
      }
      std::string payload;
      bool complete = true;
      if (h.chunked) {
        std::string l, chunk;
        complete = false;
        while (r.line(l)) {
          long n = strtol(l.c_str(), nullptr, 16);
          if (n <= 0) {
            complete = r.line(l);  // trailing CRLF after the last chunk
            break;
          }
          if (!r.exact((size_t)n, chunk)) break;
          payload += chunk;
          if (!r.line(l)) break;
        }
      } else if (h.content_length >= 0) {
        complete = r.exact((size_t)h.content_length, payload);
      } else {
        payload = r.rest_until_close();
        h.close = true;
      }
      if (!complete) {
        res.error = r.expired() ? "request timed out" : "truncated response body";
        return res;
      }
      res.code = h.code;
      if (!payload.empty()) {
        try {
          res.body = Json::parse(payload);
        } catch (...) {
          res.body = Json(payload);
        }
      }
      if (!h.close && r.buffer().empty()) give(std::move(c));
      return res;
    }
    return res;
  }

  std::unique_ptr<WatchStream> watch(const std::string& path, std::string& err) override {
    const Deadline dl = Deadline::in_ms(cfg_.timeout_ms);
    auto c = std::make_unique<Conn>(cfg_view());
    if (!c->open(dl, err)) return nullptr;
    ClusterConfig wc = cfg_view();
    wc.token = token(false, (int)dl.left_ms());
    if (!c->write_all(build_request(wc, "GET", path, "", "", true), dl)) {
      err = "write failed";
      return nullptr;
    }
    Reader r(*c, dl);
    Head h;
    if (!read_head(r, h, err)) return nullptr;
    if (h.code != 200) {
      err = "watch HTTP " + std::to_string(h.code);
      return nullptr;
    }
    std::string leftover = r.buffer();
    return std::make_unique<HttpWatch>(std::move(c), h.chunked, std::move(leftover));
  }

 private:
  static constexpr size_t kMaxIdle = 16;

  std::unique_ptr<Conn> take(bool& pooled) {
    std::lock_guard<std::mutex> g(mu_);
    while (!idle_.empty()) {
      std::unique_ptr<Conn> c = std::move(idle_.back());
      idle_.pop_back();
      if (!c->stale()) {
        pooled = true;
        return c;
      }
    }
    return nullptr;
  }
  void give(std::unique_ptr<Conn> c) {
    std::lock_guard<std::mutex> g(mu_);
    if (idle_.size() < kMaxIdle) idle_.push_back(std::move(c));
  }

  ClusterConfig cfg_view() {
    std::lock_guard<std::mutex> g(cred_mu_);
    return cfg_;
  }

  static long long mono_ms() {
    return std::chrono::duration_cast<std::chrono::milliseconds>(
               std::chrono::steady_clock::now().time_since_epoch()).count();
  }

  // with cred_mu_ held and no refresh running: run the exec plugin on the (single) refresher thread
  void start_refresh() {
    if (refresher_.joinable()) refresher_.join();  // the previous refresher has already cleared refreshing_
    refreshing_ = true;
    ClusterConfig job;
    job.exec_config = cfg_.exec_config;
    job.exec_timeout_ms = cfg_.exec_timeout_ms;
    refresher_ = std::thread([this, job]() mutable {
      std::string err;
      try {
        job.token_expiry = 0;
        refresh_exec_credential(job);
      } catch (const std::exception& e) {
        err = e.what();
      }
      std::lock_guard<std::mutex> g(cred_mu_);
      if (err.empty()) {
        if (!job.token.empty()) cfg_.token = job.token;
        if (!job.cert_data.empty()) cfg_.cert_data = job.cert_data;
        if (!job.key_data.empty()) cfg_.key_data = job.key_data;
        cfg_.token_expiry = job.token_expiry;
        backoff_ms_ = 0;
        retry_after_ms_ = 0;
        log_info("exec credential refreshed (expires %lld)", cfg_.token_expiry);
      } else {
        backoff_ms_ = backoff_ms_ ? std::min<long long>(2 * backoff_ms_, 60000) : 1000;
        retry_after_ms_ = mono_ms() + backoff_ms_;
        log_error("exec credential refresh failed: %s (cached token kept; next try in %lld ms)", err.c_str(),
                  backoff_ms_);
      }
      refreshing_ = false;
      refresh_cv_.notify_all();
    });
  }

  ClusterConfig cfg_;
  std::mutex cred_mu_;        // cfg_'s credentials change on refresh
  std::condition_variable refresh_cv_;
  bool refreshing_ = false;   // an exec-plugin run is in flight on refresher_
  std::thread refresher_;
  long long backoff_ms_ = 0, retry_after_ms_ = 0;
  long long token_read_ = 0;  // last read of cfg_.token_file
  std::mutex mu_;
  std::vector<std::unique_ptr<Conn>> idle_;
};

}  // namespace

std::unique_ptr<KubeApi> make_http_api(const ClusterConfig& cfg) { return std::make_unique<HttpKubeApi>(cfg); }

}  // namespace tfop
