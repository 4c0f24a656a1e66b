#include "informer.h"

#include <random>

#include "log.h"

namespace tfop {

Informer::Informer(KubeApi& api, std::string collection_path, std::string label_selector, InformerOptions opts)
    : api_(api), path_(std::move(collection_path)), selector_(std::move(label_selector)), opts_(opts) {}

Informer::~Informer() { stop(); }

void Informer::start() {
  if (th_.joinable()) return;
  stop_ = false;
  th_ = std::thread([this] { run(); });
}

void Informer::stop() {
  stop_ = true;
  if (th_.joinable()) th_.join();
}

void Informer::touch() {
  last_ok_ns_ = std::chrono::duration_cast<std::chrono::nanoseconds>(
                    std::chrono::steady_clock::now().time_since_epoch()).count();
}

bool Informer::fresh() const {
  if (!synced_.load()) return false;
  if (watching_.load()) return true;
  const long long now = std::chrono::duration_cast<std::chrono::nanoseconds>(
                            std::chrono::steady_clock::now().time_since_epoch()).count();
  return now - last_ok_ns_.load() <= std::chrono::duration_cast<std::chrono::nanoseconds>(opts_.stale_after).count();
}

bool Informer::wait_synced(std::chrono::milliseconds timeout) {
  std::unique_lock<std::mutex> lk(sync_mu_);
  // system_clock deadline: see JobWorker::run (ThreadSanitizer and pthread_cond_clockwait)
  return sync_cv_.wait_until(lk, std::chrono::system_clock::now() + timeout, [&] { return synced_.load(); });
}

static std::string obj_ns(const Json& obj) {
  const Json* m = obj.find("metadata");
  return m ? get_str(*m, "namespace") : "";
}

static std::string obj_key(const Json& obj) {
  const Json* m = obj.find("metadata");
  if (!m) return "";
  return get_str(*m, "namespace") + "/" + get_str(*m, "name");
}

std::string Informer::index_key(const std::string& ns, const Json& obj) {
  const Json* m = obj.find("metadata");
  const Json* l = m ? m->find("labels") : nullptr;
  if (!l || !l->is_object()) return "";
  const Json* n = l->find("tf_job_name");
  if (!n || !n->is_string()) return "";
  return ns + "/" + n->as_string();
}

bool Informer::get(const std::string& ns, const std::string& name, Json& out) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = objs_.find(ns + "/" + name);
  if (it == objs_.end()) return false;
  out = it->second;
  return true;
}

Json Informer::list(const std::string& ns, const Labels& sel) const {
  Json items = Json::array();
  std::lock_guard<std::mutex> g(mu_);
  auto match = [&](const Json& o) {
    const Json* m = o.find("metadata");
    if (!m || get_str(*m, "namespace") != ns) return false;
    const Json* l = m->find("labels");
    return labels_match(sel, l ? *l : Json::object());
  };
  auto jn = sel.find("tf_job_name");
  if (jn != sel.end()) {
    auto it = idx_.find(ns + "/" + jn->second);
    if (it == idx_.end()) return items;
    for (auto& k : it->second) {
      auto o = objs_.find(k);
      if (o != objs_.end() && match(o->second)) items.push_back(o->second);
    }
    return items;
  }
  for (auto& kv : objs_)
    if (match(kv.second)) items.push_back(kv.second);
  return items;
}

size_t Informer::size() const {
  std::lock_guard<std::mutex> g(mu_);
  return objs_.size();
}

void Informer::apply(const std::string& type, const Json& obj) {
  const std::string key = obj_key(obj);
  if (key.empty()) return;
  const std::string ns = obj_ns(obj);
  {
    std::lock_guard<std::mutex> g(mu_);
    auto old = objs_.find(key);
    if (old != objs_.end()) {  // the index entry of the previous version (labels may have changed)
      const std::string ik = index_key(ns, old->second);
      if (!ik.empty()) {
        auto s = idx_.find(ik);
        if (s != idx_.end()) {
          s->second.erase(key);
          if (s->second.empty()) idx_.erase(s);
        }
      }
    }
    if (type == "DELETED") {
      objs_.erase(key);
    } else {
      objs_[key] = obj;
      const std::string ik = index_key(ns, obj);
      if (!ik.empty()) idx_[ik].insert(key);
    }
  }
  ++events_;
  if (on_change_) on_change_(type, obj);  // outside the lock: the callback takes the controller's locks
}

bool Informer::relist(std::string& rv) {
  ++lists_;
  const std::string q = selector_.empty() ? "" : "?labelSelector=" + url_escape(selector_);
  ApiResult r = api_.get(path_ + q);
  if (!r.ok()) {
    log_warn("informer %s: list failed: HTTP %d %s", path_.c_str(), r.code, r.message().c_str());
    return false;
  }
  std::map<std::string, Json> fresh;
  if (const Json* items = r.body.find("items"); items && items->is_array())
    for (auto& it : items->as_array()) {
      const std::string k = obj_key(it);
      if (!k.empty()) fresh[k] = it;
    }
  std::vector<Json> gone;
  {
    std::lock_guard<std::mutex> g(mu_);
    for (auto& kv : objs_)
      if (!fresh.count(kv.first)) gone.push_back(kv.second);
  }
  for (auto& o : gone) apply("DELETED", o);
  for (auto& kv : fresh) {
    Json cur;
    bool had;
    {
      std::lock_guard<std::mutex> g(mu_);
      auto it = objs_.find(kv.first);
      had = it != objs_.end();
      if (had) cur = it->second;
    }
    const Json* m1 = had ? cur.find("metadata") : nullptr;
    const Json* m2 = kv.second.find("metadata");
    if (had && m1 && m2 && get_str(*m1, "resourceVersion") == get_str(*m2, "resourceVersion")) continue;
    apply(had ? "MODIFIED" : "ADDED", kv.second);
  }
  if (const Json* m = r.body.find("metadata")) rv = get_str(*m, "resourceVersion");
  touch();
  if (!synced_.exchange(true)) {
    std::lock_guard<std::mutex> g(sync_mu_);
    sync_cv_.notify_all();
  }
  return true;
}

void Informer::run() {
  std::mt19937 rng(std::random_device{}());
  using clock = std::chrono::steady_clock;
  std::string rv;
  bool need_list = true;
  int watch_failures = 0;
  clock::time_point listed_at = clock::now();
  auto pause = [&] {
    for (long i = 0; i < opts_.retry.count() / 50 && !stop_; ++i)
      std::this_thread::sleep_for(std::chrono::milliseconds(50));
  };
  auto resync_due = [&] {
    return opts_.resync_period.count() > 0 && clock::now() - listed_at >= opts_.resync_period;
  };
  while (!stop_) {
    if (need_list || resync_due()) {
      if (!relist(rv)) {
        pause();
        continue;
      }
      need_list = false;
      watch_failures = 0;
      listed_at = clock::now();
    }
    const long tmin = std::max<long>(1, (long)(opts_.watch_timeout.count() / 1000));
    long timeout_s = std::uniform_int_distribution<long>(tmin, std::max(tmin, 2 * tmin - 1))(rng);
    if (opts_.resync_period.count() > 0) {  // end the watch by the next resync
      const long left = (long)std::chrono::duration_cast<std::chrono::seconds>(
                            opts_.resync_period - (clock::now() - listed_at)).count();
      timeout_s = std::max<long>(1, std::min(timeout_s, left));
    }
    std::string q = "?watch=true&resourceVersion=" + rv + "&timeoutSeconds=" + std::to_string(timeout_s);
    if (!selector_.empty()) q += "&labelSelector=" + url_escape(selector_);
    std::string err;
    ++watches_;
    auto w = api_.watch(path_ + q, err);
    if (!w) {
      ++watch_failures;
      // the rv may be gone (410) or the watch forbidden (403): re-watching from it would fail forever, leaving the
      // cache frozen at its last list. Relist at once on those, and after a run of any other failures.
      const bool gone = err.find("HTTP 410") != std::string::npos || err.find("HTTP 403") != std::string::npos;
      if (gone || watch_failures >= opts_.relist_after_watch_failures) need_list = true;
      log_warn("informer %s: watch failed (%d in a row): %s%s", path_.c_str(), watch_failures, err.c_str(),
               need_list ? ": relisting" : "");
      pause();
      continue;
    }
    watch_failures = 0;
    watching_ = true;
    touch();
    const auto dead_after = clock::now() + std::chrono::seconds(timeout_s) + opts_.watch_idle_grace;
    while (!stop_) {
      if (clock::now() > dead_after) {
        log_warn("informer %s: watch past its timeoutSeconds: re-watching from rv=%s", path_.c_str(), rv.c_str());
        break;
      }
      if (resync_due()) break;
      Json ev;
      if (!w->next(ev, 500, err)) break;  // stream ended: re-watch from rv
      if (ev.is_null()) continue;
      const std::string type = get_str(ev, "type");
      const Json* obj = ev.find("object");
      if (!obj) continue;
      if (type == "ERROR") {
        const int code = obj->find("code") ? (int)obj->at("code").as_int() : 0;
        if (code == 410) log_v(1, "informer %s: 410 Gone at rv=%s: relisting", path_.c_str(), rv.c_str());
        else log_warn("informer %s: watch ERROR %s", path_.c_str(), obj->dump().c_str());
        need_list = true;
        break;
      }
      touch();
      if (const Json* m = obj->find("metadata")) rv = get_str(*m, "resourceVersion");
      if (type == "ADDED" || type == "MODIFIED" || type == "DELETED") apply(type, *obj);
    }
    watching_ = false;
    w->close();
  }
  watching_ = false;
}

}  // namespace tfop
