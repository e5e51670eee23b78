// Application.cpp -- reference-shaped driver of the MI355X simulator.
//
// `./Application testcases/X.conf` writes dbg.log, stats.log, msgcount.log and
// the "i-th introduced node" stdout lines exactly as the reference does
// (Application.cpp:27-202, Log.cpp, EmulNet.cpp:184-220), with every tick of
// the membership protocol executed by libgm's HIP kernels.
// Seeds (the seed contract of the parity tests): $TIME_SEED feeds srand()
// (the reference's srand(time(NULL))), $RD_SEED the per-(tick, node) mt19937
// seeds (the reference's random_device). Unset: time(NULL) / a random seed, as
// nondeterministic as the reference.
#include "Application.h"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <ctime>
#include <random>
#include <string>

static uint64_t env_u64(const char *name, uint64_t dflt) {
  const char *s = getenv(name);
  return s ? strtoull(s, nullptr, 10) : dflt;
}

Application::Application(const char *conf) {
  cfg_.abi_version = GM_ABI_VERSION;
  cfg_.mode = GM_MODE_FAITHFUL;
  rc_ = gm_parse_conf(conf, &cfg_);  // Params::setparams (Params.cpp:19-40)
  if (rc_ != GM_OK) return;
  cfg_.time_seed = (uint32_t)env_u64("TIME_SEED", (uint64_t)time(nullptr));
  cfg_.rd_seed = env_u64("RD_SEED", std::random_device{}());
  cfg_.device = (int)env_u64("GM_DEVICE", 0);
  cfg_.shard_count = 1;
  log_.reset(new Log());
  for (int i = 0; i < cfg_.n; i++) log_->LOG(i + 1, 0, "APP");  // Application.cpp:66
  const auto t0 = std::chrono::steady_clock::now();
  rc_ = gm_create(&cfg_, &ctx_);
  if (getenv("GM_APP_TIMING"))
    fprintf(stderr, "gm_create %.1f ms\n",
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
}

Application::~Application() {
  if (ctx_) gm_destroy(ctx_);
}

void Application::check(int rc) {
  if (rc != GM_OK && rc_ == GM_OK) {
    rc_ = rc;
    fprintf(stderr, "libgm: %s\n", gm_strerror(rc));
  }
}

void Application::drain() {
  size_t n = 0;
  int rc = gm_drain_events(ctx_, nullptr, 0, &n);
  if (rc == GM_ERANGE) {
    ev_.resize(n);
    rc = gm_drain_events(ctx_, ev_.data(), ev_.size(), &n);
  }
  check(rc);
  for (size_t k = 0; k < n && rc == GM_OK; k++) {
    const gm_event &e = ev_[k];
    const int32_t id = e.logger + 1;
    switch (e.kind) {
      case GM_EV_JOINED: log_->logNodeAdd(id, e.subject, e.t); break;
      case GM_EV_REMOVED: log_->logNodeRemove(id, e.subject, e.t); break;
      case GM_EV_START_GROUP: log_->LOG(id, e.t, "Starting up group..."); break;
      case GM_EV_TRY_JOIN: log_->LOG(id, e.t, "Trying to join..."); break;
      case GM_EV_TIME_MARK: log_->LOG(id, e.t, ("@@time=" + std::to_string(e.t)).c_str()); break;
      default: break;
    }
  }
}

// Ticks are enqueued without a host wait; the log is written from drained records
// before every line the host itself logs (fail) and at the end, so dbg.log keeps the
// reference's order (Application.cpp:121-164 logs inside the tick).
void Application::mp1Run() {
  check(gm_tick(ctx_));
  // "i-th introduced node" lines, in node-phase order (Application.cpp:143-147)
  for (int i = cfg_.n - 1; i >= 0; i--)
    if (t_ == (int)(0.25 * i)) printf("%d-th introduced node is assigned with the address: %d:0\n", i, i + 1);
}

void Application::fail() {
  char s[64];
  if (cfg_.drop_msg && t_ == 50) check(gm_set_dropmsg(ctx_, 1));
  if (t_ == 100) drain();  // this tick's records precede the failure lines
  if (cfg_.single_failure && t_ == 100) {
    int32_t r = 0;
    check(gm_rand(ctx_, &r));
    int32_t removed = r % cfg_.n;
    snprintf(s, sizeof s, "Node failed at time=%d", t_);
    log_->LOG(removed + 1, t_, s);
    check(gm_set_failed(ctx_, &removed, 1));
  } else if (t_ == 100) {
    int32_t r = 0;
    check(gm_rand(ctx_, &r));
    int removed = r % cfg_.n / 2;
    std::vector<int32_t> idx;
    for (int i = removed; i < removed + cfg_.n / 2; i++) {
      snprintf(s, sizeof s, "Node failed at time = %d", t_);
      log_->LOG(i + 1, t_, s);
      idx.push_back(i);
    }
    check(gm_set_failed(ctx_, idx.data(), (int32_t)idx.size()));
  }
  if (cfg_.drop_msg && t_ == 300) check(gm_set_dropmsg(ctx_, 0));
}

int Application::run() {
  if (rc_ != GM_OK) return rc_;
  const auto t0 = std::chrono::steady_clock::now();
  for (t_ = 0; t_ < TOTAL_RUNNING_TIME && rc_ == GM_OK; ++t_) {
    mp1Run();
    fail();
  }
  drain();
  if (getenv("GM_APP_TIMING"))
    fprintf(stderr, "%d ticks %.1f ms\n", t_,
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
  // ENcleanup: msgcount.log (EmulNet.cpp:184-220), node 67 special-cased
  const int n = cfg_.n, T = t_;
  std::vector<int32_t> sent((size_t)n * T), recv((size_t)n * T);
  check(gm_msgcount(ctx_, T, sent.data(), recv.data()));
  FILE *f = fopen("msgcount.log", "w+");
  for (int i = 1; i <= n && f; i++) {
    fprintf(f, "node %3d ", i);
    unsigned st = 0, rt = 0;
    for (int j = 0; j < T; j++) {
      int sv = sent[(size_t)(i - 1) * T + j], rv = recv[(size_t)(i - 1) * T + j];
      st += (unsigned)sv;
      rt += (unsigned)rv;
      if (i != 67) {
        fprintf(f, " (%4d, %4d)", sv, rv);
        if (j % 10 == 9) fprintf(f, "\n         ");
      } else {
        fprintf(f, "special %4d %4d %4d\n", j, sv, rv);
      }
    }
    fprintf(f, "\n");
    fprintf(f, "node %3d sent_total %6u  recv_total %6u\n\n", i, st, rt);
  }
  if (f) fclose(f);
  return rc_;
}

int main(int argc, char *argv[]) {
  if (argc != 2) {  // ARGS_COUNT (Application.h:26)
    printf("Configuration (i.e., *.conf) file File Required\n");
    return -1;
  }
  Application app(argv[1]);
  int rc = app.run();
  if (rc != GM_OK) fprintf(stderr, "libgm: %s\n", gm_strerror(rc));
  return rc == GM_OK ? 0 : 1;
}
