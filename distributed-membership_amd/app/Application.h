// Application.h -- the reference's driver surface (Application.h:1-52) on top of
// libgm: construct from a testcase .conf, run TOTAL_RUNNING_TIME ticks of
// mp1Run() + fail(), then write msgcount.log.
#pragma once
#include <memory>
#include <vector>

#include "Log.h"
#include "gm_abi.h"

#define TOTAL_RUNNING_TIME 700  // Application.h:27

class Application {
 public:
  explicit Application(const char *conf);
  ~Application();
  int run();     // Application.cpp:90-114
  void mp1Run(); // Application.cpp:121-164 -> one gm_tick
  void fail();   // Application.cpp:173-202 (host fault injection, same S1 stream)
  bool ok() const { return rc_ == GM_OK; }
  int rc() const { return rc_; }

 private:
  void drain();
  void check(int rc);
  gm_config cfg_{};
  gm_ctx *ctx_ = nullptr;
  std::unique_ptr<Log> log_;
  int t_ = 0, rc_ = GM_OK;
  std::vector<gm_event> ev_;
};
