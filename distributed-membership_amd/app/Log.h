// Log.h -- dbg.log writer with the reference's byte contract (Log.cpp:44-131).
#pragma once
#include <cstdint>
#include <cstdio>
#include <string>

class Log {
 public:
  explicit Log(const char *path = "dbg.log", const char *stats_path = "stats.log");
  ~Log();
  // Log::LOG: "\n <a.b.c.d:p >[t] text"; the very first record has no address
  // prefix and the file starts with the magic line "131\n" (Log.cpp:56-88).
  void LOG(int32_t id, int t, const char *text);
  void logNodeAdd(int32_t logger_id, int32_t added_id, int t);      // Log.cpp:116-120
  void logNodeRemove(int32_t logger_id, int32_t removed_id, int t); // Log.cpp:127-131
  static std::string addr(int32_t id, int16_t port = 0);            // signed-char bytes (Log.cpp:73)

 private:
  FILE *fp_ = nullptr;
  bool opened_ = false, first_ = false;
};
