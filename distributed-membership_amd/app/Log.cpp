// Log.cpp -- see Log.h.
#include "Log.h"

#include <cstring>

Log::Log(const char *path, const char *stats_path) {
  fp_ = fopen(path, "w");
  FILE *s = fopen(stats_path, "w");  // stats.log is created and stays empty (Log.cpp:66-67,90-95)
  if (s) fclose(s);
}

Log::~Log() {
  if (fp_) fclose(fp_);
}

std::string Log::addr(int32_t id, int16_t port) {
  unsigned char b[4];
  memcpy(b, &id, 4);
  char tmp[64];
  snprintf(tmp, sizeof tmp, "%d.%d.%d.%d:%d", (signed char)b[0], (signed char)b[1], (signed char)b[2],
           (signed char)b[3], (int)port);
  return tmp;
}

void Log::LOG(int32_t id, int t, const char *text) {
  if (!fp_) return;
  std::string prefix;
  if (!opened_) opened_ = true;  // first call: the address sprintf is skipped
  else prefix = addr(id) + " ";
  if (!first_) {
    int magic = 0;
    for (const char *m = "CS425"; *m; m++) magic += *m;
    fprintf(fp_, "%x\n", magic);
    first_ = true;
  }
  fprintf(fp_, "\n %s", prefix.c_str());
  fprintf(fp_, "[%d] ", t);
  fputs(text, fp_);
  fflush(fp_);  // MAXWRITES 1 (Log.h:18)
}

void Log::logNodeAdd(int32_t logger_id, int32_t added_id, int t) {
  std::string s = "Node " + addr(added_id) + " joined at time " + std::to_string(t);
  LOG(logger_id, t, s.c_str());
}

void Log::logNodeRemove(int32_t logger_id, int32_t removed_id, int t) {
  std::string s = "Node " + addr(removed_id) + " removed at time " + std::to_string(t);
  LOG(logger_id, t, s.c_str());
}
