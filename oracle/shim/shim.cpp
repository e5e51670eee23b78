/* shim.cpp -- TEST INFRASTRUCTURE ONLY: the time() wrap of the seed contract
 * (linked with -Wl,--wrap=time into oracle/_ref binaries). */
#include <ctime>
#include "seedshim.h"
long SeededRDCtx::tick = 0;
int SeededRDCtx::id = 0;
extern "C" time_t __wrap_time(time_t *t) {
  const char *s = getenv("TIME_SEED");
  time_t v = s ? (time_t)strtoll(s, 0, 10) : 0;
  if (t) *t = v;
  return v;
}
