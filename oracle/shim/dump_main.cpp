/* dump_main.cpp -- TEST INFRASTRUCTURE ONLY.
 * Drives the unmodified reference Application (compiled with -Dmain=ref_main)
 * tick by tick exactly as Application::run does (Application.cpp:90-114) and,
 * after every `mp1Run(); fail();`, prints every node's membership list and
 * protocol state so the golden fixtures can pin per-tick table parity.
 * Output (stderr-free, to $DUMP_FILE): one line per (tick, node):
 *   t i started inGroup bFailed heartbeat n id:hb:ts id:hb:ts ...
 */
#define private public
#define nodeCount dump_nodeCount_unused
#include "Application.h"
#undef nodeCount
#include <cstdio>

int main(int argc, char **argv) {
  if (argc != 2) { fprintf(stderr, "usage: dump conf\n"); return 1; }
  const char *df = getenv("DUMP_FILE");
  FILE *out = fopen(df ? df : "tables.txt", "w");
  Application *app = new Application(argv[1]);
  srand(time(NULL)); /* Application.cpp:96 */
  for (app->par->globaltime = 0; app->par->globaltime < TOTAL_RUNNING_TIME; ++app->par->globaltime) {
    app->mp1Run();
    app->fail();
    int t = app->par->globaltime;
    for (int i = 0; i < app->par->EN_GPSZ; i++) {
      Member *m = app->mp1[i]->getMemberNode();
      fprintf(out, "%d %d %d %d %d %ld %zu", t, i, (int)m->inited, (int)m->inGroup, (int)m->bFailed,
              m->heartbeat, m->memberList.size());
      for (size_t k = 0; k < m->memberList.size(); k++) {
        MemberListEntry &e = m->memberList[k];
        fprintf(out, " %d:%ld:%ld", e.id, e.heartbeat, e.timestamp);
      }
      fprintf(out, "\n");
    }
  }
  app->en->ENcleanup();
  fclose(out);
  return 0;
}
