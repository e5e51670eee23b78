/* ref_cpu_main.c -- TEST INFRASTRUCTURE: command-line driver of the oracle,
 * shaped like the reference's `./Application <conf>` (Application.cpp:27-42).
 * Writes dbg.log, stats.log (empty), msgcount.log and stdout exactly as the
 * seeded reference does. Seeds: $TIME_SEED, $RD_SEED.
 * Optional: $DUMP_FILE receives the per-tick table dump; $TICKS overrides 700. */
#include <stdio.h>
#include <stdlib.h>
#include "ref_cpu.h"

int main(int argc, char **argv) {
  if (argc != 2) {
    printf("Configuration (i.e., *.conf) file File Required\n");
    return -1;
  }
  oc_config cfg = {0};
  FILE *fp = fopen(argv[1], "r");
  if (!fp) return -1;
  /* Params::setparams, Params.cpp:22-25 */
  if (fscanf(fp, "MAX_NNB: %d", &cfg.n) != 1) cfg.n = 0;
  if (fscanf(fp, "\nSINGLE_FAILURE: %d", &cfg.single_failure) != 1) cfg.single_failure = 0;
  if (fscanf(fp, "\nDROP_MSG: %d", &cfg.drop_msg) != 1) cfg.drop_msg = 0;
  if (fscanf(fp, "\nMSG_DROP_PROB: %lf", &cfg.drop_prob) != 1) cfg.drop_prob = 0;
  fclose(fp);
  const char *s;
  cfg.mode = OC_FAITHFUL;
  cfg.time_seed = (s = getenv("TIME_SEED")) ? (uint32_t)strtoll(s, 0, 10) : 0;
  cfg.rd_seed = (s = getenv("RD_SEED")) ? strtoull(s, 0, 10) : 0;
  int ticks = (s = getenv("TICKS")) ? atoi(s) : 700; /* TOTAL_RUNNING_TIME, Application.h:27 */
  oc_ctx *c = oc_create(&cfg);
  if (!c) return 1;
  FILE *dump = (s = getenv("DUMP_FILE")) ? fopen(s, "w") : NULL;
  for (int t = 0; t < ticks; t++) {
    if (oc_tick(c)) return 2;
    if (dump) {
      size_t n;
      const char *d = oc_dump(c, &n);
      fwrite(d, 1, n, dump);
    }
  }
  if (dump) fclose(dump);
  size_t n;
  const char *p = oc_dbg_log(c, &n);
  FILE *f = fopen("dbg.log", "w");
  fwrite(p, 1, n, f);
  fclose(f);
  f = fopen("stats.log", "w");
  fclose(f);
  p = oc_msgcount(c, &n);
  f = fopen("msgcount.log", "w");
  fwrite(p, 1, n, f);
  fclose(f);
  p = oc_stdout(c, &n);
  fwrite(p, 1, n, stdout);
  oc_destroy(c);
  return 0;
}
