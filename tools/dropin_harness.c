/* Drop-in cycle latency at the C ABI (no Python): what the cgo plugin of
 * INTEGRATION.md §3 calls per pod — ksg_cycle (commit = 0), ksg_cycle_view_acquire,
 * ksg_reserve on the engine's choice, ksg_cycle_view_release — timed per call with
 * a monotonic clock, averaged over the timed pods; with the library's own split
 * of ksg_cycle's host phases (ksg_debug_cycle_times, looked up with dlsym).
 *
 * usage: dropin_harness PROFILE.json CLUSTER.json PODS.jsonl WARMUP COUNT
 *   PODS.jsonl: one v1.Pod JSON per line (names unique); the first WARMUP are
 *   untimed.  Prints one JSON object.
 * build: gcc -O2 -o dropin_harness tools/dropin_harness.c -Iinclude -Lkube-scheduler-simulator-p9_amd -lksg -ldl
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "ksg.h"

static char* slurp(const char* path, size_t* len) {
  FILE* f = fopen(path, "rb");
  if (!f) return NULL;
  fseek(f, 0, SEEK_END);
  long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  char* b = (char*)malloc((size_t)n + 1);
  if (b && fread(b, 1, (size_t)n, f) != (size_t)n) {
    free(b);
    b = NULL;
  }
  fclose(f);
  if (b) b[n] = 0;
  *len = (size_t)n;
  return b;
}

static double now_us(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec * 1e6 + (double)t.tv_nsec * 1e-3;
}

static int fail(ksg_ctx* c, const char* what, int rc) {
  fprintf(stderr, "%s: %d %s\n", what, rc, c ? ksg_last_error(c) : "");
  return 1;
}

int main(int argc, char** argv) {
  if (argc < 6) {
    fprintf(stderr, "usage: %s PROFILE.json CLUSTER.json PODS.jsonl WARMUP COUNT\n", argv[0]);
    return 2;
  }
  size_t plen = 0, clen = 0, qlen = 0;
  char* prof = slurp(argv[1], &plen);
  char* clus = slurp(argv[2], &clen);
  char* pods = slurp(argv[3], &qlen);
  const int warm = atoi(argv[4]), count = atoi(argv[5]);
  if (!prof || !clus || !pods) return fail(NULL, "read inputs", -1);
  ksg_ctx* c = NULL;
  int rc = ksg_create(prof, plen, NULL, &c);
  if (rc) return fail(c, "ksg_create", rc);
  if ((rc = ksg_load_cluster(c, clus, clen))) return fail(c, "ksg_load_cluster", rc);
  int (*cycle_times)(ksg_ctx*, double*, int) = (int (*)(ksg_ctx*, double*, int))dlsym(RTLD_DEFAULT, "ksg_debug_cycle_times");
  double t_cycle = 0, t_view = 0, t_res = 0, t_rel = 0;
  int done = 0, placed = 0;
  char* line = pods;
  for (int i = 0; i < warm + count && line && *line; ++i) {
    char* nl = strchr(line, '\n');
    const size_t len = nl ? (size_t)(nl - line) : strlen(line);
    if (i == warm && cycle_times) cycle_times(c, NULL, 1);
    ksg_pod_result r;
    const double t0 = now_us();
    if ((rc = ksg_cycle(c, line, len, 0, &r))) return fail(c, "ksg_cycle", rc);
    const double t1 = now_us();
    const uint32_t q = (uint32_t)ksg_queue_len(c) - 1;
    const ksg_cycle_view* v = NULL;
    if ((rc = ksg_cycle_view_acquire(c, q, &v))) return fail(c, "ksg_cycle_view_acquire", rc);
    const double t2 = now_us();
    if (r.selected >= 0) {
      if ((rc = ksg_reserve(c, q, r.selected))) return fail(c, "ksg_reserve", rc);
    }
    const double t3 = now_us();
    ksg_cycle_view_release(v);
    const double t4 = now_us();
    if (i >= warm) {
      t_cycle += t1 - t0;
      t_view += t2 - t1;
      t_res += t3 - t2;
      t_rel += t4 - t3;
      done++;
      placed += r.selected >= 0;
    }
    line = nl ? nl + 1 : NULL;
  }
  double ph[8] = {0};
  if (cycle_times) cycle_times(c, ph, 0);
  const double k = done ? 1.0 / done : 0;
  printf("{\"pods\": %d, \"placed\": %d, \"cycle_us\": %.2f, \"view_us\": %.2f, \"reserve_us\": %.2f, "
         "\"release_us\": %.2f, \"total_us\": %.2f",
         done, placed, t_cycle * k, t_view * k, t_res * k, t_rel * k, (t_cycle + t_view + t_res + t_rel) * k);
  if (cycle_times && ph[7] > 0) {
    const double m = 1.0 / ph[7];
    printf(", \"cycle_split_us\": {\"parse\": %.2f, \"checks_vocab\": %.2f, \"compile\": %.2f, \"append\": %.2f, "
           "\"launch\": %.2f, \"wait\": %.2f, \"postfilter\": %.2f}",
           ph[0] * m, ph[1] * m, ph[2] * m, ph[3] * m, ph[4] * m, ph[5] * m, ph[6] * m);
  }
  printf("}\n");
  ksg_destroy(c);
  free(prof);
  free(clus);
  free(pods);
  return 0;
}
