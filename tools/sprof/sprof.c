// Minimal sampling profiler (tuning aid): SIGPROF every 1/hz s of process CPU
// time records the interrupted PC; sprof_stop writes "pc" lines and a copy of
// /proc/self/maps for symbolisation (tools/sprof/report.py).
#define _GNU_SOURCE
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <sys/time.h>
#include <ucontext.h>

#define CAP (1 << 22)
static uint64_t pcs[CAP];
static volatile uint64_t npc;

static void handler(int sig, siginfo_t* si, void* uc_) {
  (void)sig;
  (void)si;
  ucontext_t* uc = (ucontext_t*)uc_;
  uint64_t k = __atomic_fetch_add(&npc, 1, __ATOMIC_RELAXED);
  if (k < CAP) pcs[k] = (uint64_t)uc->uc_mcontext.gregs[REG_RIP];
}

int sprof_start(int hz) {
  struct sigaction sa;
  memset(&sa, 0, sizeof sa);
  sa.sa_sigaction = handler;
  sa.sa_flags = SA_SIGINFO | SA_RESTART;
  sigaction(SIGPROF, &sa, 0);
  struct itimerval it = {{0, 1000000 / hz}, {0, 1000000 / hz}};
  npc = 0;
  return setitimer(ITIMER_PROF, &it, 0);
}

int sprof_stop(const char* path) {
  struct itimerval it = {{0, 0}, {0, 0}};
  setitimer(ITIMER_PROF, &it, 0);
  FILE* f = fopen(path, "w");
  if (!f) return -1;
  uint64_t n = npc < CAP ? npc : CAP;
  for (uint64_t i = 0; i < n; i++) fprintf(f, "%lx\n", (unsigned long)pcs[i]);
  fclose(f);
  char mp[4096];
  snprintf(mp, sizeof mp, "%s.maps", path);
  FILE* in = fopen("/proc/self/maps", "r");
  FILE* out = fopen(mp, "w");
  char buf[4096];
  size_t r;
  while (in && out && (r = fread(buf, 1, sizeof buf, in)) > 0) fwrite(buf, 1, r, out);
  if (in) fclose(in);
  if (out) fclose(out);
  return (int)n;
}
