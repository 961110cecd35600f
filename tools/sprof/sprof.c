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
static uint64_t ras[CAP];  // the word at the stack top: a leaf function's return address (libc memchr & co.)
#define DEPTH 12
static uint64_t chain[CAP / 16][DEPTH];  // frame-pointer chain (code built with -fno-omit-frame-pointer)
static volatile uint64_t npc;

static void handler(int sig, siginfo_t* si, void* uc_) {
  (void)sig;
  (void)si;
  ucontext_t* uc = (ucontext_t*)uc_;
  uint64_t k = __atomic_fetch_add(&npc, 1, __ATOMIC_RELAXED);
  if (k < CAP) {
    pcs[k] = (uint64_t)uc->uc_mcontext.gregs[REG_RIP];
    ras[k] = *(const uint64_t*)uc->uc_mcontext.gregs[REG_RSP];
    if (k < CAP / 16) {
      const uint64_t* fp = (const uint64_t*)uc->uc_mcontext.gregs[REG_RBP];
      const uint64_t lo = (uint64_t)uc->uc_mcontext.gregs[REG_RSP];
      for (int d = 0; d < DEPTH; d++) {
        if ((uint64_t)fp < lo || (uint64_t)fp > lo + (1 << 22) || ((uint64_t)fp & 7)) {
          chain[k][d] = 0;
          break;
        }
        chain[k][d] = fp[1];
        fp = (const uint64_t*)fp[0];
      }
    }
  }
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
  for (uint64_t i = 0; i < n; i++) {
    fprintf(f, "%lx %lx", (unsigned long)pcs[i], (unsigned long)ras[i]);
    for (int d = 0; i < CAP / 16 && d < DEPTH && chain[i][d]; d++) fprintf(f, " %lx", (unsigned long)chain[i][d]);
    fprintf(f, "\n");
  }
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
