/* Diagnostic SIGSEGV / SIGBUS reporter: loaded with ctypes by bench.py when
 * DMY_SEGV_REPORT=1.  On a fault it prints the faulting PC and data address, dladdr() of the PC (which shared object,
 * nearest symbol), the /proc/self/maps lines that contain the PC and the fault address (plus the mappings on either
 * side of the address), and a backtrace of the faulting thread, then re-raises with the default action. */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <execinfo.h>
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <ucontext.h>
#include <unistd.h>

static void report_maps(uintptr_t pc, uintptr_t addr) {
  FILE* f = fopen("/proc/self/maps", "r");
  if (!f) return;
  char line[512], prev[512] = "";
  int after = 0;
  while (fgets(line, sizeof line, f)) {
    unsigned long lo = 0, hi = 0;
    if (sscanf(line, "%lx-%lx", &lo, &hi) != 2) continue;
    if (after) { fprintf(stderr, "[segv]   next mapping:  %s", line); after = 0; }
    if (pc >= lo && pc < hi) fprintf(stderr, "[segv]   PC in:         %s", line);
    if (addr >= lo && addr < hi) fprintf(stderr, "[segv]   address in:    %s", line);
    if (prev[0]) {
      unsigned long plo = 0, phi = 0;
      sscanf(prev, "%lx-%lx", &plo, &phi);
      if (addr >= phi && addr < lo) {
        fprintf(stderr, "[segv]   address in the gap after: %s", prev);
        fprintf(stderr, "[segv]                       before: %s", line);
      }
    }
    if (addr >= lo && addr < hi) after = 1;
    strncpy(prev, line, sizeof prev - 1);
  }
  fclose(f);
}

static void handler(int sig, siginfo_t* si, void* uc_) {
  ucontext_t* uc = (ucontext_t*)uc_;
  uintptr_t pc = (uintptr_t)uc->uc_mcontext.gregs[REG_RIP];
  uintptr_t addr = (uintptr_t)si->si_addr;
  fprintf(stderr, "\n[segv] signal %d code %d tid %ld: PC 0x%lx, fault address 0x%lx\n", sig, si->si_code,
          (long)gettid(), (unsigned long)pc, (unsigned long)addr);
  Dl_info di;
  if (dladdr((void*)pc, &di) && di.dli_fname)
    fprintf(stderr, "[segv]   PC object %s (base %p) +0x%lx, symbol %s +0x%lx\n", di.dli_fname, di.dli_fbase,
            (unsigned long)(pc - (uintptr_t)di.dli_fbase), di.dli_sname ? di.dli_sname : "?",
            di.dli_saddr ? (unsigned long)(pc - (uintptr_t)di.dli_saddr) : 0ul);
  fprintf(stderr, "[segv]   registers: rdi 0x%llx rsi 0x%llx rdx 0x%llx rcx 0x%llx rax 0x%llx rsp 0x%llx\n",
          (unsigned long long)uc->uc_mcontext.gregs[REG_RDI], (unsigned long long)uc->uc_mcontext.gregs[REG_RSI],
          (unsigned long long)uc->uc_mcontext.gregs[REG_RDX], (unsigned long long)uc->uc_mcontext.gregs[REG_RCX],
          (unsigned long long)uc->uc_mcontext.gregs[REG_RAX], (unsigned long long)uc->uc_mcontext.gregs[REG_RSP]);
  report_maps(pc, addr);
  void* bt[64];
  int n = backtrace(bt, 64);
  fprintf(stderr, "[segv] backtrace (%d frames):\n", n);
  for (int i = 0; i < n; ++i) {
    Dl_info d;
    if (dladdr(bt[i], &d) && d.dli_fname)
      fprintf(stderr, "[segv]   #%d %p %s +0x%lx %s\n", i, bt[i], d.dli_fname,
              (unsigned long)((uintptr_t)bt[i] - (uintptr_t)d.dli_fbase), d.dli_sname ? d.dli_sname : "?");
    else
      fprintf(stderr, "[segv]   #%d %p\n", i, bt[i]);
  }
  fflush(stderr);
  signal(sig, SIG_DFL);
  raise(sig);
}

int segv_report_install(void) {
  struct sigaction sa;
  memset(&sa, 0, sizeof sa);
  sa.sa_sigaction = handler;
  sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
  sigemptyset(&sa.sa_mask);
  return sigaction(SIGSEGV, &sa, NULL) | sigaction(SIGBUS, &sa, NULL);
}
