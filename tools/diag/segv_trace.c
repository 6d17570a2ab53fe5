/* Diagnostics only (never loaded by the product): a SIGSEGV/SIGFPE/SIGBUS handler that
   prints the native backtrace (addresses + nearest exported symbol) to stderr and then
   re-raises with the default action.  Loaded with ctypes by tools/rp_exit.py. */
#define _GNU_SOURCE
#include <execinfo.h>
#include <signal.h>
#include <string.h>
#include <unistd.h>

static void on_fault(int sig) {
  void* frames[64];
  const char msg[] = "\n[segv_trace] fatal signal, native backtrace:\n";
  write(2, msg, sizeof(msg) - 1);
  int n = backtrace(frames, 64);
  backtrace_symbols_fd(frames, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}

int segv_trace_install(void) {
  struct sigaction sa;
  memset(&sa, 0, sizeof(sa));
  sa.sa_handler = on_fault;
  sigemptyset(&sa.sa_mask);
  sa.sa_flags = SA_RESETHAND;
  return sigaction(SIGSEGV, &sa, 0) | sigaction(SIGFPE, &sa, 0) | sigaction(SIGBUS, &sa, 0);
}
