/* SIGSEGV / SIGBUS diagnostics for a host crash whose stack is unsymbolised (the
 * kriging leg under rocprofv3 --pmc).  Loaded by ctypes (bench_kriging.py, MK_SEGV_DIAG=<path>);
 * segv_diag_install(path) installs a handler that appends to <path>: the fault address, the faulting
 * thread, the PC and every backtrace frame resolved with dladdr (object, symbol, offsets), and
 * /proc/self/maps.  It then restores the previous handler and returns, so the fault repeats and the
 * earlier handler (the profiler's) reports as before.  Not async-signal-safe in general (dladdr,
 * backtrace): a one-shot diagnostic for a process that is about to die anyway.
 *
 *   gcc -O1 -g -shared -fPIC tools/segv_diag.c -o tools/segv_diag.so -ldl
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <execinfo.h>
#include <fcntl.h>
#include <signal.h>
#include <stdio.h>
#include <string.h>
#include <sys/syscall.h>
#include <ucontext.h>
#include <unistd.h>

static char g_path[512];
static struct sigaction g_old_segv, g_old_bus;

static void put(int fd, const char* s) { (void)!write(fd, s, strlen(s)); }

static void describe(int fd, const char* tag, void* pc) {
  Dl_info di;
  char line[1024];
  if (dladdr(pc, &di) && di.dli_fname) {
    snprintf(line, sizeof line, "%s %p  %s+0x%lx  (%s+0x%lx)\n", tag, pc, di.dli_fname,
             (unsigned long)((char*)pc - (char*)di.dli_fbase), di.dli_sname ? di.dli_sname : "?",
             di.dli_saddr ? (unsigned long)((char*)pc - (char*)di.dli_saddr) : 0ul);
  } else {
    snprintf(line, sizeof line, "%s %p  (no object)\n", tag, pc);
  }
  put(fd, line);
}

static void handler(int sig, siginfo_t* si, void* uc_) {
  int fd = open(g_path, O_WRONLY | O_CREAT | O_APPEND, 0644);
  if (fd >= 0) {
    char line[512];
    ucontext_t* uc = (ucontext_t*)uc_;
    void* pc = (void*)uc->uc_mcontext.gregs[REG_RIP];
    snprintf(line, sizeof line, "=== signal %d addr %p code %d pid %d tid %ld\n", sig, si->si_addr, si->si_code,
             (int)getpid(), (long)syscall(SYS_gettid));
    put(fd, line);
    describe(fd, "PC", pc);
    snprintf(line, sizeof line, "regs rdi %llx rsi %llx rdx %llx rcx %llx rax %llx rsp %llx\n",
             (unsigned long long)uc->uc_mcontext.gregs[REG_RDI], (unsigned long long)uc->uc_mcontext.gregs[REG_RSI],
             (unsigned long long)uc->uc_mcontext.gregs[REG_RDX], (unsigned long long)uc->uc_mcontext.gregs[REG_RCX],
             (unsigned long long)uc->uc_mcontext.gregs[REG_RAX], (unsigned long long)uc->uc_mcontext.gregs[REG_RSP]);
    put(fd, line);
    void* fr[64];
    int n = backtrace(fr, 64);
    for (int i = 0; i < n; ++i) {
      snprintf(line, sizeof line, "#%d", i);
      describe(fd, line, fr[i]);
    }
    put(fd, "--- /proc/self/maps\n");
    int mf = open("/proc/self/maps", O_RDONLY);
    if (mf >= 0) {
      char buf[4096];
      ssize_t r;
      while ((r = read(mf, buf, sizeof buf)) > 0) (void)!write(fd, buf, (size_t)r);
      close(mf);
    }
    close(fd);
  }
  sigaction(SIGSEGV, &g_old_segv, NULL);
  sigaction(SIGBUS, &g_old_bus, NULL);
}

int segv_diag_install(const char* path) {
  struct sigaction sa;
  memset(&sa, 0, sizeof sa);
  snprintf(g_path, sizeof g_path, "%s", path);
  sa.sa_sigaction = handler;
  sa.sa_flags = SA_SIGINFO;
  sigemptyset(&sa.sa_mask);
  if (sigaction(SIGSEGV, &sa, &g_old_segv)) return -1;
  if (sigaction(SIGBUS, &sa, &g_old_bus)) return -1;
  return 0;
}
