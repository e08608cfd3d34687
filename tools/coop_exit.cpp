// coop_exit: where a process that made cooperative launches (lv_persist)
// faults at exit under rocprofv3. Checks C5 once through the C
// ABI, releases everything, then returns from main; each teardown stage is
// printed, and a SIGSEGV handler prints the faulting address and the native
// backtrace (with the shared object of every frame).
//   hipcc -O1 -g -I include tools/coop_exit.cpp -o tools/coop_exit \
//     -L s2_verification_amd -ls2lincheck -Wl,-rpath,$PWD/s2_verification_amd
//   rocprofv3 --kernel-trace --stats -d gpurun_out/ce -- tools/coop_exit [plain|reset]
#include <dlfcn.h>
#include <execinfo.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <hip/hip_runtime_api.h>

#include "s2lincheck.h"

static void on_segv(int sig, siginfo_t* si, void*) {
  char msg[128];
  const int n = snprintf(msg, sizeof msg, "coop_exit: signal %d at address %p\n", sig, si->si_addr);
  write(2, msg, n);
  void* fr[64];
  const int k = backtrace(fr, 64);
  for (int i = 0; i < k; ++i) {
    Dl_info di;
    char line[512];
    int m;
    if (dladdr(fr[i], &di) && di.dli_fname) {
      m = snprintf(line, sizeof line, "  #%d %p %s+0x%lx (%s)\n", i, fr[i], di.dli_sname ? di.dli_sname : "?",
                   (unsigned long)((char*)fr[i] - (char*)(di.dli_saddr ? di.dli_saddr : di.dli_fbase)),
                   di.dli_fname);
    } else {
      m = snprintf(line, sizeof line, "  #%d %p\n", i, fr[i]);
    }
    write(2, line, m);
  }
  _exit(128 + sig);
}

static void at_exit_mark() { fprintf(stderr, "coop_exit: atexit handlers running\n"); }

int main(int argc, char** argv) {
  struct sigaction sa;
  memset(&sa, 0, sizeof sa);
  sa.sa_sigaction = on_segv;
  sa.sa_flags = SA_SIGINFO;
  sigaction(SIGSEGV, &sa, nullptr);
  sigaction(SIGBUS, &sa, nullptr);
  atexit(at_exit_mark);
  const bool reset = argc > 1 && !strcmp(argv[1], "reset");
  if (argc > 1 && !strcmp(argv[1], "plain")) setenv("S2LC_PERSIST_PLAIN", "1", 1);
  s2lc_sim_params sp;
  s2lc_sim_params_default(&sp);
  sp.workflow = S2LC_WF_REGULAR;  // C5 (workloads.py)
  sp.num_clients = 32;
  sp.ops_per_client = 1000;
  sp.seed = 5;
  sp.max_client_ids = 1u << 20;
  sp.p_indefinite = 0.03;
  sp.p_definite = 0.02;
  sp.p_read_failure = 0.01;
  sp.p_check_tail_failure = 0.01;
  s2lc_history* h = nullptr;
  if (s2lc_simulate_history(&sp, &h)) return 2;
  s2lc_opts o;
  memset(&o, 0, sizeof o);
  o.struct_size = sizeof o;
  o.device = -1;
  int st = 0;
  s2lc_ctx* c = s2lc_create(&o, &st);
  if (!c) return 3;
  s2lc_result r;
  memset(&r, 0, sizeof r);
  const int rc = s2lc_check(c, h, &r);
  fprintf(stderr, "coop_exit: check rc %d verdict %d rounds %u device_ms %.2f\n", rc, r.verdict, r.rounds,
          r.device_ms);
  s2lc_result_free(&r);
  s2lc_destroy(c);
  fprintf(stderr, "coop_exit: context destroyed\n");
  s2lc_history_free(h);
  if (reset) {
    (void)hipDeviceReset();
    fprintf(stderr, "coop_exit: device reset\n");
  }
  fprintf(stderr, "coop_exit: returning from main\n");
  return rc ? 4 : 0;
}
