/* exit_hook: lets a profiled process that made cooperative launches end
 * without running the HIP runtime's library destructor.
 *
 * Under rocprofv3, ROCm's own teardown faults at exit after any
 * hipLaunchCooperativeKernel: libamdhip64's destructor (__cxa_finalize) calls
 * into libhsa-runtime64 after the profiler's finalization. tools/coop_min.hip
 * reproduces it with no libs2lincheck code at all, and hipDeviceReset() before
 * returning does not avoid it. The profiler writes its results in its own
 * finalization, which runs before the exit handlers registered early in the
 * process; the handler registered here runs after it and ends the process
 * with _exit, so the results are complete and the faulting destructor never
 * runs. Profiling harness only (tools/c5run.py with S2LC_EXIT_HOOK=1);
 * nothing in the product loads it.
 *   gcc -O2 -shared -fPIC tools/exit_hook.c -o tools/exit_hook.so */
#include <stdlib.h>
#include <unistd.h>

static volatile int g_code = 0;

static void exit_now(void) { _exit(g_code); }

/* register before the first HIP call (the profiler's handler is registered
 * later, so it runs first) */
int exit_hook_register(void) { return atexit(exit_now); }

/* the status the process should end with (default 0) */
void exit_hook_code(int code) { g_code = code; }
