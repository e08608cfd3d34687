// cli.cpp — s2-porcupine: drop-in for golang/s2-porcupine/main.go:568-640.
//   -file=<path> | -file - (stdin) | -version ; exit 0 = linearizable, 1 = not
//   linearizable (or an input error), 3 = witness certification failed,
//   4 = unknown (device capacity)
//   stderr: slog-style JSON lines ("passed: is linearizable" /
//   "failed: is NOT linearizable" with res), "failed to decode history: ..."
// The check runs on the GPU through libs2lincheck (s2lc_check).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <errno.h>

#include <string>
#include <vector>

#include "s2lincheck.h"

// main.go:565-566: Version is injected at build time from golang/VERSION
// (Makefile:5-9); here from s2_verification_amd/VERSION by the Makefile.
#ifndef S2LC_CLI_VERSION
#define S2LC_CLI_VERSION "dev"
#endif

static std::string now_rfc3339() {
  char buf[64];
  struct timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
  struct tm tm;
  localtime_r(&ts.tv_sec, &tm);
  size_t n = strftime(buf, sizeof buf, "%Y-%m-%dT%H:%M:%S", &tm);
  snprintf(buf + n, sizeof buf - n, ".%06ld", ts.tv_nsec / 1000);
  n = strlen(buf);
  strftime(buf + n, sizeof buf - n, "%z", &tm);
  std::string s(buf);
  if (s.size() >= 5) s.insert(s.size() - 2, ":");
  return s;
}

static std::string jstr(const std::string& s) {
  std::string o = "\"";
  for (char c : s) {
    if (c == '"' || c == '\\') { o += '\\'; o += c; }
    else if ((unsigned char)c < 0x20) { char b[8]; snprintf(b, sizeof b, "\\u%04x", c); o += b; }
    else o += c;
  }
  return o + "\"";
}

static void slog(const char* level, const std::string& msg, const std::string& extra = "") {
  fprintf(stderr, "{\"time\":%s,\"level\":\"%s\",\"msg\":%s%s}\n", jstr(now_rfc3339()).c_str(), level,
          jstr(msg).c_str(), extra.c_str());
}

// S2LC_CLI_TIMING=1: one stderr line with the process's phases (ms since start)
static double ms_since(const struct timespec& t0) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return 1e3 * (double)(t.tv_sec - t0.tv_sec) + 1e-6 * (double)(t.tv_nsec - t0.tv_nsec);
}

int main(int argc, char** argv) {
  struct timespec t_start;
  clock_gettime(CLOCK_MONOTONIC, &t_start);
  const bool timing = getenv("S2LC_CLI_TIMING") != nullptr;
  double t_load = 0, t_ctx = 0, t_check = 0, t_viz = 0;
  const char* file = nullptr;
  bool version = false;
  for (int i = 1; i < argc; ++i) {  // Go flag syntax: -flag, --flag, -flag=value, -flag value
    const char* a = argv[i];
    if (a[0] != '-') break;
    const char* n = a + 1;
    if (*n == '-') ++n;
    if (!strcmp(n, "version") || !strcmp(n, "version=true")) version = true;
    else if (!strncmp(n, "file=", 5)) file = n + 5;
    else if (!strcmp(n, "file") && i + 1 < argc) file = argv[++i];
    else if (!strcmp(n, "h") || !strcmp(n, "help")) {
      fprintf(stderr, "Usage of %s:\n  -file string\n    \tpath to JSONL records file (use '-' for stdin)\n  -version\n    \tshow version information\n", argv[0]);
      return 0;
    } else {
      fprintf(stderr, "flag provided but not defined: %s\n", a);
      return 2;
    }
  }
  if (version) {
    printf("s2-porcupine version %s\n", S2LC_CLI_VERSION);
    return 0;
  }
  if (!file || !*file) {
    fprintf(stderr, "usage: %s -file=records-<epoch>.jsonl\n", argv[0]);
    return 1;
  }
  char err[1024] = {0};
  s2lc_history* h = nullptr;
  int rc = s2lc_load_jsonl(file, nullptr, 0, &h, err, sizeof err);
  if (rc == S2LC_EIO) {
    slog("ERROR", "open file", ",\"path\":" + jstr(file) + ",\"err\":" + jstr(err));
    return 1;
  }
  if (rc) {
    fprintf(stderr, "failed to decode history: %s\n", err);
    return 1;
  }
  t_load = ms_since(t_start);
  s2lc_opts o;
  memset(&o, 0, sizeof o);
  o.struct_size = sizeof o;
  o.device = -1;
  int st = 0;
  s2lc_ctx* ctx = s2lc_create(&o, &st);
  if (!ctx) {
    fprintf(stderr, "s2-porcupine: no usable GPU (status %d)\n", st);
    s2lc_history_free(h);
    return 1;
  }
  t_ctx = ms_since(t_start);
  s2lc_result r;
  memset(&r, 0, sizeof r);
  rc = s2lc_check(ctx, h, &r);
  t_check = ms_since(t_start);
  if (rc == S2LC_EWITNESS) {
    // the GPU found a linearization that failed CPU-model certification: a
    // checker bug, never a verdict (exit 3, distinct from 0 / 1)
    slog("ERROR", "failed: witness certification", ",\"err\":" + jstr(s2lc_last_error(ctx)));
    s2lc_result_free(&r);
    s2lc_destroy(ctx);
    s2lc_history_free(h);
    return 3;
  }
  if (rc) {
    fprintf(stderr, "s2-porcupine: check failed: %s\n", s2lc_last_error(ctx));
    s2lc_destroy(ctx);
    s2lc_history_free(h);
    return 1;
  }
  // main.go:608-631: ./porcupine-outputs/<input base>-<random>.html (stdin-*.html)
  if (mkdir("./porcupine-outputs", 0755) != 0 && errno != EEXIST)
    slog("ERROR", "failed to create visualizations directory", ",\"err\":" + jstr(strerror(errno)));
  {
    std::string base = "stdin";
    if (strcmp(file, "-") != 0) {
      base = file;
      const size_t sl = base.find_last_of('/');
      if (sl != std::string::npos) base = base.substr(sl + 1);
      const size_t dot = base.find_last_of('.');
      if (dot != std::string::npos && dot > 0) base = base.substr(0, dot);
    }
    std::string tmpl = "porcupine-outputs/" + base + "-XXXXXX.html";
    std::vector<char> path(tmpl.begin(), tmpl.end());
    path.push_back(0);
    const int fd = mkstemps(path.data(), 5);
    if (fd < 0) {
      slog("ERROR", "failed to create temp file", ",\"err\":" + jstr(strerror(errno)));
    } else {
      close(fd);
      // Illegal: porcupine's LinearizationInfo (the longest partial
      // linearization containing each op) for the page, as main.go:606-627
      s2lc_partials info;
      memset(&info, 0, sizeof info);
      const bool have_info = r.verdict == S2LC_ILLEGAL && s2lc_check_partials(ctx, h, &info) == 0;
      if (s2lc_visualize_info(h, &r, have_info ? &info : nullptr, path.data()) != 0)
        slog("ERROR", "failed to visualize", ",\"err\":\"write\"");
      s2lc_partials_free(&info);
      slog("INFO", "wrote visualization", ",\"file\":" + jstr(path.data()));
    }
  }
  t_viz = ms_since(t_start);
  const bool ok = r.verdict == S2LC_OK;
  int code = 0;
  if (ok) {
    slog("INFO", "passed: is linearizable");
  } else if (r.verdict == S2LC_ILLEGAL) {
    // main.go:636: res is porcupine's CheckResult
    slog("ERROR", "failed: is NOT linearizable", ",\"res\":\"Illegal\"");
    code = 1;
  } else {
    // Unknown: a device capacity limit (the reference at timeout 0 never
    // returns it). Not a verdict on the history, so neither message above and
    // its own exit code (4): a DST script must not read it as a violation.
    const char* why = r.reason == S2LC_R_FRONTIER ? "frontier exceeds device capacity"
                    : r.reason == S2LC_R_TIMEOUT  ? "timeout"
                    : r.reason == S2LC_R_BUDGET   ? "budget" : "other";
    slog("ERROR", "failed: linearizability unknown",
         std::string(",\"res\":\"Unknown\",\"reason\":\"") + why + "\"");
    code = 4;
  }
  // The verdict is out and the page written: leave without tearing down the
  // HIP runtime (its exit-time teardown cost the process 70-95 ms on the
  // MI355X box, more than the check). The OS reclaims the context; Go's
  // os.Exit in main.go:636-640 likewise runs no finalizers.
  // S2LC_CLI_CLEAN_EXIT=1 frees everything and returns normally (leak checks).
  if (getenv("S2LC_CLI_CLEAN_EXIT")) {
    s2lc_result_free(&r);
    s2lc_destroy(ctx);
    s2lc_history_free(h);
  }
  if (timing)
    fprintf(stderr, "{\"cli_timing_ms\":{\"decode\":%.2f,\"create\":%.2f,\"check\":%.2f,\"viz\":%.2f,\"teardown\":%.2f,\"main\":%.2f}}\n",
            t_load, t_ctx - t_load, t_check - t_ctx, t_viz - t_check, ms_since(t_start) - t_viz, ms_since(t_start));
  if (getenv("S2LC_CLI_CLEAN_EXIT")) return code;
  fflush(stdout);
  fflush(stderr);
  _exit(code);
}
